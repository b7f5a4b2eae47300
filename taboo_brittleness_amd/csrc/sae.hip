// SAE and low-rank residual edits.
//
//  gemm_nt_epi      C = A[M,K] . W[N,K]^T on v_mfma_f32_16x16x32_bf16, LDS-tiled
//                   (128x128x64 block tile, 2x2 waves of 64x64, register-staged
//                   double buffer in 2 x (128+128) x 72 bf16 = 72 KB of static LDS --
//                   assumes gfx950's 160 KB LDS, above the 64 KB of older CDNA parts;
//                   K % 64 == 32 is handled by zero-filled chunks, so K % 32 == 0),
//                   with fused epilogues: bf16 store, fp32 store, or Gemma-Scope
//                   JumpReLU (a = pre * [pre > theta], pre = acc + b_enc; strict
//                   '>' as sae_lens).  Used for the dense SAE encode.
//  lowrank_edit     per flagged row:  c_j = f(<h - pre_bias, E_j> + bias_j) * alpha,
//                   h -= sum_j c_j D_j, then x_next = RMSNorm(h) for the next
//                   block.  With E = W_enc^T rows, D = W_dec rows, f = JumpReLU
//                   it is the error-preserving SAE latent ablation (EP:126; only the
//                   m ablated latents are ever encoded); with E = D = U rows,
//                   f = id it is the projection-out x - U U^T x (EP:148).
//  sae_decode_sparse  x_hat = sum_{a_j != 0} a_j W_dec[j] + b_dec (L0 ~ 76 of 16k)
//  latent_score     score_j = mean_{t in spikes} a_j(t) * max(0, corr_t(a_j, p_secret))
//                   per prompt segment (EP:118-124).
#include "common.h"
#include "api.h"

namespace {

constexpr int GBM = 128, GBN = 128, GBK = 64, GLDS = 72;   // padded LDS row (bf16 elements)
constexpr int GCPR = GBK / 8;                               // 16-B chunks per tile row

__device__ __forceinline__ bf16x8 as_bf16x8(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }

template <int EPI>
__global__ void __launch_bounds__(256) gemm_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                      void* __restrict__ C, const float* __restrict__ bias,
                                                      const float* __restrict__ thr, int M, int N, int K, int ldc) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2][(GBM + GBN) * GLDS];
  // XCD-aware bijective remap of the linear block id (speed only).
  const int nbn = (N + GBN - 1) / GBN, nbm = (M + GBM - 1) / GBM, nwg = nbn * nbm;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int bn = bid % nbn, bm = bid / nbn;
  const int m0 = bm * GBM, n0 = bn * GBN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int grp = lane >> 4, col = lane & 15;

  // staging: each operand tile is 128 rows x 8 chunks (16 B) = 1024 chunks, 4 per thread; chunks past K
  // (K % 64 == 32) are zero-filled, so any K % 32 == 0 works
  auto load_tile = [&](int k0, uint4 (&ra)[4], uint4 (&rw)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int id = tid + c * 256, row = id / GCPR, kk = k0 + (id % GCPR) * 8;
      const int ar = m0 + row, wr = n0 + row;
      ra[c] = (ar < M && kk < K) ? *reinterpret_cast<const uint4*>(A + (size_t)ar * K + kk) : make_uint4(0, 0, 0, 0);
      rw[c] = (wr < N && kk < K) ? *reinterpret_cast<const uint4*>(W + (size_t)wr * K + kk) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int buf, const uint4 (&ra)[4], const uint4 (&rw)[4]) {
    uint16_t* la = lds[buf];
    uint16_t* lw = lds[buf] + GBM * GLDS;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int id = tid + c * 256, off = (id / GCPR) * GLDS + (id % GCPR) * 8;
      *reinterpret_cast<uint4*>(la + off) = ra[c];
      *reinterpret_cast<uint4*>(lw + off) = rw[c];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rw[4];
  load_tile(0, ra, rw);
  store_tile(0, ra, rw);
  __syncthreads();
  const int nk = (K + GBK - 1) / GBK;
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile((kt + 1) * GBK, ra, rw);
    const uint16_t* la = lds[cur];
    const uint16_t* lw = lds[cur] + GBM * GLDS;
#pragma unroll
    for (int ks = 0; ks < GBK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = as_bf16x8(*reinterpret_cast<const uint4*>(la + (wm * 64 + i * 16 + col) * GLDS + ks * 32 + grp * 8));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = as_bf16x8(*reinterpret_cast<const uint4*>(lw + (wn * 64 + j * 16 + col) * GLDS + ks * 32 + grp * 8));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1, ra, rw);
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: C layout row = 4*grp + r, col = lane&15 inside each 16x16 tile
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + col;
      if (n >= N) continue;
      float bn_ = 0.f, th = 0.f;
      if (EPI == 2) { bn_ = bias ? bias[n] : 0.f; th = thr ? thr[n] : 0.f; }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * grp + r;
        if (m >= M) continue;
        float v = acc[i][j][r];
        if (EPI == 0) {
          reinterpret_cast<uint16_t*>(C)[(size_t)m * ldc + n] = f2bf(v);
        } else if (EPI == 1) {
          reinterpret_cast<float*>(C)[(size_t)m * ldc + n] = v;
        } else {
          v += bn_;
          reinterpret_cast<float*>(C)[(size_t)m * ldc + n] = (v > th) ? v : 0.f;
        }
      }
    }
}

// ---------------------------------------------------------------- low-rank edit
template <typename TT>
__device__ __forceinline__ void load8(const TT* p, float* f);
template <>
__device__ __forceinline__ void load8<uint16_t>(const uint16_t* p, float* f) {
  unpack8(*reinterpret_cast<const uint4*>(p), f);
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// One workgroup (256 threads) per row; D <= 256*8*VPT.
template <typename TT, int VPT>
__global__ void __launch_bounds__(256) lowrank_edit_kernel(
    uint16_t* __restrict__ h, uint16_t* __restrict__ x_next, const uint8_t* __restrict__ apply,
    const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt, int mmax, const TT* __restrict__ E,
    const TT* __restrict__ Dm, const float* __restrict__ bias, const float* __restrict__ thr,
    const float* __restrict__ pre_bias, float alpha, const uint16_t* __restrict__ w_next, float eps, int D,
    float* __restrict__ coef_out) {
  const int row = blockIdx.x;
  if (!apply[row]) return;
  __shared__ float red[16];
  __shared__ float coef[256];
  const int nvec = D >> 3;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint16_t* hr = h + (size_t)row * D;
  float v[VPT][8];
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = tid + s * 256;
    if (i < nvec) unpack8(reinterpret_cast<const uint4*>(hr)[i], v[s]);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = 0.f;
  }
  const int m = min(cnt[row], min(mmax, 256));
  const int32_t* ir = idx + (size_t)row * mmax;
  // coefficients: waves split the m directions, lanes split D
  for (int j = wid; j < m; j += 4) {
    const int e = ir[j];
    const TT* er = E + (size_t)e * D;
    float part = 0.f;
    for (int c = lane; c < nvec; c += 64) {
      float ef[8], hf[8];
      load8<TT>(er + c * 8, ef);
      unpack8(reinterpret_cast<const uint4*>(hr)[c], hf);
      if (pre_bias) {
#pragma unroll
        for (int q = 0; q < 8; ++q) hf[q] -= pre_bias[c * 8 + q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) part += hf[q] * ef[q];
    }
    part = wave_sum(part);
    if (lane == 0) {
      float pre = part + (bias ? bias[e] : 0.f);
      float a = pre;
      if (thr) a = (pre > thr[e]) ? pre : 0.f;
      coef[j] = alpha * a;
      if (coef_out) coef_out[(size_t)row * mmax + j] = a;
    }
  }
  __syncthreads();
  // an all-zero edit (every ablated latent below its threshold here, or alpha = 0) is an exact no-op: h and
  // x_next stay bit-identical to the unedited forward (no re-rounded h, no re-normalised x)
  bool any = false;
  for (int j = 0; j < m; ++j) any |= coef[j] != 0.f;
  if (!any) return;
  for (int j = 0; j < m; ++j) {
    const float cj = coef[j];
    if (cj == 0.f) continue;
    const TT* dr = Dm + (size_t)ir[j] * D;
#pragma unroll
    for (int s = 0; s < VPT; ++s) {
      const int i = tid + s * 256;
      if (i < nvec) {
        float df[8];
        load8<TT>(dr + i * 8, df);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[s][q] -= cj * df[q];
      }
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = tid + s * 256;
    if (i < nvec) {
#pragma unroll
      for (int q = 0; q < 8; ++q) { v[s][q] = rbf(v[s][q]); ss += v[s][q] * v[s][q]; }
      reinterpret_cast<uint4*>(hr)[i] = pack8(v[s]);
    }
  }
  if (x_next == nullptr) return;
  const float r = rsqrtf(block_sum(ss, red) / (float)D + eps);
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = tid + s * 256;
    if (i < nvec) {
      float wf[8], o[8];
      unpack8(reinterpret_cast<const uint4*>(w_next)[i], wf);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = v[s][q] * r * (1.f + wf[q]);
      reinterpret_cast<uint4*>(x_next + (size_t)row * D)[i] = pack8(o);
    }
  }
}

// ------------------------------------------------------------- sparse decode
template <typename TT>   // decoder table: bf16 (uint16_t) or fp32 (the Gemma Scope dtype, default)
__global__ void __launch_bounds__(256) sae_decode_sparse_kernel(const float* __restrict__ acts,
                                                                const TT* __restrict__ Wdec,
                                                                const float* __restrict__ b_dec,
                                                                uint16_t* __restrict__ out_bf16,
                                                                float* __restrict__ out_f32, int L, int D) {
  __shared__ int act_idx[1024];
  __shared__ float act_val[1024];
  __shared__ int nact;
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* ar = acts + (size_t)row * L;
  if (tid == 0) nact = 0;
  __syncthreads();
  for (int j = tid; j < L; j += blockDim.x) {
    const float a = ar[j];
    if (a != 0.f) {
      const int slot = atomicAdd(&nact, 1);
      if (slot < 1024) { act_idx[slot] = j; act_val[slot] = a; }
    }
  }
  __syncthreads();
  const int nvec = D >> 3;
  if (nact > 1024) {   // dense fallback (only reachable with a badly calibrated SAE)
    for (int c = tid; c < nvec; c += blockDim.x) {
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = b_dec ? b_dec[c * 8 + q] : 0.f;
      for (int j = 0; j < L; ++j) {
        const float a = ar[j];
        if (a == 0.f) continue;
        float wf[8];
        load8<TT>(Wdec + (size_t)j * D + c * 8, wf);
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] += a * wf[q];
      }
      if (out_bf16) reinterpret_cast<uint4*>(out_bf16 + (size_t)row * D)[c] = pack8(o);
      if (out_f32) {
        float* dst = out_f32 + (size_t)row * D + c * 8;
#pragma unroll
        for (int q = 0; q < 8; ++q) dst[q] = o[q];
      }
    }
    return;
  }
  const int n = nact;
  // deterministic order: sort the (small) active list by index (odd-even transposition)
  for (int phase = 0; phase < n; ++phase) {
    for (int k = tid * 2 + (phase & 1); k + 1 < n; k += 2 * blockDim.x) {
      if (act_idx[k] > act_idx[k + 1]) {
        const int ti = act_idx[k]; act_idx[k] = act_idx[k + 1]; act_idx[k + 1] = ti;
        const float tv = act_val[k]; act_val[k] = act_val[k + 1]; act_val[k + 1] = tv;
      }
    }
    __syncthreads();
  }
  for (int c = tid; c < nvec; c += blockDim.x) {
    float o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = b_dec ? b_dec[c * 8 + q] : 0.f;
    for (int k = 0; k < n; ++k) {
      float wf[8];
      load8<TT>(Wdec + (size_t)act_idx[k] * D + c * 8, wf);
      const float a = act_val[k];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] += a * wf[q];
    }
    if (out_bf16) reinterpret_cast<uint4*>(out_bf16 + (size_t)row * D)[c] = pack8(o);
    if (out_f32) {
      float* dst = out_f32 + (size_t)row * D + c * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) dst[q] = o[q];
    }
  }
}

// ------------------------------------------------------------- latent score
// grid (ceil(L/256), G): segment g covers rows seg[g] .. seg[g+1]-1.
__global__ void __launch_bounds__(256) latent_score_kernel(const float* __restrict__ acts,
                                                           const float* __restrict__ p,
                                                           const uint8_t* __restrict__ spike,
                                                           const int32_t* __restrict__ seg, float* __restrict__ out,
                                                           float* __restrict__ spike_mean_out,
                                                           float* __restrict__ corr_out, int L) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (j >= L) return;
  const int r0 = seg[g], r1 = seg[g + 1];
  const int n = r1 - r0;
  // two passes in fp64 (means, then centred sums): the one-pass saa - sa^2/n form cancels
  // catastrophically for offset, low-variance latents (a ~ 40 +- 0.01) and could push a noisy
  // correlation into the targeted set.  n is a prompt's length, so the second read hits L2.
  double sa = 0.0, sp = 0.0, ssp = 0.0;
  int nsp = 0;
  for (int r = r0; r < r1; ++r) {
    const double a = acts[(size_t)r * L + j];
    sa += a; sp += (double)p[r];
    if (spike[r]) { ssp += a; ++nsp; }
  }
  float corr = 0.f;
  if (n > 1) {
    const double ma = sa / n, mp = sp / n;
    double va = 0.0, vp = 0.0, cov = 0.0;
    for (int r = r0; r < r1; ++r) {
      const double ac = (double)acts[(size_t)r * L + j] - ma, pc = (double)p[r] - mp;
      va += ac * ac; vp += pc * pc; cov += ac * pc;
    }
    if (va > 1e-12 && vp > 1e-20) corr = (float)(cov / sqrt(va * vp));
  }
  const float sm = nsp ? (float)(ssp / nsp) : 0.f;
  out[(size_t)g * L + j] = sm * fmaxf(corr, 0.f);
  if (spike_mean_out) spike_mean_out[(size_t)g * L + j] = sm;
  if (corr_out) corr_out[(size_t)g * L + j] = corr;
}

}  // namespace

void tb_gemm_nt(const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr, int M, int N,
                int K, int ldc, int epi, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const int nwg = ((N + GBN - 1) / GBN) * ((M + GBM - 1) / GBM);
  if (epi == 0) hipLaunchKernelGGL(gemm_nt_kernel<0>, dim3(nwg), dim3(256), 0, st, A, W, C, bias, thr, M, N, K, ldc);
  else if (epi == 1) hipLaunchKernelGGL(gemm_nt_kernel<1>, dim3(nwg), dim3(256), 0, st, A, W, C, bias, thr, M, N, K, ldc);
  else hipLaunchKernelGGL(gemm_nt_kernel<2>, dim3(nwg), dim3(256), 0, st, A, W, C, bias, thr, M, N, K, ldc);
}

void tb_lowrank_edit(uint16_t* h, uint16_t* x_next, const uint8_t* apply, const int32_t* idx, const int32_t* cnt,
                     int mmax, const void* E, const void* Dm, int table_f32, const float* bias, const float* thr,
                     const float* pre_bias, float alpha, const uint16_t* w_next, float eps, int M, int D,
                     float* coef_out, hipStream_t st) {
  if (M <= 0) return;
  const int nvec = D >> 3;
#define TB_LR(TT, VPT)                                                                                          \
  hipLaunchKernelGGL((lowrank_edit_kernel<TT, VPT>), dim3(M), dim3(256), 0, st, h, x_next, apply, idx, cnt, mmax, \
                     (const TT*)E, (const TT*)Dm, bias, thr, pre_bias, alpha, w_next, eps, D, coef_out)
  if (table_f32) {
    if (nvec <= 256) TB_LR(float, 1); else if (nvec <= 512) TB_LR(float, 2); else TB_LR(float, 4);
  } else {
    if (nvec <= 256) TB_LR(uint16_t, 1); else if (nvec <= 512) TB_LR(uint16_t, 2); else TB_LR(uint16_t, 4);
  }
#undef TB_LR
}

void tb_sae_decode_sparse(const float* acts, const void* Wdec, int table_f32, const float* b_dec, uint16_t* out_bf16,
                          float* out_f32, int M, int L, int D, hipStream_t st) {
  if (M <= 0) return;
  if (table_f32)
    hipLaunchKernelGGL(sae_decode_sparse_kernel<float>, dim3(M), dim3(256), 0, st, acts,
                       reinterpret_cast<const float*>(Wdec), b_dec, out_bf16, out_f32, L, D);
  else
    hipLaunchKernelGGL(sae_decode_sparse_kernel<uint16_t>, dim3(M), dim3(256), 0, st, acts,
                       reinterpret_cast<const uint16_t*>(Wdec), b_dec, out_bf16, out_f32, L, D);
}

void tb_latent_score(const float* acts, const float* p, const uint8_t* spike, const int32_t* seg, float* out,
                     float* spike_mean, float* corr, int G, int L, hipStream_t st) {
  if (G <= 0) return;
  dim3 grid((L + 255) / 256, G);
  hipLaunchKernelGGL(latent_score_kernel, grid, dim3(256), 0, st, acts, p, spike, seg, out, spike_mean, corr, L);
}
