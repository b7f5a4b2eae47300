// Four-wave MFMA GEMM for gfx950: C = A[M,K] . W[N,K]^T (both operands K-contiguous, nn.Linear layout)
// with fused epilogues.  This is the hot-path GEMM of the Gemma-2 blocks (SURVEY K3 QKV, K6 o_proj,
// K7 gate|up (+GeGLU), K8 down, K10 vocab head, K11 lens unembedding).
//
// Why four waves of 128x128 (instead of gemm.hip's eight of 128x64): the MFMA operand traffic out of LDS
// is what limits the eight-wave ping-pong kernel (its no-LDS-read lab build runs ~10 % faster,
// profiles/r2/gemm_pp/lab_knobs.txt) and, under the chip's power cap, LDS read bytes also cost clock
// (cdna_hip_programming.md §5.4 rule 28).  A 128x128 wave tile reads 2/3 of the LDS bytes per MFMA of a
// 128x64 one; its 64 fp32x4 accumulators (256 registers) live in the AGPR half of the unified 512-entry
// register file, which a one-wave-per-SIMD kernel owns entirely.
//
// Structure:
//  * 256 threads = 2 (n) x 2 (m) waves; wave (wn, wm) owns output columns wn*16*WN.. and rows wm*16*WM..
//    (WN = WM = 8: 256x256 tiles; WM = 4: 256 (n) x 128 (m) tiles for the N = 3584 projections at
//    moderate M, which would otherwise leave half the CUs idle).
//  * The MFMA row operand is W (output columns n), the column operand A (output rows m), so each lane's
//    accumulator holds 4 consecutive n of one m (8-byte bf16 stores, row-wise epilogue reductions).
//  * K is consumed in 32-deep slices (one v_mfma_f32_16x16x32_bf16 k-step).  A slice's LDS image is
//    [W rows | A rows] x 64 B; NSLOT slices are resident.  Each 16-B chunk is stored at chunk ^ 3*((row>>2)&1),
//    which makes every ds_read_b128 lane group (MI355X_MICROARCH.md §LDS: {0-3,12-15,20-27}, ...) hit 16
//    distinct 16-B slots of the bank row (exhaustively checked, tools/lab/swizzle_check.py).
//  * Software pipeline, one barrier per slice: after barrier B_s the wave issues the fragment reads of
//    slice s+1 (second register set) and the staging of slice s+NSLOT-1, then runs slice s's 64 MFMAs from
//    the first register set, so LDS latency and staging issue hide behind the MFMAs.
//    Staging is LDS-DMA (global_load_lds_dwordx4, lane-linear 1 KB per wave-instruction with the swizzle
//    applied to the global source address); counted vmcnt (never 0 while more slices are in flight) + raw
//    s_barrier.  Slice s+2 is waited for before B_{s+1}; a slot is re-staged one barrier after the MFMAs
//    that consumed its last fragment reads.  The memory instructions of a slice are spread over its MFMA
//    row-groups (W4_INTERLEAVE) so their issue cost hides behind the MFMA pipe.
//  * Block ids: XCD-aware bijective remap (T1), then GROUP_M tile rows per group so the co-resident tiles
//    of an XCD share A and W panels through its L2.
// Requirements (host-checked, tb_gemm_w4_ok): N % 256 == 0, K % 64 == 0 (an even slice count), K >= 64; any M (rows past M are
// clamped on load and masked on store).
#include "../../taboo_brittleness_amd/csrc/common.h"
#include "../../taboo_brittleness_amd/csrc/api.h"

namespace {

constexpr int W4_THREADS = 256;
#ifndef W4_GROUP_M
#define W4_GROUP_M 4
#endif
#ifndef W4_INTERLEAVE
#define W4_INTERLEAVE 1  // 1: a slice's memory instructions interleaved with its MFMA row-groups
#endif

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void g2l16(const uint16_t* src, char* dst) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)dst, 16, 0, 0);
}
__device__ __forceinline__ void w4_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
// vmcnt with a run-time (wave-uniform) count: the instruction needs a literal
__device__ __forceinline__ void w4_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int N>
__device__ __forceinline__ void w4_vmcnt_c() {
  static_assert(N == 0 || N == 6 || N == 8, "vmcnt literal");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

enum { W4_BF16 = 0, W4_F32 = 1, W4_JUMPRELU = 2, W4_GEGLU = 3, W4_HEAD = 4, W4_LENS = 5 };
constexpr int W4_HEAD_COLS = 128;       // vocab columns per head partial (one wave's n range at WN = 8)
constexpr int W4_CTAB_N = 32768;        // entries of the exact bf16 softcap table (lens.hip)

template <int WM, int WN, int NSLOT, int EPI>
__global__ void __launch_bounds__(W4_THREADS, (WM == 8 ? 1 : 2))
gemm_w4_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, void* __restrict__ C,
               const float* __restrict__ bias, const float* __restrict__ thr, int M, int N, int K, int ldc,
               const uint16_t* __restrict__ ctab, const int32_t* __restrict__ tgt, float* __restrict__ tgt_logit,
               float4* __restrict__ lpart) {
  constexpr int BN = 32 * WN, BM = 32 * WM;
  constexpr int PIMG = BN * 64, QIMG = BM * 64, SLOT = PIMG + QIMG;
  constexpr int PI = BN / 64, QI = BM / 64, GL = PI + QI;     // staging wave-instructions per wave and slice
  static_assert(EPI != W4_HEAD || NSLOT * SLOT >= 2 * W4_CTAB_N, "head epilogue stages the softcap table in LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];

  const int nbn = N / BN, nbm = (M + BM - 1) / BM, nwg = nbn * nbm;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int per_group = W4_GROUP_M * nbn, first_bm = (bid / per_group) * W4_GROUP_M;
  const int gsz = min(nbm - first_bm, W4_GROUP_M), lid = bid % per_group;
  const int bm = first_bm + lid % gsz, bn = lid / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid & 1, wm = wid >> 1;

  // ---- staging: wave-instruction q of an image covers its rows 16q .. 16q+15 (64 B each, lane-linear:
  // lane -> row 16q + lane/4, physical chunk lane%4 = logical chunk (lane%4) ^ 3*((row>>2)&1)).
  // Instruction i of this wave is q = 4i + wid.
  const int lchunk = (lane & 3) ^ (3 * ((lane >> 4) & 1));
  // uniform tile bases (SGPR) + per-lane 32-bit byte offsets, so a staging instruction is the saddr form
  const char* const wbase = reinterpret_cast<const char*>(W + (size_t)n0 * K);
  const char* const abase = reinterpret_cast<const char*>(A + (size_t)m0 * K);
  uint32_t vp[PI], vq[QI];
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    const int r = (4 * i + wid) * 16 + (lane >> 2);
    vp[i] = (uint32_t)(r * K + lchunk * 8) * 2u;
  }
#pragma unroll
  for (int i = 0; i < QI; ++i) {
    const int r = (4 * i + wid) * 16 + (lane >> 2);
    vq[i] = (uint32_t)((min(m0 + r, M - 1) - m0) * K + lchunk * 8) * 2u;
  }

  // ---- fragment reads: operand row = base + (lane&15), logical chunk lane>>4 (k = 8*(lane>>4) .. +8)
  const int co = ((lane >> 4) ^ (3 * ((lane >> 2) & 1))) << 4;
  const int offp = (wn * 16 * WN + (lane & 15)) * 64 + co;
  const int offq = PIMG + (wm * 16 * WM + (lane & 15)) * 64 + co;

  f32x4 acc[WN][WM];
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 p0[WN], q0[WM], p1[WN], q1[WM];

  const int ns = K >> 5;

  auto read_frags = [&](int slot, bf16x8* pf, bf16x8* qf) {
    const char* b = smem + slot * SLOT;
#pragma unroll
    for (int i = 0; i < WN; ++i) pf[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(b + offp + i * 1024));
#pragma unroll
    for (int j = 0; j < WM; ++j) qf[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(b + offq + j * 1024));
  };
  auto mfmas = [&](const bf16x8* pf, const bf16x8* qf) {
#pragma unroll
    for (int i = 0; i < WN; ++i)
#pragma unroll
      for (int j = 0; j < WM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[i], qf[j], acc[i][j], 0, 0, 0);
  };

  // staging of slice s into slot: wave-instruction g < PI fills W-image rows, g >= PI A-image rows
  auto stage_one = [&](int g, int s, int slot) {
    char* d = smem + slot * SLOT + wid * 1024;
    const int kb = s * 64;                 // byte offset of the slice in a row
    if (g < PI) g2l16(reinterpret_cast<const uint16_t*>(wbase + kb + vp[g]), d + g * 4096);
    else g2l16(reinterpret_cast<const uint16_t*>(abase + kb + vq[g - PI]), d + PIMG + (g - PI) * 4096);
  };
  const int pre = min(ns, NSLOT - 1);
  for (int s = 0; s < pre; ++s) {
#pragma unroll
    for (int g = 0; g < GL; ++g) stage_one(g, s, s);
  }
  w4_vmcnt((pre - 1) * GL);            // slice 0 landed
  w4_bar();
  read_frags(0, p0, q0);
  w4_vmcnt(max(0, pre - 2) * GL);      // slice 1 landed
  w4_bar();
  // One slice = one basic block: the next slice's fragment reads, the staging of slice s+NSLOT-1 (past the
  // end: the last slice again, into the free slot, so no branch splits the block) and this slice's MFMAs,
  // interleaved by sched_group_barrier so each memory instruction issues in the shadow of MFMAs.
#define W4_STEP(PC, QC, PN, QN)                                                                        \
  {                                                                                                    \
    const int ss = min(s + NSLOT - 1, ns - 1), sl = (s + NSLOT - 1) % NSLOT;                           \
    read_frags((s + 1) % NSLOT, PN, QN);                                                               \
    _Pragma("unroll") for (int g = 0; g < GL; ++g) stage_one(g, ss, sl);                               \
    mfmas(PC, QC);                                                                                     \
    if (W4_INTERLEAVE) {                                                                               \
      _Pragma("unroll") for (int g = 0; g < WN; ++g) {                                                 \
        __builtin_amdgcn_sched_group_barrier(0x008, WM / 2, 0);                                        \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                             \
        __builtin_amdgcn_sched_group_barrier(0x008, WM / 2, 0);                                        \
        if (g < WM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                 \
        if (g < GL) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);                                 \
      }                                                                                                \
    }                                                                                                  \
    w4_vmcnt_c<(NSLOT - 3) * GL>();                                                                    \
    w4_bar();                                                                                          \
  }
  for (int s = 0; s < ns; ++s) {       // ns is even (host-checked)
    W4_STEP(p0, q0, p1, q1);
    ++s;
    W4_STEP(p1, q1, p0, q0);
  }
#undef W4_STEP
  w4_vmcnt(0);                         // the past-the-end re-stagings
  __syncthreads();

  // ---- epilogue.  acc[i][j][r]: n = n0 + wn*16*WN + i*16 + 4*(lane>>4) + r, m = m0 + wm*16*WM + j*16 + (lane&15)
  const int nb = n0 + wn * 16 * WN + 4 * (lane >> 4);
  const int mb = m0 + wm * 16 * WM + (lane & 15);
  if constexpr (EPI == W4_HEAD || EPI == W4_LENS) {
    static_assert(WN == 8, "head partials cover one wave's 128 columns");
    // Vocab head: bf16 logits (acc rounded like a bf16 GEMM output), then the exact bf16
    // final softcap by table (staged into the idle staging LDS), reduced per (row, 128-column wave slice) to
    // {max, sum exp(z - max), first argmax}; the row's teacher-target logit is written by the lane holding it.
    // Lens (K11): no softcap; the bf16 logits are stored and the same partials go to lpart.
    const uint16_t* ct = nullptr;
    if constexpr (EPI == W4_HEAD) {
      uint16_t* ctw = reinterpret_cast<uint16_t*>(smem);
      if (ctab != nullptr) {
        for (int i = tid; i < W4_CTAB_N / 8; i += W4_THREADS)
          reinterpret_cast<uint4*>(ctw)[i] = reinterpret_cast<const uint4*>(ctab)[i];
        ct = ctw;
      }
      __syncthreads();
    }
    float4* part = EPI == W4_HEAD ? reinterpret_cast<float4*>(C) : lpart;
    const int npart = N / W4_HEAD_COLS, pcol = (n0 + wn * 128) / W4_HEAD_COLS;
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      const int m = mb + j * 16;
      const int t = (tgt != nullptr && m < M) ? tgt[m] : -1;
      float z[WN * 4];
      float mx = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int i = 0; i < WN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t b = f2bf(acc[i][j][r]);
          const float v = ct != nullptr ? __uint_as_float(((uint32_t)ct[b & 0x7fffu] | (b & 0x8000u)) << 16)
                                        : __uint_as_float(b << 16);
          const int n = nb + i * 16 + r;
          z[i * 4 + r] = v;
          if (v > mx || (v == mx && n < bi)) { mx = v; bi = n; }
          if (EPI == W4_HEAD && n == t) tgt_logit[m] = v;
        }
      if constexpr (EPI == W4_LENS) {
        if (m < M) {
#pragma unroll
          for (int i = 0; i < WN; ++i)
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + (size_t)m * ldc + nb + i * 16) =
                make_uint2(pack2(z[4 * i], z[4 * i + 1]), pack2(z[4 * i + 2], z[4 * i + 3]));
        }
      }
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < WN * 4; ++e) s += __expf(z[e] - mx);
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {
        const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(s, o, 64);
        const int i2 = __shfl_xor(bi, o, 64);
        if (m2 > mx) { s = s * __expf(mx - m2) + s2; mx = m2; bi = i2; }
        else if (m2 == mx) { s += s2; bi = min(bi, i2); }
        else { s += s2 * __expf(m2 - mx); }
      }
      if (lane < 16 && m < M) part[(size_t)m * npart + pcol] = make_float4(mx, s, __int_as_float(bi), 0.f);
    }
  } else if constexpr (EPI == W4_GEGLU) {
    // W rows interleaved per wave (ops.geglu_interleave_index): frags 0..WN/2-1 are the gate rows of features
    // f0 .. f0+63, frags WN/2.. the up rows of the same features; gate|up are rounded to bf16 first so the
    // result equals geglu(bf16 gate|up GEMM output).
    static_assert(WN == 8, "GeGLU interleave is 64 features per wave");
    uint16_t* out = reinterpret_cast<uint16_t*>(C);
    const int fb = (n0 >> 1) + wn * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      const int m = mb + j * 16;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < WN / 2; ++i) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = rbf(acc[i][j][r]), u = rbf(acc[i + WN / 2][j][r]);
          o[r] = rbf(gelu_tanh_fast(gt)) * u;
        }
        *reinterpret_cast<uint2*>(out + (size_t)m * ldc + fb + i * 16) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < WN; ++i) {
      const int n = nb + i * 16;
      float4 bn_ = make_float4(0.f, 0.f, 0.f, 0.f), th = bn_;
      if constexpr (EPI == W4_JUMPRELU) {
        if (bias) bn_ = *reinterpret_cast<const float4*>(bias + n);
        if (thr) th = *reinterpret_cast<const float4*>(thr + n);
      }
#pragma unroll
      for (int j = 0; j < WM; ++j) {
        const int m = mb + j * 16;
        if (m >= M) continue;
        const f32x4 v = acc[i][j];
        if constexpr (EPI == W4_BF16) {
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + (size_t)m * ldc + n) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        } else if constexpr (EPI == W4_F32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          const float a0 = v[0] + bn_.x, a1 = v[1] + bn_.y, a2 = v[2] + bn_.z, a3 = v[3] + bn_.w;
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) =
              make_float4(a0 > th.x ? a0 : 0.f, a1 > th.y ? a1 : 0.f, a2 > th.z ? a2 : 0.f, a3 > th.w ? a3 : 0.f);
        }
      }
    }
  }
}

// Fold a row's N/128 head / lens partials: lse, first argmax and the NLLs (greedy token, optional teacher
// target); each output pointer may be null.
__global__ void __launch_bounds__(256) w4_head_merge_kernel(const float4* __restrict__ part, int npart,
                                                            const int32_t* __restrict__ tgt,
                                                            const float* __restrict__ tgt_logit,
                                                            int32_t* __restrict__ nxt, float* __restrict__ nll_self,
                                                            float* __restrict__ nll_tgt, float* __restrict__ lse_out,
                                                            int V) {
  __shared__ float sm[4], ss[4];
  __shared__ int si[4];
  const int r = blockIdx.x;
  const float4* p = part + (size_t)r * npart;
  float mx = -INFINITY, s = 0.f;
  int bi = 0x7fffffff;
  auto merge = [&](float m2, float s2, int i2) {
    if (m2 > mx) { s = (mx == -INFINITY ? 0.f : s * __expf(mx - m2)) + s2; mx = m2; bi = i2; }
    else if (m2 == mx) { s += s2; bi = min(bi, i2); }
    else if (m2 != -INFINITY) { s += s2 * __expf(m2 - mx); }
  };
  for (int c = threadIdx.x; c < npart; c += blockDim.x) {
    const float4 q = p[c];
    merge(q.x, q.y, __float_as_int(q.z));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(s, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    merge(m2, s2, i2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = mx; ss[wid] = s; si[wid] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = sm[0]; s = ss[0]; bi = si[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) merge(sm[w], ss[w], si[w]);
    const float lse = mx + __logf(s);
    if (lse_out != nullptr) lse_out[r] = lse;
    if (nxt != nullptr) nxt[r] = bi;
    if (nll_self != nullptr) nll_self[r] = lse - mx;
    if (nll_tgt != nullptr) {
      const int t = tgt != nullptr ? tgt[r] : -1;
      nll_tgt[r] = (t >= 0 && t < V) ? lse - tgt_logit[r] : 0.f;
    }
  }
}

// variant -> tile.  0: 256x256, 4 slices resident; 1: 256x256, 3 slices resident; 2: 256 (n) x 128 (m), 3 slices
// resident (two workgroups per CU fit in LDS and registers)
template <int EPI>
void w4_launch(int variant, const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr,
               int M, int N, int K, int ldc, const uint16_t* ctab, const int32_t* tgt, float* tgt_logit,
               float4* lpart, hipStream_t st) {
  const int bm = variant == 2 ? 128 : 256;
  const int nwg = (N / 256) * ((M + bm - 1) / bm);
#define W4_GO(WM_, NS_)                                                                                           \
  hipLaunchKernelGGL((gemm_w4_kernel<WM_, 8, NS_, EPI>), dim3(nwg), dim3(W4_THREADS), 0, st, A, W, C, bias,       \
                     thr, M, N, K, ldc, ctab, tgt, tgt_logit, lpart)
  if (variant == 2) W4_GO(4, 3);
  else if (variant == 1) W4_GO(8, 3);
  else W4_GO(8, 4);
#undef W4_GO
}

}  // namespace

bool tb_gemm_w4_ok(int M, int N, int K) { return M > 0 && N > 0 && N % 256 == 0 && K >= 64 && K % 64 == 0; }

void tb_gemm_w4(const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr, int M, int N,
                int K, int ldc, int epi, int variant, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  switch (epi) {
    case W4_BF16: w4_launch<W4_BF16>(variant, A, W, C, nullptr, nullptr, M, N, K, ldc, nullptr, nullptr, nullptr, nullptr, st); break;
    case W4_F32: w4_launch<W4_F32>(variant, A, W, C, nullptr, nullptr, M, N, K, ldc, nullptr, nullptr, nullptr, nullptr, st); break;
    case W4_JUMPRELU: w4_launch<W4_JUMPRELU>(variant, A, W, C, bias, thr, M, N, K, ldc, nullptr, nullptr, nullptr, nullptr, st); break;
    default: w4_launch<W4_GEGLU>(variant, A, W, C, nullptr, nullptr, M, N, K, ldc, nullptr, nullptr, nullptr, nullptr, st);
  }
}

void tb_head_w4(const uint16_t* A, const uint16_t* W, float* part, const uint16_t* ctab, const int32_t* tgt,
                float* tgt_logit, int32_t* nxt, float* nll_self, float* nll_tgt, int M, int N, int K, int variant,
                hipStream_t st) {
  if (M <= 0) return;
  w4_launch<W4_HEAD>(variant, A, W, part, nullptr, nullptr, M, N, K, 0, ctab, tgt, tgt_logit,
                     nullptr, st);
  hipLaunchKernelGGL(w4_head_merge_kernel, dim3(M), dim3(256), 0, st, reinterpret_cast<const float4*>(part),
                     N / W4_HEAD_COLS, tgt, tgt_logit, nxt, nll_self, nll_tgt, nullptr, N);
}

void tb_lens_w4(const uint16_t* A, const uint16_t* W, uint16_t* logits, float* part, float* lse, int M, int N, int K,
                int variant, hipStream_t st) {
  if (M <= 0) return;
  w4_launch<W4_LENS>(variant, A, W, logits, nullptr, nullptr, M, N, K, N, nullptr, nullptr,
                     nullptr, reinterpret_cast<float4*>(part), st);
  hipLaunchKernelGGL(w4_head_merge_kernel, dim3(M), dim3(256), 0, st, reinterpret_cast<const float4*>(part),
                     N / W4_HEAD_COLS, nullptr, nullptr, nullptr, nullptr, nullptr, lse, N);
}
