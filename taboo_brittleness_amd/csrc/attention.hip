// Softcapped GQA attention over the KV cache: one kernel for
// prefill, chunked prefill and decode.
//
//   s = tanh((q.k) * scale / cap) * cap,  masked to keys j <= pos (causal) and
//   pos - j < window on sliding layers;  out = softmax(s) V.
//
// Stock flash kernels have no tanh softcap, hence this kernel.  Geometry:
//  * workgroup = (16/G query positions) x (G q-heads of one kv head) = 16 MFMA
//    rows for one sequence, 4 waves;  grid = (ceil(T/P), Hkv, B).
//  * the waves split the key range in 32-key blocks (flash-decoding inside the
//    workgroup) and merge (m, l, O) through LDS at the end.
//  * S = Q K^T on v_mfma_f32_16x16x32_bf16 with K fragments loaded straight
//    from the cache (a lane's 8 k-elements are 16 contiguous bytes of one key
//    row); online softmax on the C fragment (a row spans one 16-lane group:
//    4 xor-shuffles); P goes through a 1 KB per-wave LDS tile to become the A
//    operand; V is staged per wave in LDS (row stride HD+16 halves the
//    transposed-read bank conflicts) and read with ds_read_b64_tr_b16 as the
//    B operand (cdna_hip_programming.md T10).
// Rows with pos < 0 (padding) produce zeros.
#include <stdlib.h>

#include "common.h"
#include "api.h"

// LDS: V staging [4][32][HD+16] + P tiles [4][16][40] (bf16), then 128 floats of
// merge scalars.  The fp32 merge image [4][16][HD] reuses the staging area
// (it is smaller for HD <= 256, asserted below).
int tb_attention_lds_bytes(int HD) {
  const int VSTR = HD + 16, PSTR = 40;
  const int stage = 4 * 32 * VSTR * 2 + 4 * 16 * PSTR * 2;
  return ((stage + 128 * 4 + 15) / 16) * 16;
}

namespace {

typedef short v4i16 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i16 ds_read_tr16(const uint16_t* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(lds_ptr));
}

__device__ __forceinline__ bf16x8 as_bf16x8(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }

// The 4 waves of a workgroup split one (query block, kv head) item's key range and merge through LDS.  Prefill
// (dense [B, T]) and long packed contexts; short packed rows (the sweep's teacher-forced tails) run
// attn_tail_exact_kernel, the decode's numerics.
template <int HD, int G>
__global__ void __launch_bounds__(256) attn_cache_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    uint16_t* __restrict__ out, const int32_t* __restrict__ pos, const int32_t* __restrict__ slot, int T, int Hq,
    int Hkv, int S, float scale, float softcap, int window, const int32_t* __restrict__ blk, int bw = 3,
    const uint16_t* __restrict__ pkc = nullptr, const uint16_t* __restrict__ pvc = nullptr) {
  constexpr int P = 16 / G;        // query positions per workgroup
  constexpr int KS = HD / 32;      // MFMA k-steps over head_dim
  constexpr int DT = HD / 16;      // 16-wide output dim tiles
  constexpr int VSTR = HD + 16;    // padded LDS row (elements)
  constexpr int PSTR = 40;         // padded P row (elements)
  static_assert(4 * 16 * HD * 4 <= 4 * 32 * VSTR * 2, "merge image must fit in the staging area");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* vlds_all = reinterpret_cast<uint16_t*>(smem);                    // [4][32][VSTR]
  uint16_t* plds_all = vlds_all + 4 * 32 * VSTR;                             // [4][16][PSTR]
  float* mrg = reinterpret_cast<float*>(plds_all + 4 * 16 * PSTR);           // [4][16] m, [4][16] l

  // Row geometry: dense [B, T] layout (blk == nullptr) or a ragged block table blk[i] =
  // {first row, rows (<= P), cache slot} over packed rows (varlen prefill / teacher forcing).
  // bw = 5: blk[i] also holds (prefix slot, prefix length): keys [0, plen) are read from that slot of
  // the shared prefix cache (pkc, pvc) — the pair's baseline KV — instead of the row's own slot.
  const int kh = blockIdx.y;
  int rbase, nvalid, cs, ps = 0, np = 0;
  if (blk != nullptr) {
    rbase = blk[bw * blockIdx.x];
    nvalid = blk[bw * blockIdx.x + 1];
    cs = blk[bw * blockIdx.x + 2];
    if (bw == 5) { ps = blk[bw * blockIdx.x + 3]; np = blk[bw * blockIdx.x + 4]; }
  } else {
    const int b = blockIdx.z, t0 = blockIdx.x * P;
    rbase = b * T + t0;
    nvalid = min(P, T - t0);
    cs = slot[b];
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int grp = lane >> 4, col = lane & 15;
  const uint16_t* kbase = kc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* vbase = vc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* kpre = kbase;
  const uint16_t* vpre = vbase;
  if (np > 0) {
    kpre = pkc + ((size_t)ps * Hkv + kh) * (size_t)S * HD;
    vpre = pvc + ((size_t)ps * Hkv + kh) * (size_t)S * HD;
  }

  // --- query rows: A-layout row = col; C-layout rows = 4*grp + i
  auto row_pos = [&](int r) -> int {
    const int t = r / G;
    return (t < nvalid) ? pos[(size_t)rbase + t] : -1;
  };
  const int posA = row_pos(col);
  int posC[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) posC[i] = row_pos(4 * grp + i);

  int kmax = (int)wave_max((float)posA);   // -1 when every row is padding
  float pmin = (posA >= 0) ? (float)posA : 1e30f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pmin = fminf(pmin, __shfl_xor(pmin, o, 64));
  if (kmax >= S) kmax = S - 1;
  int kmin = 0;
  if (window > 0 && pmin < 1e29f) {
    kmin = (int)pmin - window + 1;
    if (kmin < 0) kmin = 0;
  }
  const int kstart = kmin & ~31;

  // --- Q fragments (A operand), zero for invalid rows
  bf16x8 qa[KS];
  {
    const int t = col / G, h = kh * G + (col % G);
    const uint16_t* qrow = q + (((size_t)rbase + t) * Hq + h) * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 u = {0, 0, 0, 0};
      if (posA >= 0) u = *reinterpret_cast<const uint4*>(qrow + ks * 32 + grp * 8);
      qa[ks] = as_bf16x8(u);
    }
  }

  float m_r[4], l_r[4];
  f32x4 o_acc[DT];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m_r[i] = -INFINITY; l_r[i] = 0.f; }
#pragma unroll
  for (int d = 0; d < DT; ++d) o_acc[d] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint16_t* vlds = vlds_all + wid * 32 * VSTR;
  uint16_t* plds = plds_all + wid * 16 * PSTR;
  const float inv_cap = softcap > 0.f ? 1.f / softcap : 0.f;

  for (int kb = kstart + wid * 32; kb <= kmax; kb += 4 * 32) {
    // ---- stage V block (32 keys x HD) into this wave's LDS, coalesced 1 KB per instruction
    constexpr int VCH = HD / 8;                // 16-B chunks per key row
    constexpr int VIT = 32 * VCH / 64;         // instructions per lane
    uint4 vreg[VIT];
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int c = it * 64 + lane, key = c / VCH, ch = c % VCH;
      int kk = kb + key;
      kk = kk < S ? kk : S - 1;
      vreg[it] = *reinterpret_cast<const uint4*>((kk < np ? vpre : vbase) + (size_t)kk * HD + ch * 8);
    }
    // ---- S = Q K^T for two 16-key tiles
    f32x4 sacc[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      int kk = kb + tt * 16 + col;
      kk = kk < S ? kk : S - 1;
      const uint16_t* krow = (kk < np ? kpre : kbase) + (size_t)kk * HD + grp * 8;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint4 u = *reinterpret_cast<const uint4*>(krow + ks * 32);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], as_bf16x8(u), acc, 0, 0, 0);
      }
      sacc[tt] = acc;
    }
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int c = it * 64 + lane, key = c / VCH, ch = c % VCH;
      *reinterpret_cast<uint4*>(vlds + key * VSTR + ch * 8) = vreg[it];
    }
    // ---- scale, softcap, mask, online softmax (rows 4*grp+i, keys kb + 16*tt + col)
    float pr[2][4];
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pr_pos = posC[i];
      float s0, s1;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int key = kb + tt * 16 + col;
        float s = sacc[tt][i] * scale;
        if (softcap > 0.f) s = tanhf(s * inv_cap) * softcap;
        const bool ok = pr_pos >= 0 && key <= pr_pos && key < S && (window <= 0 || pr_pos - key < window);
        s = ok ? s : -INFINITY;
        if (tt == 0) s0 = s; else s1 = s;
      }
      float mx = fmaxf(s0, s1);
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
      const float mnew = fmaxf(m_r[i], mx);
      const float a = (mnew == -INFINITY) ? 1.f : __expf(m_r[i] - mnew);
      const float p0 = (mnew == -INFINITY) ? 0.f : __expf(s0 - mnew);
      const float p1 = (mnew == -INFINITY) ? 0.f : __expf(s1 - mnew);
      // P is consumed in bf16 by the PV MFMA; sum the rounded values so l matches.
      const float p0r = rbf(p0), p1r = rbf(p1);
      float rs = p0r + p1r;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) rs += __shfl_xor(rs, o, 64);
      l_r[i] = l_r[i] * a + rs;
      m_r[i] = mnew;
      alpha[i] = a;
      pr[0][i] = p0r;
      pr[1][i] = p1r;
    }
#pragma unroll
    for (int d = 0; d < DT; ++d)
#pragma unroll
      for (int i = 0; i < 4; ++i) o_acc[d][i] *= alpha[i];
    // ---- P (C layout) -> LDS -> A layout
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 4; ++i) plds[(4 * grp + i) * PSTR + tt * 16 + col] = f2bf(pr[tt][i]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 pa_u = *reinterpret_cast<const uint4*>(plds + col * PSTR + grp * 8);
    const bf16x8 pa = as_bf16x8(pa_u);
    // ---- O += P V: B fragment = V[keys 8*grp .. +8][dim tile] via two transposed reads
    const int q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const uint16_t* a0 = vlds + (8 * grp + q4) * VSTR + d * 16 + 4 * p4;
      const v4i16 lo = ds_read_tr16(a0);
      const v4i16 hi = ds_read_tr16(a0 + 4 * VSTR);
      i16x8 vb;
      vb[0] = lo[0]; vb[1] = lo[1]; vb[2] = lo[2]; vb[3] = lo[3];
      vb[4] = hi[0]; vb[5] = hi[1]; vb[6] = hi[2]; vb[7] = hi[3];
      o_acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, __builtin_bit_cast(bf16x8, vb), o_acc[d], 0, 0, 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  // ---- merge the 4 waves: publish (m, l) and O (fp32, reusing the V staging area)
  __syncthreads();
  float* ofin = reinterpret_cast<float*>(smem);   // [4][16][HD] fp32 = 64 KB for HD=256
  if (col == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mrg[wid * 16 + 4 * grp + i] = m_r[i];
      mrg[64 + wid * 16 + 4 * grp + i] = l_r[i];
    }
  }
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 4; ++i) ofin[(wid * 16 + 4 * grp + i) * HD + d * 16 + col] = o_acc[d][i];
  __syncthreads();
  // 16 rows x HD outputs, 8 contiguous dims per thread-step
  for (int e = threadIdx.x; e < 16 * (HD / 8); e += blockDim.x) {
    const int r = e / (HD / 8), c8 = (e % (HD / 8)) * 8;
    const int t = r / G, h = kh * G + (r % G);
    if (t >= nvalid) continue;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, mrg[w * 16 + r]);
    float wsc[4], L = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float mw = mrg[w * 16 + r];
      wsc[w] = (mw == -INFINITY) ? 0.f : __expf(mw - M);
      L += wsc[w] * mrg[64 + w * 16 + r];
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    float o8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) acc += wsc[w] * ofin[(w * 16 + r) * HD + c8 + j];
      o8[j] = acc * inv;
    }
    *reinterpret_cast<uint4*>(out + (((size_t)rbase + t) * Hq + h) * HD + c8) = pack8(o8);
  }
}

// ---------------------------------------------------------------------------
// Decode (one query position per sequence): one workgroup per (sequence, kv
// head), 4 waves, low register / LDS footprint so several workgroups share a
// CU.  Phase 1: S = Q K^T on MFMA (16-key tiles, tiles strided over waves; only
// the G useful query rows of the 16-row tile are kept).  Phase 2: softmax over
// the <= S scores in LDS (one wave per head).  Phase 3: O = P V on the VALU:
// each wave takes a contiguous key range, each lane owns HD/64 output dims and
// streams V rows with 8-B loads (coalesced 512 B per key), then the four
// partial O's are summed through LDS.
template <int DPL>
struct vrow_t;
template <>
struct vrow_t<4> {
  typedef uint2 type;
  __device__ static void unpack(const uint2& w, float* f) {
    f[0] = __uint_as_float(w.x << 16); f[1] = __uint_as_float(w.x & 0xffff0000u);
    f[2] = __uint_as_float(w.y << 16); f[3] = __uint_as_float(w.y & 0xffff0000u);
  }
};
template <>
struct vrow_t<2> {
  typedef uint32_t type;
  __device__ static void unpack(const uint32_t& w, float* f) {
    f[0] = __uint_as_float(w << 16); f[1] = __uint_as_float(w & 0xffff0000u);
  }
};

template <int HD, int G>
__global__ void __launch_bounds__(256) attn_decode_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    uint16_t* __restrict__ out, const int32_t* __restrict__ pos, const int32_t* __restrict__ slot, int Hq, int Hkv,
    int S, float scale, float softcap, int window, const uint16_t* __restrict__ pkc, const uint16_t* __restrict__ pvc,
    const int32_t* __restrict__ pslot, const int32_t* __restrict__ plen) {
  constexpr int KS = HD / 32;
  constexpr int DPL = HD / 64;            // output dims per lane in the PV phase
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sc = reinterpret_cast<float*>(smem);                 // [G][Smax]
  const int b = blockIdx.x, kh = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int grp = lane >> 4, col = lane & 15;
  const int p = pos[b];
  const int SS = (S + 15) & ~15;                             // score row stride (whole 16-key tiles)
  float* opart = sc + G * SS;                                 // [4][G][HD]
  float* stat = opart + 4 * G * HD;                           // [G] max, [G] 1/sum
  uint16_t* ob = out + ((size_t)b * Hq + kh * G) * HD;
  if (p < 0) {   // padding row
    for (int e = threadIdx.x; e < G * HD; e += blockDim.x) ob[e] = 0;
    return;
  }
  const int kmax = p < S ? p : S - 1;
  int kmin = 0;
  if (window > 0) { kmin = p - window + 1; if (kmin < 0) kmin = 0; }
  const int cs = slot[b];
  const uint16_t* kbase = kc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* vbase = vc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  // Shared read-only prefix (prefix-shared sweep cells): keys [0, np) come from slot pslot[b] of
  // (pkc, pvc) — the pair's baseline KV, which every cell of the pair reads (served from L2 / the
  // Infinity Cache after the first reader) instead of a private per-cell copy.
  int np = 0;
  const uint16_t* kpre = kbase;
  const uint16_t* vpre = vbase;
  if (plen != nullptr) {
    np = plen[b];
    if (np > 0) {
      const size_t po = ((size_t)pslot[b] * Hkv + kh) * (size_t)S * HD;
      kpre = pkc + po;
      vpre = pvc + po;
    }
  }
  const int own_lo = kmin;
  // Q fragments: row = col (only rows < G real)
  bf16x8 qa[KS];
  {
    const uint16_t* qrow = q + ((size_t)b * Hq + kh * G + (col < G ? col : 0)) * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 u = {0, 0, 0, 0};
      if (col < G) u = *reinterpret_cast<const uint4*>(qrow + ks * 32 + grp * 8);
      qa[ks] = as_bf16x8(u);
    }
  }
  const float inv_cap = softcap > 0.f ? 1.f / softcap : 0.f;
  const int t0 = own_lo >> 4, t1 = kmax >> 4;
  // (tried: V rows of the wave's PV range prefetched into registers here, with the Q / K loads — 25% slower
  // in the sweep bench, profiles/r2/kstats_vprefetch.txt; the kernel is not bound by its memory round trips)
  const int lo = t0 * 16, hi = kmax;     // scores live in [lo, hi]
  const int nk = hi - lo + 1;
  const int chunk = (nk + 3) >> 2;
  const int j0 = lo + wid * chunk, j1 = min(hi + 1, j0 + chunk);
  using VT = typename vrow_t<DPL>::type;
  for (int t = t0 + wid; t <= t1; t += 4) {
    int kk = t * 16 + col;
    const int kr = kk <= kmax ? (kk >= own_lo ? kk : own_lo <= kmax ? own_lo : kmax) : kmax;
    const uint16_t* krow = (kr < np ? kpre : kbase) + (size_t)kr * HD + grp * 8;
    uint4 kf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = *reinterpret_cast<const uint4*>(krow + ks * 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], as_bf16x8(kf[ks]), acc, 0, 0, 0);
    if (grp == 0) {   // rows 0..3 live in lanes 0..15 (regs 0..3)
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float s = acc[h] * scale;
        if (softcap > 0.f) s = tanhf(s * inv_cap) * softcap;
        const bool ok = kk >= own_lo && kk <= kmax;
        sc[h * SS + kk] = ok ? s : -INFINITY;
      }
    }
  }
  __syncthreads();
  if (wid < G) {
    const float* sh = sc + wid * SS;
    float m = -INFINITY;
    for (int j = lo + lane; j <= hi; j += 64) m = fmaxf(m, sh[j]);
    m = wave_max(m);
    float l = 0.f;
    if (m > -INFINITY)
      for (int j = lo + lane; j <= hi; j += 64) l += rbf(__expf(sh[j] - m));
    l = wave_sum(l);
    if (lane == 0) { stat[wid] = m; stat[G + wid] = l > 0.f ? 1.f / l : 0.f; }
  }
  __syncthreads();
  // PV: wave w takes keys [j0, j1): prefetched rows from registers, the rest streamed
  float o[G][DPL];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[h][d] = 0.f;
  float mh[G];
#pragma unroll
  for (int h = 0; h < G; ++h) mh[h] = stat[h];
  int j = j0;
  for (; j + 4 <= j1; j += 4) {
    float vf[4][DPL];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      vrow_t<DPL>::unpack(*reinterpret_cast<const VT*>((j + u < np ? vpre : vbase) + (size_t)(j + u) * HD + lane * DPL),
                          vf[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float pw = rbf(__expf(sc[h * SS + j + u] - mh[h]));
#pragma unroll
        for (int d = 0; d < DPL; ++d) o[h][d] += pw * vf[u][d];
      }
  }
  for (; j < j1; ++j) {
    float vf[DPL];
    vrow_t<DPL>::unpack(*reinterpret_cast<const VT*>((j < np ? vpre : vbase) + (size_t)j * HD + lane * DPL), vf);
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float pw = rbf(__expf(sc[h * SS + j] - mh[h]));
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[h][d] += pw * vf[d];
    }
  }
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int d = 0; d < DPL; ++d) opart[(wid * G + h) * HD + lane * DPL + d] = o[h][d];
  __syncthreads();
  for (int e = threadIdx.x; e < G * HD; e += blockDim.x) {
    const int h = e / HD;
    float v = opart[e] + opart[G * HD + e] + opart[2 * G * HD + e] + opart[3 * G * HD + e];
    ob[e] = f2bf(v * stat[G + h]);
  }
}

// ---------------------------------------------------------------------------
// Decode, one wave per (sequence, kv head): NWH waves of a workgroup take NWH kv heads of one sequence and
// never synchronise with each other (no __syncthreads, 2.5 KB of LDS per 4 waves), so many workgroups
// share a CU.  At decode lengths (tens of keys) the 4-wave-per-head kernel above spent about half of its
// time in per-workgroup latency chains (pos -> K -> scores -> softmax -> V -> cross-wave sum, three
// barriers) with 8 workgroups per CU in flight (profiles/r2/attn_scan.log: 45 us at 1 key vs 208 us at
// 67 keys for 2048 rows); here each wave streams its whole key range with the next K tile and the V
// rows prefetched (issued before the scores are known), and the softmax weights p = rbf(exp(s - m)) are
// computed once per key (not once per lane) and read back as LDS broadcasts.
// Numerics = attn_decode_kernel: bf16-rounded softmax weights, fp32 sums, out = O / l.
// K tiles are loaded one at a time (no second register set: 114 -> 82 VGPRs, 4 -> 5 waves per SIMD, 3-6 % faster at
// 1024-4096 rows than loading tile t+1 under tile t's MFMAs, profiles/r5/attn/attn_bench_variants.log); V rows are
// prefetched VCH_ ahead (4 instead of 8: 1-3 % slower)
template <int HD, int G, int VCH_ = 8, int KDB = 1>
__global__ void __launch_bounds__(256) attn_decode_wave_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    uint16_t* __restrict__ out, const int32_t* __restrict__ pos, const int32_t* __restrict__ slot, int Hq, int Hkv,
    int S, float scale, float softcap, int window, const uint16_t* __restrict__ pkc, const uint16_t* __restrict__ pvc,
    const int32_t* __restrict__ pslot, const int32_t* __restrict__ plen) {
  constexpr int KS = HD / 32;
  constexpr int DPL = HD / 64;
  constexpr int VCH = VCH_;              // V rows per prefetch chunk
  using VT = typename vrow_t<DPL>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwh = blockDim.x >> 6;
  const int b = blockIdx.x, hy = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kh = hy * nwh + w;
  const int grp = lane >> 4, col = lane & 15;
  const int SS = (S + 15) & ~15;
  float* sc = reinterpret_cast<float*>(smem) + (size_t)w * G * SS;   // this wave's [G][SS] scores / weights
  // this wave's G query rows (bf16), re-read per key tile instead of held in 32 VGPRs: 4 instead of 3 waves per SIMD
  uint16_t* ql = reinterpret_cast<uint16_t*>(reinterpret_cast<float*>(smem) + (size_t)nwh * G * SS) + (size_t)w * G * HD;
  uint16_t* ob = out + ((size_t)b * Hq + kh * G) * HD;
  const int p = pos[b];
  if (p < 0) {   // padding row
    for (int e = lane; e < G * HD; e += 64) ob[e] = 0;
    return;
  }
  const int kmax = p < S ? p : S - 1;
  int kmin = 0;
  if (window > 0) { kmin = p - window + 1; if (kmin < 0) kmin = 0; }
  const int cs = slot[b];
  const uint16_t* kbase = kc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* vbase = vc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  int np = 0;
  const uint16_t* kpre = kbase;
  const uint16_t* vpre = vbase;
  if (plen != nullptr) {
    np = plen[b];
    if (np > 0) {
      const size_t po = ((size_t)pslot[b] * Hkv + kh) * (size_t)S * HD;
      kpre = pkc + po;
      vpre = pvc + po;
    }
  }
  auto vload = [&](int j, VT (&v)[VCH]) {
#pragma unroll
    for (int u = 0; u < VCH; ++u) {
      const int jj = j + u <= kmax ? j + u : kmax;
      v[u] = *reinterpret_cast<const VT*>((jj < np ? vpre : vbase) + (size_t)jj * HD + lane * DPL);
    }
  };
  // the first V chunk is independent of the scores: issue it first
  VT va[VCH], vb[VCH];
  vload(kmin, va);
  {
    // G rows x HD bf16 = G x HD / 8 16-B chunks, one per lane and round
    const uint16_t* qrow = q + ((size_t)b * Hq + kh * G) * HD;
#pragma unroll
    for (int e = lane; e < G * HD / 8; e += 64)
      *reinterpret_cast<uint4*>(ql + e * 8) = *reinterpret_cast<const uint4*>(qrow + e * 8);
  }
  const float inv_cap = softcap > 0.f ? 1.f / softcap : 0.f;
  auto kload = [&](int t, uint4 (&kf)[KS]) {
    const int kk = t * 16 + col;
    const int kr = kk < kmin ? kmin : (kk > kmax ? kmax : kk);
    const uint16_t* krow = (kr < np ? kpre : kbase) + (size_t)kr * HD + grp * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = *reinterpret_cast<const uint4*>(krow + ks * 32);
  };
  // MFMA rows >= G (lanes col >= G) read a copy of a real query row: their outputs are never used, rows < G are
  // unchanged (each output row of the MFMA depends on its own A row only)
  const uint16_t* qlr = ql + (col % G) * HD + grp * 8;
  auto score = [&](int t, const uint4 (&kf)[KS]) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(*reinterpret_cast<const uint4*>(qlr + ks * 32)),
                                                    as_bf16x8(kf[ks]), acc, 0, 0, 0);
    const int kk = t * 16 + col;
    if (grp == 0) {   // query rows 0..3 of the 16-row tile live in lanes 0..15
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float s = acc[h] * scale;
        if (softcap > 0.f) s = tanhf(s * inv_cap) * softcap;
        sc[h * SS + kk] = (kk >= kmin && kk <= kmax) ? s : -INFINITY;
      }
    }
  };
  const int t0 = kmin >> 4, t1 = kmax >> 4;
  if constexpr (KDB == 2) {
    uint4 ka[KS], kb[KS];
    kload(t0, ka);
    for (int t = t0; t <= t1; t += 2) {
      if (t + 1 <= t1) kload(t + 1, kb);
      score(t, ka);
      if (t + 1 <= t1) {
        if (t + 2 <= t1) kload(t + 2, ka);
        score(t + 1, kb);
      }
    }
  } else {
    for (int t = t0; t <= t1; ++t) {
      uint4 ka[KS];
      kload(t, ka);
      score(t, ka);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // softmax weights, in place: p = rbf(exp(s - m)), l = sum p
  float inv_l[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float* sh = sc + h * SS;
    float m = -INFINITY;
    for (int j = kmin + lane; j <= kmax; j += 64) m = fmaxf(m, sh[j]);
    m = wave_max(m);
    float l = 0.f;
    for (int j = kmin + lane; j <= kmax; j += 64) {
      const float pw = m > -INFINITY ? rbf(__expf(sh[j] - m)) : 0.f;
      sh[j] = pw;
      l += pw;
    }
    l = wave_sum(l);
    inv_l[h] = l > 0.f ? 1.f / l : 0.f;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // O = sum_j p_j v_j over [kmin, kmax]: each lane owns DPL dims, V rows prefetched one chunk ahead
  float o[G][DPL];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[h][d] = 0.f;
  auto accum = [&](int j, const VT (&v)[VCH]) {
#pragma unroll
    for (int u = 0; u < VCH; ++u) {
      if (j + u > kmax) break;
      float vf[DPL];
      vrow_t<DPL>::unpack(v[u], vf);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float pw = sc[h * SS + j + u];
#pragma unroll
        for (int d = 0; d < DPL; ++d) o[h][d] += pw * vf[d];
      }
    }
  };
  for (int j = kmin; j <= kmax; j += 2 * VCH) {
    if (j + VCH <= kmax) vload(j + VCH, vb);
    accum(j, va);
    if (j + VCH <= kmax) {
      if (j + 2 * VCH <= kmax) vload(j + 2 * VCH, va);
      accum(j + VCH, vb);
    }
  }
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float r[DPL];
#pragma unroll
    for (int d = 0; d < DPL; ++d) r[d] = o[h][d] * inv_l[h];
    uint16_t* dst = ob + h * HD + lane * DPL;
    if constexpr (DPL == 4) {
      *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(r[0], r[1]), pack2(r[2], r[3]));
    } else {
      *reinterpret_cast<uint32_t*>(dst) = pack2(r[0], r[1]);
    }
  }
}


// Packed rows (block-table mode: the sweep's teacher-forced tails and NLL passes) with the DECODE kernel's numerics,
// bit for bit.  A tail row at position p is the same query the greedy decode computes at p (the reuse levels replay
// positions >= a cell's first edit as one packed forward instead of one decode step each), so the tail must round
// exactly like attn_decode_wave_kernel or a resumed cell's records drift from a from-scratch generation's
// (tests/test_exact_9b_gpu.py).  Per (block of P = 16 / G positions of one sequence, kv head) one wave:
//  * scores: the decode's MFMA chain (Q fragment A, K fragment B, head_dim in 32-deep steps) for the block's 16
//    (position, head) rows at once -- an MFMA output row depends on its own A row only, so every row's scores are
//    the decode's; scaled, softcapped and masked (keys in [kmin_r, pos_r]) per row, into LDS key-major;
//  * softmax per row as the decode does it: exact max, p = rbf(exp(s - m)), l = the lane-strided sum from kmin_r +
//    wave butterfly, in the same order;
//  * O = sum_j p_j v_j on the VALU in ascending key order, one fp32 FMA chain per (row, dim) -- the decode's chain;
//    keys outside a row's range carry p = 0, and adding +-0 leaves an fp32 sum unchanged;
//  * out = O * (1 / l), bf16.
// Each wave reads the block's K / V once for its 16 rows (the decode kernel would read them once per row).
template <int HD, int G>
__global__ void __launch_bounds__(256) attn_tail_exact_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    uint16_t* __restrict__ out, const int32_t* __restrict__ pos, int Hq, int Hkv, int S, float scale, float softcap,
    int window, const int32_t* __restrict__ blk, int nitems, int bw, const uint16_t* __restrict__ pkc,
    const uint16_t* __restrict__ pvc) {
  constexpr int P = 16 / G;
  constexpr int KS = HD / 32;
  constexpr int DPL = HD / 64;
  constexpr int VCH = 8;
  using VT = typename vrow_t<DPL>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wid;
  if (item >= nitems) return;                     // wave-uniform; the waves never synchronise
  const int SS = (S + 15) & ~15;
  float* sc = reinterpret_cast<float*>(smem) + (size_t)wid * 16 * SS;   // key-major [SS][16] scores / weights
  const int bi = item / Hkv, kh = item % Hkv;
  const int rbase = blk[bw * bi], nvalid = blk[bw * bi + 1], cs = blk[bw * bi + 2];
  const int ps = bw == 5 ? blk[bw * bi + 3] : 0, np = bw == 5 ? blk[bw * bi + 4] : 0;
  const int grp = lane >> 4, col = lane & 15;
  const uint16_t* kbase = kc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* vbase = vc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* kpre = kbase;
  const uint16_t* vpre = vbase;
  if (np > 0) {
    kpre = pkc + ((size_t)ps * Hkv + kh) * (size_t)S * HD;
    vpre = pvc + ((size_t)ps * Hkv + kh) * (size_t)S * HD;
  }
  // row r = (position t = r / G, head kh * G + r % G); per-row key range [kmin_r, kmax_r] as the decode computes it
  auto rpos = [&](int r) -> int { return (r / G) < nvalid ? pos[(size_t)rbase + r / G] : -1; };
  auto rkmax = [&](int p) -> int { return p < S ? p : S - 1; };
  auto rkmin = [&](int p) -> int {
    int k = 0;
    if (window > 0) { k = p - window + 1; if (k < 0) k = 0; }
    return k;
  };
  int kmaxb = -1, kminb = 1 << 30;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = rpos(r);
    if (p >= 0) { kmaxb = max(kmaxb, rkmax(p)); kminb = min(kminb, rkmin(p)); }
  }
  uint16_t* orow0 = out + (size_t)rbase * Hq * HD;
  if (kmaxb < 0) {                                  // every row is padding: zeros, as the decode writes them
    for (int e = lane; e < nvalid * G * HD; e += 64) {
      const int t = e / (G * HD), rem = e % (G * HD);
      orow0[(size_t)t * Hq * HD + kh * G * HD + rem] = 0;
    }
    return;
  }
  // ---- scores (the decode's MFMA operands: query row (r) fragments, key rows clamped into [kminb, kmaxb])
  const int pA = rpos(col);                         // this lane's A row
  bf16x8 qa[KS];
  {
    const uint16_t* qrow = q + (((size_t)rbase + col / G) * Hq + kh * G + col % G) * HD + grp * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 u = {0, 0, 0, 0};
      if (pA >= 0) u = *reinterpret_cast<const uint4*>(qrow + ks * 32);
      qa[ks] = as_bf16x8(u);
    }
  }
  int pC[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) pC[i] = rpos(4 * grp + i);
  const float inv_cap = softcap > 0.f ? 1.f / softcap : 0.f;
  for (int t = kminb >> 4; t <= kmaxb >> 4; ++t) {
    const int kk = t * 16 + col;
    const int kr = kk < kminb ? kminb : (kk > kmaxb ? kmaxb : kk);
    const uint16_t* krow = (kr < np ? kpre : kbase) + (size_t)kr * HD + grp * 8;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], as_bf16x8(*reinterpret_cast<const uint4*>(krow + ks * 32)),
                                                    acc, 0, 0, 0);
    float sv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = acc[i] * scale;
      if (softcap > 0.f) s = tanhf(s * inv_cap) * softcap;
      const int p = pC[i];
      sv[i] = (p >= 0 && kk >= rkmin(p) && kk <= rkmax(p)) ? s : -INFINITY;
    }
    if (kk < SS) *reinterpret_cast<float4*>(sc + (size_t)kk * 16 + 4 * grp) = make_float4(sv[0], sv[1], sv[2], sv[3]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // ---- softmax weights per row, the decode's order; keys of the block's range outside the row's get p = 0
  float inv_l[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = rpos(r);
    inv_l[r] = 0.f;
    if (p < 0) {
      for (int j = kminb + lane; j <= kmaxb; j += 64) sc[(size_t)j * 16 + r] = 0.f;
      continue;
    }
    const int k0 = rkmin(p), k1 = rkmax(p);
    float m = -INFINITY;
    for (int j = k0 + lane; j <= k1; j += 64) m = fmaxf(m, sc[(size_t)j * 16 + r]);
    m = wave_max(m);
    float l = 0.f;
    for (int j = k0 + lane; j <= k1; j += 64) {
      const float pw = m > -INFINITY ? rbf(__expf(sc[(size_t)j * 16 + r] - m)) : 0.f;
      sc[(size_t)j * 16 + r] = pw;
      l += pw;
    }
    l = wave_sum(l);
    inv_l[r] = l > 0.f ? 1.f / l : 0.f;
    for (int j = kminb + lane; j <= kmaxb; j += 64)
      if (j < k0 || j > k1) sc[(size_t)j * 16 + r] = 0.f;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // ---- O = sum_j p_j v_j: each lane owns DPL dims of all 16 rows, keys ascending, V rows prefetched VCH ahead
  float o[16][DPL];
#pragma unroll
  for (int r = 0; r < 16; ++r)
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[r][d] = 0.f;
  auto vload = [&](int j, VT (&v)[VCH]) {
#pragma unroll
    for (int u = 0; u < VCH; ++u) {
      const int jj = j + u <= kmaxb ? j + u : kmaxb;
      v[u] = *reinterpret_cast<const VT*>((jj < np ? vpre : vbase) + (size_t)jj * HD + lane * DPL);
    }
  };
  auto accum = [&](int j, const VT (&v)[VCH]) {
#pragma unroll
    for (int u = 0; u < VCH; ++u) {
      if (j + u > kmaxb) break;
      float vf[DPL];
      vrow_t<DPL>::unpack(v[u], vf);
      const float4* pr = reinterpret_cast<const float4*>(sc + (size_t)(j + u) * 16);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const float4 pw4 = pr[r4];
        const float pwv[4] = {pw4.x, pw4.y, pw4.z, pw4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int d = 0; d < DPL; ++d) o[4 * r4 + i][d] += pwv[i] * vf[d];
      }
    }
  };
  VT va[VCH], vb[VCH];
  vload(kminb, va);
  for (int j = kminb; j <= kmaxb; j += 2 * VCH) {
    if (j + VCH <= kmaxb) vload(j + VCH, vb);
    accum(j, va);
    if (j + VCH <= kmaxb) {
      if (j + 2 * VCH <= kmaxb) vload(j + 2 * VCH, va);
      accum(j + VCH, vb);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (r / G >= nvalid) continue;
    float v[DPL];
#pragma unroll
    for (int d = 0; d < DPL; ++d) v[d] = o[r][d] * inv_l[r];
    uint16_t* dst = out + (((size_t)rbase + r / G) * Hq + kh * G + r % G) * HD + lane * DPL;
    if constexpr (DPL == 4) {
      *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    } else {
      *reinterpret_cast<uint32_t*>(dst) = pack2(v[0], v[1]);
    }
  }
}


// Decode, one 4-wave workgroup per (row, kv head): attn_decode_wave_kernel's arithmetic spread over 4 waves, for the
// small decode buckets (<= 64 rows: 2 or fewer waves per SIMD in the wave kernel, each walking its keys alone).
// Bit-identical to the wave kernel per row (so switching kernels by row count keeps the decode batch-invariant):
// the 16-key score tiles are strided over the waves (one MFMA per tile, the same operands);
// the max is exact in any order; each wave forms the weights p = rbf(exp(s - m)) of a quarter of the keys, and every
// wave then sums them in the wave kernel's lane-strided order + butterfly; the P V chain of each output dim runs over
// the keys in ascending order in one lane, the waves taking (head, dim range) slices instead of the wave kernel's
// whole rows (tests/test_kernels_gpu.py::test_attention_decode_split_bitequal).
template <int HD, int G>
__global__ void __launch_bounds__(256) attn_decode_split_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    uint16_t* __restrict__ out, const int32_t* __restrict__ pos, const int32_t* __restrict__ slot, int Hq, int Hkv,
    int S, float scale, float softcap, int window, const uint16_t* __restrict__ pkc, const uint16_t* __restrict__ pvc,
    const int32_t* __restrict__ pslot, const int32_t* __restrict__ plen) {
  constexpr int KS = HD / 32;
  constexpr int PARTS = 4 / G;                 // waves per head in the P V phase
  constexpr int DPW = HD / PARTS / 64;         // output dims per lane
  constexpr int VCH = 8;
  static_assert(PARTS * G == 4 && (DPW == 2 || DPW == 4), "geometry");
  using VT = typename vrow_t<DPW>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, kh = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane >> 4, col = lane & 15;
  const int SS = (S + 15) & ~15;
  float* sc = reinterpret_cast<float*>(smem);                                   // [G][SS] scores, then weights
  uint16_t* ql = reinterpret_cast<uint16_t*>(sc + (size_t)G * SS);               // [G][HD] query rows
  uint16_t* ob = out + ((size_t)b * Hq + kh * G) * HD;
  const int p = pos[b];
  if (p < 0) {   // padding row
    for (int e = threadIdx.x; e < G * HD; e += 256) ob[e] = 0;
    return;
  }
  const int kmax = p < S ? p : S - 1;
  int kmin = 0;
  if (window > 0) { kmin = p - window + 1; if (kmin < 0) kmin = 0; }
  const int cs = slot[b];
  const uint16_t* kbase = kc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  const uint16_t* vbase = vc + ((size_t)cs * Hkv + kh) * (size_t)S * HD;
  int np = 0;
  const uint16_t* kpre = kbase;
  const uint16_t* vpre = vbase;
  if (plen != nullptr) {
    np = plen[b];
    if (np > 0) {
      const size_t po = ((size_t)pslot[b] * Hkv + kh) * (size_t)S * HD;
      kpre = pkc + po;
      vpre = pvc + po;
    }
  }
  // this wave's P V slice: head h, dims d0 .. d0 + DPW of each V row; its first V chunk goes out first
  const int h = w / PARTS, d0 = (w % PARTS) * (HD / PARTS) + lane * DPW;
  auto vload = [&](int j, VT (&v)[VCH]) {
#pragma unroll
    for (int u = 0; u < VCH; ++u) {
      const int jj = j + u <= kmax ? j + u : kmax;
      v[u] = *reinterpret_cast<const VT*>((jj < np ? vpre : vbase) + (size_t)jj * HD + d0);
    }
  };
  VT va[VCH], vb[VCH];
  vload(kmin, va);
  {
    const uint16_t* qrow = q + ((size_t)b * Hq + kh * G) * HD;
    for (int e = threadIdx.x; e < G * HD / 8; e += 256)
      *reinterpret_cast<uint4*>(ql + e * 8) = *reinterpret_cast<const uint4*>(qrow + e * 8);
  }
  __syncthreads();
  const float inv_cap = softcap > 0.f ? 1.f / softcap : 0.f;
  const uint16_t* qlr = ql + (col % G) * HD + grp * 8;
  const int t0 = kmin >> 4, t1 = kmax >> 4;
  for (int t = t0 + w; t <= t1; t += 4) {
    uint4 kf[KS];
    const int kk = t * 16 + col;
    const int kr = kk < kmin ? kmin : (kk > kmax ? kmax : kk);
    const uint16_t* krow = (kr < np ? kpre : kbase) + (size_t)kr * HD + grp * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = *reinterpret_cast<const uint4*>(krow + ks * 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(*reinterpret_cast<const uint4*>(qlr + ks * 32)),
                                                    as_bf16x8(kf[ks]), acc, 0, 0, 0);
    if (grp == 0) {
#pragma unroll
      for (int hh = 0; hh < G; ++hh) {
        float s = acc[hh] * scale;
        if (softcap > 0.f) s = tanhf(s * inv_cap) * softcap;
        sc[hh * SS + kk] = (kk >= kmin && kk <= kmax) ? s : -INFINITY;
      }
    }
  }
  __syncthreads();
  // row max (exact in any order; every wave for itself), then this wave's quarter of the weights
  float m[G];
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    const float* sh = sc + hh * SS;
    float mm = -INFINITY;
    for (int j = kmin + lane; j <= kmax; j += 64) mm = fmaxf(mm, sh[j]);
    m[hh] = wave_max(mm);
  }
  __syncthreads();   // every wave has read the scores it needs for its max
#pragma unroll
  for (int hh = 0; hh < G; ++hh) {
    float* sh = sc + hh * SS;
    for (int j = kmin + lane + 64 * w; j <= kmax; j += 256)
      sh[j] = m[hh] > -INFINITY ? rbf(__expf(sh[j] - m[hh])) : 0.f;
  }
  __syncthreads();
  // l in the wave kernel's order: lane-strided ascending partial sums, then the butterfly
  float inv_l;
  {
    const float* sh = sc + h * SS;
    float l = 0.f;
    for (int j = kmin + lane; j <= kmax; j += 64) l += sh[j];
    l = wave_sum(l);
    inv_l = l > 0.f ? 1.f / l : 0.f;
  }
  float o[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) o[d] = 0.f;
  const float* ph = sc + h * SS;
  auto accum = [&](int j, const VT (&v)[VCH]) {
#pragma unroll
    for (int u = 0; u < VCH; ++u) {
      if (j + u > kmax) break;
      float vf[DPW];
      vrow_t<DPW>::unpack(v[u], vf);
      const float pw = ph[j + u];
#pragma unroll
      for (int d = 0; d < DPW; ++d) o[d] += pw * vf[d];
    }
  };
  for (int j = kmin; j <= kmax; j += 2 * VCH) {
    if (j + VCH <= kmax) vload(j + VCH, vb);
    accum(j, va);
    if (j + VCH <= kmax) {
      if (j + 2 * VCH <= kmax) vload(j + 2 * VCH, va);
      accum(j + VCH, vb);
    }
  }
  float r[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) r[d] = o[d] * inv_l;
  uint16_t* dst = ob + h * HD + d0;
  if constexpr (DPW == 4) {
    *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(r[0], r[1]), pack2(r[2], r[3]));
  } else {
    *reinterpret_cast<uint32_t*>(dst) = pack2(r[0], r[1]);
  }
}

template <int HD, int G>
void launch_attn(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, uint16_t* out, const int32_t* pos,
                 const int32_t* slot, int B, int T, int Hq, int Hkv, int S, float scale, float softcap, int window,
                 hipStream_t st, const int32_t* blk = nullptr, int nblk = 0, int bw = 3,
                 const uint16_t* pkc = nullptr, const uint16_t* pvc = nullptr) {
  constexpr int P = 16 / G;
  const size_t lds = (size_t)tb_attention_lds_bytes(HD);
  static bool attr_set = false;   // > 64 KB dynamic LDS needs the opt-in (first call is never captured)
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_cache_kernel<HD, G>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  if (blk != nullptr && S <= 512) {
    // packed tails / NLL passes: the decode's numerics (attn_tail_exact_kernel), 4 independent waves per workgroup
    const size_t lds_t = (size_t)4 * 16 * ((S + 15) & ~15) * sizeof(float);
    static size_t attr_tail = 65536;
    if (lds_t > attr_tail) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_tail_exact_kernel<HD, G>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_tail = 160 * 1024;
    }
    const int nitems = nblk * Hkv;
    hipLaunchKernelGGL((attn_tail_exact_kernel<HD, G>), dim3((nitems + 3) / 4), dim3(256), lds_t, st, q, kc, vc, out,
                       pos, Hq, Hkv, S, scale, softcap, window, blk, nitems, bw, pkc, pvc);
    return;
  }
  if (blk != nullptr) {
    dim3 grid(nblk, Hkv, 1);
    hipLaunchKernelGGL((attn_cache_kernel<HD, G>), grid, dim3(256), lds, st, q, kc, vc, out, pos, slot, T, Hq, Hkv,
                       S, scale, softcap, window, blk, bw, pkc, pvc);
    return;
  }
  dim3 grid((T + P - 1) / P, Hkv, B);
  hipLaunchKernelGGL((attn_cache_kernel<HD, G>), grid, dim3(256), lds, st, q, kc, vc, out, pos, slot, T, Hq, Hkv, S,
                     scale, softcap, window, (const int32_t*)nullptr);
}


// rows at or below which the decode (S <= 2048, HD 256, G 2 / 4) runs attn_decode_split_kernel (same bits), for rows
// with their own keys only / rows reading a shared prefix: at 64 rows 15-18 % faster than the one-wave kernel (too
// few waves to cover its latency), from 128 rows on 3-20 % slower (profiles/r5/attn/attn_bench_split_own.log,
// attn_bench_split_sweep.log)
int g_attn_split_rows[2] = {64, 64};

template <int HD, int G>
void launch_attn_decode(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, uint16_t* out, const int32_t* pos,
                        const int32_t* slot, int B, int Hq, int Hkv, int S, float scale, float softcap, int window,
                        const uint16_t* pkc, const uint16_t* pvc, const int32_t* pslot, const int32_t* plen,
                        hipStream_t st) {
  if constexpr (HD == 256 && (G == 2 || G == 4)) {
    if (S <= 2048 && B <= g_attn_split_rows[pkc != nullptr ? 1 : 0]) {
      const size_t lds_s = (size_t)G * ((S + 15) & ~15) * sizeof(float) + (size_t)G * HD * 2;
      hipLaunchKernelGGL((attn_decode_split_kernel<HD, G>), dim3(B, Hkv), dim3(256), lds_s, st, q, kc, vc, out, pos,
                         slot, Hq, Hkv, S, scale, softcap, window, pkc, pvc, pslot, plen);
      return;
    }
  }
  if (S <= 2048) {
    int nwh = Hkv % 4 == 0 ? 4 : (Hkv % 2 == 0 ? 2 : 1);
    auto wave_lds = [&](int n) { return (size_t)n * G * ((S + 15) & ~15) * sizeof(float) + (size_t)n * G * HD * 2; };
    // fewer kv heads per workgroup where nwh of them would not fit the 160 KB LDS (large G near S = 2048)
    while (nwh > 1 && wave_lds(nwh) > 160 * 1024) nwh >>= 1;
    const size_t lds_w = wave_lds(nwh);
    static size_t wave_attr = 65536;       // above 64 KB of dynamic LDS the launch needs the opt-in attribute
    if (lds_w > wave_attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_decode_wave_kernel<HD, G>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      wave_attr = 160 * 1024;
    }
    hipLaunchKernelGGL((attn_decode_wave_kernel<HD, G>), dim3(B, Hkv / nwh), dim3(64 * nwh), lds_w, st, q, kc, vc, out,
                       pos, slot, Hq, Hkv, S, scale, softcap, window, pkc, pvc, pslot, plen);
    return;
  }
  const size_t lds = ((size_t)G * ((S + 15) & ~15) + 4 * G * HD + 3 * G + 2) * sizeof(float);
  static size_t attr_set = 0;
  if (lds > attr_set && lds > 65536) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_decode_kernel<HD, G>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = lds;
  }
  hipLaunchKernelGGL((attn_decode_kernel<HD, G>), dim3(B, Hkv), dim3(256), lds, st, q, kc, vc, out, pos, slot, Hq,
                     Hkv, S, scale, softcap, window, pkc, pvc, pslot, plen);
}

}  // namespace

int tb_attention_split_rows(int n, bool prefix) {
  const int old = g_attn_split_rows[prefix ? 1 : 0];
  if (n >= 0) g_attn_split_rows[prefix ? 1 : 0] = n;
  return old;
}

void tb_attention(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, uint16_t* out, const int32_t* pos,
                  const int32_t* slot, int B, int T, int Hq, int Hkv, int HD, int S, float scale, float softcap,
                  int window, hipStream_t st, const uint16_t* pkc, const uint16_t* pvc, const int32_t* pslot,
                  const int32_t* plen) {
  if (B <= 0 || T <= 0) return;
  const int G = Hq / Hkv;
  if (T == 1 && S <= 8192) {
#define TB_DEC_CASE(hd, g)                                                                                   \
  if (HD == hd && G == g) {                                                                                  \
    launch_attn_decode<hd, g>(q, kc, vc, out, pos, slot, B, Hq, Hkv, S, scale, softcap, window, pkc, pvc,    \
                              pslot, plen, st);                                                              \
    return;                                                                                                  \
  }
    TB_DEC_CASE(256, 2)
    TB_DEC_CASE(256, 1)
    TB_DEC_CASE(256, 4)
    TB_DEC_CASE(128, 2)
    TB_DEC_CASE(128, 1)
    TB_DEC_CASE(128, 4)
#undef TB_DEC_CASE
  }
#define TB_ATTN_CASE(hd, g)                                                                                   \
  if (HD == hd && G == g) {                                                                                  \
    launch_attn<hd, g>(q, kc, vc, out, pos, slot, B, T, Hq, Hkv, S, scale, softcap, window, st);             \
    return;                                                                                                  \
  }
  TB_ATTN_CASE(256, 2)
  TB_ATTN_CASE(256, 1)
  TB_ATTN_CASE(256, 4)
  TB_ATTN_CASE(128, 2)
  TB_ATTN_CASE(128, 1)
  TB_ATTN_CASE(128, 4)
#undef TB_ATTN_CASE
}

void tb_attention_varlen(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, uint16_t* out, const int32_t* pos,
                         const int32_t* blk, int nblk, int Hq, int Hkv, int HD, int S, float scale, float softcap,
                         int window, hipStream_t st, int bw, const uint16_t* pkc, const uint16_t* pvc) {
  if (nblk <= 0) return;
  const int G = Hq / Hkv;
#define TB_VL_CASE(hd, g)                                                                                    \
  if (HD == hd && G == g) {                                                                                  \
    launch_attn<hd, g>(q, kc, vc, out, pos, nullptr, 0, 0, Hq, Hkv, S, scale, softcap, window, st, blk, nblk,  \
                       bw, pkc, pvc);                                                                        \
    return;                                                                                                  \
  }
  TB_VL_CASE(256, 2)
  TB_VL_CASE(256, 1)
  TB_VL_CASE(256, 4)
  TB_VL_CASE(128, 2)
  TB_VL_CASE(128, 1)
  TB_VL_CASE(128, 4)
#undef TB_VL_CASE
}

