// Vocabulary-side readouts over bf16 logits [R, V] (SURVEY K10, K11, K12, K16,
// K17, K23).  The unembedding GEMM itself runs on hipBLASLt; everything that
// the reference does afterwards on the host over 1.6 GB fp32 arrays
// (`src/models.py:135-153`, `src/01_reproduce_logit_lens.py:35-71,147-149`)
// happens here on the device, so only [V]-sized results ever leave the GPU.
//
//  argmax_rows    greedy next token (optionally with the bf16 final-softcap
//                 rounding chain of HF generate, which can create ties)
//  row_lse        per-row log-sum-exp (online max/sum; logit-lens softmax)
//  gather_probs   p(row, id) = exp(z - lse) for secret / decoy ids
//  lens_colsum    acc[b, v] (+)= sum_t mask[b,t] * softmax(z[b,t])[v] with the
//                 reference's per-position id exclusions (2 ids per row)
//  topk_rows      per-row top-k (k <= 64), ties -> lower index
//  xent_rows      NLL of target ids under softcapped logits (fluency ΔNLL)
//  decode_head    one pass over a decode row: greedy token (argmax_rows semantics), its NLL and
//                 the NLL of an optional teacher target (the baseline's token at that column)
#include "common.h"
#include "api.h"
#include <algorithm>
#include <cstdlib>

namespace {

// tanh for the final-logit softcap: 1 - 2/(e^{2|y|} + 1) on v_exp_f32 + v_rcp_f32 (a few fp32 ulp; the
// result is rounded to bf16 right after, like HF's bf16 tanh), odd Taylor series near 0 where that
// form cancels.  ~4x cheaper than libm tanhf, which made the 256k-wide vocab passes VALU-bound.
__device__ __forceinline__ float fast_tanh(float y) {
  const float a = fabsf(y);
  float t;
  if (a < 0.0625f) {
    const float a2 = a * a;
    t = a * (1.f + a2 * (-0.33333334f + a2 * 0.13333334f));
  } else {
    const float e = __expf(2.f * a);
    t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  }
  return copysignf(t, y);
}

__device__ __forceinline__ float softcap_bf16(float x, float cap) {
  // HF: logits / cap ; tanh ; * cap, each on a bf16 tensor.
  return rbf(rbf(fast_tanh(rbf(x / cap))) * cap);
}

// ---- exact bf16 softcap by table ------------------------------------------------------------
// softcap_bf16 is a pure function of its bf16 input bits and odd, so the 32768 results for the
// non-negative bit patterns (built on the host with the reference op, registered per cap value)
// make it one LDS lookup per element instead of ~25 VALU ops (the vocab-wide passes were
// VALU-bound on it).  Every kernel that applies the emulated softcap copies the 64 KB table to LDS.
constexpr int CTAB_N = 32768;

__device__ __forceinline__ const uint16_t* stage_ctab(const uint16_t* tab, uint16_t* lds) {
  if (tab == nullptr) return nullptr;
  for (int i = threadIdx.x; i < CTAB_N / 8; i += blockDim.x)
    reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(tab)[i];
  __syncthreads();
  return lds;
}

__device__ __forceinline__ float ctab_get(const uint16_t* ct, uint32_t b) {
  return __uint_as_float(((uint32_t)ct[b & 0x7fffu] | (b & 0x8000u)) << 16);
}

// ---- compact exact softcap (decode_head) ------------------------------------------------------------------
// The chain rbf(rbf(tanh(rbf(x/cap))) * cap) equals rbf(rbf(x * (1/cap)) * cap) for |x| below `lo` (2.703 at cap 30:
// tanh(y) rounds to y there) and saturates at `sat` from `hi` on (104 at cap 30), both checked exhaustively against
// the reference table on the host (ops._softcap_table, tests/test_softcap_compact_cpu.py).  Only the hi - lo
// (~675) bit patterns in between need the table: 1.35 KB of LDS instead of 64 KB, read only by the lanes whose
// logit falls there — no bank-conflicted 64 KB gather, and the small LDS footprint lets full occupancy stream.
struct CapC {
  const uint16_t* tab;   // [hi - lo] bf16 magnitudes
  int lo, hi;
  float sat, rc, cap;
};
constexpr int CAPC_MAX = 2048;   // table entries staged (host-checked)

__device__ __forceinline__ float capc1(uint32_t b, const uint16_t* lt, const CapC& c) {
  const uint32_t ab = b & 0x7fffu;
  const float x = __uint_as_float(b << 16);
  const float a = rbf(rbf(x * c.rc) * c.cap);
  if (ab < (uint32_t)c.lo) return a;
  float mag;
  if (ab < (uint32_t)c.hi) mag = __uint_as_float((uint32_t)lt[ab - c.lo] << 16);
  else if (ab <= 0x7f80u) mag = c.sat;
  else return x;   // NaN stays NaN
  return (b & 0x8000u) ? -mag : mag;
}

// 8 logits of a uint4 -> capped fp32 (table, emulated compute, fp32 tanh, or none)
__device__ __forceinline__ void capped8(const uint4& v, float* f, const uint16_t* ct, float cap, int emu) {
  if (ct != nullptr) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = ctab_get(ct, w[k] & 0xffffu);
      f[2 * k + 1] = ctab_get(ct, w[k] >> 16);
    }
    return;
  }
  unpack8(v, f);
  if (cap > 0.f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = emu ? softcap_bf16(f[j], cap) : fast_tanh(f[j] / cap) * cap;
  }
}

__device__ __forceinline__ float capped1(uint16_t b, const uint16_t* ct, float cap, int emu) {
  if (ct != nullptr) return ctab_get(ct, b);
  const float x = bf2f(b);
  if (cap <= 0.f) return x;
  return emu ? softcap_bf16(x, cap) : fast_tanh(x / cap) * cap;
}

// Streams one row's 16-B vectors c = tid, tid + stride, ... with UNR loads in flight per thread before the first
// is consumed: with the 64 KB softcap table in LDS only 2 blocks (16 waves) fit on a CU, and one outstanding 16-B
// load per lane cannot cover HBM latency.  f(v, c) runs in the plain loop's order (bit-identical reductions).
// (UNR = 1: the plain loop)
template <int UNR, typename F>
__device__ __forceinline__ void stream_row(const uint4* __restrict__ p, int nv, F&& f) {
  const int st = blockDim.x;
  int c = threadIdx.x;
  for (; c + (UNR - 1) * st < nv; c += UNR * st) {
    uint4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = p[c + u * st];
#pragma unroll
    for (int u = 0; u < UNR; ++u) f(v[u], c + u * st);
  }
  for (; c < nv; c += st) f(p[c], c);
}
constexpr int ROW_UNR = 4;
inline int row_unr() { return ROW_UNR; }

struct ArgBest {
  float v;
  int i;
};
__device__ __forceinline__ ArgBest better(ArgBest a, ArgBest b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

template <int UNR>
__global__ void __launch_bounds__(512) argmax_rows_kernel(const uint16_t* __restrict__ logits,
                                                          int32_t* __restrict__ out, int V, float cap,
                                                          const uint16_t* __restrict__ tab) {
  __shared__ float sv[8];
  __shared__ int si[8];
  extern __shared__ __attribute__((aligned(16))) uint16_t ctab_lds[];
  const uint16_t* ct = stage_ctab(tab, ctab_lds);
  const uint16_t* row = logits + (size_t)blockIdx.x * V;
  ArgBest best{-INFINITY, 0x7fffffff};
  const int nv = V >> 3;
  stream_row<UNR>(reinterpret_cast<const uint4*>(row), nv, [&](const uint4& v, int c) {
    float f[8];
    capped8(v, f, ct, cap, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) best = better(best, ArgBest{f[j], c * 8 + j});
  });
  for (int c = nv * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float x = capped1(row[c], ct, cap, 1);
    best = better(best, ArgBest{x, c});
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgBest oth{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, oth);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = best.v; si[wid] = best.i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    ArgBest b{sv[0], si[0]};
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) b = better(b, ArgBest{sv[w], si[w]});
    out[blockIdx.x] = b.i;
  }
}

__device__ __forceinline__ void online_add(float& m, float& s, float x) {
  if (x > m) {
    s = s * __expf(m - x) + 1.f;
    m = x;
  } else {
    s += __expf(x - m);
  }
}
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else { s += s2 * __expf(m2 - m); }
}

template <int UNR>
__global__ void __launch_bounds__(512) row_lse_kernel(const uint16_t* __restrict__ logits, float* __restrict__ lse,
                                                      int V, float cap, int emulate_bf16,
                                                      const uint16_t* __restrict__ tab) {
  __shared__ float sm[8], ss[8];
  extern __shared__ __attribute__((aligned(16))) uint16_t ctab_lds[];
  const uint16_t* ct = stage_ctab(tab, ctab_lds);
  const uint16_t* row = logits + (size_t)blockIdx.x * V;
  float m = -INFINITY, s = 0.f;
  const int nv = V >> 3;
  stream_row<UNR>(reinterpret_cast<const uint4*>(row), nv, [&](const uint4& v, int) {
    float f[8];
    capped8(v, f, ct, cap, emulate_bf16);
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) lm = fmaxf(lm, f[j]);
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(f[j] - lm);
    online_merge(m, s, lm, ls);
  });
  for (int c = nv * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float x = capped1(row[c], ct, cap, emulate_bf16);
    if (m == -INFINITY) { m = x; s = 1.f; } else online_add(m, s, x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) online_merge(M, Ssum, sm[w], ss[w]);
    lse[blockIdx.x] = M + __logf(Ssum);
  }
}

// ``rowmap`` (optional): logical row r reads logits / lse row rowmap[r] (rows deduplicated upstream).
__global__ void gather_probs_kernel(const uint16_t* __restrict__ logits, const float* __restrict__ lse,
                                    const int32_t* __restrict__ ids, float* __restrict__ out, int R, int K, int V,
                                    int round_bf16, const int32_t* __restrict__ rowmap) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R * K) return;
  const int r = rowmap ? rowmap[e / K] : e / K;
  const int id = ids[e];
  if (id < 0 || id >= V) { out[e] = 0.f; return; }
  float p = __expf(bf2f(logits[(size_t)r * V + id]) - lse[r]);
  out[e] = round_bf16 ? rbf(p) : p;
}

// grid (ceil(V / (8*256)), B); rows of sequence b are b*T .. b*T+T-1.
// Rows of sequence b: [b*T, b*T+T) (dense, mask may skip rows) or [offs[b], offs[b+1]) (packed).
// With ``cum`` the running sum after each row is also written to cum[b, t+1, :] (cum[b, 0] = start),
// so later consumers can take any prefix sum of a sequence's lens probabilities with one row read.
__global__ void __launch_bounds__(256) lens_colsum_kernel(const uint16_t* __restrict__ logits,
                                                          const float* __restrict__ lse,
                                                          const uint8_t* __restrict__ mask,
                                                          const int32_t* __restrict__ excl, float* __restrict__ acc,
                                                          int T, int V, int accumulate, int round_bf16,
                                                          const int32_t* __restrict__ offs, float* __restrict__ cum,
                                                          const int32_t* __restrict__ rowmap) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;   // 8-column group
  const int col0 = c * 8;
  if (col0 >= V) return;
  const bool full = col0 + 8 <= V;
  float a[8];
  float* dst = acc + (size_t)b * V + col0;
  if (accumulate && full) {
    const float4 x0 = reinterpret_cast<const float4*>(dst)[0], x1 = reinterpret_cast<const float4*>(dst)[1];
    a[0] = x0.x; a[1] = x0.y; a[2] = x0.z; a[3] = x0.w; a[4] = x1.x; a[5] = x1.y; a[6] = x1.z; a[7] = x1.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (accumulate && col0 + j < V) ? dst[j] : 0.f;
  }
  auto put = [&](float* d) {
    if (full) {
      reinterpret_cast<float4*>(d)[0] = make_float4(a[0], a[1], a[2], a[3]);
      reinterpret_cast<float4*>(d)[1] = make_float4(a[4], a[5], a[6], a[7]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (col0 + j < V) d[j] = a[j];
    }
  };
  const int r0 = offs ? offs[b] : b * T, r1 = offs ? offs[b + 1] : b * T + T;
  float* cb = cum ? cum + (size_t)b * (T + 1) * V + col0 : nullptr;
  if (cb) put(cb);
  for (int r = r0; r < r1; ++r) {
    if (mask == nullptr || mask[r]) {
      const int pr = rowmap ? rowmap[r] : r;             // physical logits row (deduplicated rows)
      const float l = lse[pr];
      const int e0 = excl[2 * r], e1 = excl[2 * r + 1];
      const uint16_t* row = logits + (size_t)pr * V;
      float f[8];
      if (full) {
        unpack8(*reinterpret_cast<const uint4*>(row + col0), f);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (col0 + j < V) ? bf2f(row[col0 + j]) : -INFINITY;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(f[j] - l);
        if (round_bf16) p = rbf(p);
        const int id = col0 + j;
        if (id == e0 || id == e1) p = 0.f;
        a[j] += p;
      }
    }
    if (cb) put(cb + (size_t)(r - r0 + 1) * V);
  }
  put(dst);
}

// Per-row top-k by k rounds of block argmax over per-thread sorted candidate lists (ties: lower column first).
// Workgroup b takes chunk b % C (CH columns) of row b / C and writes its k best to vals / idx[b * K ..]; with xi the
// row holds candidates whose columns are xi (the second pass of a chunked top-k: the same order, so the same set).
template <int KMAX>
__global__ void __launch_bounds__(256) topk_rows_kernel(const float* __restrict__ x, const int32_t* __restrict__ xi,
                                                        float* __restrict__ vals, int32_t* __restrict__ idx, int V,
                                                        int K, int CH, int C) {
  __shared__ float sv[4];
  __shared__ int si[4];
  __shared__ int win;
  const int r = blockIdx.x / C, ch = blockIdx.x - r * C;
  const float* row = x + (size_t)r * V;
  const int32_t* rowi = xi != nullptr ? xi + (size_t)r * V : nullptr;
  const int cend = min(V, (ch + 1) * CH);
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) { tv[j] = -INFINITY; ti[j] = 0x7fffffff; }
  // the list's last entry in registers: the common case (no insertion) reads no dynamically indexed list entry
  float thv = -INFINITY;
  int thi = 0x7fffffff;
  auto ins = [&](float v, int c) {
    if (!(v > thv || (v == thv && c < thi))) return;
    // insertion into the sorted list (descending, ties by lower index first) as an unrolled shift network: every
    // list index is a compile-time constant (a loop with a per-lane index became a waterfall over the lanes)
#pragma unroll
    for (int j = KMAX - 1; j >= 0; --j) {
      const bool here = v > tv[j] || (v == tv[j] && c < ti[j]);
      bool above = false;
      if (j > 0) above = v > tv[j - 1] || (v == tv[j - 1] && c < ti[j - 1]);
      if (j > 0 && above) { tv[j] = tv[j - 1]; ti[j] = ti[j - 1]; }
      else if (here) { tv[j] = v; ti[j] = c; }
    }
    thv = tv[K - 1];
    thi = ti[K - 1];
  };
  const int cbeg = ch * CH;
  if (rowi == nullptr && (V & 3) == 0 && (CH & 3) == 0) {
    // 16-B loads, 4 in flight per thread before any compare
    const float4* row4 = reinterpret_cast<const float4*>(row);
    const int b4 = cbeg >> 2, e4 = cend >> 2;
    for (int p = b4 + threadIdx.x; p < e4; p += 4 * blockDim.x) {
      float4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = p + u * blockDim.x;
        a[u] = q < e4 ? row4[q] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = 4 * (p + u * blockDim.x);
        if (c >= cend) break;
        ins(a[u].x, c);
        ins(a[u].y, c + 1);
        ins(a[u].z, c + 2);
        ins(a[u].w, c + 3);
      }
    }
  } else {
    for (int p = cbeg + threadIdx.x; p < cend; p += blockDim.x) ins(row[p], rowi != nullptr ? rowi[p] : p);
  }
  // K rounds of block argmax over the lists' heads; the winning list shifts left (constant indices, as above).
  // Entries past K are dropped first, so a list never offers more than its K best.
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j >= K) { tv[j] = -INFINITY; ti[j] = 0x7fffffff; }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = 0; k < K; ++k) {
    ArgBest b{tv[0], ti[0]};
    // ties: prefer lower index
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ArgBest oth{__shfl_xor(b.v, o, 64), __shfl_xor(b.i, o, 64)};
      b = better(b, oth);
    }
    if (lane == 0) { sv[wid] = b.v; si[wid] = b.i; }
    __syncthreads();
    if (threadIdx.x == 0) {
      ArgBest bb{sv[0], si[0]};
      for (int w = 1; w < 4; ++w) bb = better(bb, ArgBest{sv[w], si[w]});
      vals[(size_t)blockIdx.x * K + k] = bb.v;
      idx[(size_t)blockIdx.x * K + k] = bb.i;
      win = bb.i;
    }
    __syncthreads();
    if (ti[0] == win) {
#pragma unroll
      for (int j = 0; j + 1 < KMAX; ++j) { tv[j] = tv[j + 1]; ti[j] = ti[j + 1]; }
      tv[KMAX - 1] = -INFINITY;
      ti[KMAX - 1] = 0x7fffffff;
    }
    __syncthreads();
  }
}

template <int UNR>
__global__ void __launch_bounds__(512) xent_rows_kernel(const uint16_t* __restrict__ logits,
                                                        const int32_t* __restrict__ tgt, float* __restrict__ nll,
                                                        int V, float cap, int emulate_bf16,
                                                        const uint16_t* __restrict__ tab) {
  __shared__ float sm[8], ss[8];
  const int r = blockIdx.x;
  const int t = tgt[r];
  if (t < 0 || t >= V) {
    if (threadIdx.x == 0) nll[r] = 0.f;
    return;
  }
  extern __shared__ __attribute__((aligned(16))) uint16_t ctab_lds[];
  const uint16_t* ct = stage_ctab(tab, ctab_lds);
  const uint16_t* row = logits + (size_t)r * V;
  float m = -INFINITY, s = 0.f;
  const int nv = V >> 3;
  stream_row<UNR>(reinterpret_cast<const uint4*>(row), nv, [&](const uint4& v, int) {
    float f[8];
    capped8(v, f, ct, cap, emulate_bf16);
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) lm = fmaxf(lm, f[j]);
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(f[j] - lm);
    online_merge(m, s, lm, ls);
  });
  for (int c = nv * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float x = capped1(row[c], ct, cap, emulate_bf16);
    if (m == -INFINITY) { m = x; s = 1.f; } else online_add(m, s, x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) online_merge(M, Ssum, sm[w], ss[w]);
    const float zt = capped1(row[t], ct, cap, emulate_bf16);
    nll[r] = (M + __logf(Ssum)) - zt;
  }
}

template <int UNR>
__global__ void __launch_bounds__(512) decode_head_kernel(const uint16_t* __restrict__ logits,
                                                          const int32_t* __restrict__ tgt, int32_t* __restrict__ nxt,
                                                          float* __restrict__ nll_self, float* __restrict__ nll_tgt,
                                                          int V, float cap, const uint16_t* __restrict__ tab) {
  __shared__ float sm[8], ss[8], sv[8];
  __shared__ int si[8];
  extern __shared__ __attribute__((aligned(16))) uint16_t ctab_lds[];
  const uint16_t* ct = stage_ctab(tab, ctab_lds);
  const int r = blockIdx.x;
  const uint16_t* row = logits + (size_t)r * V;
  float m = -INFINITY, s = 0.f;
  ArgBest best{-INFINITY, 0x7fffffff};
  const int nv = V >> 3;
  stream_row<UNR>(reinterpret_cast<const uint4*>(row), nv, [&](const uint4& v, int c) {
    float f[8];
    capped8(v, f, ct, cap, 1);
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lm = fmaxf(lm, f[j]);
      best = better(best, ArgBest{f[j], c * 8 + j});
    }
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(f[j] - lm);
    online_merge(m, s, lm, ls);
  });
  for (int c = nv * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float x = capped1(row[c], ct, cap, 1);
    best = better(best, ArgBest{x, c});
    if (m == -INFINITY) { m = x; s = 1.f; } else online_add(m, s, x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
    ArgBest oth{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, oth);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; sv[wid] = best.v; si[wid] = best.i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    ArgBest b{sv[0], si[0]};
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      online_merge(M, Ssum, sm[w], ss[w]);
      b = better(b, ArgBest{sv[w], si[w]});
    }
    const float lse = M + __logf(Ssum);
    nxt[r] = b.i;
    nll_self[r] = lse - b.v;
    if (nll_tgt != nullptr) {
      const int t = tgt[r];
      float zt = 0.f;
      if (t >= 0 && t < V) zt = capped1(row[t], ct, cap, 1);
      nll_tgt[r] = (t >= 0 && t < V) ? lse - zt : 0.f;
    }
  }
}

// decode_head on the compact softcap (see CapC): same outputs as decode_head_kernel with the full table
template <int UNR>
__global__ void __launch_bounds__(512) decode_head_c_kernel(const uint16_t* __restrict__ logits,
                                                            const int32_t* __restrict__ tgt, int32_t* __restrict__ nxt,
                                                            float* __restrict__ nll_self, float* __restrict__ nll_tgt,
                                                            int V, CapC cc) {
  __shared__ float sm[8], ss[8], sv[8];
  __shared__ int si[8];
  __shared__ __attribute__((aligned(16))) uint16_t lt[CAPC_MAX];
  for (int i = threadIdx.x; i < cc.hi - cc.lo; i += blockDim.x) lt[i] = cc.tab[i];
  __syncthreads();
  const int r = blockIdx.x;
  const uint16_t* row = logits + (size_t)r * V;
  float m = -INFINITY, s = 0.f;
  ArgBest best{-INFINITY, 0x7fffffff};
  const int nv = V >> 3;
  stream_row<UNR>(reinterpret_cast<const uint4*>(row), nv, [&](const uint4& v, int c) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float f[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = capc1(w[k] & 0xffffu, lt, cc);
      f[2 * k + 1] = capc1(w[k] >> 16, lt, cc);
    }
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lm = fmaxf(lm, f[j]);
      best = better(best, ArgBest{f[j], c * 8 + j});
    }
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(f[j] - lm);
    online_merge(m, s, lm, ls);
  });
  for (int c = nv * 8 + threadIdx.x; c < V; c += blockDim.x) {
    const float x = capc1(row[c], lt, cc);
    best = better(best, ArgBest{x, c});
    if (m == -INFINITY) { m = x; s = 1.f; } else online_add(m, s, x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
    ArgBest oth{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = better(best, oth);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; sv[wid] = best.v; si[wid] = best.i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    ArgBest b{sv[0], si[0]};
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      online_merge(M, Ssum, sm[w], ss[w]);
      b = better(b, ArgBest{sv[w], si[w]});
    }
    const float lse = M + __logf(Ssum);
    nxt[r] = b.i;
    nll_self[r] = lse - b.v;
    if (nll_tgt != nullptr) {
      const int t = tgt[r];
      const float zt = (t >= 0 && t < V) ? capc1(row[t], lt, cc) : 0.f;
      nll_tgt[r] = (t >= 0 && t < V) ? lse - zt : 0.f;
    }
  }
}

// decode_head for 0 < cap <= DH_FIXED_CAP, the default: the same outputs as decode_head_kernel (argmax bit-exact,
// NLLs to fp32 summation order) on about half the VALU work per logit, which is what bound the row pass
// (2.9 TB/s).  (1) Capped logits lie in [-cap, cap], so sum(exp(z)) over the row can neither
// overflow nor underflow in fp32: no running max, no rescaling, one exp + add per logit.  (2) The argmax keeps
// the best 8-logit chunk (its max against the thread's best, strict > so the earliest chunk wins) and resolves
// the index inside the winning chunk once per row by re-reading its 16 B — first index of the max, as torch.
// (3) Persistent: 2 blocks per CU loop over the rows, so the 64 KB table is staged once per block instead of once
// per row (+12.5 % HBM/L2 traffic at the Gemma-2 vocab).
constexpr float DH_FIXED_CAP = 40.f;   // e^40 * 2^20 columns < FLT_MAX; e^-40 a normal float

// 8 capped logits of a uint4 through the 64 KB table at ~4 VALU ops per logit (the generic capped8 path costs ~5):
// the 15-bit magnitudes come from v_bfe (opaque to the compiler, which otherwise rewrites the index math into three
// ops), the two lookups of a dword are packed with one v_lshl_or, one v_and_or puts both signs back, a shift / a
// mask unpack them.  (ds_read_u16_d16_hi cannot pack them: with SRAM ECC on, d16 loads zero the other half.)
__device__ __forceinline__ void capped8_tab(const uint4& v, float* f, const uint16_t* ct) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t ilo, ihi, q;
    asm("v_bfe_u32 %0, %1, 0, 15" : "=v"(ilo) : "v"(w[k]));
    asm("v_bfe_u32 %0, %1, 16, 15" : "=v"(ihi) : "v"(w[k]));
    const uint32_t p = ((uint32_t)ct[ihi] << 16) | ct[ilo];   // table entries are magnitudes (bit 15 clear)
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(q) : "v"(w[k]), "s"(0x80008000u), "v"(p));
    f[2 * k] = __uint_as_float(q << 16);
    f[2 * k + 1] = __uint_as_float(q & 0xffff0000u);
  }
}

// v_max3_f32 / v_max_f32 without the canonicalising v_max x, x the compiler puts before fmaxf on bit-cast inputs
// (table values are never signalling NaNs)
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float fmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr f2 LOG2E2 = {1.4426950408889634f, 1.4426950408889634f};

// stats != nullptr (vocab-parallel TP head, models/gemma2.py): instead of the token / NLLs, per row the float4
// {log-sum-exp, best capped logit, its global vocab id (local + off), the capped logit of the teacher target
// tgt - off if it falls in this rank's [0, V) slice, else -inf}, merged over the ranks by vp_head_merge (vp.hip)
template <int UNR>
__global__ void __launch_bounds__(512) decode_head_f_kernel(const uint16_t* __restrict__ logits,
                                                            const int32_t* __restrict__ tgt, int32_t* __restrict__ nxt,
                                                            float* __restrict__ nll_self, float* __restrict__ nll_tgt,
                                                            int R, int V, const uint16_t* __restrict__ tab,
                                                            float4* __restrict__ stats, int off) {
  __shared__ float ss[8], sv[8];
  __shared__ int si[8];
  extern __shared__ __attribute__((aligned(16))) uint16_t ctab_lds[];
  const uint16_t* ct = stage_ctab(tab, ctab_lds);
  const int nv = V >> 3;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int r = blockIdx.x; r < R; r += gridDim.x) {
    const uint16_t* row = logits + (size_t)r * V;
    float s = 0.f, bv = -INFINITY;
    int bc = -1;
    f2 s2 = {0.f, 0.f};
    stream_row<UNR>(reinterpret_cast<const uint4*>(row), nv, [&](const uint4& v, int c) {
      float f[8];
      capped8_tab(v, f, ct);
      const float cm = max3_raw(max3_raw(f[0], f[1], f[2]), max3_raw(f[3], f[4], f[5]), fmax_raw(f[6], f[7]));
#pragma unroll
      for (int j = 0; j < 8; j += 2) {   // packed scale / add (v_pk_mul_f32, v_pk_add_f32), exp2 per lane
        const f2 y = f2{f[j], f[j + 1]} * LOG2E2;
        s2 += f2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
      }
      if (cm > bv) { bv = cm; bc = c; }
    });
    s = s2.x + s2.y;
    ArgBest best{bv, 0x7fffffff};
    if (bc >= 0) {
      float f[8];
      capped8(reinterpret_cast<const uint4*>(row)[bc], f, ct, 0.f, 1);
#pragma unroll
      for (int j = 7; j >= 0; --j)
        if (f[j] == bv) best.i = bc * 8 + j;
    }
    for (int c = nv * 8 + threadIdx.x; c < V; c += blockDim.x) {
      const float x = capped1(row[c], ct, 0.f, 1);
      s += __expf(x);
      best = better(best, ArgBest{x, c});
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 64);
      ArgBest oth{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
      best = better(best, oth);
    }
    if (lane == 0) { ss[wid] = s; sv[wid] = best.v; si[wid] = best.i; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float Ssum = ss[0];
      ArgBest b{sv[0], si[0]};
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
        Ssum += ss[w];
        b = better(b, ArgBest{sv[w], si[w]});
      }
      const float lse = __logf(Ssum);
      if (stats != nullptr) {
        const int t = tgt != nullptr ? tgt[r] - off : -1;
        const float tl = (tgt != nullptr && tgt[r] >= 0 && t >= 0 && t < V) ? capped1(row[t], ct, 0.f, 1) : -INFINITY;
        stats[r] = make_float4(lse, b.v, (float)(b.i + off), tl);   // vocab ids < 2^24: exact in fp32
      } else {
        nxt[r] = b.i;
        nll_self[r] = lse - b.v;
        if (nll_tgt != nullptr) {
          const int t = tgt[r];
          nll_tgt[r] = (t >= 0 && t < V) ? lse - capped1(row[t], ct, 0.f, 1) : 0.f;
        }
      }
    }
    __syncthreads();   // ss / sv / si are rewritten by the next row
  }
}

// elementwise exact softcap through the compact path (ops.softcap_values; the exhaustive GPU test)
__global__ void softcap_c_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int n, CapC cc) {
  __shared__ uint16_t lt[CAPC_MAX];
  for (int i = threadIdx.x; i < cc.hi - cc.lo; i += blockDim.x) lt[i] = cc.tab[i];
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = capc1(x[i], lt, cc);
}

struct CapCEntry {
  int dev;
  uint32_t capbits;
  CapC c;
};
CapCEntry g_capc[16];
int g_ncapc = 0;

const CapC* find_capc(float cap) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint32_t cb = __builtin_bit_cast(uint32_t, cap);
  for (int i = 0; i < g_ncapc; ++i)
    if (g_capc[i].dev == dev && g_capc[i].capbits == cb) return &g_capc[i].c;
  return nullptr;
}

// softcap tables registered from the host, keyed by (device, cap bits)
struct CapTab {
  int dev;
  uint32_t capbits;
  const uint16_t* ptr;
};
CapTab g_tabs[16];
int g_ntabs = 0;

const uint16_t* find_tab(float cap, int emulate) {
  if (!(cap > 0.f) || !emulate) return nullptr;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint32_t cb = __builtin_bit_cast(uint32_t, cap);
  for (int i = 0; i < g_ntabs; ++i)
    if (g_tabs[i].dev == dev && g_tabs[i].capbits == cb) return g_tabs[i].ptr;
  return nullptr;
}

size_t tab_lds(const void* kernel, const uint16_t* tab, bool& attr_done) {
  if (tab == nullptr) return 0;
  if (!attr_done) {   // > 64 KB of LDS needs the opt-in; first call is never inside a graph capture
    (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, CTAB_N * 2 + 256);
    attr_done = true;
  }
  return CTAB_N * 2;
}

}  // namespace

void tb_register_softcap_table(float cap, const uint16_t* tab) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint32_t cb = __builtin_bit_cast(uint32_t, cap);
  for (int i = 0; i < g_ntabs; ++i)
    if (g_tabs[i].dev == dev && g_tabs[i].capbits == cb) { g_tabs[i].ptr = tab; return; }
  if (g_ntabs < 16) g_tabs[g_ntabs++] = CapTab{dev, cb, tab};
}

const uint16_t* tb_find_softcap_table(float cap) { return find_tab(cap, 1); }

bool tb_register_softcap_compact(float cap, const uint16_t* tab, int lo, int hi, float sat) {
  if (hi < lo || hi - lo > CAPC_MAX || !(cap > 0.f)) return false;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint32_t cb = __builtin_bit_cast(uint32_t, cap);
  const CapC c{tab, lo, hi, sat, 1.0f / cap, cap};
  for (int i = 0; i < g_ncapc; ++i)
    if (g_capc[i].dev == dev && g_capc[i].capbits == cb) { g_capc[i].c = c; return true; }
  if (g_ncapc >= 16) return false;
  g_capc[g_ncapc++] = CapCEntry{dev, cb, c};
  return true;
}

bool tb_softcap_compact_params(float cap, const uint16_t** tab, int* lo, int* hi, float* sat) {
  const CapC* c = find_capc(cap);
  if (c == nullptr) return false;
  *tab = c->tab;
  *lo = c->lo;
  *hi = c->hi;
  *sat = c->sat;
  return true;
}

bool tb_softcap_compact(const uint16_t* x, float* y, int n, float cap, hipStream_t st) {
  const CapC* c = find_capc(cap);
  if (c == nullptr || n <= 0) return c != nullptr;
  hipLaunchKernelGGL(softcap_c_kernel, dim3(std::min((n + 255) / 256, 4096)), dim3(256), 0, st, x, y, n, *c);
  return true;
}

bool tb_decode_head_stats(const uint16_t* logits, const int32_t* tgt, int off, float* stats, int R, int V, float cap,
                          hipStream_t st) {
  const uint16_t* tab = find_tab(cap, 1);
  if (tab == nullptr || !(cap <= DH_FIXED_CAP)) return false;
  if (R <= 0) return true;
  static bool attr = false;
  static const int ncu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  hipLaunchKernelGGL(decode_head_f_kernel<1>, dim3(std::min(R, 2 * ncu)), dim3(512),
                     tab_lds(reinterpret_cast<const void*>(&decode_head_f_kernel<1>), tab, attr), st, logits, tgt,
                     nullptr, nullptr, nullptr, R, V, tab, reinterpret_cast<float4*>(stats), off);
  return true;
}

void tb_decode_head(const uint16_t* logits, const int32_t* tgt, int32_t* nxt, float* nll_self, float* nll_tgt, int R,
                    int V, float cap, hipStream_t st) {
  if (R <= 0) return;
  // TB_DECODE_HEAD: "t" the per-row 64 KB-table kernel, "c" the compact-softcap kernel (A/B; both keep a running
  // max), default "f": decode_head_f_kernel where the cap allows it
  static const char mode = [] {
    const char* e = getenv("TB_DECODE_HEAD");
    return e != nullptr && (e[0] == 't' || e[0] == 'c') ? e[0] : 'f';
  }();
  const uint16_t* tab = find_tab(cap, 1);
  if (mode == 'f' && tab != nullptr && cap <= DH_FIXED_CAP) {
    static bool attr = false, attr1 = false;
    static const int ncu = [] {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return n > 0 ? n : 256;
    }();
    const int grid = std::min(R, 2 * ncu);
    if (row_unr() == 1)   // (8 loads in flight per lane measured 2-5 % slower than 4: profiles/r3/dh5)
      hipLaunchKernelGGL(decode_head_f_kernel<1>, dim3(grid), dim3(512),
                         tab_lds(reinterpret_cast<const void*>(&decode_head_f_kernel<1>), tab, attr1), st, logits, tgt,
                         nxt, nll_self, nll_tgt, R, V, tab, nullptr, 0);
    else
      hipLaunchKernelGGL(decode_head_f_kernel<ROW_UNR>, dim3(grid), dim3(512),
                         tab_lds(reinterpret_cast<const void*>(&decode_head_f_kernel<ROW_UNR>), tab, attr), st, logits,
                         tgt, nxt, nll_self, nll_tgt, R, V, tab, nullptr, 0);
    return;
  }
  if (const CapC* cc = find_capc(cap); cc != nullptr && mode != 't') {
    if (row_unr() == 1)
      hipLaunchKernelGGL(decode_head_c_kernel<1>, dim3(R), dim3(512), 0, st, logits, tgt, nxt, nll_self, nll_tgt, V, *cc);
    else
      hipLaunchKernelGGL(decode_head_c_kernel<ROW_UNR>, dim3(R), dim3(512), 0, st, logits, tgt, nxt, nll_self, nll_tgt, V,
                         *cc);
    return;
  }
  static bool attr_decode_head_kernel = false, attr_decode_head_kernel1 = false;
  if (row_unr() == 1)
    hipLaunchKernelGGL(decode_head_kernel<1>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&decode_head_kernel<1>), tab, attr_decode_head_kernel1), st, logits, tgt, nxt,
                     nll_self, nll_tgt, V, cap, tab);
  else
    hipLaunchKernelGGL(decode_head_kernel<ROW_UNR>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&decode_head_kernel<ROW_UNR>), tab, attr_decode_head_kernel), st, logits, tgt, nxt,
                     nll_self, nll_tgt, V, cap, tab);
}

void tb_argmax_rows(const uint16_t* logits, int32_t* out, int R, int V, float cap, hipStream_t st) {
  if (R <= 0) return;
  const uint16_t* tab = find_tab(cap, 1);
  static bool attr_argmax_rows_kernel = false, attr_argmax_rows_kernel1 = false;
  if (row_unr() == 1)
    hipLaunchKernelGGL(argmax_rows_kernel<1>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&argmax_rows_kernel<1>), tab, attr_argmax_rows_kernel1), st, logits, out, V, cap,
                     tab);
  else
    hipLaunchKernelGGL(argmax_rows_kernel<ROW_UNR>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&argmax_rows_kernel<ROW_UNR>), tab, attr_argmax_rows_kernel), st, logits, out, V, cap,
                     tab);
}

void tb_row_lse(const uint16_t* logits, float* lse, int R, int V, float cap, int emulate_bf16, hipStream_t st) {
  if (R <= 0) return;
  const uint16_t* tab = find_tab(cap, emulate_bf16);
  static bool attr_row_lse_kernel = false, attr_row_lse_kernel1 = false;
  if (row_unr() == 1)
    hipLaunchKernelGGL(row_lse_kernel<1>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&row_lse_kernel<1>), tab, attr_row_lse_kernel1), st, logits, lse, V, cap,
                     emulate_bf16, tab);
  else
    hipLaunchKernelGGL(row_lse_kernel<ROW_UNR>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&row_lse_kernel<ROW_UNR>), tab, attr_row_lse_kernel), st, logits, lse, V, cap,
                     emulate_bf16, tab);
}

void tb_gather_probs(const uint16_t* logits, const float* lse, const int32_t* ids, float* out, int R, int K, int V,
                     int round_bf16, const int32_t* rowmap, hipStream_t st) {
  if (R <= 0 || K <= 0) return;
  const int n = R * K;
  hipLaunchKernelGGL(gather_probs_kernel, dim3((n + 255) / 256), dim3(256), 0, st, logits, lse, ids, out, R, K, V,
                     round_bf16, rowmap);
}

void tb_lens_colsum(const uint16_t* logits, const float* lse, const uint8_t* mask, const int32_t* excl, float* acc,
                    int B, int T, int V, int accumulate, int round_bf16, const int32_t* offs, float* cum,
                    const int32_t* rowmap, hipStream_t st) {
  if (B <= 0) return;
  const int groups = (V + 7) / 8;
  dim3 grid((groups + 255) / 256, B);
  hipLaunchKernelGGL(lens_colsum_kernel, grid, dim3(256), 0, st, logits, lse, mask, excl, acc, T, V, accumulate,
                     round_bf16, offs, cum, rowmap);
}

int tb_topk_chunks(int R, int V) { return (R >= 512 || V <= 4096) ? 1 : (V + 2047) / 2048; }

namespace {
void topk_launch(const float* x, const int32_t* xi, float* vals, int32_t* idx, int R, int V, int K, int CH, int C,
                 hipStream_t st) {
  const dim3 g(R * C);
  if (K <= 8) hipLaunchKernelGGL(topk_rows_kernel<8>, g, dim3(256), 0, st, x, xi, vals, idx, V, K, CH, C);
  else if (K <= 16) hipLaunchKernelGGL(topk_rows_kernel<16>, g, dim3(256), 0, st, x, xi, vals, idx, V, K, CH, C);
  else hipLaunchKernelGGL(topk_rows_kernel<64>, g, dim3(256), 0, st, x, xi, vals, idx, V, K, CH, C);
}
}  // namespace

// few long rows (the lens top-k over the vocabulary: a few hundred workgroups streaming 1 MB rows cannot fill the
// chip): C chunks of each row give C * K candidates each, then one pass over the candidates per row
void tb_topk_rows(const float* x, float* vals, int32_t* idx, int R, int V, int K, float* wv, int32_t* wi, int C,
                  hipStream_t st) {
  if (R <= 0) return;
  if (C <= 1 || wv == nullptr || wi == nullptr) {
    topk_launch(x, nullptr, vals, idx, R, V, K, V, 1, st);
    return;
  }
  const int CH = (((V + C - 1) / C) + 3) & ~3;
  topk_launch(x, nullptr, wv, wi, R, V, K, CH, C, st);
  topk_launch(wv, wi, vals, idx, R, C * K, K, C * K, 1, st);
}

void tb_xent_rows(const uint16_t* logits, const int32_t* tgt, float* nll, int R, int V, float cap, int emulate_bf16,
                  hipStream_t st) {
  if (R <= 0) return;
  const uint16_t* tab = find_tab(cap, emulate_bf16);
  static bool attr_xent_rows_kernel = false, attr_xent_rows_kernel1 = false;
  if (row_unr() == 1)
    hipLaunchKernelGGL(xent_rows_kernel<1>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&xent_rows_kernel<1>), tab, attr_xent_rows_kernel1), st, logits, tgt, nll, V,
                     cap, emulate_bf16, tab);
  else
    hipLaunchKernelGGL(xent_rows_kernel<ROW_UNR>, dim3(R), dim3(512), tab_lds(reinterpret_cast<const void*>(&xent_rows_kernel<ROW_UNR>), tab, attr_xent_rows_kernel), st, logits, tgt, nll, V,
                     cap, emulate_bf16, tab);
}
