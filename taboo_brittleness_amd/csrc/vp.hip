// Vocab-parallel merges for tensor parallelism ("vocab-parallel lm_head (128000 per rank) ... the
// logit lens needs a softmax max/sum all-reduce [42·T] plus a top-k candidate all-gather").
//
// Under TP each rank unembeds its V/tp rows of lm_head (a row slice of the tied embedding); the group then
// exchanges a few numbers per row with one all-gather (parallel/p2p.py, capturable) and every rank merges them
// in rank order = vocab order, so all ranks hold bit-identical results:
//   * head (decode step): {log-sum-exp, best capped logit, its index, target logit} per
//     (rank, row) -> greedy token, its NLL, the teacher target's NLL;
//   * lens: the local log-sum-exp per (rank, row) -> the row's global log-sum-exp, which the
//     lens readouts (gather_probs / lens_colsum) then apply to their local vocab slice;
//   * lens top-k: each rank's top-k of its local response sums (global ids) -> the global top-k,
//     ties to the lower vocab index (the single-GPU topk_rows order).
// One thread per row: the data is tp x a few floats per row, the launches are latency-, not bandwidth-bound.
#include "common.h"
#include "api.h"

namespace {

// log-sum-exp pair (m, s) <- merge (m2, s2); -inf parts are empty
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
  else s += s2 * __expf(m2 - m);
}

__global__ void __launch_bounds__(256) vp_head_merge_kernel(const float4* __restrict__ st, int tp, int R,
                                                            const int32_t* __restrict__ tgt, int V,
                                                            int32_t* __restrict__ nxt, float* __restrict__ nll_self,
                                                            float* __restrict__ nll_tgt) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float m = -INFINITY, s = 0.f, best = -INFINITY, bidx = 0.f, tl = -INFINITY;
  for (int k = 0; k < tp; ++k) {           // rank order = vocab order
    const float4 q = st[(size_t)k * R + r];
    lse_merge(m, s, q.x, 1.f);             // a rank's lse is log(sum) at scale 0: (lse, 1)
    if (q.y > best) { best = q.y; bidx = q.z; }   // strict: on a tie the lower rank (lower vocab id) keeps it
    tl = fmaxf(tl, q.w);
  }
  const float lse = m + __logf(s);
  if (nxt) nxt[r] = (int32_t)bidx;
  if (nll_self) nll_self[r] = lse - best;
  if (nll_tgt) {
    const int t = tgt ? tgt[r] : -1;
    nll_tgt[r] = (t >= 0 && t < V) ? lse - tl : 0.f;
  }
}

__global__ void __launch_bounds__(256) vp_lse_merge_kernel(const float* __restrict__ lse, int tp, int R,
                                                           float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float m = -INFINITY, s = 0.f;
  for (int k = 0; k < tp; ++k) lse_merge(m, s, lse[(size_t)k * R + r], 1.f);
  out[r] = m + __logf(s);
}

template <int KMAX>
__global__ void __launch_bounds__(256) vp_topk_merge_kernel(const float* __restrict__ vals,
                                                            const int32_t* __restrict__ ids, int tp, int n, int k,
                                                            float* __restrict__ ov, int32_t* __restrict__ oi) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) { tv[j] = -INFINITY; ti[j] = 0x7fffffff; }
  for (int q = 0; q < tp; ++q)
    for (int c = 0; c < k; ++c) {
      const float v = vals[((size_t)q * n + r) * k + c];
      const int id = ids[((size_t)q * n + r) * k + c];
      if (!(v > tv[k - 1] || (v == tv[k - 1] && id < ti[k - 1]))) continue;
      int j = k - 1;                        // insertion: descending, ties by lower id first
      while (j > 0 && (v > tv[j - 1] || (v == tv[j - 1] && id < ti[j - 1]))) {
        tv[j] = tv[j - 1];
        ti[j] = ti[j - 1];
        --j;
      }
      tv[j] = v;
      ti[j] = id;
    }
  for (int j = 0; j < k; ++j) {
    ov[(size_t)r * k + j] = tv[j];
    oi[(size_t)r * k + j] = ti[j];
  }
}

}  // namespace

void tb_vp_head_merge(const float* st, int tp, int R, const int32_t* tgt, int V, int32_t* nxt, float* nll_self,
                      float* nll_tgt, hipStream_t stream) {
  if (R <= 0) return;
  hipLaunchKernelGGL(vp_head_merge_kernel, dim3((R + 255) / 256), dim3(256), 0, stream,
                     reinterpret_cast<const float4*>(st), tp, R, tgt, V, nxt, nll_self, nll_tgt);
}

void tb_vp_lse_merge(const float* lse, int tp, int R, float* out, hipStream_t stream) {
  if (R <= 0) return;
  hipLaunchKernelGGL(vp_lse_merge_kernel, dim3((R + 255) / 256), dim3(256), 0, stream, lse, tp, R, out);
}

void tb_vp_topk_merge(const float* vals, const int32_t* ids, int tp, int n, int k, float* ov, int32_t* oi,
                      hipStream_t stream) {
  if (n <= 0) return;
  if (k <= 8)
    hipLaunchKernelGGL(vp_topk_merge_kernel<8>, dim3((n + 255) / 256), dim3(256), 0, stream, vals, ids, tp, n, k, ov,
                       oi);
  else
    hipLaunchKernelGGL(vp_topk_merge_kernel<64>, dim3((n + 255) / 256), dim3(256), 0, stream, vals, ids, tp, n, k, ov,
                       oi);
}
