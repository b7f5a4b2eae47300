// Per-step bookkeeping of the batched greedy decode (runtime/generation.py), one thread per row, and the bf16 row
// moves around it (residual capture into the sweep's store, group-residual gathers).  In PyTorch these
// were ~15 tiny kernels per captured decode step (gather / where / three scatters / compare + any / copies / adds)
// and ~8 more per prefix-trie step; each cost a launch slot and a few microseconds of an otherwise idle GPU inside
// the hipGraph.  Reference: the greedy `generate` loop of /root/reference/src/models.py:74-79 (argmax token,
// stop on <end_of_turn>/<eos>).
#include "common.h"
#include "api.h"

namespace {

constexpr int DS_THREADS = 256;

// teacher target of the column this step writes: tf_step[r] = tf_tgt[r, min(step_idx[r], W - 1)]
__global__ void __launch_bounds__(DS_THREADS) decode_pre_kernel(const int64_t* __restrict__ step_idx,
                                                                const int32_t* __restrict__ tf_tgt,
                                                                int32_t* __restrict__ tf_step, int nb, int W) {
  const int r = blockIdx.x * DS_THREADS + threadIdx.x;
  if (r >= nb) return;
  const int64_t c = min(step_idx[r], (int64_t)(W - 1));
  tf_step[r] = tf_tgt[(size_t)r * W + c];
}

// after the head: the row's token (pad once done), its NLLs into the output columns, the stop check, and the next
// step's inputs (token, position + 1, column + 1)
__global__ void __launch_bounds__(DS_THREADS) decode_post_kernel(
    const int32_t* __restrict__ nxt, const float* __restrict__ nll, const float* __restrict__ tf_nll,
    uint8_t* __restrict__ done, int64_t* __restrict__ step_idx, int32_t* __restrict__ out_tok,
    float* __restrict__ out_nll, float* __restrict__ out_tf_nll, const int32_t* __restrict__ stop, int nstop,
    int32_t* __restrict__ tok, int32_t* __restrict__ pos, int nb, int W, int pad) {
  const int r = blockIdx.x * DS_THREADS + threadIdx.x;
  if (r >= nb) return;
  const int64_t si = step_idx[r];
  const size_t o = (size_t)r * W + min(si, (int64_t)(W - 1));
  const bool d = done[r] != 0;
  const int32_t n = d ? pad : nxt[r];
  out_tok[o] = n;
  out_nll[o] = nll[r];
  out_tf_nll[o] = tf_nll[r];
  bool s = false;
  for (int i = 0; i < nstop; ++i) s |= n == stop[i];
  done[r] = (uint8_t)(d || s);
  tok[r] = n;
  pos[r] += 1;
  step_idx[r] = si + 1;
}

// prefix-trie decode, blocks 0..l: the representative row rep[i] of each group i < U feeds lo row i (rows >= U
// are parked at position S)
__global__ void __launch_bounds__(DS_THREADS) share_lo_gather_kernel(
    const int64_t* __restrict__ rep, const int64_t* __restrict__ U, const int32_t* __restrict__ tok,
    const int32_t* __restrict__ pos, const int32_t* __restrict__ slot, int32_t* __restrict__ s_tok,
    int32_t* __restrict__ s_pos, int32_t* __restrict__ s_slot, const int32_t* __restrict__ kp_slot,
    const int32_t* __restrict__ kp_len_lo, int32_t* __restrict__ l_slot, int32_t* __restrict__ l_len_lo, int nb,
    int B, int S) {
  const int i = blockIdx.x * DS_THREADS + threadIdx.x;
  if (i >= nb) return;
  const int64_t r = min(max(rep[i], (int64_t)0), (int64_t)(B - 1));
  s_tok[i] = tok[r];
  s_pos[i] = i < *U ? pos[r] : S;
  s_slot[i] = slot[r];
  if (kp_slot != nullptr) {
    l_slot[i] = kp_slot[r];
    l_len_lo[i] = kp_len_lo[r];
  }
}

// store row slot[b] * S1 + (pos valid ? pos : S1 - 1) <- h row b * T + t (16-B vectors; padding rows land in each
// slot's scratch row S1 - 1)
__global__ void __launch_bounds__(DS_THREADS) capture_rows_kernel(uint16_t* __restrict__ store,
                                                                  const uint16_t* __restrict__ h,
                                                                  const int32_t* __restrict__ pos,
                                                                  const int32_t* __restrict__ slot, int T, int S1,
                                                                  int D) {
  const int i = blockIdx.x;
  const int p = pos[i];
  const int pp = (p >= 0 && p < S1 - 1) ? p : S1 - 1;
  const size_t dst = ((size_t)slot[i / T] * S1 + pp) * D, src = (size_t)i * D;
  for (int c = threadIdx.x * 8; c < D; c += DS_THREADS * 8)
    *reinterpret_cast<uint4*>(store + dst + c) = *reinterpret_cast<const uint4*>(h + src + c);
}

// out row i <- src row idx[i]
template <typename I>
__global__ void __launch_bounds__(DS_THREADS) row_gather_kernel(uint16_t* __restrict__ out,
                                                                const uint16_t* __restrict__ src,
                                                                const I* __restrict__ idx, int D) {
  const int i = blockIdx.x;
  const size_t s = (size_t)idx[i] * D, d = (size_t)i * D;
  for (int c = threadIdx.x * 8; c < D; c += DS_THREADS * 8)
    *reinterpret_cast<uint4*>(out + d + c) = *reinterpret_cast<const uint4*>(src + s + c);
}

inline int ds_grid(int n) { return (n + DS_THREADS - 1) / DS_THREADS; }

}  // namespace

void tb_decode_pre(const int64_t* step_idx, const int32_t* tf_tgt, int32_t* tf_step, int nb, int W, hipStream_t st) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(decode_pre_kernel, dim3(ds_grid(nb)), dim3(DS_THREADS), 0, st, step_idx, tf_tgt, tf_step, nb, W);
}

void tb_decode_post(const int32_t* nxt, const float* nll, const float* tf_nll, uint8_t* done, int64_t* step_idx,
                    int32_t* out_tok, float* out_nll, float* out_tf_nll, const int32_t* stop, int nstop, int32_t* tok,
                    int32_t* pos, int nb, int W, int pad, hipStream_t st) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(decode_post_kernel, dim3(ds_grid(nb)), dim3(DS_THREADS), 0, st, nxt, nll, tf_nll, done, step_idx,
                     out_tok, out_nll, out_tf_nll, stop, nstop, tok, pos, nb, W, pad);
}

void tb_share_lo_gather(const int64_t* rep, const int64_t* U, const int32_t* tok, const int32_t* pos,
                        const int32_t* slot, int32_t* s_tok, int32_t* s_pos, int32_t* s_slot, const int32_t* kp_slot,
                        const int32_t* kp_len_lo, int32_t* l_slot, int32_t* l_len_lo, int nb, int B, int S,
                        hipStream_t st) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(share_lo_gather_kernel, dim3(ds_grid(nb)), dim3(DS_THREADS), 0, st, rep, U, tok, pos, slot, s_tok,
                     s_pos, s_slot, kp_slot, kp_len_lo, l_slot, l_len_lo, nb, B, S);
}

void tb_capture_rows(uint16_t* store, const uint16_t* h, const int32_t* pos, const int32_t* slot, int n, int T, int S1,
                     int D, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(capture_rows_kernel, dim3(n), dim3(DS_THREADS), 0, st, store, h, pos, slot, T, S1, D);
}

void tb_row_gather(uint16_t* out, const uint16_t* src, const void* idx, bool idx64, int n, int D, hipStream_t st) {
  if (n <= 0) return;
  if (idx64)
    hipLaunchKernelGGL(row_gather_kernel<int64_t>, dim3(n), dim3(DS_THREADS), 0, st, out, src,
                       static_cast<const int64_t*>(idx), D);
  else
    hipLaunchKernelGGL(row_gather_kernel<int32_t>, dim3(n), dim3(DS_THREADS), 0, st, out, src,
                       static_cast<const int32_t*>(idx), D);
}
