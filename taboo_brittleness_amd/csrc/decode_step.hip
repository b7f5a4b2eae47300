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

// Prefix-trie regrouping after a decode step (runtime/generation.py _share_group), one workgroup: rows i < nb keyed
// by (group, emitted token) (rows >= act: one parked group) are grouped through a 16384-slot LDS hash table; each
// group's representative is its first row, dense group ids follow the representatives' row order (a block scan),
// so the result is deterministic.  Replaces torch.unique's sort + scatter-reduce + ~8 small kernels per step.
constexpr int SG_THREADS = 1024, SG_TAB = 16384, SG_RMAX = 8;   // rows <= SG_THREADS * SG_RMAX
__global__ void __launch_bounds__(SG_THREADS) share_group_kernel(int64_t* __restrict__ gid,
                                                                 const int32_t* __restrict__ tok,
                                                                 int64_t* __restrict__ rep, int64_t* __restrict__ grp,
                                                                 int32_t* __restrict__ src, int64_t* __restrict__ U,
                                                                 int nb, int act, int first, int64_t V) {
  __shared__ unsigned long long tab[SG_TAB];   // keys, then (reused) the slot's first row, then its dense id
  __shared__ int scan[SG_THREADS];
  constexpr unsigned long long EMPTY = 0x8000000000000000ull;   // keys are >= -1
  const int t = threadIdx.x;
  const int R = (nb + SG_THREADS - 1) / SG_THREADS;
  for (int s = t; s < SG_TAB; s += SG_THREADS) tab[s] = EMPTY;
  __syncthreads();
  int slot[SG_RMAX];
#pragma unroll
  for (int k = 0; k < SG_RMAX; ++k) {
    const int i = t * R + k;
    slot[k] = -1;
    if (k < R && i < nb) {
      const long long key = i >= act ? -1ll : (first ? (long long)gid[i] : (long long)gid[i] * V + tok[i]);
      const unsigned long long uk = (unsigned long long)key;
      unsigned h = (unsigned)((uk * 0x9E3779B97F4A7C15ull) >> 50) & (SG_TAB - 1);
      for (;;) {
        const unsigned long long prev = atomicCAS(&tab[h], EMPTY, uk);
        if (prev == EMPTY || prev == uk) break;
        h = (h + 1) & (SG_TAB - 1);
      }
      slot[k] = (int)h;
    }
  }
  __syncthreads();
  int* first_row = reinterpret_cast<int*>(tab);
  for (int s = t; s < SG_TAB; s += SG_THREADS) first_row[s] = 0x7fffffff;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SG_RMAX; ++k)
    if (slot[k] >= 0) atomicMin(&first_row[slot[k]], t * R + k);
  __syncthreads();
  int r[SG_RMAX], cnt = 0;
#pragma unroll
  for (int k = 0; k < SG_RMAX; ++k) {
    r[k] = slot[k] >= 0 ? first_row[slot[k]] : -1;
    cnt += slot[k] >= 0 && r[k] == t * R + k;
  }
  scan[t] = cnt;
  __syncthreads();
  for (int off = 1; off < SG_THREADS; off <<= 1) {   // inclusive scan (Hillis-Steele)
    const int v = t >= off ? scan[t - off] : 0;
    __syncthreads();
    scan[t] += v;
    __syncthreads();
  }
  int d = scan[t] - cnt;   // this thread's first dense id
  int* dense = first_row;  // (every first_row read is done: the scan's barriers)
#pragma unroll
  for (int k = 0; k < SG_RMAX; ++k) {
    const int i = t * R + k;
    if (slot[k] >= 0 && r[k] == i) {
      dense[slot[k]] = d;
      rep[d] = i;
      ++d;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SG_RMAX; ++k) {
    const int i = t * R + k;
    if (slot[k] >= 0) {
      const int g = dense[slot[k]];
      grp[i] = g;
      gid[i] = g;
      src[i] = (r[k] == i || i >= act) ? -1 : r[k];
    }
  }
  if (t == SG_THREADS - 1) *U = scan[SG_THREADS - 1];
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

int tb_share_group_max_rows() { return SG_THREADS * SG_RMAX; }

void tb_share_group(int64_t* gid, const int32_t* tok, int64_t* rep, int64_t* grp, int32_t* src, int64_t* U, int nb,
                    int act, int first, int64_t V, hipStream_t st) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(share_group_kernel, dim3(1), dim3(SG_THREADS), 0, st, gid, tok, rep, grp, src, U, nb, act, first,
                     V);
}
