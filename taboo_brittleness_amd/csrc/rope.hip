// RoPE on q/k + KV-cache scatter.
//
// Input is the fused QKV projection output [M, (Hq + 2*Hkv) * HD] (one GEMM).
// Per row: rotate q heads into q_out [M, Hq, HD], rotate k heads and copy v
// heads into the layer's cache slot at the row's absolute position.  Rows with
// pos < 0 are padding: their q is zeroed and nothing is written to the cache.
//
// Rounding mirrors transformers' bf16 apply_rotary_pos_emb: cos/sin tables are
// fp32 (HF computes them in fp32) rounded to bf16, and each product and the
// sum are bf16-rounded: out = bf16(bf16(x*cos) + bf16(rot(x)*sin)).
#include "common.h"
#include "api.h"

namespace {

// 8 consecutive qkv values of a row: bf16 from the projection output, or (PART) the ordered sum of the ks fp32
// split-K partials [ks, M, N] of the projection (gemm4.hip tb_gemm4_splitk_part) rounded to bf16 -- exactly what
// the split-K reduction kernel would have stored
template <bool PART>
__device__ __forceinline__ void qkv_load8(const uint16_t* row, const float* prow, int ks, size_t plane, int off,
                                          float (&x)[8]) {
  if constexpr (PART) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = 0.f;
    sum_splits8(prow + off, plane, ks, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = rbf(x[j]);
  } else {
    unpack8(*reinterpret_cast<const uint4*>(row + off), x);
  }
}

template <bool PART>
__global__ void __launch_bounds__(256) rope_qkv_cache_kernel(
    const uint16_t* __restrict__ qkv, const float* __restrict__ part, int ks, int M, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ slot_of_row, const float* __restrict__ cos_t, const float* __restrict__ sin_t,
    uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc, uint16_t* __restrict__ vc, int Hq, int Hkv, int HD, int S,
    int max_pos) {
  const int m = blockIdx.x;
  const int p = pos[m];
  const int half = HD >> 1, gph = half >> 3;            // 8-element groups per half head
  const int nrot = (Hq + Hkv) * gph, nv = Hkv * (HD >> 3);
  const int N = (Hq + 2 * Hkv) * HD;
  const uint16_t* row = PART ? nullptr : qkv + (size_t)m * N;
  const float* prow = PART ? part + (size_t)m * N : nullptr;
  const size_t plane = (size_t)M * N;
  const int slot = slot_of_row[m];
  for (int it = threadIdx.x + blockIdx.y * blockDim.x; it < nrot + nv; it += blockDim.x * gridDim.y) {
    if (it < nrot) {
      const int head = it / gph, g = it % gph;
      const bool is_q = head < Hq;
      const int src = head * HD + g * 8;
      if (p < 0) {
        if (is_q) {
          uint4 z = {0, 0, 0, 0};
          uint16_t* dq = q_out + ((size_t)m * Hq + head) * HD + g * 8;
          *reinterpret_cast<uint4*>(dq) = z;
          *reinterpret_cast<uint4*>(dq + half) = z;
        }
        continue;
      }
      const int pp = p < max_pos ? p : max_pos - 1;
      float x1[8], x2[8], o1[8], o2[8];
      qkv_load8<PART>(row, prow, ks, plane, src, x1);
      qkv_load8<PART>(row, prow, ks, plane, src + half, x2);
      const float* ct = cos_t + (size_t)pp * half + g * 8;
      const float* st = sin_t + (size_t)pp * half + g * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = rbf(ct[j]), s = rbf(st[j]);
        o1[j] = rbf(rbf(x1[j] * c) + rbf(-x2[j] * s));
        o2[j] = rbf(rbf(x2[j] * c) + rbf(x1[j] * s));
      }
      uint16_t* dst;
      if (is_q) {
        dst = q_out + ((size_t)m * Hq + head) * HD + g * 8;
      } else {
        if (p >= S) continue;
        const int kh = head - Hq;
        dst = kc + (((size_t)slot * Hkv + kh) * S + p) * HD + g * 8;
      }
      *reinterpret_cast<uint4*>(dst) = pack8(o1);
      *reinterpret_cast<uint4*>(dst + half) = pack8(o2);
    } else {
      if (p < 0 || p >= S) continue;
      const int j = it - nrot;
      const int kh = j / (HD >> 3), g = j % (HD >> 3);
      const int src = (Hq + Hkv + kh) * HD + g * 8;
      uint16_t* dst = vc + (((size_t)slot * Hkv + kh) * S + p) * HD + g * 8;
      if constexpr (PART) {
        float x[8];
        qkv_load8<true>(row, prow, ks, plane, src, x);
        *reinterpret_cast<uint4*>(dst) = pack8(x);
      } else {
        *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(row + src);
      }
    }
  }
}

}  // namespace

void tb_rope_qkv_cache(const uint16_t* qkv, const int32_t* pos, const int32_t* slot_of_row, const float* cos_t,
                       const float* sin_t, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M, int Hq, int Hkv,
                       int HD, int S, int max_pos, hipStream_t st) {
  if (M <= 0) return;
  hipLaunchKernelGGL(rope_qkv_cache_kernel<false>, dim3(M), dim3(256), 0, st, qkv, nullptr, 0, M, pos, slot_of_row,
                     cos_t, sin_t, q_out, kc, vc, Hq, Hkv, HD, S, max_pos);
}

void tb_rope_qkv_cache_part(const float* part, int ks, const int32_t* pos, const int32_t* slot_of_row,
                            const float* cos_t, const float* sin_t, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M,
                            int Hq, int Hkv, int HD, int S, int max_pos, hipStream_t st) {
  if (M <= 0) return;
  // a row's items over 4 workgroups: a decode-sized M fills the chip, each item sums ks partials
  hipLaunchKernelGGL(rope_qkv_cache_kernel<true>, dim3(M, 4), dim3(256), 0, st, nullptr, part, ks, M, pos, slot_of_row,
                     cos_t, sin_t, q_out, kc, vc, Hq, Hkv, HD, S, max_pos);
}

// KV fan-out of a prefix-trie decode step (runtime/generation.py, shared decode): rows that share their
// whole token sequence with a representative row (same pair, same tokens) compute blocks 0..nl-1 only
// through that representative; this copies the K/V the representative just wrote at its position into
// every member row's own slot, for those layers, so any member can become a representative later (when
// its group splits) with its full history in place.  One workgroup per (row, layer); src_row < 0 = skip.
namespace {

__global__ void __launch_bounds__(256) kv_fanout_kernel(uint16_t* __restrict__ kc, uint16_t* __restrict__ vc,
                                                        const int32_t* __restrict__ src_row,
                                                        const int32_t* __restrict__ slot,
                                                        const int32_t* __restrict__ pos, int slots, int Hkv, int S,
                                                        int HD) {
  const int r = blockIdx.x, l = blockIdx.y;
  const int s = src_row[r];
  if (s < 0 || s == r) return;
  const int pd = pos[r], ps = pos[s];
  if (pd < 0 || pd >= S || ps < 0 || ps >= S) return;
  const int gph = HD >> 3, nvec = Hkv * gph;
  const size_t lay = (size_t)l * slots * Hkv;
  const size_t sd = lay + (size_t)slot[r] * Hkv, ss = lay + (size_t)slot[s] * Hkv;
  for (int i = threadIdx.x; i < nvec; i += blockDim.x) {
    const int h = i / gph, g = i % gph;
    const size_t od = ((sd + h) * S + pd) * HD + g * 8, os = ((ss + h) * S + ps) * HD + g * 8;
    *reinterpret_cast<uint4*>(kc + od) = *reinterpret_cast<const uint4*>(kc + os);
    *reinterpret_cast<uint4*>(vc + od) = *reinterpret_cast<const uint4*>(vc + os);
  }
}

}  // namespace

void tb_kv_fanout(uint16_t* kc, uint16_t* vc, const int32_t* src_row, const int32_t* slot, const int32_t* pos, int M,
                  int nlayers, int slots, int Hkv, int S, int HD, hipStream_t st) {
  if (M <= 0 || nlayers <= 0) return;
  hipLaunchKernelGGL(kv_fanout_kernel, dim3(M, nlayers), dim3(256), 0, st, kc, vc, src_row, slot, pos, slots, Hkv,
                     S, HD);
}
