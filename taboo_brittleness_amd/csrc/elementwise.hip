// GeGLU activation: act = bf16( bf16(gelu_tanh(gate)) * up ).
//
// Gemma-2's MLP is gelu_pytorch_tanh(gate_proj(x)) * up_proj(x) — GeGLU, not
// SwiGLU.  The fused gate|up GEMM output is [M, 2F] (gate in
// columns [0, F), up in [F, 2F)); this kernel reads both halves with 16-B
// vector loads and writes [M, F].  Rounding points follow the bf16 PyTorch
// graph (GELU output rounded, product rounded).
#include "common.h"
#include "api.h"

namespace {

// grid (M, ceil(F / 8 / 256)): one 16-B vector of gate and of up per thread, no index division
__global__ void __launch_bounds__(256) geglu_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out, int F) {
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= (F >> 3)) return;
  const size_t m = blockIdx.x;
  const uint16_t* row = gu + m * 2 * (size_t)F;
  float g[8], u[8], o[8];
  unpack8(reinterpret_cast<const uint4*>(row)[c], g);
  unpack8(reinterpret_cast<const uint4*>(row + F)[c], u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = rbf(gelu_tanh_fast(g[j])) * u[j];
  reinterpret_cast<uint4*>(out + m * (size_t)F)[c] = pack8(o);
}

// Whole-slot copies between two [L, slots, inner] bf16 tensors (KV caches: inner = Hkv * S * HD):
// dst[l, dslot[i]] = src[l0 + l, sslot[i]] for i < n, l < nl.  One pass (a torch index_select + index_copy_ pair
// moves every byte twice through a temporary); grid (n, nl, ceil(inner / 8 / (256 * VPB))).
constexpr int SLOT_VPB = 8;   // 16-B vectors per thread
__global__ void __launch_bounds__(256) slot_copy_kernel(uint16_t* __restrict__ dst, const uint16_t* __restrict__ src,
                                                        const int32_t* __restrict__ dslot,
                                                        const int32_t* __restrict__ sslot, int64_t inner,
                                                        int dst_slots, int src_slots, int dst_l0, int src_l0) {
  const int i = blockIdx.x, l = blockIdx.y;
  const int64_t nv = inner >> 3;
  const u32x4* s = reinterpret_cast<const u32x4*>(src + ((int64_t)(src_l0 + l) * src_slots + sslot[i]) * inner);
  u32x4* d = reinterpret_cast<u32x4*>(dst + ((int64_t)(dst_l0 + l) * dst_slots + dslot[i]) * inner);
  const int64_t v0 = (int64_t)blockIdx.z * 256 * SLOT_VPB + threadIdx.x;
  u32x4 r[SLOT_VPB];
#pragma unroll
  for (int k = 0; k < SLOT_VPB; ++k)
    if (v0 + k * 256 < nv) r[k] = __builtin_nontemporal_load(s + v0 + k * 256);
#pragma unroll
  for (int k = 0; k < SLOT_VPB; ++k)
    if (v0 + k * 256 < nv) d[v0 + k * 256] = r[k];
}

}  // namespace

void tb_slot_copy(uint16_t* dst, const uint16_t* src, const int32_t* dslot, const int32_t* sslot, int n, int nl,
                  int64_t inner, int dst_slots, int src_slots, int dst_l0, int src_l0, hipStream_t st) {
  if (n <= 0 || nl <= 0 || inner <= 0) return;
  const int64_t nz = ((inner >> 3) + 256 * SLOT_VPB - 1) / (256 * SLOT_VPB);
  hipLaunchKernelGGL(slot_copy_kernel, dim3(n, nl, (unsigned)nz), dim3(256), 0, st, dst, src, dslot, sslot, inner,
                     dst_slots, src_slots, dst_l0, src_l0);
}

void tb_geglu(const uint16_t* gu, uint16_t* out, int M, int F, hipStream_t st) {
  if (M <= 0) return;
  const int fv = F >> 3;
  hipLaunchKernelGGL(geglu_kernel, dim3(M, (fv + 255) / 256), dim3(256), 0, st, gu, out, F);
}
