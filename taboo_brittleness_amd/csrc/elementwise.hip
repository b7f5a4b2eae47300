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

// Row combination out[b] = sum_t coef[b, t] * row(ptr[b, t]) of fp32 rows of length V (the sweep's lens base: a
// cell's reused response lens sum is its pair's running sum at the divergence minus the re-evaluated spike terms,
// pipelines/sweep_readout.py _lens_base).  The rows live in separate per-pair tensors, so each term is a device row
// address; the T terms of a row are summed in their given order (fp32 FMA chain): the result of a row never depends
// on the other rows of the launch.  grid (B, ceil(V / 4 / 256)).
__global__ void __launch_bounds__(256) row_combine_kernel(const int64_t* __restrict__ ptr, const float* __restrict__ coef,
                                                          float* __restrict__ out, int T, int V) {
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= (V >> 2)) return;
  const size_t b = blockIdx.x;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int t = 0; t < T; ++t) {
    const float w = coef[b * T + t];
    if (w == 0.f) continue;                  // padding terms (uniform per row)
    const float4 x = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(ptr[b * T + t]))[c];
    acc.x = fmaf(w, x.x, acc.x);
    acc.y = fmaf(w, x.y, acc.y);
    acc.z = fmaf(w, x.z, acc.z);
    acc.w = fmaf(w, x.w, acc.w);
  }
  reinterpret_cast<float4*>(out + b * (size_t)V)[c] = acc;
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

void tb_row_combine(const int64_t* ptr, const float* coef, float* out, int B, int T, int V, hipStream_t st) {
  if (B <= 0 || V <= 0) return;
  hipLaunchKernelGGL(row_combine_kernel, dim3(B, (V / 4 + 255) / 256), dim3(256), 0, st, ptr, coef, out, T, V);
}

void tb_geglu(const uint16_t* gu, uint16_t* out, int M, int F, hipStream_t st) {
  if (M <= 0) return;
  const int fv = F >> 3;
  hipLaunchKernelGGL(geglu_kernel, dim3(M, (fv + 255) / 256), dim3(256), 0, st, gu, out, F);
}
