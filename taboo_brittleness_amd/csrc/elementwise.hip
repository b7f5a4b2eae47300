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

}  // namespace

void tb_geglu(const uint16_t* gu, uint16_t* out, int M, int F, hipStream_t st) {
  if (M <= 0) return;
  const int fv = F >> 3;
  hipLaunchKernelGGL(geglu_kernel, dim3(M, (fv + 255) / 256), dim3(256), 0, st, gu, out, F);
}
