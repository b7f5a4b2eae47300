// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * bf16 tensors are passed as `uint16_t*` (raw bits); conversions go through
//    clang's `__bf16` type, which hipcc lowers to v_cvt_pk_bf16_f32 (RNE,
//    NaN-preserving) on gfx950.
//  * Wave width is 64 (hard-coded; `warpSize` is not used in constant contexts).
//  * Vector memory traffic is 16 B per lane (8 x bf16) wherever the row length
//    allows (cdna_hip_programming.md Guideline 13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TB_WAVE 64

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}
// Round-trip through bf16 (emulates a bf16-typed PyTorch intermediate).
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

// gelu_tanh(x) = 0.5 x (1 + tanh(y)) = x / (1 + exp(-2y)), y = k0 (x + k1 x^3): one v_exp + one v_rcp instead
// of a libm tanhf (the kernel then streams at HBM rate); differs from the tanhf form by ~1e-6 relative before
// the bf16 rounding.  exp overflow gives x * rcp(inf) = 0 (the x -> -inf limit), underflow gives x.  The bare
// v_rcp_f32 (1 ulp): a correctly rounded reciprocal (__frcp_rn) expands to a 9-instruction division sequence,
// which in the fused GeGLU GEMM epilogue was ~1300 VALU instructions per tile.
__device__ __forceinline__ float gelu_tanh_fast(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float y = k0 * (x + k1 * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * y));
}

// v[0..8) += sum over s < ks of p[s * plane + 0..8) (fp32 split-K partials), added in split order; the loads
// of 4 splits are issued before their adds (a plain loop waits for each split's load before the next one's)
__device__ __forceinline__ void sum_splits8(const float* __restrict__ p, size_t plane, int ks, float (&v)[8]) {
  int s = 0;
  for (; s + 4 <= ks; s += 4) {
    float4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = *reinterpret_cast<const float4*>(p + (s + u) * plane);
      b[u] = *reinterpret_cast<const float4*>(p + (s + u) * plane + 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[0] += a[u].x; v[1] += a[u].y; v[2] += a[u].z; v[3] += a[u].w;
      v[4] += b[u].x; v[5] += b[u].y; v[6] += b[u].z; v[7] += b[u].w;
    }
  }
  for (; s < ks; ++s) {
    const float4 a = *reinterpret_cast<const float4*>(p + s * plane);
    const float4 b = *reinterpret_cast<const float4*>(p + s * plane + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
}

struct bf16x8_u {
  uint4 v;
  __device__ __forceinline__ float get(int i) const {
    uint32_t w = (i < 2) ? v.x : (i < 4) ? v.y : (i < 6) ? v.z : v.w;
    return (i & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
  }
};

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` needs >= 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// tanh via exp; accurate to ~1 ulp-ish in fp32 for the softcap range.
__device__ __forceinline__ float tanh_f(float x) { return tanhf(x); }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

#define TB_CHECK_LAUNCH() (void)hipGetLastError()
