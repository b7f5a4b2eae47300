// Gemma RMSNorm family + scaled embedding gather.
//
// Gemma-2 RMSNorm: y = bf16( x * rsqrt(mean(x^2) + eps) * (1 + w) ), fp32 math
// (transformers gemma2 Gemma2RMSNorm).  A decoder block contains
//   h = h + post_norm(branch(pre_norm(h)))
// twice, so the hot kernel here is `add_rmsnorm2`: it applies the post-norm
// to the branch output, adds it into the residual IN PLACE and emits the next
// pre-norm, i.e. one HBM pass instead of three.  Rounding points mirror the
// bf16 PyTorch graph exactly (post-norm output rounded, residual add rounded).
//
// One workgroup per row; each lane owns 8 contiguous bf16 (one 16-B load) per
// vector slot; VPT slots per lane keep the row in registers between the
// reduction and the write.
#include "common.h"
#include "api.h"

namespace {

template <int VPT>
__device__ __forceinline__ void load_row(const uint16_t* __restrict__ p, int nvec, float (&v)[VPT][8]) {
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = threadIdx.x + s * blockDim.x;
    if (i < nvec) {
      uint4 u = reinterpret_cast<const uint4*>(p)[i];
      unpack8(u, v[s]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = 0.f;
    }
  }
}

template <int VPT>
__device__ __forceinline__ float sumsq(const float (&v)[VPT][8]) {
  float a = 0.f;
#pragma unroll
  for (int s = 0; s < VPT; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) a += v[s][j] * v[s][j];
  return a;
}

// out = bf16(v * r * (1 + w)), v fp32 register row.
template <int VPT>
__device__ __forceinline__ void norm_store(const float (&v)[VPT][8], float r, const uint16_t* __restrict__ w,
                                           uint16_t* __restrict__ out, int nvec, float (*keep)[8] = nullptr) {
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = threadIdx.x + s * blockDim.x;
    if (i < nvec) {
      float wf[8], o[8];
      unpack8(reinterpret_cast<const uint4*>(w)[i], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[s][j] * r * (1.f + wf[j]);
      reinterpret_cast<uint4*>(out)[i] = pack8(o);
    }
  }
}

template <int VPT>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                       uint16_t* __restrict__ y, int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, nvec = D >> 3;
  float v[VPT][8];
  load_row<VPT>(x + (size_t)row * D, nvec, v);
  const float ss = block_sum(sumsq<VPT>(v), red);
  const float r = rsqrtf(ss / (float)D + eps);
  norm_store<VPT>(v, r, w, y + (size_t)row * D, nvec);
}

// h <- bf16(h + bf16(norm(o, w_post)));  x <- norm(h, w_next)
template <int VPT>
__global__ void __launch_bounds__(1024) add_rmsnorm2_kernel(uint16_t* __restrict__ h, const uint16_t* __restrict__ o,
                                                            const uint16_t* __restrict__ w_post,
                                                            const uint16_t* __restrict__ w_next,
                                                            uint16_t* __restrict__ x, int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, nvec = D >> 3;
  float v[VPT][8];
  load_row<VPT>(o + (size_t)row * D, nvec, v);
  const float r1 = rsqrtf(block_sum(sumsq<VPT>(v), red) / (float)D + eps);
  uint16_t* hr = h + (size_t)row * D;
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = threadIdx.x + s * blockDim.x;
    if (i < nvec) {
      float wf[8], hf[8];
      unpack8(reinterpret_cast<const uint4*>(w_post)[i], wf);
      unpack8(reinterpret_cast<const uint4*>(hr)[i], hf);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = rbf(hf[j] + rbf(v[s][j] * r1 * (1.f + wf[j])));
      reinterpret_cast<uint4*>(hr)[i] = pack8(v[s]);
    }
  }
  const float r2 = rsqrtf(block_sum(sumsq<VPT>(v), red) / (float)D + eps);
  norm_store<VPT>(v, r2, w_next, x + (size_t)row * D, nvec);
}

// add_rmsnorm2 whose branch output o arrives as the ks fp32 split-K partials of the projection (gemm4.hip
// tb_gemm4_splitk_part, [ks, M, D]): o = bf16(sum over the splits in order), exactly what the split-K reduction
// kernel would have stored -- the reduction, its bf16 store and this kernel's re-read of o are one pass.
template <int VPT>
__global__ void __launch_bounds__(1024) add_rmsnorm2_part_kernel(uint16_t* __restrict__ h, const float* __restrict__ part,
                                                                 int ks, int M, const uint16_t* __restrict__ w_post,
                                                                 const uint16_t* __restrict__ w_next,
                                                                 uint16_t* __restrict__ x, int D, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, nvec = D >> 3;
  float v[VPT][8];
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = threadIdx.x + s * blockDim.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[s][j] = 0.f;
    if (i < nvec) {
      sum_splits8(part + (size_t)row * D + i * 8, (size_t)M * D, ks, v[s]);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = rbf(v[s][j]);
    }
  }
  const float r1 = rsqrtf(block_sum(sumsq<VPT>(v), red) / (float)D + eps);
  uint16_t* hr = h + (size_t)row * D;
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = threadIdx.x + s * blockDim.x;
    if (i < nvec) {
      float wf[8], hf[8];
      unpack8(reinterpret_cast<const uint4*>(w_post)[i], wf);
      unpack8(reinterpret_cast<const uint4*>(hr)[i], hf);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = rbf(hf[j] + rbf(v[s][j] * r1 * (1.f + wf[j])));
      reinterpret_cast<uint4*>(hr)[i] = pack8(v[s]);
    }
  }
  const float r2 = rsqrtf(block_sum(sumsq<VPT>(v), red) / (float)D + eps);
  norm_store<VPT>(v, r2, w_next, x + (size_t)row * D, nvec);
}

// h <- bf16(E[id] * bf16(scale));  x <- norm(h, w)
template <int VPT>
__global__ void __launch_bounds__(1024) embed_rmsnorm_kernel(const int32_t* __restrict__ ids,
                                                             const uint16_t* __restrict__ E,
                                                             const uint16_t* __restrict__ w, uint16_t* __restrict__ h,
                                                             uint16_t* __restrict__ x, int D, int V, float scale,
                                                             float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x, nvec = D >> 3;
  int id = ids[row];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  float v[VPT][8];
  load_row<VPT>(E + (size_t)id * D, nvec, v);
  const float sc = rbf(scale);
  uint16_t* hr = h + (size_t)row * D;
#pragma unroll
  for (int s = 0; s < VPT; ++s) {
    const int i = threadIdx.x + s * blockDim.x;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[s][j] = rbf(v[s][j] * sc);
      reinterpret_cast<uint4*>(hr)[i] = pack8(v[s]);
    }
  }
  const float r = rsqrtf(block_sum(sumsq<VPT>(v), red) / (float)D + eps);
  norm_store<VPT>(v, r, w, x + (size_t)row * D, nvec);
}

inline int threads_for(int nvec, int vpt) {
  int t = (nvec + vpt - 1) / vpt;
  t = (t + 63) / 64 * 64;
  return t < 64 ? 64 : t;
}

}  // namespace

// D must be a multiple of 8.  VPT = 1 covers D <= 8192, VPT = 4 covers D <= 32768.
#define TB_DISPATCH_VPT(D, KERNEL_LAUNCH)            \
  do {                                               \
    const int nvec_ = (D) >> 3;                      \
    if (nvec_ <= 1024) { constexpr int VPT = 1; KERNEL_LAUNCH; } \
    else { constexpr int VPT = 4; KERNEL_LAUNCH; }   \
  } while (0)

void tb_rmsnorm(const uint16_t* x, const uint16_t* w, uint16_t* y, int M, int D, float eps, hipStream_t st) {
  if (M <= 0) return;
  TB_DISPATCH_VPT(D, {
    const int thr = threads_for(nvec_, VPT);
    hipLaunchKernelGGL(rmsnorm_kernel<VPT>, dim3(M), dim3(thr), 0, st, x, w, y, D, eps);
  });
}

void tb_add_rmsnorm2(uint16_t* h, const uint16_t* o, const uint16_t* w_post, const uint16_t* w_next, uint16_t* x,
                     int M, int D, float eps, hipStream_t st) {
  if (M <= 0) return;
  TB_DISPATCH_VPT(D, {
    const int thr = threads_for(nvec_, VPT);
    hipLaunchKernelGGL(add_rmsnorm2_kernel<VPT>, dim3(M), dim3(thr), 0, st, h, o, w_post, w_next, x, D, eps);
  });
}

void tb_add_rmsnorm2_part(uint16_t* h, const float* part, int ks, const uint16_t* w_post, const uint16_t* w_next,
                          uint16_t* x, int M, int D, float eps, hipStream_t st) {
  if (M <= 0) return;
  TB_DISPATCH_VPT(D, {
    const int thr = threads_for(nvec_, VPT);
    hipLaunchKernelGGL(add_rmsnorm2_part_kernel<VPT>, dim3(M), dim3(thr), 0, st, h, part, ks, M, w_post, w_next, x, D,
                       eps);
  });
}

void tb_embed_rmsnorm(const int32_t* ids, const uint16_t* E, const uint16_t* w, uint16_t* h, uint16_t* x, int M,
                      int D, int V, float scale, float eps, hipStream_t st) {
  if (M <= 0) return;
  TB_DISPATCH_VPT(D, {
    const int thr = threads_for(nvec_, VPT);
    hipLaunchKernelGGL(embed_rmsnorm_kernel<VPT>, dim3(M), dim3(thr), 0, st, ids, E, w, h, x, D, V, scale, eps);
  });
}
