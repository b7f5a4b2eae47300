// Standalone timing harness for csrc/gemm.hip variants (one executable per compile-time knob setting,
// cdna_hip_programming.md §5.4 rule 19).  Operands are uniform [-1, 1) bf16 (rule 25).
//   gemm_lab <M> <N> <K> [epi] [reps]   -> one JSON line {us, TF}
#include "../../taboo_brittleness_amd/csrc/gemm.hip"
#include <cstdio>
#ifndef TILE_ROWS
#define TILE_ROWS 256
#endif
#include <cstdlib>

__global__ void fill_kernel(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = f2bf(((h & 0xffffff) / 8388608.f) - 1.f);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]);
  const int epi = argc > 4 ? atoi(argv[4]) : 0, reps = argc > 5 ? atoi(argv[5]) : 20;
  if (!tb_gemm_pp_ok(M, N, K)) { fprintf(stderr, "bad shape\n"); return 1; }
  uint16_t *A, *W; void* C; float *b, *t;
  CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&W, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 4)); CK(hipMalloc(&b, N * 4)); CK(hipMalloc(&t, N * 4));
  CK(hipMemset(b, 0, N * 4)); CK(hipMemset(t, 0, N * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, A, (size_t)M * K, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, W, (size_t)N * K, 7u);
  const int ldc = epi == 3 ? N / 2 : N;
  for (int i = 0; i < 3; ++i) tb_gemm_pp(A, W, C, b, t, M, N, K, ldc, epi, TILE_ROWS, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30f, tot = 0.f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) tb_gemm_pp(A, W, C, b, t, M, N, K, ldc, epi, TILE_ROWS, 0);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const float us = ms * 1000.f / reps; tot += us; if (us < best) best = us;
  }
  const double flop = 2.0 * M * N * K;
  printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"epi\": %d, \"us_best\": %.1f, \"us_mean\": %.1f, \"TF_best\": %.1f}\n",
         M, N, K, epi, best, tot / 5, flop / best / 1e6);
  return 0;
}
