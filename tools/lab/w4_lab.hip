// Standalone check + timing harness for csrc/gemm_w4.hip (and, for an in-process A/B, csrc/gemm.hip's
// ping-pong kernel).  Operands are uniform [-1, 1) bf16 (cdna_hip_programming.md §5.4 rule 25).
//   w4_lab check                      -> exactness vs an fp32 reference kernel, every variant and epilogue
//   w4_lab time <M> <N> <K> [reps]    -> one JSON line per kernel {us, TF}, interleaved rounds (rule 24)
#include "gemm_w4_experiment.hip"
#include "../../taboo_brittleness_amd/csrc/gemm.hip"
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <algorithm>
#include <cstring>
#include <string>

__global__ void fill_kernel(uint16_t* p, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = f2bf(((h & 0xffffff) / 8388608.f) - 1.f);
  }
}
__global__ void ref_kernel(const uint16_t* A, const uint16_t* W, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(size_t)m * K + k]) * bf2f(W[(size_t)n * K + k]);
  C[(size_t)m * N + n] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float bfh(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }

static int check() {
  const int shapes[][3] = {{1, 256, 64}, {37, 512, 128}, {300, 768, 256}, {513, 1024, 3584}, {256, 256, 640}, {700, 3584, 4096}};
  int bad = 0;
  for (auto& s : shapes) {
    const int M = s[0], N = s[1], K = s[2];
    uint16_t *A, *W; float *R, *Cf; uint16_t* Cb; float *b, *t;
    CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&W, (size_t)N * K * 2)); CK(hipMalloc(&R, (size_t)M * N * 4));
    CK(hipMalloc(&Cf, (size_t)M * N * 4)); CK(hipMalloc(&Cb, (size_t)M * N * 2)); CK(hipMalloc(&b, N * 4)); CK(hipMalloc(&t, N * 4));
    hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, A, (size_t)M * K, 3u);
    hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, W, (size_t)N * K, 9u);
    CK(hipMemset(b, 0, N * 4)); CK(hipMemset(t, 0, N * 4));
    hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, A, W, R, M, N, K);
    std::vector<float> hr((size_t)M * N), hf((size_t)M * N);
    std::vector<uint16_t> hb((size_t)M * N);
    CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
    for (int variant = 0; variant < 3; ++variant) {
      CK(hipMemset(Cf, 0xff, (size_t)M * N * 4)); CK(hipMemset(Cb, 0xff, (size_t)M * N * 2));
      tb_gemm_w4(A, W, Cf, b, t, M, N, K, N, 1, variant, 0);
      tb_gemm_w4(A, W, Cb, b, t, M, N, K, N, 0, variant, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(hf.data(), Cf, hf.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hb.data(), Cb, hb.size() * 2, hipMemcpyDeviceToHost));
      double ef = 0, eb = 0, den = 0;
      for (size_t i = 0; i < hr.size(); ++i) {
        den = std::max(den, (double)fabsf(hr[i]));
        ef = std::max(ef, (double)fabsf(hf[i] - hr[i]));
        eb = std::max(eb, (double)fabsf(bfh(hb[i]) - hr[i]));
      }
      const bool ok = ef / den < 1e-5 && eb / den < 8e-3 && std::isfinite(ef) && std::isfinite(eb);
      bad += !ok;
      printf("{\"check\": [%d, %d, %d], \"variant\": %d, \"f32_rel\": %.3g, \"bf16_rel\": %.3g, \"ok\": %s}\n", M, N, K,
             variant, ef / den, eb / den, ok ? "true" : "false");
    }
    hipFree(A); hipFree(W); hipFree(R); hipFree(Cf); hipFree(Cb); hipFree(b); hipFree(t);
  }
  printf("{\"check_ok\": %s}\n", bad ? "false" : "true");
  return bad ? 1 : 0;
}

static int timing(int M, int N, int K, int reps) {
  uint16_t *A, *W; void* C;
  CK(hipMalloc(&A, (size_t)M * K * 2)); CK(hipMalloc(&W, (size_t)N * K * 2)); CK(hipMalloc(&C, (size_t)M * N * 2));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, A, (size_t)M * K, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, W, (size_t)N * K, 7u);
  const char* names[] = {"w4_256_s4", "w4_256_s3", "w4_128m_s3", "pp"};
  const int nk = 4;
  auto run = [&](int v) {
    if (v < 3) tb_gemm_w4(A, W, C, nullptr, nullptr, M, N, K, N, 0, v, 0);
    else tb_gemm_pp(A, W, C, nullptr, nullptr, M, N, K, N, 0, 256, 0);
  };
  for (int v = 0; v < nk; ++v) for (int i = 0; i < 3; ++i) run(v);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> us(nk);
  for (int round = 0; round < 7; ++round)
    for (int v = 0; v < nk; ++v) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) run(v);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      us[v].push_back(ms * 1000.f / reps);
    }
  const double flop = 2.0 * M * N * K;
  for (int v = 0; v < nk; ++v) {
    std::sort(us[v].begin(), us[v].end());
    printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"kernel\": \"%s\", \"us_med\": %.1f, \"us_min\": %.1f, \"TF_med\": %.1f}\n", M,
           N, K, names[v], us[v][3], us[v][0], flop / us[v][3] / 1e6);
  }
  hipFree(A); hipFree(W); hipFree(C);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "check") return check();
  if (argc > 4) return timing(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), argc > 5 ? atoi(argv[5]) : 10);
  fprintf(stderr, "usage: w4_lab check | time M N K [reps]\n");
  return 2;
}
