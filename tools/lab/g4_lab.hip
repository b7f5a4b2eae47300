// ctypes shim over csrc/gemm4.hip for tools/lab/g4_bench.py (in-process A/B against hipBLASLt and the extension)
#include "../../taboo_brittleness_amd/csrc/gemm4.hip"
// the lab never runs the fused head: its softcap-table lookup (csrc/lens.hip) is stubbed
bool tb_softcap_compact_params(float, const uint16_t**, int*, int*, float*) { return false; }
extern "C" int g4_gemm(const void* A, const void* W, void* C, int M, int N, int K, int ldc, int epi, int rows,
                       void* stream) {
  if (!tb_gemm4_ok(M, N, K)) return 1;
  tb_gemm4((const uint16_t*)A, (const uint16_t*)W, C, nullptr, nullptr, M, N, K, ldc, epi, rows, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
