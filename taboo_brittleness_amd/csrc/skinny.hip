// Weight-streaming GEMM for decode-sized M (<= 64 rows): C[M, N] = A[M, K] · W[N, K]^T, bf16 in,
// fp32 MFMA accumulation, bf16 out.
//
// At M <= 64 a decode projection is a pass over the weights (16.7 GB per Gemma-2-9B step): the
// kernel is built to stream W from HBM once at near peak bandwidth, not to reuse it.
//  * A workgroup owns NT x 16 rows of W; its 8 waves split K (each wave a contiguous 1/8 of the
//    128-wide k-blocks), so even N = 3584 launches 224 x 8 = 1792 waves (7 per CU) without a
//    cross-workgroup split-K reduction; the 8 partial tiles are summed through LDS at the end.
//  * k-permuted MFMA fragments: v_mfma_f32_16x16x32_bf16 wants lane l to hold k = 8*(l>>4)..+8 of
//    row (l&15).  Any permutation of k applied to both operands leaves the dot product unchanged, so
//    within a 128-wide k-block lane group g owns k = 32g..32g+32 and MFMA step j uses its j-th
//    16-byte piece: every lane issues 4 contiguous 16-B loads (64 B) per W row per k-block instead
//    of 16-B scattered ones.
//  * A (the activations, <= 64 x K, L2-resident) is read with the same permuted fragments; the
//    next k-block's W and A are loaded before the current block's MFMAs (register double buffer).
//  * Loads go straight to VGPRs: W is used once per workgroup, an LDS round trip would be pure
//    overhead (cdna_hip_programming.md §5, "GEMV / M <= 16 decode weights").
#include "common.h"
#include "api.h"

namespace {

__device__ __forceinline__ bf16x8 bits8(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }

template <int MT, int NT>
__global__ void __launch_bounds__(512) gemm_skinny_kernel(const uint16_t* __restrict__ A,
                                                          const uint16_t* __restrict__ W, uint16_t* __restrict__ C,
                                                          int M, int N, int K) {
  __shared__ float red[8 * MT * NT * 4 * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (NT * 16);
  const int nkb = K >> 7;
  const int kb0 = (nkb * wid) >> 3, kb1 = (nkb * (wid + 1)) >> 3;

  const uint16_t* wp[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wp[nt] = W + (size_t)(n0 + nt * 16 + col) * K + 32 * g;
  const uint16_t* ap[MT];
  bool av[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int r = mt * 16 + col;
    av[mt] = r < M;
    ap[mt] = A + (size_t)(av[mt] ? r : 0) * K + 32 * g;
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint4 wc[NT][4], ac[MT][4];
  const uint4 z = {0u, 0u, 0u, 0u};
#define TB_SKINNY_LOAD(KB, WD, AD)                                                                   \
  {                                                                                                \
    const int ko_ = (KB) << 7;                                                                     \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt)                                              \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                \
        WD[nt][j] = *reinterpret_cast<const uint4*>(wp[nt] + ko_ + 8 * j);                         \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                              \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                \
        AD[mt][j] = av[mt] ? *reinterpret_cast<const uint4*>(ap[mt] + ko_ + 8 * j) : z;            \
  }
  if (kb0 < kb1) TB_SKINNY_LOAD(kb0, wc, ac)
  for (int kb = kb0; kb < kb1; ++kb) {
    uint4 wn[NT][4], an[MT][4];
    if (kb + 1 < kb1) TB_SKINNY_LOAD(kb + 1, wn, an)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bits8(ac[mt][j]), bits8(wc[nt][j]), acc[mt][nt], 0,
                                                                0, 0);
    if (kb + 1 < kb1) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int j = 0; j < 4; ++j) wc[nt][j] = wn[nt][j];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) ac[mt][j] = an[mt][j];
    }
  }
#undef TB_SKINNY_LOAD

  // cross-wave reduction of the 8 K-slices: red[wave][tile*4 + i][lane]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[((wid * MT * NT + mt * NT + nt) * 4 + i) * 64 + lane] = acc[mt][nt][i];
  __syncthreads();
  constexpr int OUT = MT * NT * 4 * 64;
  for (int o = threadIdx.x; o < OUT; o += 512) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[w * OUT + o];
    const int ln = o & 63, q = o >> 6, i = q & 3, tile = q >> 2;
    const int mt = tile / NT, nt = tile % NT;
    const int m = mt * 16 + 4 * (ln >> 4) + i, n = n0 + nt * 16 + (ln & 15);
    if (m < M) C[(size_t)m * N + n] = f2bf(s);
  }
}

template <int MT>
void launch_mt(const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, hipStream_t st) {
  if (N % 32 == 0 && N / 32 >= 1024) {
    hipLaunchKernelGGL((gemm_skinny_kernel<MT, 2>), dim3(N / 32), dim3(512), 0, st, A, W, C, M, N, K);
  } else {
    hipLaunchKernelGGL((gemm_skinny_kernel<MT, 1>), dim3(N / 16), dim3(512), 0, st, A, W, C, M, N, K);
  }
}

}  // namespace

bool tb_gemm_skinny_ok(int M, int N, int K) { return M >= 1 && M <= 64 && N % 16 == 0 && K % 128 == 0 && K >= 1024; }

void tb_gemm_skinny(const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, hipStream_t st) {
  if (M <= 16) launch_mt<1>(A, W, C, M, N, K, st);
  else if (M <= 32) launch_mt<2>(A, W, C, M, N, K, st);
  else launch_mt<4>(A, W, C, M, N, K, st);
}
