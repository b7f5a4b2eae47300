// Random orthonormal bases for the projection sweep's random-subspace controls (EP:150): per cell, r
// directions of a Gaussian D x r matrix orthonormalised by Gram-Schmidt (classical, twice), written straight into
// the edit plan's basis table (the rows the lowrank_edit kernel projects out).  A sweep step of BASELINE config 4 draws ~4200
// of them (5 random trials x ranks 1..64 x 120 pairs); drawn on the host (randn + LAPACK QR) they took ~5 ms each
// and made the projection sweep host-bound (profiles/r6/side/lowrank_prof.err).
//
// One workgroup per basis, 256 threads; thread t owns elements d = t + 256 e of every vector (e < EPT), so the
// vectors it reads back are the ones it wrote (no cross-thread visibility question).  The Gaussian entries come from
// a counter-based hash of (seed, vector, element) -- splitmix64 finaliser, Box-Muller in fp64 -- so a basis is a pure
// function of (seed, r, D): it does not depend on the launch, the batch or the device (ops.reference.random_basis
// is the same algorithm in numpy).  Orthogonalisation: classical Gram-Schmidt applied twice, in fp64, against the
// fp32-rounded earlier directions (what the table holds), 64 directions per chunk; every dot product / norm is
// reduced in a fixed order (lane butterfly, then the 4 waves in order).  Modified Gram-Schmidt (one block reduction
// per earlier direction, each waiting on the last) cost ~28 ms per 5040-basis sweep step; CGS2 has two barriers per
// chunk of 64.
#include "common.h"
#include "api.h"

namespace {

constexpr int RB_QCH = 64;               // earlier directions per Gram-Schmidt chunk

__device__ __forceinline__ uint64_t rb_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double rb_gauss(uint64_t seed, int j, int d) {
  const uint64_t key = seed * 0x9E3779B97F4A7C15ULL + (((uint64_t)(uint32_t)j << 32) | (uint32_t)d);
  const uint64_t a = rb_mix64(key), b = rb_mix64(key ^ 0xD1B54A32D192ED03ULL);
  const double u1 = ((double)(a >> 11) + 1.0) * 0x1.0p-53;   // (0, 1]
  const double u2 = (double)(b >> 11) * 0x1.0p-53;           // [0, 1)
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

__device__ __forceinline__ double rb_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();                       // the previous reduction's readers are done with red
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

// QU: earlier directions whose table rows are loaded together (each direction's own arithmetic and order unchanged,
// so every QU gives the same bits; tools/basis_bench.py)
template <int EPT, int QU>
__global__ void __launch_bounds__(256) random_basis_kernel(const uint64_t* __restrict__ seeds,
                                                           const int32_t* __restrict__ ranks,
                                                           const int64_t* __restrict__ rows, int D,
                                                           float* __restrict__ table) {
  __shared__ double red[4];
  __shared__ double dots[RB_QCH][4];     // per (earlier direction, wave) partial dot products
  const int i = blockIdx.x;
  const uint64_t seed = seeds[i];
  const int r = ranks[i];
  float* out = table + (size_t)rows[i] * D;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  double v[EPT];
  for (int j = 0; j < r; ++j) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int d = t + 256 * e;
      v[e] = d < D ? rb_gauss(seed, j, d) : 0.0;
    }
    // classical Gram-Schmidt, twice ("twice is enough"), against the stored (fp32) directions in chunks of RB_QCH:
    // a chunk's dot products are independent (no per-direction barrier chain as in modified Gram-Schmidt)
    for (int pass = 0; pass < 2; ++pass)
      for (int q0 = 0; q0 < j; q0 += RB_QCH) {
        const int nq = j - q0 < RB_QCH ? j - q0 : RB_QCH;
        // dot products QU directions at a time: their table loads in flight together (each direction's own
        // arithmetic and order unchanged, so the bits are those of one direction at a time)
        for (int qb = 0; qb < nq; qb += QU) {
          float a[QU][EPT];
#pragma unroll
          for (int u = 0; u < QU; ++u) {
            const float* qr = out + (size_t)(q0 + (qb + u < nq ? qb + u : nq - 1)) * D;
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
              const int d = t + 256 * e;
              a[u][e] = d < D ? qr[d] : 0.f;
            }
          }
#pragma unroll
          for (int u = 0; u < QU; ++u) {
            double part = 0.0;
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
              const int d = t + 256 * e;
              if (d < D) part = fma((double)a[u][e], v[e], part);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
            if (lane == 0 && qb + u < nq) dots[qb + u][w] = part;
          }
        }
        __syncthreads();
        for (int qb = 0; qb < nq; qb += QU) {   // v -= c_q q in direction order, loads batched likewise
          float a[QU][EPT];
#pragma unroll
          for (int u = 0; u < QU; ++u) {
            const float* qr = out + (size_t)(q0 + (qb + u < nq ? qb + u : nq - 1)) * D;
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
              const int d = t + 256 * e;
              a[u][e] = d < D ? qr[d] : 0.f;
            }
          }
#pragma unroll
          for (int u = 0; u < QU; ++u) {
            if (qb + u >= nq) break;
            const double c = ((dots[qb + u][0] + dots[qb + u][1]) + dots[qb + u][2]) + dots[qb + u][3];
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
              const int d = t + 256 * e;
              if (d < D) v[e] = fma(-c, (double)a[u][e], v[e]);
            }
          }
        }
        __syncthreads();                 // dots is rewritten by the next chunk
      }
    double ss = 0.0;
#pragma unroll
    for (int e = 0; e < EPT; ++e) ss = fma(v[e], v[e], ss);
    const double inv = 1.0 / sqrt(rb_block_sum(ss, red));
    float* oj = out + (size_t)j * D;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int d = t + 256 * e;
      if (d < D) oj[d] = (float)(v[e] * inv);
    }
  }
}

}  // namespace

bool tb_random_basis_ok(int D) { return D > 0 && D <= 256 * 16; }

void tb_random_basis(const uint64_t* seeds, const int32_t* ranks, const int64_t* rows, int n, int D, float* table,
                     hipStream_t st, int qu) {
  if (n <= 0) return;
  const int ept = (D + 255) / 256;
#define RB_GO(E_, Q_) hipLaunchKernelGGL((random_basis_kernel<E_, Q_>), dim3(n), dim3(256), 0, st, seeds, ranks, rows, D, table)
#define RB_Q(E_)                  \
  if (qu >= 4) RB_GO(E_, 4);      \
  else if (qu == 2) RB_GO(E_, 2); \
  else RB_GO(E_, 1);
  if (ept <= 4) {
    RB_Q(4)
  } else if (ept <= 8) {
    RB_Q(8)
  } else {
    RB_Q(16)
  }
#undef RB_Q
#undef RB_GO
}
