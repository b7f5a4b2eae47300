// Ping-pong 256x256x64 MFMA GEMM for gfx950: C = A[M,K] . W[N,K]^T (both operands K-contiguous,
// nn.Linear layout) with fused epilogues.  SURVEY K7 (gate/up + GeGLU) and K15 (SAE encode +
// JumpReLU): the epilogue works on the fp32 accumulators, so the [M, 2F] gate|up or the
// pre-activation never round-trips through HBM.
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", T1/T2/T3/T4/T5):
//  * 512 threads = 8 waves in two groups of 4 (group g owns output rows g*128..g*128+127, wave wc of
//    the group owns columns wc*64..wc*64+63, i.e. 128x64 per wave = 2x2 quadrants of 64x32).
//  * One K-tile (64 deep) = 4 phases, one quadrant each (16 x mfma_f32_16x16x32_bf16 per wave and
//    phase).  Quadrant order (0,0) (0,1) (1,1) (1,0): A fragments are read twice and B fragments
//    twice per K-tile (12 + 4 + 8 + 0 ds_read_b128), the minimum for this register budget.
//  * LDS = 2 stages x 4 half-tile images (A0 A1 B0 B1, 128 rows x 128 B each) = 128 KB, the kernel's
//    only __shared__ object.  Half-tile q of K-tile t+1 is staged during phase q of K-tile t with
//    two global_load_lds_dwordx4 per thread (lane-linear 1 KB per wave-instruction); the XOR swizzle
//    (chunk ^= (row>>1)&7) is applied to the global SOURCE address and to the ds_read address, which
//    makes every 16-lane ds_read_b128 group hit 16 distinct 16-B slots (conflict-free).
//  * Ping-pong: group 1 runs one barrier behind group 0, so on every SIMD (one wave of each group)
//    one wave issues its ds_reads + staging while the other runs its MFMA cluster.
//  * Synchronisation is counted, never drained in the main loop: after staging in phase q a wave
//    waits vmcnt(4) (its phases <= q-2 have landed), then a raw s_barrier.  Data staged in phase s
//    is first read in phase s+3; with the one-barrier stagger the last wait that covers it (the
//    other group's, phase s+2) precedes a barrier the reader passes before reading.  A stage buffer
//    is re-staged >= 2 phases after its last ds_read completed (lgkmcnt before the MFMA cluster).
//  * Block ids: XCD-aware bijective remap (T1), then GROUP_M = 4 tile-rows per group so the 32
//    co-resident tiles of an XCD share 4 A panels and 8 W panels through its L2.
// Requirements (host-checked): N % 256 == 0, K % 64 == 0, K >= 64; any M (rows past M are clamped
// on load and masked on store).
#include "common.h"
#include "api.h"

namespace {

constexpr int PBN = 256, PBK = 64, PTHREADS = 512;
constexpr int PHALF = 128 * PBK * 2;   // bytes of one half-tile image (128 rows x 64 bf16)
constexpr int PSTAGE = 4 * PHALF;      // A0 A1 B0 B1
#ifndef PP_GROUP_M
#define PP_GROUP_M 4
#endif
// lab knobs (tools/gemm_lab.sh builds one executable per setting; the extension uses the defaults)
#ifndef PP_SETPRIO
#define PP_SETPRIO 1
#endif
#ifndef PP_STAGGER
#define PP_STAGGER 1
#endif
#ifndef PP_PHASES
#define PP_PHASES 4
#endif
#ifndef PP_NO_LDS_READ
#define PP_NO_LDS_READ 0
#endif
#ifndef PP_MFMA32
#define PP_MFMA32 0      // 1: v_mfma_f32_32x32x16_bf16 (same wave tile, same reads, half the MFMA count)
#endif
constexpr int PGROUP_M = PP_GROUP_M;

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const uint16_t* src, char* dst) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 0, 0);
}
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ bf16x8 lds8(const char* p) {
#if PP_NO_LDS_READ
  // lab: MFMA/barrier/staging cost without LDS reads (operand = the address bits, kept live)
  const uint32_t a = (uint32_t)(uintptr_t)p;
  return __builtin_bit_cast(bf16x8, make_uint4(a, a ^ 1u, a ^ 2u, a ^ 3u));
#else
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
#endif
}

enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_JUMPRELU = 2, EPI_GEGLU = 3 };
constexpr int HEAD_COLS = 128;          // vocab columns per head / lens partial (gemm4.hip G4_HEAD / G4_LENS)

// QROWS = output rows (m) per tile: 256, or 128 for grids that would otherwise leave CUs idle (the N = 3584
// projections at moderate M).  Every variant accumulates each output element over K in the same order with
// the same MFMA (16x16x32, 32-deep steps in K order), so C does not depend on the tile shape or on M: a row
// gets bit-identical results whatever batch it runs in (batch invariance, tests/test_engine_gpu.py).
template <int EPI, int QROWS>
__global__ void __launch_bounds__(PTHREADS, 1)
gemm_pp_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, void* __restrict__ C,
               const float* __restrict__ bias, const float* __restrict__ thr, int M, int N, int K, int ldc) {
  static_assert(QROWS == 256 || QROWS == 128, "tile rows");
  static_assert(QROWS == 256 || !PP_MFMA32, "32x32 MFMA lab build: 256-row tiles only");
  constexpr int QW = QROWS / 4;          // output rows per wave (64 | 32)
  constexpr int QJ = QW / 2;             // of them per Q half-image (32 | 16)
  constexpr int NJ = QJ / 16;            // 16-row MFMA blocks per half (2 | 1)
  constexpr int QL = QROWS / 128;        // glds per thread per Q half-image (2 | 1)
  __shared__ __attribute__((aligned(1024))) char smem[2 * PSTAGE];
  const int nbn = N / PBN, nbm = (M + QROWS - 1) / QROWS, nwg = nbn * nbm;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int per_group = PGROUP_M * nbn, first_bm = (bid / per_group) * PGROUP_M;
  const int gsz = min(nbm - first_bm, PGROUP_M), lid = bid % per_group;
  const int bm = first_bm + lid % gsz, bn = lid / gsz;
  const int m0 = bm * QROWS, n0 = bn * PBN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wc = wid & 3;

  // ---- staging sources.  The MFMA row operand P is W (tile rows = output columns n), the column
  // operand Q is A (tile columns = output rows m), so each lane's accumulator holds 4 consecutive n of
  // one m: the epilogue stores 8 / 16 contiguous bytes per lane with no LDS round trip.
  // This thread fills image rows r_s = 8*(2*wid+s) + lane/8 (s = 0, 1) at physical 16-B chunk lane%8,
  // which holds logical chunk (lane%8) ^ ((r_s>>1)&7) of that row.
  //   P-half h, image row i  ->  tile row (i>>6)*128 + h*64 + (i&63)   (wave group g reads rows g*64..)
  //   Q-half h, image row i  ->  tile col (i/QJ)*QW + h*QJ + (i%QJ) (wave wc reads rows wc*QJ..)
  // (a 128-row tile's Q images are 64 rows: one glds per thread, rows 8*wid + lane/8)
  const uint16_t* sp[2][2];   // [half][s]
  const uint16_t* sq[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int r = 8 * (2 * wid + s) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int rq = QL == 2 ? r : 8 * wid + (lane >> 3);
    const int cq = (lane & 7) ^ ((rq >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int wn = n0 + (r >> 6) * 128 + h * 64 + (r & 63);
      sp[h][s] = W + (size_t)wn * K + c * 8;
      const int am = min(m0 + (rq / QJ) * QW + h * QJ + (rq % QJ), M - 1);
      sq[h][s] = A + (size_t)am * K + cq * 8;
    }
  }
  char* const dst0 = smem + wid * 2048;   // + stage*PSTAGE + image*PHALF (+1024 for s = 1)

  // ---- fragment read offsets (the swizzle term ((row>>1)&7) = (lane&15)>>1 for every row read)
  const int xr = (lane & 15) >> 1;
#if PP_MFMA32
  // 32x32x16: lane l holds row (l&31), k = 16*s + 8*(l>>5) .. +8 of k-step s, i.e. logical chunk 2s + (l>>5)
  int co[4];
#pragma unroll
  for (int k4 = 0; k4 < 4; ++k4) co[k4] = ((2 * k4 + (lane >> 5)) ^ xr) << 4;
  const int offp = (grp * 64 + (lane & 31)) * 128;
  const int offq = (wc * 32 + (lane & 31)) * 128;
  f32x16 acc[2][2][2];   // [qm][qn][32-row block of the 64-row P half]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][b][i][e] = 0.f;
  bf16x8 pf[2][4], qf0[4], qf1[4];
#else
  const int co0 = (((lane >> 4)) ^ xr) << 4, co1 = ((4 + (lane >> 4)) ^ xr) << 4;
  const int offp = (grp * 64 + (lane & 15)) * 128;
  const int offq = (wc * QJ + (lane & 15)) * 128;

  f32x4 acc[2][2][4][NJ];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 pf[4][2], qf0[NJ][2], qf1[NJ][2];
#endif

  // images: 0 = P0, 1 = P1, 2 = Q0, 3 = Q1
#define PP_STAGE(stg, img, SRC, k0)                                         \
  do {                                                                      \
    char* d_ = dst0 + (stg) * PSTAGE + (img) * PHALF;                       \
    if ((img) < 2 || QL == 2) {                                             \
      glds16(SRC[0] + (k0), d_);                                            \
      glds16(SRC[1] + (k0), d_ + 1024);                                     \
    } else {                                                                \
      glds16(SRC[0] + (k0), smem + (stg) * PSTAGE + (img) * PHALF + wid * 1024); \
    }                                                                       \
  } while (0)
#if PP_MFMA32
#define PP_READ_P(sb, qm)                                                   \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) {                           \
    const char* p_ = (sb) + (qm) * PHALF + offp + i * 4096;                 \
    _Pragma("unroll") for (int k4 = 0; k4 < 4; ++k4) pf[i][k4] = lds8(p_ + co[k4]); \
  }
#define PP_READ_Q(sb, qn, dstf)                                             \
  {                                                                         \
    const char* p_ = (sb) + (2 + (qn)) * PHALF + offq;                      \
    _Pragma("unroll") for (int k4 = 0; k4 < 4; ++k4) dstf[k4] = lds8(p_ + co[k4]); \
  }
#define PP_MFMA(qm, qn, qfr)                                                \
  if (PP_SETPRIO) __builtin_amdgcn_s_setprio(1);                            \
  _Pragma("unroll") for (int k4 = 0; k4 < 4; ++k4)                          \
  _Pragma("unroll") for (int i = 0; i < 2; ++i)                             \
    acc[qm][qn][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[i][k4], qfr[k4], acc[qm][qn][i], 0, 0, 0); \
  if (PP_SETPRIO) __builtin_amdgcn_s_setprio(0);
#else
#define PP_READ_P(sb, qm)                                                   \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) {                           \
    const char* p_ = (sb) + (qm) * PHALF + offp + i * 2048;                 \
    pf[i][0] = lds8(p_ + co0);                                              \
    pf[i][1] = lds8(p_ + co1);                                              \
  }
#define PP_READ_Q(sb, qn, dstf)                                             \
  _Pragma("unroll") for (int j = 0; j < NJ; ++j) {                          \
    const char* p_ = (sb) + (2 + (qn)) * PHALF + offq + j * 2048;           \
    dstf[j][0] = lds8(p_ + co0);                                            \
    dstf[j][1] = lds8(p_ + co1);                                            \
  }
#define PP_MFMA(qm, qn, qfr)                                                \
  if (PP_SETPRIO) __builtin_amdgcn_s_setprio(1);                            \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                          \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)                             \
  _Pragma("unroll") for (int j = 0; j < NJ; ++j)                            \
    acc[qm][qn][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[i][ks], qfr[j][ks], acc[qm][qn][i][j], 0, 0, 0); \
  if (PP_SETPRIO) __builtin_amdgcn_s_setprio(0);
#endif
#define PP_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
  // counted waits: after staging in phase q the loads of phases q-2..q stay in flight (P images: 2 glds per
  // thread, Q images: QL): after a P stage 2P + Q, after a Q stage P + 2Q, phase 3 without a stage P + Q
#define PP_VM_AFTER_P() do { if constexpr (QL == 2) PP_VMCNT(6); else PP_VMCNT(5); } while (0)
#define PP_VM_AFTER_Q() do { if constexpr (QL == 2) PP_VMCNT(6); else PP_VMCNT(4); } while (0)
#define PP_VM_TAIL() do { if constexpr (QL == 2) PP_VMCNT(4); else PP_VMCNT(3); } while (0)

  // Staging schedule (every image >= 4 phases ahead of its first read; each phase stages one image):
  //   phase 0: P0 of K-tile t+1   phase 1: Q1 of t+1   phase 2: P1 of t+1   phase 3: Q0 of t+2
  // (Q0 of t+2 goes into the stage K-tile t is using: its Q0 image was read in phase 0 and is held in
  // registers for phase 3.)  After a staging phase vmcnt(6) leaves the last 3 staged images in flight.
  const int nk = K / PBK;
#if PP_PHASES == 4
  PP_STAGE(0, 0, sp[0], 0);
  PP_STAGE(0, 1, sp[1], 0);
  PP_STAGE(0, 2, sq[0], 0);
  PP_STAGE(0, 3, sq[1], 0);
  if (nk > 1) PP_STAGE(1, 2, sq[0], PBK);
  PP_VMCNT(0);
  bar();
  if (PP_STAGGER && grp == 1) bar();   // ping-pong: group 1 runs one barrier behind

  for (int t = 0; t < nk; ++t) {
    const char* sb = smem + (t & 1) * PSTAGE;
    const int ns = (t + 1) & 1;
    const bool more = t + 1 < nk;
    const int kn = (t + 1) * PBK;
    // phase 0: quadrant (0,0) -- read P0 + Q0
    PP_READ_P(sb, 0);
    PP_READ_Q(sb, 0, qf0);
    if (more) { PP_STAGE(ns, 0, sp[0], kn); PP_VM_AFTER_P(); } else { PP_VMCNT(0); }
    bar();
    PP_MFMA(0, 0, qf0);
    bar();
    // phase 1: quadrant (0,1) -- read Q1
    PP_READ_Q(sb, 1, qf1);
    if (more) { PP_STAGE(ns, 3, sq[1], kn); PP_VM_AFTER_Q(); } else { PP_VMCNT(0); }
    bar();
    PP_MFMA(0, 1, qf1);
    bar();
    // phase 2: quadrant (1,1) -- read P1
    PP_READ_P(sb, 1);
    if (more) { PP_STAGE(ns, 1, sp[1], kn); PP_VM_AFTER_P(); } else { PP_VMCNT(0); }
    bar();
    PP_MFMA(1, 1, qf1);
    bar();
    // phase 3: quadrant (1,0) -- no reads (P1 and Q0 are in registers)
    if (t + 2 < nk) { PP_STAGE(t & 1, 2, sq[0], kn + PBK); PP_VM_AFTER_Q(); }
    else if (more) { PP_VM_TAIL(); }
    else { PP_VMCNT(0); }
    bar();
    PP_MFMA(1, 0, qf0);
    bar();
  }
#else
  static_assert(QROWS == 256, "two-phase lab schedule: 256-row tiles only");
  // Two phases per K-tile (two quadrants = 32 MFMAs per wave each, 4 barriers per K-tile):
  //   phase 0: quadrants (0,0) (0,1), reads P0 Q0 Q1, stages P0 Q0 Q1 of K-tile t+1, then vmcnt(6)
  //   phase 1: quadrants (1,1) (1,0), reads P1,       stages P1 of t+1,          then vmcnt(2)
  // i.e. after every phase only that phase's loads are in flight: an image staged in phase s is read
  // in phase s+2, after the other group's wait at the end of phase s+1 and the barrier behind it;
  // a stage slot is re-staged 2 phases after its last read.
  PP_STAGE(0, 0, sp[0], 0);
  PP_STAGE(0, 1, sp[1], 0);
  PP_STAGE(0, 2, sq[0], 0);
  PP_STAGE(0, 3, sq[1], 0);
  PP_VMCNT(0);
  bar();
  if (PP_STAGGER && grp == 1) bar();   // ping-pong: group 1 runs one barrier behind

  for (int t = 0; t < nk; ++t) {
    const char* sb = smem + (t & 1) * PSTAGE;
    const int ns = (t + 1) & 1;
    const bool more = t + 1 < nk;
    const int kn = (t + 1) * PBK;
    PP_READ_P(sb, 0);
    PP_READ_Q(sb, 0, qf0);
    PP_READ_Q(sb, 1, qf1);
    if (more) {
      PP_STAGE(ns, 0, sp[0], kn);
      PP_STAGE(ns, 2, sq[0], kn);
      PP_STAGE(ns, 3, sq[1], kn);
      PP_VMCNT(6);
    } else {
      PP_VMCNT(0);
    }
    bar();
    PP_MFMA(0, 0, qf0);
    PP_MFMA(0, 1, qf1);
    bar();
    PP_READ_P(sb, 1);
    if (more) { PP_STAGE(ns, 1, sp[1], kn); PP_VMCNT(2); } else { PP_VMCNT(0); }
    bar();
    PP_MFMA(1, 1, qf1);
    PP_MFMA(1, 0, qf0);
    bar();
  }
#endif
  if (PP_STAGGER && grp == 0) bar();   // every wave executes the same number of barriers
#undef PP_STAGE
#undef PP_READ_P
#undef PP_READ_Q
#undef PP_MFMA
#undef PP_VMCNT
#undef PP_VM_AFTER_P
#undef PP_VM_AFTER_Q
#undef PP_VM_TAIL

  // ---- epilogue.  Every lane holds, per (qm, qn), accumulator groups of 4 consecutive output columns n of one
  // output row m:  E_M(qn, rj) is the row, E_N(qm, g) the first column of group g, E_V(...) its r-th value.
  //   16x16x32: acc[qm][qn][i][j][r]: n = n0 + grp*128 + qm*64 + i*16 + 4*(lane>>4) + r,
  //             m = m0 + wc*64 + qn*32 + j*16 + (lane&15)             (g = i, rj = j; 4 lanes share a row)
  //   32x32x16: acc[qm][qn][b][4*q + r]: n = n0 + grp*128 + qm*64 + b*32 + 8*q + 4*(lane>>5) + r,
  //             m = m0 + wc*64 + qn*32 + (lane&31)                     (g = 4b + q; 2 lanes share a row)
#if PP_MFMA32
  constexpr int E_RJ = 1, E_G = 8, E_LO = 32;
#define E_M(qn, rj) (m0 + wc * 64 + (qn) * 32 + (lane & 31))
#define E_N(qm, g) (n0 + grp * 128 + (qm) * 64 + ((g) >> 2) * 32 + 8 * ((g) & 3) + 4 * (lane >> 5))
#define E_V(qm, qn, rj, g, r) acc[qm][qn][(g) >> 2][4 * ((g) & 3) + (r)]
#else
  constexpr int E_RJ = NJ, E_G = 4, E_LO = 16;
#define E_M(qn, rj) (m0 + wc * QW + (qn) * QJ + (rj) * 16 + (lane & 15))
#define E_N(qm, g) (n0 + grp * 128 + (qm) * 64 + (g) * 16 + 4 * (lane >> 4))
#define E_V(qm, qn, rj, g, r) acc[qm][qn][g][rj][r]
#endif
  if constexpr (EPI == EPI_GEGLU) {
    // P rows are gate (qm = 0) / up (qm = 1) of feature E_N(0, g) - n0/2 - grp*64 + r; the gate|up values are
    // rounded to bf16 first so the result equals geglu(bf16 gate|up GEMM output)
    uint16_t* out = reinterpret_cast<uint16_t*>(C);
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int rj = 0; rj < E_RJ; ++rj) {
        const int m = E_M(qn, rj);
        if (m >= M) continue;
#pragma unroll
        for (int g = 0; g < E_G; ++g) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gt = rbf(E_V(0, qn, rj, g, r)), u = rbf(E_V(1, qn, rj, g, r));
            o[r] = rbf(gelu_tanh_fast(gt)) * u;
          }
          const int f = E_N(0, g) - (n0 >> 1) - grp * 64;
          *reinterpret_cast<uint2*>(out + (size_t)m * ldc + f) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
        }
      }
  } else {
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int g = 0; g < E_G; ++g) {
        const int n = E_N(qm, g);
        float4 bn_ = make_float4(0.f, 0.f, 0.f, 0.f), th = bn_;
        if constexpr (EPI == EPI_JUMPRELU) {
          if (bias) bn_ = *reinterpret_cast<const float4*>(bias + n);
          if (thr) th = *reinterpret_cast<const float4*>(thr + n);
        }
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int rj = 0; rj < E_RJ; ++rj) {
            const int m = E_M(qn, rj);
            if (m >= M) continue;
            const float v0 = E_V(qm, qn, rj, g, 0), v1 = E_V(qm, qn, rj, g, 1), v2 = E_V(qm, qn, rj, g, 2),
                        v3 = E_V(qm, qn, rj, g, 3);
            if constexpr (EPI == EPI_BF16) {
              *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + (size_t)m * ldc + n) =
                  make_uint2(pack2(v0, v1), pack2(v2, v3));
            } else if constexpr (EPI == EPI_F32) {
              *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) = make_float4(v0, v1, v2, v3);
            } else {
              const float a0 = v0 + bn_.x, a1 = v1 + bn_.y, a2 = v2 + bn_.z, a3 = v3 + bn_.w;
              *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) =
                  make_float4(a0 > th.x ? a0 : 0.f, a1 > th.y ? a1 : 0.f, a2 > th.z ? a2 : 0.f, a3 > th.w ? a3 : 0.f);
            }
          }
      }
  }
#undef E_M
#undef E_N
#undef E_V
}

}  // namespace

bool tb_gemm_pp_ok(int M, int N, int K) { return M > 0 && N > 0 && N % PBN == 0 && K >= PBK && K % PBK == 0; }

#define PP_LAUNCH_T(E_, Q_)                                                                                        \
  hipLaunchKernelGGL((gemm_pp_kernel<E_, Q_>), dim3((N / PBN) * ((M + (Q_) - 1) / (Q_))), dim3(PTHREADS), 0, st, A, W, \
                     C, bias, thr, M, N, K, ldc)
#define PP_LAUNCH(E_) PP_LAUNCH_T(E_, 256)

// tile_rows: 256 or 128 (output rows per tile; identical numerics, see gemm_pp_kernel)
void tb_gemm_pp(const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr, int M, int N,
                int K, int ldc, int epi, int tile_rows, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  if (tile_rows == 128) {
    switch (epi) {
      case EPI_BF16: PP_LAUNCH_T(EPI_BF16, 128); break;
      case EPI_F32: PP_LAUNCH_T(EPI_F32, 128); break;
      case EPI_JUMPRELU: PP_LAUNCH_T(EPI_JUMPRELU, 128); break;
      default: PP_LAUNCH_T(EPI_GEGLU, 128);
    }
    return;
  }
  switch (epi) {
    case EPI_BF16: PP_LAUNCH(EPI_BF16); break;
    case EPI_F32: PP_LAUNCH(EPI_F32); break;
    case EPI_JUMPRELU: PP_LAUNCH(EPI_JUMPRELU); break;
    default: PP_LAUNCH(EPI_GEGLU);
  }
}

namespace {

// Fold a row's N/128 head / lens partials: lse, first argmax, and the NLLs (greedy token, optional teacher
// target); each output pointer may be null.
__global__ void __launch_bounds__(256) head_merge_kernel(const float4* __restrict__ part, int npart,
                                                         const int32_t* __restrict__ tgt,
                                                         const float* __restrict__ tgt_logit, int32_t* __restrict__ nxt,
                                                         float* __restrict__ nll_self, float* __restrict__ nll_tgt,
                                                         float* __restrict__ lse_out, int V) {
  __shared__ float sm[4], ss[4];
  __shared__ int si[4];
  const int r = blockIdx.x;
  const float4* p = part + (size_t)r * npart;
  float mx = -INFINITY, s = 0.f;
  int bi = 0x7fffffff;
  auto merge = [&](float m2, float s2, int i2) {
    if (m2 > mx) { s = (mx == -INFINITY ? 0.f : s * __expf(mx - m2)) + s2; mx = m2; bi = i2; }
    else if (m2 == mx) { s += s2; bi = min(bi, i2); }
    else if (m2 != -INFINITY) { s += s2 * __expf(m2 - mx); }
  };
  for (int c = threadIdx.x; c < npart; c += blockDim.x) {
    const float4 q = p[c];
    merge(q.x, q.y, __float_as_int(q.z));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(s, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    merge(m2, s2, i2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = mx; ss[wid] = s; si[wid] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = sm[0]; s = ss[0]; bi = si[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) merge(sm[w], ss[w], si[w]);
    const float lse = mx + __logf(s);
    if (lse_out != nullptr) lse_out[r] = lse;
    if (nxt != nullptr) nxt[r] = bi;
    if (nll_self != nullptr) nll_self[r] = lse - mx;
    if (nll_tgt != nullptr) {
      const int t = tgt != nullptr ? tgt[r] : -1;
      nll_tgt[r] = (t >= 0 && t < V) ? lse - tgt_logit[r] : 0.f;
    }
  }
}

}  // namespace

void tb_head_merge(const float* part, int npart, const int32_t* tgt, const float* tgt_logit, int32_t* nxt,
                   float* nll_self, float* nll_tgt, float* lse, int M, int V, hipStream_t st) {
  if (M <= 0) return;
  hipLaunchKernelGGL(head_merge_kernel, dim3(M), dim3(256), 0, st, reinterpret_cast<const float4*>(part), npart, tgt,
                     tgt_logit, nxt, nll_self, nll_tgt, lse, V);
}

