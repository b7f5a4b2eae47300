// Four-wave 256 x BM x 64 MFMA GEMM for gfx950: C = A[M,K] . W[N,K]^T (both operands K-contiguous, the
// nn.Linear layout).  The projection GEMMs of the Gemma-2 blocks (SURVEY K3 QKV, K6 o_proj, K7 gate|up,
// K8 down, K10 vocab head, K11 lens unembedding) run on this kernel.
//
// Why four waves of 128 x (BM/2) (the round-2/3 ping-pong kernel used eight of 128 x 64): a 128 x 128 wave
// tile reads 2/3 of the LDS bytes per MFMA of a 128 x 64 one, and LDS read bytes cost clock under the
// chip's power cap (cdna_hip_programming.md §5.4 rule 28).  Its 64 f32x4 accumulators (256 registers)
// live in the AGPR half of the 512-entry register file a one-wave-per-SIMD kernel owns.
//
// Structure:
//  * 256 threads = 2 (n) x 2 (m) waves; wave (wn, wm) owns output columns n0 + wn*128 .. +127 and rows
//    m0 + wm*BM/2 .. (8 x BM/32 accumulators of 16 x 16).  The MFMA row operand P is W (output columns),
//    the column operand Q is A (output rows), so each lane's accumulator holds 4 consecutive n of one m.
//  * K tiles are 64 deep: a stage's LDS image is [256 W rows | BM A rows] x 128 B, two stages (128 KB at
//    BM = 256).  Each 16-B chunk c of row r is stored at c ^ ((r>>1)&7), so every ds_read_b128 lane group
//    hits 16 distinct 16-B slots of the 256-B bank row.
//  * Staging is LDS-DMA through buffer descriptors (buffer_load_dwordx4 ... lds): one wave-instruction writes
//    8 whole rows (8 full 128-B lines; 16 half-line rows per instruction, the 32-deep layout measured first,
//    took 25 % longer: profiles/r3/gemm4/); the swizzle is applied to the per-lane source offset (a VGPR
//    fixed for the whole K loop), the tile's K offset is the scalar soffset.
//  * One period per K tile t (two k32 steps, 2 x 64 MFMAs per wave at BM = 256), tile t+2 staged during it:
//      - step-0 MFMAs, the first WN+WM of them each followed by a read of a step-1 fragment (all of tile t is
//        then in registers);
//      - lgkmcnt(0) + barrier #1: no wave reads stage t&1 any more, so the LDS-DMA of tile t+2 into it is
//        spread over the following MFMAs;
//      - WN+WM MFMAs before the end: vmcnt(GL) (this wave's tile t+1 landed, t+2 in flight) + barrier #2,
//        then the step-0 fragment reads of tile t+1 (stage (t+1)&1) ride behind the last MFMAs.
//    The MFMAs are volatile asm statements (AGPR-tied accumulators; they also pin this source order).
//  * Block ids: XCD-aware bijective remap (T1), then GROUP_M tile rows per group so the tiles an XCD runs
//    together share A and W panels through its L2.
// Every output element is accumulated over K in the same order with the same MFMA (16x16x32, 32-deep steps in K
// order) whatever BM, M or the tile -- and the same as gemm_ring.hip's narrow tiles: a row's result does not depend
// on the batch it runs in.
// Requirements (host-checked, tb_gemm4_ok): N % 256 == 0, K % 64 == 0, K >= 64; any M.
#include "common.h"
#include "api.h"
#include <algorithm>
#include <cstdlib>
#include <utility>

namespace {

constexpr int G4_THREADS = 256, G4_BN = 256;
constexpr int G4_GROUP_M = 4;   // tile rows per group of the block-id remap
constexpr int G4_SLACK1 = 4;    // MFMAs between the last step-1 fragment read and barrier #1 (its lgkmcnt(0))
constexpr int G4_SLACK2 = 0;    // MFMAs after the last step-0 fragment read of the next tile
// (Measured and dropped ablations -- K-loop staging / reads removed, W-only staging, A staged through registers,
// A-major MFMA order, s_setprio in the K loop, nt / sc0 cache policy on the LDS-DMA, the GeGLU output through the
// LDS epilogue, the epilogue round trip in stage 1, builtin MFMAs -- live in git history and profiles/r3-r4/gemm4.)
// The one build switch: G4_CNT (set by build.py from the ISA check, taboo_brittleness_amd/isa_check.py).
#ifndef G4_CNT
#define G4_CNT 1         // 1: the 256-row tile's K-loop fragment reads as asm, each MFMA waits only for its own
                         // fragments (counted lgkmcnt); 0 (and the 128 / 64-row tiles): compiler-visible reads,
                         // drained (lgkmcnt(0)) at the end of every period
#endif

typedef __attribute__((address_space(3))) void g4_lds_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) char g4_lds_char;

template <int N>
__device__ __forceinline__ void g4_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int OFF>
__device__ __forceinline__ void g4_ds_write_b64(uint32_t a, const u32x2& v) {
  asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(a), "v"(v), "n"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ void g4_ds_read_b128(u32x4& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
// a K-loop fragment read at 2048-B row block k of the address (k a constant once the loops are unrolled)
__device__ __forceinline__ void g4_rd(bf16x8& d, uint32_t a, int k) {
  u32x4 t;
  switch (k) {
#define G4_RDC(n) case n: g4_ds_read_b128<(n) * 2048>(t, a); break;
    G4_RDC(0) G4_RDC(1) G4_RDC(2) G4_RDC(3) G4_RDC(4) G4_RDC(5) G4_RDC(6) G4_RDC(7)
    G4_RDC(8) G4_RDC(9) G4_RDC(10) G4_RDC(11) G4_RDC(12) G4_RDC(13) G4_RDC(14) G4_RDC(15)
    G4_RDC(16) G4_RDC(17) G4_RDC(18) G4_RDC(19) G4_RDC(20) G4_RDC(21) G4_RDC(22) G4_RDC(23)
    G4_RDC(24) G4_RDC(25) G4_RDC(26) G4_RDC(27) G4_RDC(28) G4_RDC(29) G4_RDC(30) G4_RDC(31)
#undef G4_RDC
    default: __builtin_unreachable();
  }
  d = __builtin_bit_cast(bf16x8, t);
}
// G4_HEAD's softcap-table reads: asm (a compiler-visible LDS read would get a vmcnt(0) in front of it, i.e. wait for
// the next tile's LDS-DMA) and held by g4_lgkm_hold4 so no use is scheduled before its wait
__device__ __forceinline__ void g4_ds_read_u16(uint32_t& d, uint32_t a) {
  asm volatile("ds_read_u16 %0, %1" : "=v"(d) : "v"(a));
}
template <int N>
__device__ __forceinline__ void g4_lgkm_hold4(uint32_t (&t)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : "n"(N));
}
template <typename F, int... I>
__device__ __forceinline__ void g4_unroll_seq(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void g4_unroll(F&& f) {
  g4_unroll_seq(f, std::make_integer_sequence<int, N>{});
}
// s_waitcnt vmcnt(n) (expcnt / lgkmcnt left at their maxima), gfx9 encoding: vmcnt[3:0] -> [3:0], vmcnt[5:4] -> [15:14]
constexpr int g4_vmcnt_enc(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
__device__ __forceinline__ void g4_bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

enum { G4_BF16 = 0, G4_F32 = 1, G4_JUMPRELU = 2, G4_GEGLU = 3, G4_ROPE = 4, G4_HEAD = 5, G4_LENS = 6 };

// Fused QKV epilogue (G4_ROPE, SURVEY K3 + K4): the projection's bf16 output is never stored; each 256-column tile is
// one head (head_dim 256): q heads are rotated into q_out [M, Hq, 256], k heads rotated and v heads copied into
// the layer's KV cache at the row's slot / position, with rope_qkv_cache_kernel's exact bf16 rounding chain
// (csrc/rope.hip).  Rows with pos < 0 are padding: q zeroed, no cache write.
struct G4Rope {
  const int32_t* pos;
  const int32_t* slot;
  const uint16_t* cs;   // bf16 (cos, sin) pairs [max_pos, 128, 2]: the fp32 tables rounded as the chain rounds them
  uint16_t* q_out;
  uint16_t* kc;
  uint16_t* vc;
  int Hq, Hkv, S, max_pos;
  // G4_HEAD (vocab head): bf16 logits -> exact bf16 final softcap, per (row, 128-column wave slice)
  // {max, sum exp(z - max), first argmax} into part[m * (N/128) + n/128]; the row's teacher-target logit into
  // tgt_logit.  The logits never reach memory.  The softcap is the compact exact form of csrc/lens.hip (CapC):
  // arithmetic below clo, the ctab[0, chi - clo) magnitudes in between (<= 4 KB, staged ONCE per workgroup into
  // LDS beside the stages), saturated above chi -- no per-tile table staging, no extra barrier.
  const uint16_t* ctab;
  int clo, chi;
  float csat, crc, ccap;
  const int32_t* tgt;
  float* tgt_logit;
  // G4_LENS (logit lens): the bf16 logits are stored (row-coalesced, as G4_BF16) AND each (row,
  // 128-column wave slice) is reduced to {max, sum exp(z - max), first argmax} into part (G4_HEAD's layout,
  // no softcap), so the row log-sum-exp needs no second pass over the logits (tb_head_merge folds the slices)
  float* part;
  // split-K (G4_F32 only, tb_gemm4_splitk): the K tiles are cut into ksplit ranges of kchunk tiles; virtual tile v is
  // (split v / nwg, output tile v % nwg) and split s writes its fp32 partial tile to C + s * M * ldc
  int ksplit, kchunk;
  // two-source A (the L2A instantiations, multi-adapter LoRA): columns [0, k0) of the GEMM's A operand are A (row
  // stride k0), columns [k0, K) are a2 (row stride K - k0); W is [N, K].  K tiles below k0 / 64 stage from A, the
  // rest from a2 -- the same K chain as one contiguous [M, K] operand, so the result is the GEMM of the
  // concatenation [A | a2] bit for bit, with no copy of A
  const uint16_t* a2;
  int k0;
};
constexpr int G4_CTAB_N = 32768;

template <int BM, int EPI, bool L2A = false>
__global__ void __launch_bounds__(G4_THREADS, 1)
gemm4_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, void* __restrict__ C,
             const float* __restrict__ bias, const float* __restrict__ thr, int M, int N, int K, int ldc, G4Rope rp) {
#if defined(__HIP_DEVICE_COMPILE__)   // the host pass only needs the signature (for the launch stub); some builtins and
                                     // the "a" asm constraint in the body make it silently drop the stub
  static_assert(BM == 256 || BM == 128 || (BM == 64 && EPI == G4_F32), "tile rows (64: the split-K decode tile)");
  // (asm fragment reads: the compiler takes their results as ready at once, so any copy it makes of one before the
  // counted wait copies stale data.  With 256 rows the accumulators fill the AGPRs and the fragments stay put; the
  // smaller tiles leave registers free and hipcc parks fragments in AGPRs -- checked in the ISA, and by the tests)
  constexpr bool G4C = G4_CNT && BM == 256;
  constexpr int WN = 8, WM = BM / 32;                 // 16-row fragments per wave: n, m
  constexpr int PIMG = G4_BN * 128, QIMG = BM * 128, STG = PIMG + QIMG;
  constexpr int PI = G4_BN / 32, QI = BM / 32, GL = PI + QI;   // LDS-DMA instructions per wave and K tile
  // row-coalesced bf16 epilogue (see the tile's end): a wave's output rows are RB bytes (bf16: its 128 columns;
  // GeGLU: its 64 features), ERPI rows per 16-B-per-lane store, ERR rows per LDS round trip, ENR stores per lane
  constexpr bool LEPI = EPI == G4_BF16 || EPI == G4_LENS;
  constexpr int RB = EPI == G4_GEGLU ? 128 : 256, ECH = RB / 16, ERPI = 64 / ECH;
  constexpr bool SPARE = LEPI;
  constexpr int EXB = SPARE ? 32768 : 0;                    // spare round-trip LDS (4 waves x ERR rows x RB)
  constexpr int ERR = SPARE ? EXB / (4 * RB) : EPI == G4_GEGLU ? BM / 2 : BM / 4;
  constexpr int ENR = LEPI ? (BM / 2) / ERPI : 1;
  constexpr int CTB = EPI == G4_HEAD ? 4096 : 0;            // compact softcap table bytes (G4_HEAD)
  static_assert(2 * STG + CTB + EXB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STG + CTB + EXB];   // one array: glds trap (a)

  const int nbn = N / G4_BN, nbm = (M + BM - 1) / BM, nwg = nbn * nbm;
  const int NT = K >> 6, KS = EPI == G4_F32 && rp.ksplit > 1 ? rp.ksplit : 1, KC = KS > 1 ? rp.kchunk : NT;
  const int nwgv = nwg * KS;   // virtual tiles (x K splits)
  // Persistent: this workgroup runs the virtual tiles blockIdx.x, blockIdx.x + gridDim.x, ...  A virtual id v keeps
  // v % 8 = blockIdx.x % 8 (gridDim.x is a multiple of 8), i.e. the XCD the workgroup runs on; the bijective
  // remap (T1) gives each XCD a contiguous range of tiles, grouped GROUP_M tile rows deep (shared A / W panels).
#define G4_TILE(v, m0_, n0_)                                                                              \
  do {                                                                                                    \
    const int q_ = nwgv / 8, r_ = nwgv % 8, x_ = (v) % 8;                                                 \
    int b_ = (x_ < r_ ? x_ * (q_ + 1) : r_ * (q_ + 1) + (x_ - r_) * q_) + (v) / 8;                        \
    sk = b_ / nwg;                                                                                        \
    b_ -= sk * nwg;                                                                                       \
    const int pg_ = G4_GROUP_M * nbn, fb_ = (b_ / pg_) * G4_GROUP_M;                                      \
    const int gs_ = min(nbm - fb_, G4_GROUP_M), l_ = b_ % pg_;                                            \
    m0_ = (fb_ + l_ % gs_) * BM;                                                                          \
    n0_ = (l_ / gs_) * G4_BN;                                                                             \
  } while (0)
  int tile = blockIdx.x, m0, n0, sk;
  G4_TILE(tile, m0, n0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid & 1, wm = wid >> 1;

  // ---- staging: instruction i of this wave fills image rows 8*(4i + wid) + lane/8 at physical chunk lane%8, which
  // holds logical chunk (lane%8) ^ ((row>>1)&7) = (lane%8) ^ ((4*wid + lane/16) & 7) (the same for every i)
  const int lchunk = (lane & 7) ^ ((4 * wid + (lane >> 4)) & 7);
  const int wbytes = G4_BN * K * 2;
  // A's row stride (L2A: the first source's k0 columns; the second source a2 holds the other K - k0)
  const int KA = L2A ? rp.k0 : K, K2 = K - KA, NT0 = KA >> 6;
  uint32_t vp[PI], vq[QI], vq2[L2A ? QI : 1];
#pragma unroll
  for (int i = 0; i < PI; ++i) vp[i] = (uint32_t)((8 * (4 * i + wid) + (lane >> 3)) * K + lchunk * 8) * 2u;
  int mrows, abytes, abytes2 = 0, nt;
  void *wtile, *atile, *atile2 = nullptr;
#define G4_DESC()                                                                                 \
  do {                                                                                            \
    mrows = min(BM, M - m0);                                                                      \
    wtile = (void*)(W + (size_t)n0 * K + sk * KC * 64);                                           \
    atile = (void*)(A + (size_t)m0 * KA + sk * KC * 64);                                          \
    nt = min(KC, NT - sk * KC);                                                                   \
    abytes = mrows * KA * 2;                                                                      \
    int ln_ = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));   /* opaque copy: the offsets are recomputed per tile, not hoisted and spilled */ \
    asm volatile("" : "+v"(ln_));                                                                 \
    const int lc_ = (ln_ & 7) ^ ((4 * wid + (ln_ >> 4)) & 7);                                     \
    _Pragma("unroll") for (int i = 0; i < QI; ++i)                                                \
      vq[i] = (uint32_t)(min(8 * (4 * i + wid) + (ln_ >> 3), mrows - 1) * KA + lc_ * 8) * 2u;     \
    if constexpr (L2A) {                                                                          \
      atile2 = (void*)(rp.a2 + (size_t)m0 * K2);                                                  \
      abytes2 = mrows * K2 * 2;                                                                   \
      _Pragma("unroll") for (int i = 0; i < QI; ++i)                                              \
        vq2[L2A ? i : 0] = (uint32_t)(min(8 * (4 * i + wid) + (ln_ >> 3), mrows - 1) * K2 + lc_ * 8) * 2u; \
    }                                                                                             \
  } while (0)
  G4_DESC();

  // ---- fragment reads: operand row = base + (lane&15) (base % 16 == 0, so (row>>1)&7 = (lane&15)>>1), logical
  // chunk 4*step + (lane>>4)
  const int xr = (lane & 15) >> 1;
  const int co0 = ((lane >> 4) ^ xr) << 4, co1 = ((4 + (lane >> 4)) ^ xr) << 4;
  // W-fragment i of wave wn covers tile rows (output columns) wn*128 + 16 i .. (G4_ROPE: wn*64 + 128 (i/4) + 16 (i%4),
  // so a lane holds both columns d and d + 128 of each rotation pair)
  constexpr bool RP = EPI == G4_ROPE;
  const int offp = (wn * (RP ? 64 : 128) + (lane & 15)) * 128;
#define G4_PROW(i) (RP ? (((i) >> 2) * 128 + ((i) & 3) * 16) : (i) * 16)
  const int offq = PIMG + (wm * (BM / 2) + (lane & 15)) * 128;

  f32x4 acc[WN][WM];
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 p0[WN], q0[WM], p1[WN], q1[WM];   // step-0 / step-1 fragments of the current K tile

  auto frag = [&](int stg, int off) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(smem + stg * STG + off));
  };
  // (macros, not lambdas: a lambda holding the buffer builtins makes the host pass drop the kernel's launch stub)
#define G4_STAGE_ONE(g, t, stg)                                                                                    \
  do {                                                                                                             \
    char* d_ = smem + (stg) * STG + wid * 1024;                                                                    \
    if ((g) < PI)                                                                                                  \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc(wtile, 0, wbytes, 0x00020000),    \
                                               (g4_lds_t*)(d_ + (g) * 4096), 16, vp[(g) < PI ? (g) : 0], (t) * 128, 0, 0); \
    else if constexpr (L2A) {   /* the second A source from K tile NT0 on: descriptor, row offsets and K offset    \
                                   picked by uniform selects, not a branch in the scheduled K loop */              \
      const bool s2_ = (t) >= NT0;                                                                                 \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                                    \
          __builtin_amdgcn_make_buffer_rsrc(s2_ ? atile2 : atile, 0, s2_ ? abytes2 : abytes, 0x00020000),          \
          (g4_lds_t*)(d_ + PIMG + ((g) - PI) * 4096), 16,                                                          \
          s2_ ? vq2[(g) >= PI ? (g) - PI : 0] : vq[(g) >= PI ? (g) - PI : 0], s2_ ? ((t) - NT0) * 128 : (t) * 128,  \
          0, 0);                                                                                                   \
    } else                                                                                                         \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc(atile, 0, abytes, 0x00020000),    \
                                               (g4_lds_t*)(d_ + PIMG + ((g) - PI) * 4096), 16,                      \
                                               vq[(g) >= PI ? (g) - PI : 0], (t) * 128, 0, 0);                      \
  } while (0)
#define G4_STAGE(t, stg) _Pragma("unroll") for (int g_ = 0; g_ < GL; ++g_) G4_STAGE_ONE(g_, t, stg)
  // MFMAs as asm statements with AGPR-tied accumulators: with the builtin, hipcc keeps the 256 accumulators in AGPRs
  // but re-homes them (and parks fragments in AGPRs) with hundreds of v_accvgpr_read/write/mov per K tile.  An
  // accumulate chain (D -> a later MFMA's C) needs no wait states; the epilogue's first accumulator read is padded.
#define G4_MFMA(i, j, pc, qc) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(pc[i]), "v"(qc[j]))
#define G4_MF(u)                                                          \
  do {                                                                    \
    if ((u) < NMF) G4_MFMA((u) / WM, (u) % WM, p0, q0);                   \
    else G4_MFMA(((u) - NMF) / WM, ((u) - NMF) % WM, p1, q1);             \
  } while (0)
  constexpr int NR = WN + WM, NMF = WN * WM, NT2 = 2 * NMF;
  constexpr int BAR1 = NR + G4_SLACK1;           // barrier #1 after this many MFMAs
  constexpr int BAR2 = NT2 - NR - G4_SLACK2;     // barrier #2 before MFMA BAR2
  constexpr int GSP = (NT2 - BAR1) / GL;         // MFMAs per LDS-DMA instruction, spread to the period's end
  constexpr int N2S = (BAR2 - BAR1) / GSP < GL ? (BAR2 - BAR1) / GSP : GL;   // slots issued before barrier #2
  // VMEM instructions younger than tile t+1's at barrier #2: the LDS-DMA slots issued before it
  constexpr int N2 = N2S;
  static_assert(GSP >= 1 && BAR1 < NMF && BAR1 < BAR2, "schedule");
  // G4C: the step-0 reads of a K tile are issued in order R = p0[0], q0[0..WM), p0[1..WN) behind the previous
  // period's last MFMAs (or the tile prologue), and one step-1 read follows each of the period's first NR MFMAs.
  // MFMA u < WM needs R[1 + u], MFMA u >= WM (fragment i = u / WM >= 1) R[WM + i]; LDS reads complete in order, so
  // "at most NR - 2 reads outstanding" in front of every MFMA before barrier #1 (whose lgkmcnt(0) covers the rest)
  // is exactly the wait for the first ones and a no-op later -- instead of draining all NR reads at the period's end.
  static_assert(NR - 2 <= 15 && BAR1 >= NR, "lgkmcnt range");
#define G4_PK(i) (G4_PROW(i) / 16)
#define G4_QK(j) (PIMG / 2048 + (j))
#define G4_WAIT()                                                        \
  do {                                                                   \
    if (G4C) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NR - 2));     \
  } while (0)
  const uint32_t lds0 = (uint32_t)(uintptr_t)((g4_lds_char*)smem);
  const uint32_t bp0 = lds0 + offp + co0, bp1 = lds0 + offp + co1;
  const uint32_t bq0 = lds0 + offq - PIMG + co0, bq1 = lds0 + offq - PIMG + co1;

  if constexpr (EPI == G4_HEAD) {
    if (rp.ctab != nullptr) {
      uint16_t* lt = reinterpret_cast<uint16_t*>(smem + 2 * STG);
      for (int i = tid; i < rp.chi - rp.clo; i += G4_THREADS) lt[i] = rp.ctab[i];
    }
    __syncthreads();
  }
  // prologue of the first tile: K tiles 0 and 1 in flight
  G4_STAGE(0, 0);
  G4_STAGE(min(1, nt - 1), 1);
  bool first_tile = true;
  for (;;) {
  // K tile 0 landed, its step-0 fragments read.  After a row-coalesced epilogue K tile 1 and the ENR row stores
  // (always issued: out-of-range rows are dropped by the buffer bounds) are younger than K tile 0.
  if (first_tile || !LEPI) g4_vmcnt<GL>();
  else g4_vmcnt<GL + ENR>();
  first_tile = false;
  g4_bar();
  if (G4C) {
    // order R (p0[0], q0[0..WM), p0[1..WN)): the first MFMAs' fragments first; see G4_WAIT
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    g4_rd(p0[0], bp0, G4_PK(0));
#pragma unroll
    for (int j = 0; j < WM; ++j) g4_rd(q0[j], bq0, G4_QK(j));
#pragma unroll
    for (int i = 1; i < WN; ++i) g4_rd(p0[i], bp0, G4_PK(i));
  } else {
#pragma unroll
    for (int i = 0; i < WN; ++i) p0[i] = frag(0, offp + G4_PROW(i) * 128 + co0);
#pragma unroll
    for (int j = 0; j < WM; ++j) q0[j] = frag(0, offq + j * 2048 + co0);
  }

  // The MFMAs after barrier #1: barrier #2 in front of MFMA BAR2 (vmcnt leaves the N2 instructions of tile t+2
  // issued so far in flight), the next tile's step-0 fragment reads behind the MFMAs from BAR2 on.
#define G4_POST(u)                                                                              \
  do {                                                                                          \
    if ((u) == BAR2) {                                                                          \
      __builtin_amdgcn_s_waitcnt(g4_vmcnt_enc(N2));                                             \
      g4_bar();                                                                                 \
    }                                                                                           \
    G4_MF(u);                                                                                   \
    const int v_ = (u) - BAR2;                                                                  \
    if (v_ >= 0 && v_ < NR) {                                                                   \
      if (G4C) {                                                                             \
        const uint32_t o_ = (sb ^ 1) * STG;                                                     \
        if (v_ == 0) g4_rd(p0[0], bp0 + o_, G4_PK(0));                                          \
        else if (v_ <= WM) g4_rd(q0[v_ >= 1 && v_ <= WM ? v_ - 1 : 0], bq0 + o_, G4_QK(v_ - 1)); \
        else g4_rd(p0[v_ > WM && v_ < NR ? v_ - WM : 0], bp0 + o_, G4_PK(v_ - WM));             \
      } else if (v_ < WN) p0[v_ >= 0 && v_ < WN ? v_ : 0] = frag(sb ^ 1, offp + G4_PROW(v_) * 128 + co0); \
      else q0[v_ >= WN && v_ < NR ? v_ - WN : 0] = frag(sb ^ 1, offq + (v_ - WN) * 2048 + co0); \
    }                                                                                           \
  } while (0)

  // Every period is branch-free: past the end, tile nt-1 is re-staged into the free stage and the last reads
  // fill the idle step-0 set.
  for (int t = 0; t < nt; ++t) {
    const int sb = t & 1, tn = min(t + 2, nt - 1);
    // (phases as short unrolled loops: hipcc will not fully unroll one 128-step loop, and a rolled one would index
    // the accumulators at run time)
#pragma unroll
    for (int u = 0; u < NR; ++u) {   // step-0 MFMAs, step-1 fragment reads
      G4_WAIT();
      G4_MF(u);
      if (G4C) {
        if (u < WN) g4_rd(p1[u < WN ? u : 0], bp1 + sb * STG, G4_PK(u));
        else g4_rd(q1[u >= WN ? u - WN : 0], bq1 + sb * STG, G4_QK(u - WN));
      } else if (u < WN) p1[u < WN ? u : 0] = frag(sb, offp + G4_PROW(u) * 128 + co1);
      else q1[u >= WN ? u - WN : 0] = frag(sb, offq + (u - WN) * 2048 + co1);
    }
#pragma unroll
    for (int u = NR; u < BAR1; ++u) {
      G4_WAIT();
      G4_MF(u);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // every wave holds all of tile t: its stage may be overwritten
    g4_bar();
#pragma unroll
    for (int g = 0; g < GL; ++g) {        // the LDS-DMA of tile t+2, one instruction per GSP MFMAs
#pragma unroll
      for (int k = 0; k < GSP; ++k) G4_POST(BAR1 + g * GSP + k);
      G4_STAGE_ONE(g, tn, sb);
    }
#pragma unroll
    for (int u = BAR1 + GL * GSP; u < NT2; ++u) G4_POST(u);
    // drain the reads here, with a memory clobber: otherwise hipcc sinks the last one into the next period and
    // waits for it (lgkmcnt(0)) in front of that period's first MFMA
    if (!G4C) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  if (G4C) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the last period's (redundant) step-0 reads
#undef G4_WAIT
#undef G4_POST
#undef G4_MF
#undef G4_MFMA
  // the stages are free once every wave is past its last fragment read and its (redundant) tail LDS-DMA: the next
  // tile's first two K tiles load while this tile's epilogue stores run
  g4_vmcnt<0>();
  g4_bar();
  const int em0 = m0, en0 = n0, esk = sk;
  const int next = tile + (int)gridDim.x;
  // Row-coalesced bf16 epilogue (G4_BF16): a lane's accumulators are 4 consecutive columns of one row, so direct
  // stores put 16 rows x 32 B into every store instruction, one address translation per lane (the UTCL1 request
  // and stall counters were 1.3x / 1.9x hipBLASLt's; 7-8 % of the kernel with the stores removed,
  // profiles/r4/gemm4/).  Each wave packs its 128 x 128 tile into its own 32 KB of the (now idle) stage LDS
  // (16-B chunks XOR-swizzled by row: conflict-free row reads), reads it back as whole 256-B row segments, and
  // stores them after the next tile's first LDS-DMA is issued.  (The GeGLU output is half as wide: its direct
  // stores measured faster than the round trip, which holds the gelu math in front of the next tile's loads.)
  if constexpr (LEPI) {
    // K tile 0 of the next tile loads into stage 0 under the round trip, which uses stage 1 (ERR rows per wave
    // and round); the LDS accesses are asm, or hipcc would wait for that LDS-DMA (vmcnt(0)) in front of them
    if (next < nwgv) {
      tile = next;
      G4_TILE(tile, m0, n0);
      G4_DESC();
      G4_STAGE(0, 0);
      if constexpr (SPARE) G4_STAGE(min(1, nt - 1), 1);
    }
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");   // last MFMA's D -> the accumulator reads below
    const uint32_t reg = (uint32_t)(uintptr_t)((g4_lds_char*)smem) + (SPARE ? 2 * STG + CTB : STG) + wid * ERR * RB;
    uint16_t* obase = reinterpret_cast<uint16_t*>(C) + (size_t)(em0 + wm * (BM / 2)) * ldc;
    const int nrow = min(BM / 2, M - em0 - wm * (BM / 2));
    const auto ors = __builtin_amdgcn_make_buffer_rsrc(obase, 0, nrow > 0 ? nrow * ldc * 2 : 0, 0x00020000);
    // write address of fragment column i (row lane&15 of a 16-row block; the block is the immediate offset), read
    // address of row group k%4 (rows 4k + lane/16; k/4 is the immediate offset)
    // (computed here from an opaque copy of the lane id: hoisted out of the tile loop they would be spilled)
    int ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(ln));
    const int oc0 = (EPI == G4_GEGLU ? (en0 >> 1) + wn * 64 : en0 + wn * 128) + (ln % ECH) * 8;
    // write address of fragment column i (row lane&15 of a 16-row block, chunk XOR-swizzled by the row; the block
    // is the immediate offset), read address of row group k % NRA (rows ERPI*k + lane/ECH)
    constexpr int NI = EPI == G4_GEGLU ? WN / 2 : WN, NRA = ECH / ERPI;
    uint32_t wa[NI], ra[NRA];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int cb = 32 * i + 8 * (ln >> 4);
      wa[i] = reg + (ln & 15) * RB + (((cb >> 4) ^ (ln & 15 & (ECH - 1))) << 4) + (cb & 15);
    }
#pragma unroll
    for (int k = 0; k < NRA; ++k) {
      const int r = ERPI * k + ln / ECH;
      ra[k] = reg + r * RB + (((ln % ECH) ^ (r & (ECH - 1))) << 4);
    }
    g4_unroll<(BM / 2) / ERR>([&](auto rc) {     // (a wave's LDS accesses run in order: the next round's writes
      constexpr int rnd = decltype(rc)::value;   // cannot pass this round's reads)
      g4_unroll<ERR / 16>([&](auto jc) {
        constexpr int jj = decltype(jc)::value, j = rnd * (ERR / 16) + jj;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          u32x2 w;
          if constexpr (EPI == G4_GEGLU) {
            // W rows interleaved per 128-row wave slice (ops.geglu_interleave_index):
            // fragments 0..3 are the gate rows of features f0 .. f0+63, fragments 4..7 the up rows of the same
            // features; gate|up are rounded to bf16 first so the result equals geglu(bf16 gate|up GEMM output)
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float gt = rbf(acc[i][j][q]), u = rbf(acc[i + WN / 2][j][q]);
              o[q] = rbf(gelu_tanh_fast(gt)) * u;
            }
            w = (u32x2){pack2(o[0], o[1]), pack2(o[2], o[3])};
          } else {
            w = (u32x2){pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3])};
          }
          g4_ds_write_b64<jj * 16 * RB>(wa[i], w);
        }
      });
      u32x4 ev[ERR / ERPI];
      g4_unroll<ERR / ERPI>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        g4_ds_read_b128<(k / NRA) * NRA * ERPI * RB>(ev[k], ra[k % NRA]);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // the round's rows as whole RB-byte segments (lane -> row ERPI*k + lane/ECH, 16-B chunk lane%ECH); buffer
      // stores bounded by the output's last row: every one is issued (an exact vmcnt count for the next tile's
      // first wait), rows past M are dropped by the bounds check
#pragma unroll
      for (int k = 0; k < ERR / ERPI; ++k)
        __builtin_amdgcn_raw_buffer_store_b128(ev[k], ors, ((rnd * ERR + ERPI * k + ln / ECH) * ldc + oc0) * 2, 0, 0);
    });
    if constexpr (!SPARE) {
      g4_bar();   // every wave's rows are out of stage 1
      if (next < nwgv) G4_STAGE(min(1, nt - 1), 1);
    }
  }
  // G4_HEAD: the rows' teacher targets, loaded before the next tile's LDS-DMA is issued (their wait then leaves
  // that DMA in flight)
  int tj[EPI == G4_HEAD ? WM : 1];
  if constexpr (EPI == G4_HEAD) {
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      const int m = em0 + wm * (BM / 2) + (lane & 15) + j * 16;
      tj[j] = -1;
      if (rp.tgt != nullptr) {
        const int t = rp.tgt[min(m, M - 1)];
        tj[j] = m < M ? t : -1;
      }
    }
  }
  // G4_ROPE: each lane's rows' positions / cache slots and their (cos, sin) pairs, loaded before the next tile's
  // LDS-DMA is issued -- the epilogue then waits for these alone (two dependent round trips per tile; loading them
  // per 16-row block behind that DMA cost ~15 % of the QKV GEMM, profiles/r5/gemm_dispatch/gs.jsonl e4 vs e0)
  constexpr int RWM = EPI == G4_ROPE ? WM : 1, RWN = EPI == G4_ROPE ? WN / 2 : 1;
  constexpr int RPF = RWM < 2 ? RWM : 2;   // row blocks whose (cos, sin) are loaded ahead of the DMA (more of them
                                            // at once, e.g. all 8: 128 VGPRs, spill)
  int rpos[RWM], rslt[RWM];
  uint4 rcs[RWM][RWN];
  if constexpr (EPI == G4_ROPE) {
    const int mb_ = em0 + wm * (BM / 2) + (lane & 15);
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      const int m = min(mb_ + j * 16, M - 1);
      rpos[j] = mb_ + j * 16 < M ? rp.pos[m] : -1;
      rslt[j] = rp.slot[m];
    }
#pragma unroll
    for (int j = 0; j < RPF; ++j) {
      const int pp = min(max(rpos[j], 0), rp.max_pos - 1);
#pragma unroll
      for (int i = 0; i < WN / 2; ++i)
        rcs[j][i] = *reinterpret_cast<const uint4*>(rp.cs + ((size_t)pp * 128 + wn * 64 + i * 16 + 4 * (lane >> 4)) * 2);
    }
  }
  if (!LEPI && next < nwgv) {
    tile = next;
    G4_TILE(tile, m0, n0);
    G4_DESC();
    G4_STAGE(0, 0);
    G4_STAGE(min(1, nt - 1), 1);
  }
  const uint16_t* ct = reinterpret_cast<const uint16_t*>(smem + 2 * STG);   // G4_HEAD's softcap table
  if constexpr (!LEPI) asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");   // last MFMA's D -> the accumulator reads

  // ---- epilogue.  acc[i][j][r]: n = n0 + wn*128 + i*16 + 4*(lane>>4) + r, m = m0 + wm*BM/2 + j*16 + (lane&15)
  {
  const int nb = en0 + wn * 128 + 4 * (lane >> 4);
  const int mb = em0 + wm * (BM / 2) + (lane & 15);
  if constexpr (EPI == G4_HEAD || EPI == G4_LENS) {
    // lane: columns nb + 16 i + r (i < 8, r < 4) of rows mb + 16 j; the 4 lanes lane&15 + 16 q share a row
    float4* part = reinterpret_cast<float4*>(EPI == G4_LENS ? rp.part : reinterpret_cast<float*>(C));
    const int npart = N / 128, pcol = (en0 >> 7) + wn;
    // branch-free: every element takes the same instruction path (selects, one table read), the table reads run
    // 2 fragments ahead of their use, the target logit is stored once per row
    const uint32_t ctb = (uint32_t)(uintptr_t)((g4_lds_char*)smem) + 2 * STG;
    constexpr float L2E = 1.4426950408889634f;
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      const int m = mb + j * 16;
      uint32_t bq[WN][4], tq[WN][4];
#pragma unroll
      for (int i = 0; i < WN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) bq[i][r] = f2bf(acc[i][j][r]);
      if constexpr (EPI == G4_HEAD) {
        auto rd = [&](auto ic) {
          constexpr int i = decltype(ic)::value;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            g4_ds_read_u16(tq[i][r], ctb + 2 * min(max((int)(bq[i][r] & 0x7fffu) - rp.clo, 0), rp.chi - rp.clo - 1));
        };
        rd(std::integral_constant<int, 0>{});
        rd(std::integral_constant<int, 1>{});
        g4_unroll<WN>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          if constexpr (i + 2 < WN) rd(std::integral_constant<int, i + 2>{});
          g4_lgkm_hold4<4 * (WN - 1 - i < 2 ? WN - 1 - i : 2)>(tq[i]);
        });
      }
      float z[WN * 4];
      float mx = -INFINITY, tl = 0.f;
      int bi = nb;
#pragma unroll
      for (int i = 0; i < WN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t b = bq[i][r];
          float v = __uint_as_float(b << 16);
          if constexpr (EPI == G4_HEAD) {   // compact exact softcap (csrc/lens.hip capc1); NaN passes through
            const uint32_t ab = b & 0x7fffu;
            const float mag = ab < (uint32_t)rp.chi ? __uint_as_float(tq[i][r] << 16) : rp.csat;
            const float cp = __uint_as_float(__float_as_uint(mag) | (b & 0x8000u) << 16);
            const float ln = rbf(rbf(v * rp.crc) * rp.ccap);
            v = ab < (uint32_t)rp.clo ? ln : (ab <= 0x7f80u ? cp : v);
          }
          const int n = nb + i * 16 + r;
          z[i * 4 + r] = v;
          if constexpr (EPI == G4_HEAD) {
            if (v > mx) { mx = v; bi = n; }   // the lane's columns ascend: the first maximum stays
            tl = n == tj[j] ? v : tl;
          } else {
            mx = fmaxf(mx, v);                // G4_LENS: no argmax (the lens needs the row LSE only)
          }
        }
      if constexpr (EPI == G4_HEAD) {
        const int d = tj[j] - nb;
        if (d >= 0 && d < WN * 16 && (d & 15) < 4) rp.tgt_logit[m] = tl;
      }
      const float mxl = mx * L2E;
      float sum = 0.f;
#pragma unroll
      for (int e = 0; e < WN * 4; ++e) sum += __builtin_amdgcn_exp2f(fmaf(z[e], L2E, -mxl));
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {   // the 4 lanes of a row; ties keep the lower column
        const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(sum, o, 64);
        const float nm = fmaxf(mx, m2);
        sum = sum * __builtin_amdgcn_exp2f((mx - nm) * L2E) + s2 * __builtin_amdgcn_exp2f((m2 - nm) * L2E);
        if constexpr (EPI == G4_HEAD) {
          const int i2 = __shfl_xor(bi, o, 64);
          bi = m2 > mx ? i2 : (m2 == mx ? min(bi, i2) : bi);
        }
        mx = nm;
      }
      if (lane < 16 && m < M) part[(size_t)m * npart + pcol] = make_float4(mx, sum, __int_as_float(bi), 0.f);
    }
  } else if constexpr (EPI == G4_ROPE) {
    // lane: d = wn*64 + 16 i + 4 (lane>>4) + r (i < 4) and d + 128 from fragment i + 4
    const int head = en0 >> 8, half = 128;
    const bool is_q = head < rp.Hq, is_k = !is_q && head < rp.Hq + rp.Hkv;
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      if (j + RPF < WM) {   // row block j + RPF's (cos, sin): in flight while this one is stored
        const int pp = min(max(rpos[j + RPF], 0), rp.max_pos - 1);
#pragma unroll
        for (int i = 0; i < WN / 2; ++i)
          rcs[j + RPF < WM ? j + RPF : 0][i] =
              *reinterpret_cast<const uint4*>(rp.cs + ((size_t)pp * 128 + wn * 64 + i * 16 + 4 * (lane >> 4)) * 2);
      }
      const int m = mb + j * 16;
      const int p = rpos[j];
      if (m >= M || (!is_q && (p < 0 || p >= rp.S))) continue;
      uint16_t* dst = is_q ? rp.q_out + ((size_t)m * rp.Hq + head) * 256
                           : (is_k ? rp.kc : rp.vc) +
                                 (((size_t)rslt[j] * rp.Hkv + (head - rp.Hq - (is_k ? 0 : rp.Hkv))) * rp.S + p) * 256;
#pragma unroll
      for (int i = 0; i < WN / 2; ++i) {
        const int d = wn * 64 + i * 16 + 4 * (lane >> 4);
        float o1[4], o2[4];
        if (p < 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o1[r] = o2[r] = 0.f;
        } else if (!is_q && !is_k) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { o1[r] = acc[i][j][r]; o2[r] = acc[i + WN / 2][j][r]; }
        } else {
          const uint32_t cws[4] = {rcs[j][i].x, rcs[j][i].y, rcs[j][i].z, rcs[j][i].w};   // cos(d+r) | sin(d+r) << 16
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x1 = rbf(acc[i][j][r]), x2 = rbf(acc[i + WN / 2][j][r]);
            const float c = __uint_as_float(cws[r] << 16), sn = __uint_as_float(cws[r] & 0xffff0000u);
            o1[r] = rbf(rbf(x1 * c) + rbf(-x2 * sn));
            o2[r] = rbf(rbf(x2 * c) + rbf(x1 * sn));
          }
        }
        *reinterpret_cast<uint2*>(dst + d) = make_uint2(pack2(o1[0], o1[1]), pack2(o1[2], o1[3]));
        *reinterpret_cast<uint2*>(dst + d + half) = make_uint2(pack2(o2[0], o2[1]), pack2(o2[2], o2[3]));
      }
    }
  } else if constexpr (EPI == G4_GEGLU && !LEPI) {
    // W rows interleaved per 128-row wave slice (ops.geglu_interleave_index): fragments 0..3 are the gate rows of
    // features f0 .. f0+63, fragments 4..7 the up rows of the same features; gate|up are rounded to bf16 first so
    // the result equals geglu(bf16 gate|up GEMM output).
    uint16_t* out = reinterpret_cast<uint16_t*>(C);
    const int fb = (en0 >> 1) + wn * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < WM; ++j) {
      const int m = mb + j * 16;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < WN / 2; ++i) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = rbf(acc[i][j][r]), u = rbf(acc[i + WN / 2][j][r]);
          o[r] = rbf(gelu_tanh_fast(gt)) * u;
        }
        *reinterpret_cast<uint2*>(out + (size_t)m * ldc + fb + i * 16) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  } else if constexpr (LEPI) {
    // stored above, from the LDS round trip
  } else {
#pragma unroll
    for (int i = 0; i < WN; ++i) {
      const int n = nb + i * 16;
      float4 bn_ = make_float4(0.f, 0.f, 0.f, 0.f), th = bn_;
      if constexpr (EPI == G4_JUMPRELU) {
        if (bias) bn_ = *reinterpret_cast<const float4*>(bias + n);
        if (thr) th = *reinterpret_cast<const float4*>(thr + n);
      }
#pragma unroll
      for (int j = 0; j < WM; ++j) {
        const int m = mb + j * 16;
        if (m >= M) continue;
        const f32x4 v = acc[i][j];
        if constexpr (EPI == G4_F32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + ((size_t)esk * M + m) * ldc + n) =
              make_float4(v[0], v[1], v[2], v[3]);
        } else {
          const float a0 = v[0] + bn_.x, a1 = v[1] + bn_.y, a2 = v[2] + bn_.z, a3 = v[3] + bn_.w;
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) =
              make_float4(a0 > th.x ? a0 : 0.f, a1 > th.y ? a1 : 0.f, a2 > th.z ? a2 : 0.f, a3 > th.w ? a3 : 0.f);
        }
      }
    }
  }
  }
  if (next >= nwgv) break;
#pragma unroll
  for (int i = 0; i < WN; ++i)
#pragma unroll
    for (int j = 0; j < WM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }   // tiles
  g4_vmcnt<0>();   // (nothing in flight: no LDS-DMA may land after the workgroup's LDS is handed to another one)
#undef G4_STAGE
#undef G4_STAGE_ONE
#undef G4_TILE
#undef G4_DESC
#endif
}

// Split-K reduction: out = sum over the ks fp32 partials in split order (deterministic), then bf16 (epi 0) or the
// GeGLU of the gate|up column pairs (epi 3, the interleaved layout of G4_GEGLU; same rounding chain).  8 outputs per
// thread.
template <int EPI>
__global__ void __launch_bounds__(256) g4_splitk_reduce_kernel(const float* __restrict__ part, uint16_t* __restrict__ out,
                                                               int M, int N, int ks, int ldo) {
  const int nout = EPI == G4_GEGLU ? N / 2 : N;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = nout / 8;
  if (i >= (size_t)M * per_row) return;
  const int m = (int)(i / per_row), c8 = (int)(i % per_row) * 8;
  const size_t plane = (size_t)M * N;
  float o[8];
  if constexpr (EPI == G4_GEGLU) {
    // output features f = c8 .. c8+7 live in 128-column block f/64: gate column 128*(f/64) + f%64, up +64
    const int blk = c8 >> 6, fi = c8 & 63;
    const float* g = part + (size_t)m * N + blk * 128 + fi;
    float gs[8], us[8];
    for (int e = 0; e < 8; ++e) gs[e] = us[e] = 0.f;
    sum_splits8(g, plane, ks, gs);
    sum_splits8(g + 64, plane, ks, us);
    for (int e = 0; e < 8; ++e) o[e] = rbf(gelu_tanh_fast(rbf(gs[e]))) * rbf(us[e]);
  } else {
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    sum_splits8(part + (size_t)m * N + c8, plane, ks, o);
  }
  *reinterpret_cast<uint4*>(out + (size_t)m * ldo + c8) =
      make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
}

}  // namespace

namespace {
// Persistent grid: one workgroup per CU (the kernel's LDS and registers allow one), a multiple of 8 so a
// workgroup's virtual tile ids stay on its XCD.
int g4_grid(int nwg) {
  static const int cap = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max(8, cus - cus % 8);
  }();
  return std::min(nwg, cap);
}
}  // namespace

bool tb_gemm4_ok(int M, int N, int K) { return M > 0 && N > 0 && N % G4_BN == 0 && K >= 64 && K % 64 == 0; }

// tile_rows: 256 or 128 (output rows per tile; identical numerics)
void tb_gemm4(const uint16_t* A, const uint16_t* W, void* C, const float* bias, const float* thr, int M, int N, int K,
              int ldc, int epi, int tile_rows, hipStream_t st, const uint16_t* a2, int k0) {
  if (M <= 0 || N <= 0) return;
  G4Rope rp{};
#define G4_GO(BM_, E_)                                                                                          \
  hipLaunchKernelGGL((gemm4_kernel<BM_, E_>), dim3(g4_grid((N / G4_BN) * ((M + (BM_) - 1) / (BM_)))),            \
                     dim3(G4_THREADS), 0, st, A, W, C, bias, thr, M, N, K, ldc, rp)
#define G4_GO2(BM_, E_)                                                                                         \
  hipLaunchKernelGGL((gemm4_kernel<BM_, E_, true>), dim3(g4_grid((N / G4_BN) * ((M + (BM_) - 1) / (BM_)))),      \
                     dim3(G4_THREADS), 0, st, A, W, C, bias, thr, M, N, K, ldc, rp)
#define G4_EPI(BM_)                                   \
  switch (epi) {                                      \
    case G4_BF16: G4_GO(BM_, G4_BF16); break;         \
    case G4_F32: G4_GO(BM_, G4_F32); break;           \
    case G4_JUMPRELU: G4_GO(BM_, G4_JUMPRELU); break; \
    default: G4_GO(BM_, G4_GEGLU);                    \
  }
  if (a2 != nullptr) {     // two-source A (host-checked: epi 0 / 3, 0 < k0 < K, both multiples of 64)
    rp.a2 = a2;
    rp.k0 = k0;
    if (tile_rows == 128) {
      if (epi == G4_GEGLU) G4_GO2(128, G4_GEGLU);
      else G4_GO2(128, G4_BF16);
    } else {
      if (epi == G4_GEGLU) G4_GO2(256, G4_GEGLU);
      else G4_GO2(256, G4_BF16);
    }
    return;
  }
  if (tile_rows == 128) {
    G4_EPI(128)
  } else {
    G4_EPI(256)
  }
#undef G4_EPI
}

// Split-K for thin grids (few output tiles: o_proj / down at N = 3584, any projection at decode M): ks K ranges per
// output tile, fp32 partials into ws [ks, M, N], then the ordered reduction (bf16, or GeGLU for epi 3).  Not batch
// invariant against tb_gemm4 (the K sum is split), so the dispatch uses it only in "auto" mode.
int tb_gemm4_splitk_ks(int M, int N, int K, int tile_rows) {
  const int nwg = (N / G4_BN) * ((M + tile_rows - 1) / tile_rows), NT = K / 64;
  int ks = std::max(1, std::min(g4_grid(1 << 30) / std::max(nwg, 1), NT / 4));
  const int kc = (NT + ks - 1) / ks;
  return (NT + kc - 1) / kc;
}

// The split GEMM alone: fp32 partials [ks, M, N] into ws (a consumer that folds the ordered sum into its own pass,
// e.g. tb_add_rmsnorm2_part).  Returns the split count actually used (ks rounded so every split is non-empty).
int tb_gemm4_splitk_part(const uint16_t* A, const uint16_t* W, float* ws, int M, int N, int K, int tile_rows, int ks,
                         hipStream_t st) {
  const int NT = K / 64;
  ks = std::max(1, std::min(ks, NT));
  const int kc = (NT + ks - 1) / ks;
  ks = (NT + kc - 1) / kc;
  if (M <= 0 || N <= 0) return ks;
  G4Rope rp{};
  rp.ksplit = ks;
  rp.kchunk = kc;
  void* C = ws;
  const float* bias = nullptr;
  const float* thr = nullptr;
  const int ldc = N;
  const int nwg = (N / G4_BN) * ((M + tile_rows - 1) / tile_rows) * ks;
  if (tile_rows == 64)      // decode row counts: a 64-row tile wastes 4x fewer MFMAs on rows past M than 128
    hipLaunchKernelGGL((gemm4_kernel<64, G4_F32>), dim3(g4_grid(nwg)), dim3(G4_THREADS), 0, st, A, W, C, bias, thr, M, N,
                       K, ldc, rp);
  else if (tile_rows == 128)
    hipLaunchKernelGGL((gemm4_kernel<128, G4_F32>), dim3(g4_grid(nwg)), dim3(G4_THREADS), 0, st, A, W, C, bias, thr, M, N,
                       K, ldc, rp);
  else
    hipLaunchKernelGGL((gemm4_kernel<256, G4_F32>), dim3(g4_grid(nwg)), dim3(G4_THREADS), 0, st, A, W, C, bias, thr, M, N,
                       K, ldc, rp);
  return ks;
}

void tb_gemm4_splitk(const uint16_t* A, const uint16_t* W, uint16_t* out, float* ws, int M, int N, int K, int ldo,
                     int epi, int tile_rows, int ks, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  ks = tb_gemm4_splitk_part(A, W, ws, M, N, K, tile_rows, ks, st);
  const size_t nthr = (size_t)M * ((epi == G4_GEGLU ? N / 2 : N) / 8);
  const dim3 grid((unsigned)((nthr + 255) / 256));
  if (epi == G4_GEGLU)
    hipLaunchKernelGGL(g4_splitk_reduce_kernel<G4_GEGLU>, grid, dim3(256), 0, st, ws, out, M, N, ks, ldo);
  else
    hipLaunchKernelGGL(g4_splitk_reduce_kernel<G4_BF16>, grid, dim3(256), 0, st, ws, out, M, N, ks, ldo);
}

void tb_head_fused4(const uint16_t* A, const uint16_t* W, float* part, float cap, const int32_t* tgt,
                    float* tgt_logit, int32_t* nxt, float* nll_self, float* nll_tgt, int M, int N, int K, hipStream_t st) {
  if (M <= 0) return;
  void* C = part;
  const float* bias = nullptr;
  const float* thr = nullptr;
  const int ldc = 0;
  G4Rope rp{};
  if (cap > 0.f) {
    const uint16_t* ct = nullptr;
    int lo = 0, hi = 0;
    float sat = 0.f;
    if (!tb_softcap_compact_params(cap, &ct, &lo, &hi, &sat) || hi - lo > 2048) return;   // host-checked
    rp.ctab = ct;
    rp.clo = lo;
    rp.chi = hi;
    rp.csat = sat;
    rp.crc = 1.0f / cap;
    rp.ccap = cap;
  } else {            // no softcap: every finite value takes the (identity) arithmetic branch
    rp.clo = 0x7f81;
    rp.chi = 0x7f82;
    rp.crc = rp.ccap = 1.f;
  }
  rp.tgt = tgt;
  rp.tgt_logit = tgt_logit;
  G4_GO(256, G4_HEAD);
  tb_head_merge(reinterpret_cast<const float*>(part), N / 128, tgt, tgt_logit, nxt, nll_self, nll_tgt, nullptr, M, N, st);
}

// Logit-lens unembedding: bf16 logits [M, N] (no softcap) and the row log-sum-exp, with no second
// pass over the logits: G4_LENS's per-slice {max, sum exp} partials folded by tb_head_merge.
void tb_lens_gemm4(const uint16_t* A, const uint16_t* W, uint16_t* logits, float* part, float* lse, int M, int N,
                   int K, hipStream_t st) {
  if (M <= 0) return;
  void* C = logits;
  const float* bias = nullptr;
  const float* thr = nullptr;
  const int ldc = N;
  G4Rope rp{};
  rp.part = part;
  G4_GO(256, G4_LENS);
  tb_head_merge(part, N / 128, nullptr, nullptr, nullptr, nullptr, nullptr, lse, M, N, st);
}

void tb_gemm4_qkv_rope(const uint16_t* A, const uint16_t* W, const int32_t* pos, const int32_t* slot_of_row,
                       const uint16_t* cs, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M, int K,
                       int Hq, int Hkv, int S, int max_pos, int tile_rows, hipStream_t st, const uint16_t* a2, int k0) {
  if (M <= 0) return;
  const int N = (Hq + 2 * Hkv) * 256, ldc = 0;
  void* C = nullptr;
  const float* bias = nullptr;
  const float* thr = nullptr;
  G4Rope rp{pos, slot_of_row, cs, q_out, kc, vc, Hq, Hkv, S, max_pos};
  if (a2 != nullptr) {
    rp.a2 = a2;
    rp.k0 = k0;
    if (tile_rows == 128) G4_GO2(128, G4_ROPE);
    else G4_GO2(256, G4_ROPE);
    return;
  }
  if (tile_rows == 128) G4_GO(128, G4_ROPE);
  else G4_GO(256, G4_ROPE);
#undef G4_GO
#undef G4_GO2
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
