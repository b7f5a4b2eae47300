// Ring GEMM for decode-to-mid row counts on gfx950: C = A[M,K] . W[N,K]^T with small output tiles (BM x BN from
// 16 x 16 to 128 x 128, and 16..256 x 112 for the N = 3584 projections) and a deep LDS-DMA ring, batch-invariant by construction (SURVEY K3/K6/K7/K8 at the row
// counts of the greedy decode and the ride-along baselines).
//
// Why: at M <= ~2k rows the N = 3584 / 8192 projections have too few 256-wide column tiles to fill 256 CUs, and the
// usual cure (split-K: fp32 partials of K ranges summed afterwards) changes a row's summation order with M, so a
// row's bf16 result depends on the batch it runs in (the reuse levels of the sweep are then exact only in the
// unsplit mode).  This kernel fills the chip with NARROW tiles instead and keeps gemm4.hip's exact per-output K
// chain: every output element is one fp32 accumulator fed by v_mfma_f32_16x16x32_bf16 in 32-deep K steps in K
// order, W fragment as the MFMA's first operand, A fragment as its second -- the same instruction sequence per
// element as gemm4_kernel / gemm_pp_kernel, so all three agree bit for bit at every M and every tile shape
// (tests/test_kernels_gpu.py::test_gemm_ring_bitexact).  The throughput model (MI355X_MICROARCH.md,
// ring-gemm / ring-vs-splitk): a decode projection is bound by the per-CU L2->LDS rate, total traffic
// 2KNM (1/BM + 1/BN), so the tile is chosen per (N, K, M) by measurement (tools/gemm_dispatch_tune.py).
//
// Structure:
//  * 256 threads = 4 waves; WGM x WGN of them own (BM/WGM) x (BN/WGN) sub-tiles, the rest (tiny tiles) only stage.
//  * K tiles are 64 deep.  Stage image: [BN W rows | BM A rows] x 128 B, 16-B chunk c of image row r stored at
//    c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 fragment reads, gemm4's layout).  A ring stage holds KU such
//    K-tile images; NS stages fill the LDS budget (64 KB: two workgroups per CU; 144 KB: one, for thin grids) so that
//    NS-1 stages are in flight per workgroup: at decode M the kernel is a latency-bound stream (Little's law: the
//    chip's in-flight bytes over its bandwidth is the load latency) and bytes in flight per CU set its rate; KU > 1
//    amortises the per-stage wait + barrier over more bytes.
//  * Staging: global_load_lds_dwordx4, one wave-instruction = 8 whole image rows; instruction j is issued by wave
//    j % 4.  One barrier per K tile: wait (counted vmcnt) for this wave's part of tile t+1, barrier, stage
//    t+NS-1 into the slot stage t-1 left, MFMAs of stage t, read stage t+1's fragments into the second register set.
//  * Pair epilogues keep both halves of a pair in one lane: GeGLU (gate | up of the same feature, the interleaved
//    gate|up weight of ops.geglu_interleave_index) and RoPE (head dims d and d + 128 of the QKV projection, then
//    the KV-cache scatter with rope_qkv_cache_kernel's bf16 chain; csrc/rope.hip).  A tile of BN/2 pair units maps
//    its image rows onto the two halves, wave by wave.
//  * Block ids: XCD-aware (consecutive tile ids on one XCD), column tile major, so the row tiles of one column tile
//    read its W panel through the same L2.
// Requirements (host-checked, tb_gemm_ring_ok): K % 128 == 0, N % BN == 0 (pair epilogues: (N / 2) % (BN / 2) == 0),
// any M.
//
// The 112-column tiles: at mid M (256 .. ~2k rows) a narrow-tile GEMM is bound by each CU's L2 -> LDS fill rate
// (MI355X_MICROARCH.md: 66-73 GB/s per CU from an L2-resident panel), so its time is rounds x (BM + BN) K bytes: N =
// 3584 = 32 x 112 columns with the row tile BM ~ M / 8 gives one round of ~256 tiles at the fewest bytes per tile (e.g.
// M = 768: 96 x 112 tiles, 208 image rows per CU, vs 256 rows for 168 tiles of 128 x 128).
#include "common.h"
#include "api.h"
#include <utility>

namespace {

typedef __attribute__((address_space(3))) void rg_lds_t;
typedef const __attribute__((address_space(1))) void rg_gbl_t;

enum { RG_BF16 = 0, RG_GEGLU = 3, RG_ROPE = 4, RG_LMASK = 5 };

struct RingArgs {   // RG_ROPE operands (gemm4.hip G4Rope's subset)
  const int32_t* pos;
  const int32_t* slot;
  const uint16_t* cs;   // bf16 (cos, sin) pairs [max_pos, 128, 2]
  uint16_t* q_out;
  uint16_t* kc;
  uint16_t* vc;
  int Hq, Hkv, S, max_pos;
  // two-source A (L2A instantiations, multi-adapter LoRA; gemm4.hip G4Rope::a2): columns [0, k0) of A from A (row
  // stride k0), [k0, K) from a2 (row stride K - k0)
  const uint16_t* a2;
  int k0;
  // RG_LMASK (the LoRA down-projection T = x A_all^T of the multi-adapter bank, models/lora.py): output column c is
  // kept only where it belongs to the row's adapter -- c < nsr and (c % nr) / r == adapter[m] -- else 0
  const int32_t* adapter;
  int nsr, nr, r;
  // RG_LMASK chunk structure (batch invariance of T at every M): K is cut into chunks of kct K tiles; a chunk's
  // dot products run one MFMA chain from zero and T = bf16(((0 + c_0) + c_1) + ...) in chunk order.  nch == 0: one
  // workgroup runs every chunk of its tile and folds them in registers (large M); nch > 0: one workgroup per (tile,
  // chunk) writes its chunk's fp32 sums to part[chunk][M][N] and lora_t_reduce_kernel folds them in the same order
  // (decode M: nch x more workgroups for the K = 3584 .. 14336 chains).  Both give the same bits.
  float* part;
  int kct, nch;
};

template <int N_>
__device__ __forceinline__ void rg_vmcnt() {
  static_assert(N_ >= 0 && N_ < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}
// wait until at most G * n of this wave's staging instructions are outstanding (n <= NMAX, wave-uniform)
template <int G, int NMAX>
__device__ __forceinline__ void rg_wait_tiles(int n) {
  if constexpr (NMAX <= 0) {
    rg_vmcnt<0>();
  } else {
    if (n >= NMAX) rg_vmcnt<G * NMAX>();
    else rg_wait_tiles<G, NMAX - 1>(n);
  }
}
// raw s_barrier (no fence: __syncthreads' fence would drain the ring with vmcnt(0)); the empty asm statements keep
// the compiler from moving LDS reads or staging across it
__device__ __forceinline__ void rg_bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// wave grid of a tile: as many computing waves (<= 4, not necessarily a power of two: a 96-row tile runs 3) as the
// 16-row / 16-column (pair epilogues: 32-column) fragments allow, then the squarest wave tile
constexpr int rg_wgn(int BM, int BN, bool pair) {
  int best = 1, bestc = -1, bestd = 1 << 30;
  const int fn = pair ? 32 : 16;
  for (int wn = 1; wn <= 4; ++wn) {
    if (BN % (wn * fn)) continue;
    for (int wm = 1; wm * wn <= 4; ++wm) {
      if (BM % (wm * 16)) continue;
      const int c = wm * wn, tm = BM / wm, tn = BN / wn, d = tm > tn ? tm - tn : tn - tm;
      if (c > bestc || (c == bestc && (d < bestd || (d == bestd && tn > BN / best)))) {
        best = wn;
        bestc = c;
        bestd = d;
      }
    }
  }
  return best;
}
constexpr int rg_wgm(int BM, int BN, bool pair) {
  const int wn = rg_wgn(BM, BN, pair);
  int wm = 1;
  for (int w = 1; w * wn <= 4; ++w)
    if (BM % (w * 16) == 0) wm = w;
  return wm;
}
// ring depth: the LDS budget (LKB KB) in stages of KU K-tile images, 3 .. 32, and the counted waits must fit
// vmcnt's 6 bits
constexpr int rg_ns(int BM, int BN, int KU, int LKB) {
  const int R = BN + BM, ni = R / 8, g = KU * ((ni + 3) / 4);
  int ns = LKB * 1024 / (R * 128 * KU);
  ns = ns < 3 ? 3 : ns > 32 ? 32 : ns;
  while (ns > 3 && g * (ns - 2) > 63) --ns;
  return ns;
}

template <int BM, int BN, int EPI, int KU, int LKB, bool L2A = false>
__global__ void __launch_bounds__(256, LKB <= 80 ? 2 : 1)
gemm_ring_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, uint16_t* __restrict__ C, int M,
                 int N, int K, int ldc, RingArgs ra) {
  constexpr bool PAIR = EPI == RG_GEGLU || EPI == RG_ROPE;
  constexpr int WGN = rg_wgn(BM, BN, PAIR), WGM = rg_wgm(BM, BN, PAIR), NS = rg_ns(BM, BN, KU, LKB);
  constexpr int R = BN + BM, IB = R * 128, SB = KU * IB, NI = R / 8, GLO = NI / 4, GX = NI % 4, GMAX = GLO + (GX ? 1 : 0);
  constexpr int TM = BM / WGM, TN = BN / WGN, FM = TM / 16, FN = TN / 16;
  static_assert(BM % 16 == 0 && BN % 16 == 0 && R % 8 == 0 && NS >= 3, "tile");
  static_assert(!PAIR || (FN % 2 == 0 && BN / 2 <= 64), "pair epilogue tile");
  static_assert(KU * GMAX * (NS - 2) <= 63, "vmcnt");
  __shared__ __attribute__((aligned(1024))) char smem[NS * SB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = (M + BM - 1) / BM, ntn = N / BN, ntile = ntm * ntn;
  constexpr bool LM = EPI == RG_LMASK;
  const int nch = LM ? ra.nch : 0;
  int bid = blockIdx.x, chunk = 0;
  if (LM && nch > 0) {   // split chunks: block = chunk * ntile + tile
    chunk = bid / ntile;
    bid -= chunk * ntile;
  }
  // XCD-aware tile id: block b runs on XCD b % 8 (round-robin dispatch, a speed assumption only); each XCD takes a
  // contiguous range of tile ids, row tiles fastest
  int u;
  {
    const int b = bid, x = b % 8, q = ntile / 8, r = ntile % 8;
    u = x * q + min(x, r) + b / 8;
  }
  const int tn = u / ntm, tm = u - tn * ntm;
  const int m0 = tm * BM, n0 = tn * BN, u0 = tn * (BN / 2);
  const int kt0 = LM ? chunk * ra.kct : 0;                                  // first K tile (split chunks)
  const int nt = LM && nch > 0 ? ra.kct / KU : K / (64 * KU);               // ring stages over K
  const int spc = LM ? ra.kct / KU : 0;                                     // stages per chunk

  // W row of tile image row r (pair epilogues: wave-by-wave halves of BN/2 pair units)
  auto wrow = [&](int r) -> int {
    if constexpr (!PAIR) {
      return n0 + r;
    } else {
      const int wn = r / TN, rr = r % TN, half = rr >= TN / 2 ? 1 : 0, unit = u0 + wn * (TN / 2) + rr - half * (TN / 2);
      if constexpr (EPI == RG_GEGLU) return (unit >> 6) * 128 + (unit & 63) + half * 64;
      else return (unit >> 7) * 256 + (unit & 127) + half * 128;
    }
  };

  // ---- staging sources: instruction j = wid + 4 q covers image rows 8j .. 8j+7; lane -> row 8j + lane/8, physical
  // chunk lane % 8 holding logical chunk (lane % 8) ^ ((row >> 1) & 7)
  // (L2A: A rows have stride k0 and K tiles from k0 / 64 on come from a2; an instruction's 8 image rows are all W or
  // all A rows, BN % 8 == 0)
  const int KA = L2A ? ra.k0 : K, K2 = K - KA, NT0 = KA >> 6;
  const uint16_t* src[GMAX];
  // (L2A: per instruction the byte offset from its first-source row to its second-source row at the same K tile,
  // 0 for W rows -- added under a uniform mask from K tile k0 / 64 on, no per-instruction select)
  int64_t dlt[L2A ? GMAX : 1];
#pragma unroll
  for (int q = 0; q < GMAX; ++q) {
    const int j = wid + 4 * q, lr = min(8 * j + (lane >> 3), R - 1);
    const int lc = (lane & 7) ^ ((lr >> 1) & 7);
    const int am = min(m0 + lr - BN, M - 1);
    const uint16_t* row = lr < BN ? W + (size_t)wrow(lr) * K : A + (size_t)am * KA;
    src[q] = row + lc * 8 + kt0 * 64;
    if constexpr (L2A) {
      const bool isa = 8 * j >= BN;
      const uint16_t* s2 = ra.a2 + (size_t)(isa ? am : 0) * K2 + lc * 8;   // K tile NT0 of the second source
      dlt[q] = isa ? (int64_t)((uintptr_t)s2 - (uintptr_t)(src[q] + (size_t)NT0 * 64)) : 0;
    }
  }
  const bool gx = wid < GX;   // this wave issues GLO + 1 instructions per K tile
  auto issue = [&](int t, int stg) {
#pragma unroll
    for (int kk = 0; kk < KU; ++kk)
#pragma unroll
      for (int q = 0; q < GMAX; ++q) {
        if (q < GLO || gx) {
          const int kt = t * KU + kk;
          const uint16_t* p = src[q] + kt * 64;
          if constexpr (L2A) p = (const uint16_t*)((const char*)p + (dlt[q] & -(int64_t)(kt >= NT0)));
          __builtin_amdgcn_global_load_lds((rg_gbl_t*)p,
                                           (rg_lds_t*)(smem + stg * SB + kk * IB + (wid + 4 * q) * 1024), 16, 0, 0);
        }
      }
  };
  auto wait_tiles = [&](int n) {   // n stages of this wave's staging left in flight
    if constexpr (GX > 0) {
      if (gx) rg_wait_tiles<KU * (GLO + 1), NS - 2>(n);
      else rg_wait_tiles<KU * GLO, NS - 2>(n);
    } else {
      rg_wait_tiles<KU * GLO, NS - 2>(n);
    }
  };

  // ---- fragments: operand row = base + (lane & 15), logical chunk 4 s + (lane >> 4) of K step s
  const bool active = wid < WGM * WGN;
  const int wm = active ? wid / WGN : 0, wn = active ? wid % WGN : 0;
  const int xr = (lane & 15) >> 1;
  const int c0 = ((lane >> 4) ^ xr) << 4, c1 = ((4 + (lane >> 4)) ^ xr) << 4;
  const int offw = (wn * TN + (lane & 15)) * 128, offa = (BN + wm * TM + (lane & 15)) * 128;
  bf16x8 fw[2][2 * KU][FN], fa[2][2 * KU][FM];   // [register set][K step of the stage][fragment]
  f32x4 acc[FN][FM];
  f32x4 sum[LM ? FN : 1][LM ? FM : 1];   // RG_LMASK: the folded chunks
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if constexpr (LM) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) sum[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  auto ld = [&](int off) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(smem + off)); };
  auto read = [&](auto setc, int stg) {
    constexpr int S_ = decltype(setc)::value;
#pragma unroll
    for (int kk = 0; kk < KU; ++kk) {
      const int b = stg * SB + kk * IB;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        fw[S_][2 * kk][i] = ld(b + offw + i * 2048 + c0);
        fw[S_][2 * kk + 1][i] = ld(b + offw + i * 2048 + c1);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        fa[S_][2 * kk][j] = ld(b + offa + j * 2048 + c0);
        fa[S_][2 * kk + 1][j] = ld(b + offa + j * 2048 + c1);
      }
    }
  };
  auto mfma = [&](auto setc) {
    constexpr int S_ = decltype(setc)::value;
#pragma unroll
    for (int s = 0; s < 2 * KU; ++s)   // K order: the stage's 32-deep steps in sequence, for every accumulator
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[S_][s][i], fa[S_][s][j], acc[i][j], 0, 0, 0);
  };

  // ---- prologue: tiles 0 .. NS-2 in flight, tile 0's fragments in set 0
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nt) issue(p, p);
  wait_tiles(min(NS - 2, nt - 1));
  rg_bar();
  if (active) read(std::integral_constant<int, 0>{}, 0);

  // ---- main loop (two K tiles per trip so the register sets are static)
  int st1 = 1 % NS, stn = NS - 1;   // stage of tile t+1, stage tile t+NS-1 goes to
  auto body = [&](auto setc, int t) {
    constexpr int S_ = decltype(setc)::value;
    if (t + 1 < nt) {
      wait_tiles(min(NS - 3, nt - 2 - t));   // this wave's part of tile t+1 landed ...
      rg_bar();                              // ... everyone's, and every wave is done with tile t-1's stage
    }
    if (t + NS - 1 < nt) issue(t + NS - 1, stn);
    if (active) {   // MFMAs first: the reads of tile t+1 then overlap the next trip's wait and barrier
      mfma(setc);
      if (t + 1 < nt) read(std::integral_constant<int, S_ ^ 1>{}, st1);
      if constexpr (LM) {
        if (nch == 0 && (t + 1) % spc == 0) {   // end of a chunk: fold it in, next chunk's chain from zero
#pragma unroll
          for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) {
              sum[i][j] += acc[i][j];
              acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
            }
        }
      }
    }
    st1 = st1 + 1 == NS ? 0 : st1 + 1;
    stn = stn + 1 == NS ? 0 : stn + 1;
  };
  for (int t = 0; t < nt; t += 2) {
    body(std::integral_constant<int, 0>{}, t);
    if (t + 1 < nt) body(std::integral_constant<int, 1>{}, t + 1);
  }
  if (!active) return;

  // ---- epilogue.  acc[i][j][r]: wave image row wn*TN + 16 i + 4 (lane >> 4) + r, output row m0 + wm*TM + 16 j + (lane & 15)
  const int mb = m0 + wm * TM + (lane & 15);
  if constexpr (EPI == RG_BF16) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * TN + i * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = mb + j * 16;
        if (m < M)
          *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) =
              make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
      }
    }
  } else if constexpr (EPI == RG_LMASK) {
    if (nch > 0) {   // this chunk's fp32 sums, unmasked (lora_t_reduce_kernel folds and masks)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = mb + j * 16;
        if (m >= M) continue;
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int n = n0 + wn * TN + i * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(ra.part + ((size_t)chunk * M + m) * N + n) = acc[i][j];
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = mb + j * 16;
      if (m >= M) continue;
      const int ad = ra.adapter[m];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * TN + i * 16 + 4 * (lane >> 4);
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = n + q;
          o[q] = (ad >= 0 && c < ra.nsr && (c % ra.nr) / ra.r == ad) ? sum[i][j][q] : 0.f;
        }
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  } else if constexpr (EPI == RG_GEGLU) {
    // gate|up rounded to bf16 first: the result equals geglu(bf16 gate|up GEMM output), as gemm4's G4_GEGLU
#pragma unroll
    for (int i = 0; i < FN / 2; ++i) {
      const int f = u0 + wn * (TN / 2) + i * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = mb + j * 16;
        if (m >= M) continue;
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float gt = rbf(acc[i][j][q]), up = rbf(acc[i + FN / 2][j][q]);
          o[q] = rbf(gelu_tanh_fast(gt)) * up;
        }
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + f) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
      }
    }
  } else {
    // RoPE + KV scatter (gemm4.hip G4_ROPE / rope.hip chain); the tile's units lie in one head
    const int head = u0 >> 7, half = 128;
    const bool is_q = head < ra.Hq, is_k = !is_q && head < ra.Hq + ra.Hkv;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = mb + j * 16;
      if (m >= M) continue;
      const int p = ra.pos[m];
      if (!is_q && (p < 0 || p >= ra.S)) continue;
      const int pp = p < ra.max_pos ? p : ra.max_pos - 1;
      uint16_t* dst;
      if (is_q) dst = ra.q_out + ((size_t)m * ra.Hq + head) * 256;
      else
        dst = (is_k ? ra.kc : ra.vc) +
              (((size_t)ra.slot[m] * ra.Hkv + (head - ra.Hq - (is_k ? 0 : ra.Hkv))) * ra.S + p) * 256;
#pragma unroll
      for (int i = 0; i < FN / 2; ++i) {
        const int d = ((u0 + wn * (TN / 2)) & 127) + i * 16 + 4 * (lane >> 4);
        float o1[4], o2[4];
        if (p < 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o1[r] = o2[r] = 0.f;
        } else if (!is_q && !is_k) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { o1[r] = acc[i][j][r]; o2[r] = acc[i + FN / 2][j][r]; }
        } else {
          const uint4 cw = *reinterpret_cast<const uint4*>(ra.cs + ((size_t)pp * half + d) * 2);
          const uint32_t cws[4] = {cw.x, cw.y, cw.z, cw.w};   // word r: cos(d + r) | sin(d + r) << 16
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x1 = rbf(acc[i][j][r]), x2 = rbf(acc[i + FN / 2][j][r]);
            const float c = __uint_as_float(cws[r] << 16), sn = __uint_as_float(cws[r] & 0xffff0000u);
            o1[r] = rbf(rbf(x1 * c) + rbf(-x2 * sn));
            o2[r] = rbf(rbf(x2 * c) + rbf(x1 * sn));
          }
        }
        *reinterpret_cast<uint2*>(dst + d) = make_uint2(pack2(o1[0], o1[1]), pack2(o1[2], o1[3]));
        *reinterpret_cast<uint2*>(dst + d + half) = make_uint2(pack2(o2[0], o2[1]), pack2(o2[2], o2[3]));
      }
    }
  }
}

// (BM, BN) tiles built per epilogue; tb_gemm_ring_tiles() lists them for the tuner
#define RG_PLAIN_TILES(X) X(16, 16) X(16, 32) X(16, 64) X(32, 32) X(32, 64) X(64, 32) X(64, 64) X(128, 32) X(64, 128) \
  X(128, 64) X(128, 128)
// 112-column tiles for the N = 3584 projections (o_proj, down): 32 column tiles, and the row tile from the set
// below chosen per M (measured, tools/ring_bench.py) so the grid is about one tile per CU; 144 KB ring only
#define RG_N112_TILES(X) X(16, 112) X(32, 112) X(48, 112) X(64, 112) X(96, 112) X(128, 112) X(144, 112) X(192, 112) \
  X(256, 112)
#define RG_PAIR_TILES(X) X(16, 32) X(16, 64) X(32, 32) X(32, 64) X(64, 32) X(64, 64) X(128, 32) X(64, 128) X(128, 64) \
  X(128, 128)

// ring variants: 0 = one K tile per stage, 64 KB (two workgroups per CU); 1 = two K tiles per stage (one for the
// largest tiles), 144 KB (thin grids); 2 = the small tiles (<= 64 image rows) with 4 or 8 K tiles per stage, 144 KB:
// at decode row counts a stage of a 16 x 16 tile is 4 KB, and the per-stage wait + barrier + dependent MFMA chain
// (~600 cycles), not the bytes, set the rate -- deeper stages amortise it (rg_ku2)
#ifndef RG_LKB1
#define RG_LKB1 144   // (160 KB, one more stage in flight: no faster at mid M, profiles/r5/gemm_dispatch/ring_lkb160.jsonl)
#endif
constexpr int rg_ku1(int BM, int BN) { return (BM + BN) * 128 * 2 * 3 <= 144 * 1024 ? 2 : 1; }   // (>= 3 stages)
constexpr int rg_ku2(int BM, int BN) {
  return (BM + BN) * 128 * 8 * 4 <= 144 * 1024 ? 8 : (BM + BN) * 128 * 4 * 4 <= 144 * 1024 ? 4 : rg_ku1(BM, BN);
}
template <int BM, int BN, int EPI>
void rg_launch(int var, const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, int ldc,
               const RingArgs& ra, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  constexpr int KU1 = rg_ku1(BM, BN), KU2 = rg_ku2(BM, BN);
  if (ra.a2 != nullptr) {   // two-source A (multi-adapter LoRA): the 144 KB ring only (host-checked)
    if constexpr (EPI != RG_LMASK)
      hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, EPI, KU1, RG_LKB1, true>), dim3(tiles), dim3(256), 0, st, A, W, C, M,
                         N, K, ldc, ra);
    return;
  }
  if (var == 2) {
    if constexpr (KU2 > KU1)
      hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, EPI, KU2, 144>), dim3(tiles), dim3(256), 0, st, A, W, C, M, N, K, ldc,
                         ra);
  } else if (var == 1) {
    hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, EPI, KU1, RG_LKB1>), dim3(tiles), dim3(256), 0, st, A, W, C, M, N, K, ldc, ra);
  } else {
    hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, EPI, 1, 64>), dim3(tiles), dim3(256), 0, st, A, W, C, M, N, K, ldc, ra);
  }
}
// whether variant 2 exists for a tile (deeper stages than variant 1)
bool rg_has_var2(int bm, int bn) { return rg_ku2(bm, bn) > rg_ku1(bm, bn); }

template <int BM, int BN>
void rg_launch_wide(const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, int ldc, const RingArgs& ra,
                    hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  if (ra.a2 != nullptr)
    hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, RG_BF16, 1, RG_LKB1, true>), dim3(tiles), dim3(256), 0, st, A, W, C, M,
                       N, K, ldc, ra);
  else
    hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, RG_BF16, 1, RG_LKB1>), dim3(tiles), dim3(256), 0, st, A, W, C, M, N, K,
                       ldc, ra);
}

template <int EPI>
bool rg_dispatch(int bm, int bn, int var, const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, int ldc,
                 const RingArgs& ra, hipStream_t st) {
#define RG_CASE(BM_, BN_)                                         \
  if (bm == BM_ && bn == BN_) {                                   \
    rg_launch<BM_, BN_, EPI>(var, A, W, C, M, N, K, ldc, ra, st); \
    return true;                                                  \
  }
  if constexpr (EPI == RG_BF16) {
    RG_PLAIN_TILES(RG_CASE)
#define RG_CASE_W(BM_, BN_)                                     \
  if (bm == BM_ && bn == BN_) {                                 \
    if (var != 1) return false;                                 \
    rg_launch_wide<BM_, BN_>(A, W, C, M, N, K, ldc, ra, st);    \
    return true;                                                \
  }
    RG_N112_TILES(RG_CASE_W)
#undef RG_CASE_W
  } else {
    RG_PAIR_TILES(RG_CASE)
  }
#undef RG_CASE
  return false;
}

bool rg_has(int epi, int bm, int bn) {
#define RG_HAS(BM_, BN_) if (bm == BM_ && bn == BN_) return true;
  if (epi == RG_BF16) {
    RG_PLAIN_TILES(RG_HAS)
    RG_N112_TILES(RG_HAS)
  } else if (epi == RG_GEGLU || epi == RG_ROPE) {
    RG_PAIR_TILES(RG_HAS)
  }
#undef RG_HAS
  return false;
}

}  // namespace

// the LoRA down-projection's tiles (RG_LMASK, N = the bank's padded width, 144 KB ring)
#define RG_LMASK_TILES(X) X(16, 32) X(32, 32) X(64, 32) X(128, 32) X(16, 64) X(32, 64) X(64, 64) X(128, 64) X(16, 96) \
  X(32, 96) X(64, 96)

namespace {
// K tiles per chunk of the T chain: 512-deep where K allows (the Gemma-2 projections: 7 / 8 / 28 chunks), else 128;
// a function of K alone, so every M and both launch forms share one summation order
int lora_kct(int K) { return K % 512 == 0 ? 8 : 2; }

// T[m, n..n+3] = bf16(((0 + part[0]) + part[1]) + ...) on the row's adapter's columns, else 0 (the fold of the
// split form, in gemm_ring_kernel's nch == 0 order)
__global__ void __launch_bounds__(256) lora_t_reduce_kernel(const float* __restrict__ part, uint16_t* __restrict__ t,
                                                            const int32_t* __restrict__ adapter, int M, int N, int ldt,
                                                            int nch, int nsr, int nr, int r) {
  const int ng = N / 4, i = blockIdx.x * 256 + threadIdx.x;
  if (i >= M * ng) return;
  const int m = i / ng, n = (i - m * ng) * 4;
  const float* p = part + (size_t)m * N + n;
  const size_t cs = (size_t)M * N;
  f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f};
  int c = 0;
  for (; c + 4 <= nch; c += 4) {   // four loads in flight, then the adds in chunk order
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(p + c * cs), v1 = *reinterpret_cast<const f32x4*>(p + (c + 1) * cs),
                v2 = *reinterpret_cast<const f32x4*>(p + (c + 2) * cs), v3 = *reinterpret_cast<const f32x4*>(p + (c + 3) * cs);
    s += v0;
    s += v1;
    s += v2;
    s += v3;
  }
  for (; c < nch; ++c) s += *reinterpret_cast<const f32x4*>(p + c * cs);
  const int ad = adapter[m];
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = n + q;
    o[q] = (ad >= 0 && c < nsr && (c % nr) / r == ad) ? s[q] : 0.f;
  }
  *reinterpret_cast<uint2*>(t + (size_t)m * ldt + n) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
}
}  // namespace

bool tb_lora_t_ok(int M, int N, int K, int bm, int bn) {
  bool has = false;
#define RG_HAS_L(BM_, BN_) if (bm == BM_ && bn == BN_) has = true;
  RG_LMASK_TILES(RG_HAS_L)
#undef RG_HAS_L
  return has && M > 0 && N % bn == 0 && K >= 128 && K % 128 == 0;
}

int tb_lora_t_chunks(int K) { return K / (64 * lora_kct(K)); }

void tb_lora_t(const uint16_t* x, const uint16_t* a_all, uint16_t* t, const int32_t* adapter, int M, int N, int K,
               int nsr, int nr, int r, int bm, int bn, hipStream_t st, int ldt, float* part) {
  if (M <= 0) return;
  if (ldt <= 0) ldt = N;
  RingArgs ra{};
  ra.adapter = adapter;
  ra.nsr = nsr;
  ra.nr = nr;
  ra.r = r;
  ra.kct = lora_kct(K);
  ra.nch = part != nullptr ? tb_lora_t_chunks(K) : 0;
  ra.part = part;
  const int tiles = ((M + bm - 1) / bm) * (N / bn) * (ra.nch > 0 ? ra.nch : 1);
#define RG_CASE_L(BM_, BN_)                                                                                        \
  if (bm == BM_ && bn == BN_) {                                                                                    \
    static_assert(8 % rg_ku1(BM_, BN_) == 0 && 2 % rg_ku1(BM_, BN_) == 0, "chunk of whole stages");               \
    hipLaunchKernelGGL((gemm_ring_kernel<BM_, BN_, RG_LMASK, rg_ku1(BM_, BN_), RG_LKB1>), dim3(tiles), dim3(256),  \
                       0, st, x, a_all, t, M, N, K, ldt, ra);                                                        \
  }
  RG_LMASK_TILES(RG_CASE_L)
#undef RG_CASE_L
  if (part != nullptr) {
    const int ng = M * (N / 4);
    hipLaunchKernelGGL(lora_t_reduce_kernel, dim3((ng + 255) / 256), dim3(256), 0, st, part, t, adapter, M, N, ldt,
                       ra.nch, nsr, nr, r);
  }
}

bool tb_gemm_ring_ok(int M, int N, int K, int epi, int bm, int bn, int var) {
  if (M <= 0 || N <= 0 || K < 128 || K % 128 || var < 0 || var > 2 || !rg_has(epi, bm, bn) || N % bn) return false;
  if (var == 2 && (!rg_has_var2(bm, bn) || K % (64 * rg_ku2(bm, bn)))) return false;
  if ((size_t)N * K * 2 >= ((size_t)1 << 40)) return false;
  if (bn == 112 && var != 1) return false;   // the 112-column tiles are built with the 144 KB ring only
  if (epi == RG_ROPE) return N % 256 == 0;
  return true;
}

int tb_gemm_ring_tiles(int epi, int* bm, int* bn, int cap) {
  int n = 0;
#define RG_LIST(BM_, BN_) if (n < cap) { bm[n] = BM_; bn[n] = BN_; } ++n;
  if (epi == RG_BF16) {
    RG_PLAIN_TILES(RG_LIST)
    RG_N112_TILES(RG_LIST)
  } else {
    RG_PAIR_TILES(RG_LIST)
  }
#undef RG_LIST
  return n;
}

void tb_gemm_ring(const uint16_t* A, const uint16_t* W, uint16_t* C, int M, int N, int K, int ldc, int epi, int bm,
                  int bn, int var, hipStream_t st, const uint16_t* a2, int k0) {
  if (M <= 0) return;
  RingArgs ra{};
  ra.a2 = a2;
  ra.k0 = k0;
  if (epi == RG_GEGLU) rg_dispatch<RG_GEGLU>(bm, bn, var, A, W, C, M, N, K, ldc, ra, st);
  else rg_dispatch<RG_BF16>(bm, bn, var, A, W, C, M, N, K, ldc, ra, st);
}

void tb_gemm_ring_qkv_rope(const uint16_t* A, const uint16_t* W, const int32_t* pos, const int32_t* slot_of_row,
                           const uint16_t* cs, uint16_t* q_out, uint16_t* kc, uint16_t* vc, int M,
                           int K, int Hq, int Hkv, int S, int max_pos, int bm, int bn, int var, hipStream_t st,
                           const uint16_t* a2, int k0) {
  if (M <= 0) return;
  RingArgs ra{pos, slot_of_row, cs, q_out, kc, vc, Hq, Hkv, S, max_pos};
  ra.a2 = a2;
  ra.k0 = k0;
  rg_dispatch<RG_ROPE>(bm, bn, var, A, W, nullptr, M, (Hq + 2 * Hkv) * 256, K, 0, ra, st);
}
