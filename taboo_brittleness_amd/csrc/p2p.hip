// One-shot peer-to-peer all-reduce over xGMI for tensor parallelism.
//
// TP moves 2 x [M, 3584] bf16 per Gemma-2 block (≈7 KB per token): small, latency-bound
// messages.  A ring all-reduce pays 2(N-1) dependent hops, each bound by ONE xGMI link; on the
// MI355X's point-to-point fabric every GPU has a direct link to each of its 7 peers, so a one-shot
// reduce — every rank reads all N inputs straight out of the peers' HBM (N-1 links in parallel)
// and sums locally — finishes in one hop.
//
// Per rank, one IPC-exported region (fine-grained, uncached: peers read it over the fabric and the
// data changes every call, so no GPU caches a stale line of it):
//
//   [ start flags  TB_P2P_MAXB x TB_P2P_MAXR u32 ]  start[b][src] : set by rank src's block b
//   [ end flags    TB_P2P_MAXB x TB_P2P_MAXR u32 ]
//   [ counters     TB_P2P_MAXB u32               ]  call counter of this rank's block b (local)
//   [ error word   u32, padding to 4 KB          ]
//   [ data         max_bytes                     ]  this rank's staged input
//
// A call (all ranks launch the same grid for the same numel):
//   1. each block copies its share of the input into the rank's own data area (in-kernel: no extra
//      launch, and the flag release below orders these stores);
//   2. block b of every rank bumps its counter to f and stores f into start[b][rank] of every peer
//      (system-scope release), then waits until start[b][src] == f for every src (system-scope
//      acquire) — all inputs are staged;
//   3. block b sums its grid-stride share of 16-byte vectors over ranks 0..N-1 IN RANK ORDER in fp32
//      and rounds once, so every rank produces bit-identical output (TP replicas stay in lockstep);
//   4. end barrier (same protocol on end[][]): no rank returns — and so no rank can restage its
//      data area for the next call — while a peer may still be reading it.
// Counters live in device memory, so the launch is graph-capturable (no per-call kernel argument).
// Every wait is bounded (spin_max polls): a missing peer sets the error word and the grid drains
// instead of hanging the GPU.
#include <cstring>

#include "common.h"

#define TB_P2P_MAXB 128
#define TB_P2P_MAXR 8
#define TB_P2P_START 0
#define TB_P2P_END (TB_P2P_MAXB * TB_P2P_MAXR)
#define TB_P2P_CTR (2 * TB_P2P_MAXB * TB_P2P_MAXR)
#define TB_P2P_ERR (TB_P2P_CTR + TB_P2P_MAXB)
#define TB_P2P_HDR 16384   // bytes before the data area (>= (TB_P2P_ERR + 1) * 4, 4 KB aligned)

static_assert((TB_P2P_ERR + 1) * 4 <= TB_P2P_HDR, "p2p header overflow");

struct P2PBases {
  char* p[TB_P2P_MAXR];
};

__device__ __forceinline__ uint32_t ld_acq_sys(uint32_t* a) {
  return __hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_rel_sys(uint32_t* a, uint32_t v) {
  __hip_atomic_store(a, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Streaming 16-byte load of a peer's staged data (read once per call: no cache allocation).
__device__ __forceinline__ uint4 ld_nt16(const u32x4* p) {
  const u32x4 v = __builtin_nontemporal_load(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Block-level barrier across ranks on flag area `slot` (START or END).  Lanes 0..world-1 of wave 0
// each signal one peer and wait for one peer.
__device__ __forceinline__ void p2p_barrier(const P2PBases& B, int rank, int world, int slot, uint32_t f,
                                            int spin_max) {
  const int t = threadIdx.x;
  if (t < world) {
    uint32_t* peer = reinterpret_cast<uint32_t*>(B.p[t]);
    uint32_t* mine = reinterpret_cast<uint32_t*>(B.p[rank]);
    st_rel_sys(peer + slot + blockIdx.x * TB_P2P_MAXR + rank, f);
    uint32_t* w = mine + slot + blockIdx.x * TB_P2P_MAXR + t;
    int n = 0;
    while (ld_acq_sys(w) != f) {
      __builtin_amdgcn_s_sleep(2);
      if (++n >= spin_max) {
        __hip_atomic_fetch_or(mine + TB_P2P_ERR, 1u << t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
}

template <bool BF16>
__global__ void __launch_bounds__(512) p2p_allreduce_kernel(P2PBases B, const void* in, void* out, int64_t nvec,
                                                            int rank, int world, int spin_max, int barriers) {
  __shared__ uint32_t s_flag;
  uint32_t* mine = reinterpret_cast<uint32_t*>(B.p[rank]);
  if (threadIdx.x == 0) {
    const uint32_t f = __hip_atomic_load(mine + TB_P2P_CTR + blockIdx.x, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_flag = f;
  }
  __syncthreads();
  const uint32_t f = s_flag;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int per = BF16 ? 1 : 2;    // 16-byte vectors per 8-element iteration index
  // stage this block's share of the input in the own region: block b of every rank stages and later
  // reads exactly the same indices, so block b's barrier orders exactly the data it reads
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(in);
    u32x4* dst = reinterpret_cast<u32x4*>(B.p[rank] + TB_P2P_HDR);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride)
      for (int k = 0; k < per; ++k) dst[per * i + k] = src[per * i + k];
  }
  __syncthreads();
  if (barriers) p2p_barrier(B, rank, world, TB_P2P_START, f, spin_max);
  // system-scope acquire in every wave: drop any line of a staging area this GPU's caches hold from
  // an earlier call (or an earlier allocation at the same address) before reading the new data
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int r = 0; r < world; ++r) {      // fixed rank order: bit-identical result on every rank
      const u32x4* src = reinterpret_cast<const u32x4*>(B.p[r] + TB_P2P_HDR);
      if (BF16) {
        const uint4 v = ld_nt16(src + i);
        float x[8];
        unpack8(v, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[j];
      } else {
        // fp32: one 16-byte vector = 4 floats; two vectors per iteration index
        const uint4 v0 = ld_nt16(src + 2 * i);
        const uint4 v1 = ld_nt16(src + 2 * i + 1);
        acc[0] += __uint_as_float(v0.x); acc[1] += __uint_as_float(v0.y);
        acc[2] += __uint_as_float(v0.z); acc[3] += __uint_as_float(v0.w);
        acc[4] += __uint_as_float(v1.x); acc[5] += __uint_as_float(v1.y);
        acc[6] += __uint_as_float(v1.z); acc[7] += __uint_as_float(v1.w);
      }
    }
    if (BF16) {
      reinterpret_cast<uint4*>(out)[i] = pack8(acc);
    } else {
      float4* o = reinterpret_cast<float4*>(out);
      o[2 * i] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      o[2 * i + 1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
  }
  __syncthreads();
  if (barriers) p2p_barrier(B, rank, world, TB_P2P_END, f, spin_max);
  if (threadIdx.x == 0)
    __hip_atomic_store(mine + TB_P2P_CTR + blockIdx.x, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// All-gather (raw 16-byte vectors of any dtype): the same stage / barrier / read / barrier protocol, each rank's
// staged input copied to out[r] in rank order -- a real gather, not a sum of zero-padded slots.  TP's
// vocab-parallel head and lens exchange a few floats per row through it (csrc/vp.hip merges them).
__global__ void __launch_bounds__(512) p2p_allgather_kernel(P2PBases B, const u32x4* in, u32x4* out, int64_t nvec,
                                                            int rank, int world, int spin_max, int barriers) {
  __shared__ uint32_t s_flag;
  uint32_t* mine = reinterpret_cast<uint32_t*>(B.p[rank]);
  if (threadIdx.x == 0) {
    const uint32_t f = __hip_atomic_load(mine + TB_P2P_CTR + blockIdx.x, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_flag = f;
  }
  __syncthreads();
  const uint32_t f = s_flag;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  {
    u32x4* dst = reinterpret_cast<u32x4*>(B.p[rank] + TB_P2P_HDR);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) dst[i] = in[i];
  }
  __syncthreads();
  if (barriers) p2p_barrier(B, rank, world, TB_P2P_START, f, spin_max);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  for (int r = 0; r < world; ++r) {
    const u32x4* src = reinterpret_cast<const u32x4*>(B.p[r] + TB_P2P_HDR);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
      const uint4 v = ld_nt16(src + i);
      out[(int64_t)r * nvec + i] = (u32x4){v.x, v.y, v.z, v.w};
    }
  }
  __syncthreads();
  if (barriers) p2p_barrier(B, rank, world, TB_P2P_END, f, spin_max);
  if (threadIdx.x == 0)
    __hip_atomic_store(mine + TB_P2P_CTR + blockIdx.x, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- host side

int tb_p2p_header_bytes() { return TB_P2P_HDR; }
int tb_p2p_max_ranks() { return TB_P2P_MAXR; }

void* tb_p2p_alloc(size_t bytes, int uncached) {
  void* p = nullptr;
  hipError_t e = uncached ? hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) : hipMalloc(&p, bytes);
  if (e != hipSuccess) return nullptr;
  if (hipMemset(p, 0, bytes) != hipSuccess) return nullptr;
  if (hipDeviceSynchronize() != hipSuccess) return nullptr;
  return p;
}

int tb_p2p_free(void* p) { return (int)hipFree(p); }

int tb_p2p_get_handle(void* p, void* handle_out /* sizeof(hipIpcMemHandle_t) bytes */) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

int tb_p2p_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

void* tb_p2p_open_handle(const void* handle) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  return p;
}

int tb_p2p_close_handle(void* p) { return (int)hipIpcCloseMemHandle(p); }

// Reduce `nbytes` of `in` (bf16 or fp32, 16-byte multiple) across `world` ranks into `out`.
// bases[r] = rank r's region as mapped in this process (bases[rank] = own allocation).
int tb_p2p_allreduce(void* const* bases, int rank, int world, const void* in, void* out, size_t nbytes, int is_bf16,
                     int blocks, int spin_max, int barriers, hipStream_t st) {
  if (world < 1 || world > TB_P2P_MAXR || blocks < 1 || blocks > TB_P2P_MAXB || (nbytes % (is_bf16 ? 16 : 32)))
    return -1;
  P2PBases B;
  for (int r = 0; r < TB_P2P_MAXR; ++r) B.p[r] = r < world ? reinterpret_cast<char*>(bases[r]) : nullptr;
  const int64_t nvec = (int64_t)(nbytes / 16) / (is_bf16 ? 1 : 2);
  const int threads = 256;
  if (is_bf16)
    hipLaunchKernelGGL(p2p_allreduce_kernel<true>, dim3(blocks), dim3(threads), 0, st, B, in, out, nvec, rank, world,
                       spin_max, barriers);
  else
    hipLaunchKernelGGL(p2p_allreduce_kernel<false>, dim3(blocks), dim3(threads), 0, st, B, in, out, nvec, rank, world,
                       spin_max, barriers);
  return (int)hipGetLastError();
}

// Gather `nbytes` (16-byte multiple) of `in` from `world` ranks into out[world * nbytes], rank order.
int tb_p2p_allgather(void* const* bases, int rank, int world, const void* in, void* out, size_t nbytes, int blocks,
                     int spin_max, int barriers, hipStream_t st) {
  if (world < 1 || world > TB_P2P_MAXR || blocks < 1 || blocks > TB_P2P_MAXB || (nbytes % 16)) return -1;
  P2PBases B;
  for (int r = 0; r < TB_P2P_MAXR; ++r) B.p[r] = r < world ? reinterpret_cast<char*>(bases[r]) : nullptr;
  hipLaunchKernelGGL(p2p_allgather_kernel, dim3(blocks), dim3(256), 0, st, B, reinterpret_cast<const u32x4*>(in),
                     reinterpret_cast<u32x4*>(out), (int64_t)(nbytes / 16), rank, world, spin_max, barriers);
  return (int)hipGetLastError();
}

// Error word of this rank's region (bit r = timed out waiting for rank r); cleared when read.
uint32_t tb_p2p_read_error(void* own_base) {
  uint32_t v = 0;
  uint32_t* w = reinterpret_cast<uint32_t*>(own_base) + TB_P2P_ERR;
  const uint32_t z = 0;
  if (hipMemcpy(&v, w, 4, hipMemcpyDeviceToHost) != hipSuccess) return 0xFFFFFFFFu;
  if (hipMemcpy(w, &z, 4, hipMemcpyHostToDevice) != hipSuccess) return 0xFFFFFFFFu;
  return v;
}
