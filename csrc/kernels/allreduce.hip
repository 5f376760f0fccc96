// One-shot tensor-parallel all-reduce (and all-gather) over IPC-mapped peer buffers.
//
// Decode-size TP all-reduces (B x d f32 = 16 KiB .. 512 KiB, 2 per layer) are latency-bound on
// xGMI: a generic ring pays n-1 dependent hops plus a collective launch.  Here every rank PUSHES its
// whole tensor straight into a receive slot of every peer (one xGMI link per peer on the MI355X
// mesh, all links at once), raises one flag per (block, source) in the peer's signal area, waits for
// the peers' flags of the same block, then sums the slots locally in rank order (bitwise identical
// results on every rank, so TP replicas never diverge in argmax).
//
// Region layout (one hipExtMallocWithFlags(hipDeviceMallocUncached) allocation per rank, opened by
// the peers with hipIpcOpenMemHandle):
//   [0,      8 KiB)  flags[AR_MAX_BLOCKS][AR_MAX_WORLD]  u32, written by peers (epoch numbers)
//   [8 KiB, 9 KiB)   epoch[AR_MAX_BLOCKS]                u32, this rank's per-block call counter
//   [9 KiB, +4)      abort                               u32, set by ANY rank whose wait timed out
//   [16 KiB, ...)    recv[2 parities][world][maxb]       pushed payloads
//   then             res[2 parities][maxb]               two-shot: the owners' reduced chunks (all-gather phase)
//
// Payload (round 5): f32, or bf16 (each rank rounds its contribution to bf16 -- its own copy too -- and the sums run
// in f32 in rank order, so every rank still gets bitwise the same result): half the xGMI bytes per all-reduce.
// Two-shot (round 5, TP >= 4 or large messages): reduce-scatter + all-gather -- every rank pushes each peer only the
// chunk that peer owns, the owner sums it and pushes the sum to every peer: (W - 1) / W of the tensor per link-hop
// pair instead of the whole tensor to each of W - 1 peers, at the price of a second flag round.
// Uncached memory keeps remote pushes coherent with the receiver's reads (no stale L2 lines of a slot
// from two calls ago).  The epoch lives on the device, so the launch has fixed arguments and replays
// inside a captured hipGraph.  Protocol invariants (per block b):
//   * a peer can be at most one epoch ahead (it needs our flag to finish), so flags are compared
//     with (int)(flag - target) >= 0 and payload slots alternate by epoch parity; the flag targets of epoch ep are
//     2 ep (one-shot) and 2 ep - 1, 2 ep (two-shot's two phases): one monotonic sequence whatever the mix of calls;
//   * pushing into parity p at epoch ep is safe: reaching ep means the peer raised ep-1, which it
//     does only after finishing ep-2 (the previous user of parity p).
// Every wait is bounded by a wall-clock timeout that sets *err and drains the grid, so a missing
// peer can never leave waves spinning on the GPU.  A rank that times out also raises the abort word in
// every peer's region; every later call on every rank reads its own abort word first and then poisons its
// result and sets its *err too, so the leader of a TP replica learns of a FOLLOWER's timeout at its next
// host sync (engine/runner.py read_rows) instead of committing tokens computed from the follower's NaNs.
#include "common.h"
#include <cstring>

#define AR_MAX_WORLD 8
#define AR_MAX_BLOCKS 256
#define AR_FLAGS_OFF 0
#define AR_EPOCH_OFF 8192
#define AR_ABORT_OFF 9216
#define AR_DATA_OFF 16384
#define AR_THREADS 256

__device__ __forceinline__ uint32_t ld_relaxed_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_release_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Residual epilogue of a row-parallel projection under TP (RES = 1, rows of D floats, D % 256 == 0): instead of
// writing the sum back, h[i] += sum; xn = bf16(h) (fragment-major with xmt row tiles, else row-major [rows][D]); and
// ss[row] += sum over the row of h^2 (Q24 int64 atomics, one per wave and 256 columns): the all-reduce, the residual
// add and the folded RMSNorm's row sums in ONE launch, so a TP decode layer issues as many launches as a TP = 1 one
// (engine/runner.py _reduce_add; the next GEMM scales its rows by rsqrt(ss / D + eps), gammas in its weights).
struct ArRes {
  float* h;
  uint16_t* xn;
  long long* ss;
  int D, xmt;
};

// GATHER = 0: sum into data (slab 0).  GATHER = 1: all-gather, out[p * n4 + i] = rank p's data[i].
// nslab > 1 (sum only): data holds nslab split-K partial slabs [nslab][n] (slab stride slab4 float4s,
// e.g. a row-parallel GEMM's f32 split-K output); each rank first sums its own slabs in slab order, so
// the split-K reduction rides along and the GEMM keeps its split-K parallelism under TP.
__device__ __forceinline__ uint2 pack4bf(const float4 v) { return make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w)); }
__device__ __forceinline__ float4 unpack4bf(const uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float4 round4bf(const float4 v) { return unpack4bf(pack4bf(v)); }

// payload slot access: f32 slots hold float4 per element, bf16 slots uint2 (same slot, half the bytes)
template <int BF16>
__device__ __forceinline__ void slot_put(uint8_t* slot, long i, const float4 v) {
  if constexpr (BF16) reinterpret_cast<uint2*>(slot)[i] = pack4bf(v);
  else reinterpret_cast<float4*>(slot)[i] = v;
}
template <int BF16>
__device__ __forceinline__ float4 slot_get(const uint8_t* slot, long i) {
  if constexpr (BF16) return unpack4bf(reinterpret_cast<const uint2*>(slot)[i]);
  else return reinterpret_cast<const float4*>(slot)[i];
}

// residual epilogue for element (float4) i of the reduced tensor: h += sum, xn = bf16(h), ss[row] += h^2 (the 64 lanes
// of a wave hold 256 consecutive columns of one row: D % 256 == 0, wave-aligned strides)
__device__ __forceinline__ void ar_res_epilogue(const ArRes& res, long i, const float4 acc) {
  float4* hp = reinterpret_cast<float4*>(res.h) + i;
  float4 hv = *hp;
  hv.x += acc.x; hv.y += acc.y; hv.z += acc.z; hv.w += acc.w;
  *hp = hv;
  const long e = i * 4;
  const int m = (int)(e / res.D), c = (int)(e - (long)m * res.D);
  uint2 pk;
  pk.x = pack2bf(hv.x, hv.y);
  pk.y = pack2bf(hv.z, hv.w);
  *reinterpret_cast<uint2*>(res.xn + (res.xmt ? xf_off(m, c, res.xmt) : (size_t)m * res.D + c)) = pk;
  // the row's wave sum on DPP / permlane (common.h), not __shfl_xor's ds_bpermute LDS round trips (whole wave active)
  const float sq = wave_sum(hv.x * hv.x + hv.y * hv.y + hv.z * hv.z + hv.w * hv.w);
  if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(res.ss) + m, (unsigned long long)ss_to_q24(sq));
}

template <int W, int GATHER, int RES, int BF16>
__global__ __launch_bounds__(AR_THREADS) void ar_oneshot_kernel(float4* __restrict__ data, const long n4,
                                                                 float4* __restrict__ out,
                                                                 uint8_t* const* __restrict__ regions, const int rank,
                                                                 const size_t maxb, const long long timeout_ticks,
                                                                 int* __restrict__ err, const int nslab,
                                                                 const long slab4, const ArRes res) {
  const int b = blockIdx.x, tid = threadIdx.x;
  uint8_t* mine = regions[rank];
  uint32_t* my_epoch = reinterpret_cast<uint32_t*>(mine + AR_EPOCH_OFF);
  __shared__ uint32_t s_ep;
  __shared__ int s_timeout;
  if (tid == 0) {
    s_ep = my_epoch[b] + 1u;
    // a peer (or this rank) timed out in an earlier call: the group is out of step for good
    s_timeout = ld_relaxed_sys(reinterpret_cast<const uint32_t*>(mine + AR_ABORT_OFF)) != 0u;
    if (s_timeout) atomicExch(err, 1);
  }
  __syncthreads();
  const uint32_t ep = s_ep;
  const size_t slot_off = AR_DATA_OFF + (size_t)(ep & 1u) * W * maxb;
  const long stride = (long)gridDim.x * AR_THREADS;

  auto own = [&](long i) {  // this rank's contribution: its slabs summed in slab order
    float4 v = data[i];
    for (int sl = 1; sl < nslab; ++sl) {
      const float4 u = data[(long)sl * slab4 + i];
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    return v;
  };
  // the group is already broken (an earlier call timed out somewhere): no push, no flag wait -- poison at once, so a
  // captured step's remaining ~2L all-reduces each cost a launch, not a full timeout
  if (s_timeout) goto poison;
  // 1. push this block's chunk into every peer's recv[parity][rank]
  for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
    const float4 v = own(i);
#pragma unroll
    for (int p = 0; p < W; ++p) {
      if (p == rank) continue;
      slot_put<BF16>(regions[p] + slot_off + (size_t)rank * maxb, i, v);
    }
  }
  __threadfence_system();  // this thread's pushes are visible system-wide before any flag below
  __syncthreads();

  // 2. raise our flag for block b at every peer, then wait for theirs
  // flag value 2 ep: the same sequence the two-shot kernel's final phase raises, so one-shot and two-shot calls can
  // alternate on one region (a flag left at 2 ep' by a two-shot call must not satisfy a later one-shot wait early)
  if (tid < W && tid != rank) {
    uint32_t* f = reinterpret_cast<uint32_t*>(regions[tid] + AR_FLAGS_OFF) + b * AR_MAX_WORLD + rank;
    st_release_sys(f, 2u * ep);
    const uint32_t* mf = reinterpret_cast<const uint32_t*>(mine + AR_FLAGS_OFF) + b * AR_MAX_WORLD + tid;
    const long long t0 = wall_clock64();
    while ((int)(ld_relaxed_sys(mf) - 2u * ep) < 0) {  // relaxed spin, one acquire fence after it
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > timeout_ticks) {
        atomicExch(err, 1);
        s_timeout = 1;
        for (int p = 0; p < W; ++p)  // tell every rank (this one included) that the group is broken
          st_release_sys(reinterpret_cast<uint32_t*>(regions[p] + AR_ABORT_OFF), 1u);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();

  if (s_timeout) {  // a peer never arrived: poison this block's result (NaN), never a silent partial sum
  poison:
    const float nan = __builtin_nanf("");
    const float4 nv = make_float4(nan, nan, nan, nan);
    for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
      if (GATHER) {
        for (int p = 0; p < W; ++p) out[(long)p * n4 + i] = nv;
      } else if (RES) {
        reinterpret_cast<float4*>(res.h)[i] = nv;  // the residual stream itself is poisoned: every later token NaN
      } else {
        data[i] = nv;
      }
    }
    if (tid == 0) my_epoch[b] = ep;
    return;
  }

  if (GATHER) {  // 3'. concatenate the slots in rank order
    for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
#pragma unroll
      for (int p = 0; p < W; ++p)
        out[(long)p * n4 + i] = (p == rank) ? data[i]
                                            : reinterpret_cast<const float4*>(mine + slot_off + (size_t)p * maxb)[i];
    }
    if (tid == 0) my_epoch[b] = ep;
    return;
  }
  // 3. rank-ordered sum of the local slots (own contribution read from data, rounded like the pushed copies)
  for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const float4 v = (p == rank) ? (BF16 ? round4bf(own(i)) : own(i))
                                   : slot_get<BF16>(mine + slot_off + (size_t)p * maxb, i);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if constexpr (RES) ar_res_epilogue(res, i, acc);
    else data[i] = acc;
  }
  if (tid == 0) my_epoch[b] = ep;
}

// Two-shot all-reduce (sum; RES as above).  Element (float4) i is owned by rank i / ch (ch a multiple of 64, so a
// wave's elements share one owner).  Phase 1 (reduce-scatter): every rank pushes each element it does not own into
// the owner's recv[parity][rank] slot and raises flag 2 ep - 1 at every peer; after every peer's phase-1 flag, the
// owner sums its elements in rank order (its own contribution rounded like the pushed copies), keeps the sum in data
// and pushes it into every peer's res[parity] area.  Phase 2 (all-gather): flag 2 ep at every peer; after every
// peer's phase-2 flag each rank reads the sums it does not own.  A peer can be at most one phase ahead of the
// slowest rank, so flags compare with (int)(flag - target) >= 0 and slots alternate by epoch parity as in one-shot.
template <int W, int RES, int BF16>
__global__ __launch_bounds__(AR_THREADS) void ar_twoshot_kernel(float4* __restrict__ data, const long n4,
                                                                 uint8_t* const* __restrict__ regions, const int rank,
                                                                 const size_t maxb, const long long timeout_ticks,
                                                                 int* __restrict__ err, const int nslab,
                                                                 const long slab4, const ArRes res) {
  const int b = blockIdx.x, tid = threadIdx.x;
  uint8_t* mine = regions[rank];
  uint32_t* my_epoch = reinterpret_cast<uint32_t*>(mine + AR_EPOCH_OFF);
  __shared__ uint32_t s_ep;
  __shared__ int s_timeout;
  if (tid == 0) {
    s_ep = my_epoch[b] + 1u;
    s_timeout = ld_relaxed_sys(reinterpret_cast<const uint32_t*>(mine + AR_ABORT_OFF)) != 0u;
    if (s_timeout) atomicExch(err, 1);
  }
  __syncthreads();
  const uint32_t ep = s_ep;
  const size_t slot_off = AR_DATA_OFF + (size_t)(ep & 1u) * W * maxb;
  const size_t res_off = AR_DATA_OFF + 2 * (size_t)W * maxb + (size_t)(ep & 1u) * maxb;
  const long stride = (long)gridDim.x * AR_THREADS;
  const long ch = ((n4 + W - 1) / W + 63) / 64 * 64;  // elements per owner, whole waves
  auto own = [&](long i) {
    float4 v = data[i];
    for (int sl = 1; sl < nslab; ++sl) {
      const float4 u = data[(long)sl * slab4 + i];
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    return v;
  };
  // raise `target` at every peer for this block, wait for theirs (bounded; a timeout breaks the group)
  auto exchange = [&](uint32_t target) {
    __threadfence_system();  // this thread's pushes are visible system-wide before any flag below
    __syncthreads();
    if (tid < W && tid != rank) {
      uint32_t* f = reinterpret_cast<uint32_t*>(regions[tid] + AR_FLAGS_OFF) + b * AR_MAX_WORLD + rank;
      st_release_sys(f, target);
      const uint32_t* mf = reinterpret_cast<const uint32_t*>(mine + AR_FLAGS_OFF) + b * AR_MAX_WORLD + tid;
      const long long t0 = wall_clock64();
      while ((int)(ld_relaxed_sys(mf) - target) < 0) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > timeout_ticks) {
          atomicExch(err, 1);
          s_timeout = 1;
          for (int p = 0; p < W; ++p) st_release_sys(reinterpret_cast<uint32_t*>(regions[p] + AR_ABORT_OFF), 1u);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
  };
  if (!s_timeout) {
    // phase 1: push the elements others own
    for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
      const int o = (int)(i / ch);
      if (o != rank) slot_put<BF16>(regions[o] + slot_off + (size_t)rank * maxb, i, own(i));
    }
    exchange(2u * ep - 1u);
  }
  if (!s_timeout) {
    // owner: rank-ordered sum of its elements, kept in data (slab 0) and pushed to every peer
    for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
      if ((int)(i / ch) != rank) continue;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const float4 v = (p == rank) ? (BF16 ? round4bf(own(i)) : own(i))
                                     : slot_get<BF16>(mine + slot_off + (size_t)p * maxb, i);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      if (BF16) acc = round4bf(acc);  // the peers receive the bf16 sum: use the same value here
      data[i] = acc;
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (p != rank) slot_put<BF16>(regions[p] + res_off, i, acc);
    }
    exchange(2u * ep);
  }
  if (s_timeout) {
    const float nan = __builtin_nanf("");
    const float4 nv = make_float4(nan, nan, nan, nan);
    for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
      if (RES) reinterpret_cast<float4*>(res.h)[i] = nv;
      else data[i] = nv;
    }
    if (tid == 0) my_epoch[b] = ep;
    return;
  }
  // phase 2 result: own elements from data, the others from the res area
  for (long i = (long)b * AR_THREADS + tid; i < n4; i += stride) {
    const float4 acc = (int)(i / ch) == rank ? data[i] : slot_get<BF16>(mine + res_off, i);
    if constexpr (RES) ar_res_epilogue(res, i, acc);
    else data[i] = acc;
  }
  if (tid == 0) my_epoch[b] = ep;
}

extern "C" {

int lsa_ar_alloc(size_t bytes, void** out) {
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, bytes);
  if (e != hipSuccess) return (int)e;
  e = hipDeviceSynchronize();
  *out = p;
  return (int)e;
}

int lsa_ar_free(void* p) { return (int)hipFree(p); }

int lsa_ar_handle(void* p, char* out64) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
  std::memcpy(out64, &h, 64);
  return 0;
}

int lsa_ar_open(const char* in64, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, in64, 64);
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int lsa_ar_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

int lsa_ar_max_world() { return AR_MAX_WORLD; }

// constant-rate clock read by wall_clock64() (s_memrealtime), in kHz, of the current device
int lsa_ar_wallclock_khz(int* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceGetAttribute(out, hipDeviceAttributeWallClockRate, dev);
}
int lsa_ar_header_bytes() { return AR_DATA_OFF; }

// data: n floats (n % 4 == 0, 16-B aligned), regions: device array of `world` region pointers;
// out == nullptr: in-place all-reduce; otherwise all-gather into out[world * n]
// res (nullable): the residual epilogue (ArRes above) instead of writing the sum back into data
// mode: bit 0 = bf16 payload (sums only), bit 1 = two-shot (sums only; the region must hold the res area:
// AR_DATA_OFF + (2 world + 2) maxb bytes)
int lsa_ar_run(float* data, long n, float* out, uint8_t* const* regions, int rank, int world, size_t maxb,
               int nblocks, long long timeout_ticks, int* err, int nslab, long slab_stride, const float* res_h,
               void* res_xn, long long* res_ss, int res_d, int res_xmt, int mode, hipStream_t s) {
  if (n % 4 || (size_t)n * 4 > maxb || world < 2 || world > AR_MAX_WORLD || rank < 0 || rank >= world) return -1;
  if (mode < 0 || mode > 3 || (mode && out)) return -3;
  if (nslab < 1 || (nslab > 1 && (out || slab_stride % 4 || slab_stride < n))) return -1;
  const bool rs = res_h != nullptr;
  if (rs && (out || !res_xn || !res_ss || res_d <= 0 || res_d % 256 || n % res_d)) return -2;
  const ArRes res{const_cast<float*>(res_h), reinterpret_cast<uint16_t*>(res_xn), res_ss, res_d, res_xmt};
  const long n4 = n / 4;
  long want = (n4 + AR_THREADS - 1) / AR_THREADS;
  int grid = (int)(want < nblocks ? want : nblocks);
  if (grid < 1) grid = 1;
  if (grid > AR_MAX_BLOCKS) grid = AR_MAX_BLOCKS;
#define AR_SUM(WV, RS, BF)                                                                                      \
  if (mode & 2)                                                                                                \
    hipLaunchKernelGGL((ar_twoshot_kernel<WV, RS, BF>), dim3(grid), dim3(AR_THREADS), 0, s,                    \
                       reinterpret_cast<float4*>(data), n4, regions, rank, maxb, timeout_ticks, err, nslab,    \
                       slab_stride / 4, res);                                                                  \
  else                                                                                                         \
    hipLaunchKernelGGL((ar_oneshot_kernel<WV, 0, RS, BF>), dim3(grid), dim3(AR_THREADS), 0, s,                 \
                       reinterpret_cast<float4*>(data), n4, nullptr, regions, rank, maxb, timeout_ticks, err, nslab, \
                       slab_stride / 4, res)
#define AR_LAUNCH(WV)                                                                                        \
  if (out)                                                                                                     \
    hipLaunchKernelGGL((ar_oneshot_kernel<WV, 1, 0, 0>), dim3(grid), dim3(AR_THREADS), 0, s,                   \
                       reinterpret_cast<float4*>(data), n4, reinterpret_cast<float4*>(out), regions, rank, maxb, \
                       timeout_ticks, err, 1, 0L, res);                                                        \
  else if (rs) {                                                                                               \
    if (mode & 1) AR_SUM(WV, 1, 1); else AR_SUM(WV, 1, 0);                                                      \
  } else {                                                                                                     \
    if (mode & 1) AR_SUM(WV, 0, 1); else AR_SUM(WV, 0, 0);                                                      \
  }
  switch (world) {
    case 2: AR_LAUNCH(2); break;
    case 3: AR_LAUNCH(3); break;
    case 4: AR_LAUNCH(4); break;
    case 5: AR_LAUNCH(5); break;
    case 6: AR_LAUNCH(6); break;
    case 7: AR_LAUNCH(7); break;
    case 8: AR_LAUNCH(8); break;
    default: return -1;
  }
#undef AR_LAUNCH
#undef AR_SUM
  return (int)hipGetLastError();
}

}  // extern "C"
