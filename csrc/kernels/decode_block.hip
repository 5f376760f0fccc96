// Persistent post-attention decode block on an LDS-DMA weight ring (TP = 1, decode batch <= 64,
// fragment-major activations), gfx950.
//
// ONE launch per layer runs, in order,
//   PO  o projection + residual   attn (xf) @ Wo: h += o; x = bf16(h) (xf); ss1[m] += sum h^2
//   PG  gate_up                   x @ Wgu, rows scaled by rsqrt(ss1 / d + eps), SiLU(gate) * up -> act (xf)
//   PD  down + residual           act @ Wd: h += y; x = bf16(h) (xf); ss2[m] += sum h^2
//   PQ  next qkv (optional)       x @ Wqkv, rows scaled by rsqrt(ss2 / d + eps) -> qout [B][nq] f32
// in place of six launches (o GEMM, add_rmsnorm, gate_up, down, add_rmsnorm, next qkv); the RMSNorm gammas are
// folded into Wgu / Wqkv at load time (models/llama.py), so a norm is a row scale in the consumer's epilogue.
//
// Engine (MI355X_MICROARCH.md price list: ldsdma-fill, prefetch-credit, ring-gemm; one workgroup per CU):
//   * ONE loader wave per CU streams this CU's weights for ALL four phases, in consumption order, into a ring of
//     DB_RING 16 KiB LDS slots with global_load_lds (nt: read once per step), DB_INFLIGHT slots in flight, and
//     publishes a slot (an LDS FULL word) behind a counted vmcnt.  Weights never depend on activations, so the
//     loader never waits for a phase hand-off: while this CU's consumers wait for the previous phase to complete
//     on every CU, its loader keeps filling the ring with the next phase's weights (the seam is hidden behind the
//     ring's ~5 us of stream).  It only waits for ring slots its consumers have not released yet (FREE words).
//   * C consumer waves split every slot's k-blocks (wave c takes k-blocks c, c + C, ..): per k-block one
//     ds_read_b128 per n-block, then the slot is released, then MT MFMA 16x16x32 per n-block against the
//     activation fragments the wave prefetched from L2 (sc1 loads) one slot ahead.  Partial sums of the C waves
//     meet in LDS at the end of each work item for the epilogue.
//   * Work is assigned statically: workgroup i owns items i, i + grid, .. of every phase (an item = NB 16-column
//     n-blocks over the full k range), so loader and consumers walk the same schedule with no claims.
//   * Phase hand-off (MI355X_MICROARCH.md 'Valid forms' row 1): every byte another workgroup reads inside the
//     launch (h, the bf16 activations x / act) is stored write-through (sc1) and loaded with sc1 loads; each
//     consumer wave drains its stores (s_waitcnt vmcnt(0)) and adds to an LDS counter, the wave whose add is last
//     adds the workgroup's item count to its XCD's done slot (agent scope); consumer wave 0 polls the 8 slots
//     (relaxed agent loads, s_sleep between polls) and then sets an LDS word the other consumer waves wait for.
//   * No __syncthreads after the prologue (the loader runs ahead of every consumer barrier): consumer waves meet
//     through LDS counters.  The loader's own LDS traffic is inline asm, so the compiler never drains its
//     LDS-DMA queue (vmcnt(0)) in front of a flag access.
// The grid is clamped to the co-resident capacity (occupancy x CUs), so every statically owned item belongs to a
// workgroup that is resident, or becomes resident as soon as another stream's kernels drain (they never wait on
// this one): no grid barrier, no deadlock.  Every wait is bounded: on timeout the kernel sets *err, raises an LDS
// abort word that releases the other waves, and returns.  Row sums of squares are int64 Q24 agent-scope atomics
// (exact and order-independent: batched decoding stays bit-reproducible; every item reduces its k range in a
// fixed order whichever workgroup runs it).
//
// Measured on MI355X (profiles/r3/decode_block_ring_mi355x.jsonl, scripts/bench_decode_block.py --stamps): 7B per
// block 86.8 us at batch 1 and 105 us at batch 32 (the register-streaming v2 with dynamic claims: 98 / 111 us), i.e.
// still slower than the launch chain it replaces (bench 7B b32 7,089 vs 8,103 tok/s), so it stays opt-in
// (LSA_DECODE_BLOCK=1).  The stamps say why: every in-launch phase hand-off costs 4-6 us after the last
// producer's item (store drain ~2 us under the weight stream + counter + poll), more than the ring's ~4.5 us of
// prefetch credit, and gate_up's 688 items leave a third of the CUs one item (~10 us) short; a kernel boundary
// costs ~1.7 us.  Pausing the loader during the poll did not shorten the hand-off (86.8 vs 87.6 us).
#include "common.h"

#ifndef DB_RING
#define DB_RING 7       // 16 KiB weight slots (the guide: >= 3 more than the slots in flight)
#endif
#ifndef DB_HOLD
#define DB_HOLD 1       // pause the loader while consumer wave 0 polls a phase hand-off
#endif
#define DB_INFLIGHT 3   // slots the loader keeps in flight: 48 LDS-DMA ops <= the 63 vmcnt can count
#define DB_SC1 16       // buffer aux: sc1 (write-through store / L1-bypassing load)
#define DB_NT 2         // LDS-DMA aux: nt (weights streamed once per step)
#define DB_LINE 32      // ints per counter line (128 B)
#define DB_SLOTS 8      // done counters per phase: one per XCD (workgroup i runs on XCD i % 8)
// per-layer counter block, one 128-B line each: phase p's done slots at lines 9p + 1 .. 9p + 8 (line 9p unused)
#define DB_CNT_INTS (4 * (1 + DB_SLOTS) * DB_LINE)

namespace {

typedef __attribute__((address_space(1))) int db_g_i32;
typedef __attribute__((address_space(1))) long long db_g_i64;
typedef __attribute__((address_space(3))) void* db_lds_t;
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

struct DbArgs {
  const uint16_t* attn;  // xf [HD / 32][MT][64][8]
  const uint4* wo;       // fragment-major [d / 16][HD / 32][64]
  float* h;              // [B][d]
  uint16_t* x;           // xf [d / 32][MT][64][8]
  long long* ss1;        // [B] Q24
  long long* ss2;        // [B] Q24
  const uint4* wgu;      // [2 ffn / 16][d / 32][64], gate / up n-blocks interleaved
  uint16_t* act;         // xf [ffn / 32][MT][64][8]
  const uint4* wd;       // [d / 16][ffn / 32][64]
  const uint4* wq;       // [nq / 16][d / 32][64] (nullptr: no next-layer projection)
  float* qout;           // [B][nq]
  int B, d, hd, ffn, nq;
  float eps;
  int* cnt;              // DB_CNT_INTS, zeroed before the launch
  int* err;
  long long timeout_ticks;
  long long* stamps;     // optional [nwg][16] wall-clock stamps of the phase boundaries (scripts/bench_decode_block.py)
  int mode;              // 0: the whole block; 1: PO alone = one residual GEMM h += X @ W (lsa_res_gemm)
};

// LDS control words (zeroed in the prologue)
struct DbCtl {
  int full[DB_RING];   // slot r holds its (full[r])-th use: the loader's publication
  int free_[DB_RING];  // consumer releases of slot r (C per use)
  int cb;              // consumer barrier arrivals (2 per consumer wave per work item)
  int pub;             // consumer waves done with their phase's stores
  int ready;           // phases handed off (set by consumer wave 0 after its poll)
  int hold;            // consumer wave 0 polls a hand-off: the loader keeps its DMA queue empty meanwhile
  int abort;           // a bounded wait timed out: every wave returns
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(db_lds_t)p; }
// LDS flag accesses as inline asm: invisible to the waitcnt pass, so no vmcnt(0) drain of the LDS-DMA queue
__device__ __forceinline__ int lds_ld(const int* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_inc1(int* p, int lane) {  // one lane adds 1
  if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(lds_addr(p)), "v"(1) : "memory");
}

// one 1 KiB wave-instruction of LDS-DMA (16 B per lane, nt); a non-template wrapper (the builtin inside a
// template trips hipcc's host pass)
__device__ __forceinline__ void glds_nt(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (db_lds_t)l, 16, 0, DB_NT);
}

__device__ __forceinline__ u32x4_t ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, DB_SC1);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ db_g_i32* done_ctr(const DbArgs& a, int p, int slot) {
  return (db_g_i32*)a.cnt + (p * (1 + DB_SLOTS) + 1 + slot) * DB_LINE;
}

// bounded LDS spin until *p >= v; false (abort raised, err set) on timeout or when another wave aborted
__device__ __forceinline__ bool spin_ge(const DbArgs& a, DbCtl* ctl, const int* p, int v) {
  if (lds_ld(p) >= v) return true;
  const long long t0 = wall_clock64();
  while (true) {
    __builtin_amdgcn_s_sleep(1);
    if (lds_ld(p) >= v) return true;
    if (lds_ld(&ctl->abort)) return false;
    if (wall_clock64() - t0 > a.timeout_ticks) {
      __hip_atomic_store((db_g_i32*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lds_st(&ctl->abort, 1);
      return false;
    }
  }
}

// bounded LDS spin until *p == 0
__device__ __forceinline__ bool spin_le0(const DbArgs& a, DbCtl* ctl, const int* p) {
  const long long t0 = wall_clock64();
  while (lds_ld(p) > 0) {
    __builtin_amdgcn_s_sleep(1);
    if (lds_ld(&ctl->abort)) return false;
    if (wall_clock64() - t0 > a.timeout_ticks) {
      __hip_atomic_store((db_g_i32*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lds_st(&ctl->abort, 1);
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ void stamp(const DbArgs& a, int k, long long v = -1) {
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 16 + k] = v < 0 ? wall_clock64() : v;
}

__device__ __forceinline__ float row_scale(const long long* ss, int m, float inv_d, float eps) {
  const long long v = __hip_atomic_load((db_g_i64*)(ss + m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return rsqrtf((float)v * (1.0f / LSA_Q24) * inv_d + eps);
}

// ------------------------------------------------------------------------------------------------------------
// Loader: this workgroup's items of one phase, slot by slot.  Slot = NB n-blocks x KS = 16 / NB k-blocks, 16
// fragments of 1 KiB in [n-block][k-block] order; k-blocks past KB re-read the last one (an L2 hit; the
// consumers mask them).  q counts slots over the whole launch, pub the published ones.
// (Measured and not kept, scripts/bench_decode_block.py, 7B batch 1: one flat schedule over all phases with
// division-free cursors 87.6 -> 102.7 us per block; the same plus 4-byte "touch" reads of the next 8 slots into
// L2 / Infinity Cache while the ring is full 110.9 us -- the touches queue in front of the hand-off polls.)
// ------------------------------------------------------------------------------------------------------------
template <int NB, int C>
__device__ __forceinline__ bool db_load_phase(const DbArgs& a, DbCtl* ctl, uint4* ring, const uint4* W, int KB,
                                              int n_items, int& q, int& pub, int lane) {
  constexpr int KS = 16 / NB;
  const int nsl = (KB + KS - 1) / KS;
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    const uint4* wi[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) wi[i] = W + (size_t)(item * NB + i) * KB * 64 + lane;
    for (int s = 0; s < nsl; ++s, ++q) {
      const int r = q % DB_RING;
      if (q - pub >= DB_INFLIGHT) {  // the oldest slot in flight has landed once <= DB_INFLIGHT - 1 remain
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        lds_st(&ctl->full[pub % DB_RING], pub / DB_RING + 1);
        ++pub;
      }
      if (q >= DB_RING) {
        const int need = (q / DB_RING) * C;  // every consumer released the slot's previous use
        if (lds_ld(&ctl->free_[r]) < need) {
          // the consumers are behind: publish everything in flight, then wait for the slot
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          for (; pub < q; ++pub) lds_st(&ctl->full[pub % DB_RING], pub / DB_RING + 1);
          if (!spin_ge(a, ctl, &ctl->free_[r], need)) return false;
        }
      }
#if DB_HOLD
      if (lds_ld(&ctl->hold)) {
        // a hand-off poll is in flight on this CU: its loads (and the activation loads right after it) would
        // queue behind this wave's LDS-DMA (MI355X_MICROARCH.md gather-pass / handoff-1to1), so drain and pause
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (; pub < q; ++pub) lds_st(&ctl->full[pub % DB_RING], pub / DB_RING + 1);
        if (!spin_le0(a, ctl, &ctl->hold)) return false;
      }
#endif
      uint4* dst = ring + r * 1024;
#pragma unroll
      for (int f = 0; f < 16; ++f) {
        const int i = f / KS, kk = f % KS;
        const int kb = min(s * KS + kk, KB - 1);
        glds_nt(wi[i] + (size_t)kb * 64, dst + f * 64);
      }
    }
  }
  return true;
}

// ------------------------------------------------------------------------------------------------------------
// Consumers: this workgroup's items of one phase.  Wave c (of C) reads fragments (i, c + C kw) of every slot
// (KW = KS / C k-blocks x NB n-blocks), prefetches the next slot's activation fragments (sc1, L2) one slot ahead,
// and at the end of an item the C partial accumulators meet in LDS (red) for the epilogue epi(nb0, red).
// e counts items over the launch (consumer-barrier generations).  Returns false on abort.
// ------------------------------------------------------------------------------------------------------------
template <int MT, int NB, int C, typename Epi>
__device__ __forceinline__ bool db_consume_phase(const DbArgs& a, DbCtl* ctl, const uint4* ring, f32x4_t* red,
                                                 const void* xin, int KB, int n_items, int& q, int& e, int& ndone,
                                                 int c, int lane, Epi epi) {
  constexpr int KS = 16 / NB, KW = KS / C;
  static_assert(KW >= 1 && KS % C == 0, "a slot's k-blocks split evenly over the consumer waves");
  const int nsl = (KB + KS - 1) / KS;
  const __amdgpu_buffer_rsrc_t rx = rsrc(xin);
  auto xload = [&](uint4 (&xr)[KW][MT], int s) {
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) {
      const int kb = min(s * KS + kw * C + c, KB - 1);  // masked at use (a select here would wait for the load)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const u32x4_t v = ld_sc1(rx, (uint32_t)((((size_t)kb * MT + j) * 64 + lane) * 16));
        xr[kw][j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto step = [&](f32x4_t (&acc)[NB][MT], const uint4 (&xr)[KW][MT], int s) -> bool {
    const int r = q % DB_RING;
    if (!spin_ge(a, ctl, &ctl->full[r], q / DB_RING + 1)) return false;
    const uint4* slot = ring + r * 1024;
    uint4 w[NB][KW];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) w[i][kw] = slot[(i * KS + kw * C + c) * 64 + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_inc1(&ctl->free_[r], lane);  // the slot's fragments are in registers: the loader may refill it
    ++q;
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) {
      const bool live = s * KS + kw * C + c < KB;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        uint4 xv = xr[kw][j];
        xv.x = live ? xv.x : 0u; xv.y = live ? xv.y : 0u; xv.z = live ? xv.z : 0u; xv.w = live ? xv.w : 0u;
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i][j] = mfma16x16x32(w[i][kw], xv, acc[i][j]);
      }
    }
    return true;
  };

  uint4 xa[KW][MT], xb[KW][MT];
  bool first = true;
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    f32x4_t acc[NB][MT];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (first) xload(xa, 0);
    first = false;
    const bool more = item + (int)gridDim.x < n_items;  // the next item starts at slot 0 (the same k-blocks)
    int s = 0;
    for (; s + 1 < nsl; s += 2) {
      xload(xb, s + 1);
      if (!step(acc, xa, s)) return false;
      if (s + 2 < nsl || more) xload(xa, s + 2 < nsl ? s + 2 : 0);
      if (!step(acc, xb, s + 1)) return false;
    }
    if (s < nsl) {  // odd slot count: the tail runs from xa, the next item's first slot lands in xb
      if (more) xload(xb, 0);
      if (!step(acc, xa, s)) return false;
#pragma unroll
      for (int kw = 0; kw < KW; ++kw)
#pragma unroll
        for (int j = 0; j < MT; ++j) xa[kw][j] = xb[kw][j];
    }
    // partial sums -> LDS once every consumer is done reading the previous item's (barrier generation 2e)
    if (e > 0 && !spin_ge(a, ctl, &ctl->cb, 2 * C * e)) return false;
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) red[((c * NB + i) * MT + j) * 64 + lane] = acc[i][j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_inc1(&ctl->cb, lane);
    if (!spin_ge(a, ctl, &ctl->cb, 2 * C * e + C)) return false;
    epi(item * NB, red);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_inc1(&ctl->cb, lane);
    ++e;
    ++ndone;
  }
  return true;
}

template <int NB, int MT, int C>
__device__ __forceinline__ f32x4_t lds_sum(const f32x4_t* red, int t, int l) {
  f32x4_t s = red[t * 64 + l];
#pragma unroll
  for (int ww = 1; ww < C; ++ww) s += red[(ww * NB * MT + t) * 64 + l];
  return s;
}

// residual epilogue of o / down for n-blocks nb0 .. nb0 + NB - 1: h += y; x = bf16(h) (xf); ss[m] += sum h^2
template <int NB, int MT, int C>
__device__ __forceinline__ void residual_epi(const DbArgs& a, const f32x4_t* red, int nb0, long long* ss) {
  const __amdgpu_buffer_rsrc_t rh = rsrc(a.h), rx = rsrc(a.x);
  for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * C) {
    const int l = idx & 63, t = idx >> 6;
    const int j = t % MT, i = t / MT;
    const int m = j * 16 + (l & 15);
    const int n = (nb0 + i) * 16 + 4 * (l >> 4);
    float hs = 0.f;
    if (m < a.B) {
      const f32x4_t s = lds_sum<NB, MT, C>(red, t, l);
      const uint32_t ho = (uint32_t)(((size_t)m * a.d + n) * 4);
      const u32x4_t hv = ld_sc1(rh, ho);
      const float v0 = __uint_as_float(hv[0]) + s[0], v1 = __uint_as_float(hv[1]) + s[1];
      const float v2 = __uint_as_float(hv[2]) + s[2], v3 = __uint_as_float(hv[3]) + s[3];
      const u32x4_t hn = {__float_as_uint(v0), __float_as_uint(v1), __float_as_uint(v2), __float_as_uint(v3)};
      __builtin_amdgcn_raw_buffer_store_b128(hn, rh, ho, 0, DB_SC1);
      const u32x2_t xb = {pack2bf(v0, v1), pack2bf(v2, v3)};
      __builtin_amdgcn_raw_buffer_store_b64(xb, rx, (int)(xf_off(m, n, MT) * 2), 0, DB_SC1);
      hs = v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
    }
    // the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 hold the same row's 16 columns of this n-block
    hs += __shfl_xor(hs, 16, 64);
    hs += __shfl_xor(hs, 32, 64);
    if (m < a.B && l < 16)
      __hip_atomic_fetch_add((db_g_i64*)(ss + m), ss_to_q24(hs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// end of phase p: every consumer wave drains its write-through stores, adds to the LDS counter; the wave whose add
// is last adds the workgroup's item count to its XCD's done slot (8 slots: no 256-way same-address storm)
template <int C>
__device__ __forceinline__ void publish(const DbArgs& a, DbCtl* ctl, int p, int ndone, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (p == 0) stamp(a, 13);  // wave 0's stores of the o phase drained
  if (lane == 0) {
    const int old = __hip_atomic_fetch_add(&ctl->pub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (old == C * (p + 1) - 1 && ndone)
      __hip_atomic_fetch_add(done_ctr(a, p, blockIdx.x % DB_SLOTS), ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// wait until phase p has n items done on every CU: consumer wave 0 polls the 8 slots (lanes 0-7, the sum
// broadcast from lane 0 so the loop stays wave-uniform), then sets ready; the other consumer waves wait for it
__device__ __forceinline__ bool wait_phase(const DbArgs& a, DbCtl* ctl, int p, int n, int c, int lane) {
  if (c != 0) return spin_ge(a, ctl, &ctl->ready, p + 1);
  if (DB_HOLD) lds_st(&ctl->hold, 1);
  const long long t0 = wall_clock64();
  while (true) {
    int v = lane < DB_SLOTS ? __hip_atomic_load(done_ctr(a, p, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    if (__shfl(v, 0, 64) >= n) break;
    if (lds_ld(&ctl->abort)) return false;
    if (wall_clock64() - t0 > a.timeout_ticks) {
      if (lane == 0) __hip_atomic_store((db_g_i32*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lds_st(&ctl->abort, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  lds_st(&ctl->ready, p + 1);
  if (DB_HOLD) lds_st(&ctl->hold, 0);
  return true;
}

}  // namespace

// NBx: n-blocks per work item of each phase (NBG counts gate + up blocks: even); MT: 16-row tiles (B <= 16 MT);
// C: consumer waves (+ 1 loader wave)
template <int MT, int NBO, int NBG, int NBD, int NBQ, int C>
__global__ __launch_bounds__(64 * (C + 1)) void decode_block_kernel(DbArgs a) {
  constexpr int NBMAX = (NBO > NBG ? NBO : NBG) > (NBD > NBQ ? NBD : NBQ) ? (NBO > NBG ? NBO : NBG) : (NBD > NBQ ? NBD : NBQ);
  constexpr int RED = C * NBMAX * MT * 64;  // f32x4 partial sums of one item
  // ONE __shared__ object: ring | red | control words
  __shared__ __attribute__((aligned(16))) uint4 smem[DB_RING * 1024 + RED + 8];
  static_assert(sizeof(DbCtl) <= 8 * 16, "control words");
  uint4* ring = smem;
  f32x4_t* red = reinterpret_cast<f32x4_t*>(smem + DB_RING * 1024);
  DbCtl* ctl = reinterpret_cast<DbCtl*>(smem + DB_RING * 1024 + RED);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  stamp(a, 0);
  if (threadIdx.x < sizeof(DbCtl) / 4) reinterpret_cast<int*>(ctl)[threadIdx.x] = 0;
  __syncthreads();  // the only workgroup barrier: the loader runs ahead of the consumers from here on
  stamp(a, 1);
  const float inv_d = 1.0f / (float)a.d;
  const int KBo = a.hd / 32, KBg = a.d / 32, KBd = a.ffn / 32, KBq = a.d / 32;
  const int nO = a.d / 16 / NBO, nG = (2 * a.ffn / 16) / NBG, nD = a.d / 16 / NBD;
  const int nQ = a.wq ? (a.nq / 16) / NBQ : 0;

  if (wv == C) {  // ---------------- the loader wave: the whole launch's weight stream
    int q = 0, pub = 0;
    const bool ok = db_load_phase<NBO, C>(a, ctl, ring, a.wo, KBo, nO, q, pub, lane) && (a.mode == 1 ||
                    db_load_phase<NBG, C>(a, ctl, ring, a.wgu, KBg, nG, q, pub, lane) &&
                    db_load_phase<NBD, C>(a, ctl, ring, a.wd, KBd, nD, q, pub, lane) &&
                    (nQ == 0 || db_load_phase<NBQ, C>(a, ctl, ring, a.wq, KBq, nQ, q, pub, lane)));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the wave
    if (ok)
      for (; pub < q; ++pub) lds_st(&ctl->full[pub % DB_RING], pub / DB_RING + 1);
    return;
  }

  // ---------------- consumer waves
  const int c = wv;
  int q = 0, e = 0, nd = 0;
  // PO: o projection + residual (ss1)
  if (!db_consume_phase<MT, NBO, C>(a, ctl, ring, red, a.attn, KBo, nO, q, e, nd, c, lane,
                                    [&](int nb0, const f32x4_t* r) { residual_epi<NBO, MT, C>(a, r, nb0, a.ss1); }))
    return;
  stamp(a, 2);
  stamp(a, 9, nd);
  if (a.mode == 1) return;
  publish<C>(a, ctl, 0, nd, lane);
  if (!wait_phase(a, ctl, 0, nO, c, lane)) return;
  stamp(a, 3);
  // PG: gate_up (rows scaled by ss1, SiLU * up -> act)
  nd = 0;
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.act);
  if (!db_consume_phase<MT, NBG, C>(a, ctl, ring, red, a.x, KBg, nG, q, e, nd, c, lane,
                                    [&](int nb0, const f32x4_t* r) {
    for (int idx = threadIdx.x; idx < (NBG / 2) * MT * 64; idx += 64 * C) {
      const int l = idx & 63, t = idx >> 6;
      const int j = t % MT, pr = t / MT;
      const int m = j * 16 + (l & 15);
      if (m >= a.B) continue;
      const f32x4_t gs = lds_sum<NBG, MT, C>(r, (2 * pr) * MT + j, l);
      const f32x4_t us = lds_sum<NBG, MT, C>(r, (2 * pr + 1) * MT + j, l);
      const float sc = row_scale(a.ss1, m, inv_d, a.eps);
      const int n = ((nb0 + 2 * pr) >> 1) * 16 + 4 * (l >> 4);
      const u32x2_t pk = {pack2bf(silu(gs[0] * sc) * (us[0] * sc), silu(gs[1] * sc) * (us[1] * sc)),
                          pack2bf(silu(gs[2] * sc) * (us[2] * sc), silu(gs[3] * sc) * (us[3] * sc))};
      __builtin_amdgcn_raw_buffer_store_b64(pk, ra, (int)(xf_off(m, n, MT) * 2), 0, DB_SC1);
    }
  }))
    return;
  stamp(a, 4);
  stamp(a, 10, nd);
  publish<C>(a, ctl, 1, nd, lane);
  if (!wait_phase(a, ctl, 1, nG, c, lane)) return;
  stamp(a, 5);
  // PD: down + residual (ss2)
  nd = 0;
  if (!db_consume_phase<MT, NBD, C>(a, ctl, ring, red, a.act, KBd, nD, q, e, nd, c, lane,
                                    [&](int nb0, const f32x4_t* r) { residual_epi<NBD, MT, C>(a, r, nb0, a.ss2); }))
    return;
  stamp(a, 6);
  stamp(a, 11, nd);
  if (!nQ) return;
  publish<C>(a, ctl, 2, nd, lane);
  if (!wait_phase(a, ctl, 2, nD, c, lane)) return;
  stamp(a, 7);
  // PQ: next layer's qkv (rows scaled by ss2) -> f32 [B][nq] for the fused-RoPE attention
  nd = 0;
  const __amdgpu_buffer_rsrc_t rq = rsrc(a.qout);
  if (!db_consume_phase<MT, NBQ, C>(a, ctl, ring, red, a.x, KBq, nQ, q, e, nd, c, lane,
                                    [&](int nb0, const f32x4_t* r) {
    for (int idx = threadIdx.x; idx < NBQ * MT * 64; idx += 64 * C) {
      const int l = idx & 63, t = idx >> 6;
      const int j = t % MT, i = t / MT;
      const int m = j * 16 + (l & 15);
      if (m >= a.B) continue;
      const f32x4_t s = lds_sum<NBQ, MT, C>(r, t, l) * row_scale(a.ss2, m, inv_d, a.eps);
      const int n = (nb0 + i) * 16 + 4 * (l >> 4);
      const u32x4_t u = {__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])};
      __builtin_amdgcn_raw_buffer_store_b128(u, rq, (int)(((size_t)m * a.nq + n) * 4), 0, 0);
    }
  }))
    return;
  stamp(a, 8);
  stamp(a, 12, nd);
}

extern "C" int lsa_decode_block_cnt_ints() { return DB_CNT_INTS; }

// co-resident workgroups of a kernel on this device: occupancy per CU x CUs
static int db_capacity(const void* kernel, int threads) {
  int per_cu = 0, dev = 0, ncu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess) per_cu = 1;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 1;
  return (per_cu > 0 ? per_cu : 1) * (ncu > 0 ? ncu : 1);
}

static int db_launch(const DbArgs& a, int nwg, int nbo, int nbg, int nbd, int nbq, int cw, hipStream_t s);

extern "C" int lsa_decode_block(const void* attn, const void* wo, float* h, void* x, long long* ss1, long long* ss2,
                                const void* wgu, void* act, const void* wd, const void* wq, float* qout, int B, int d,
                                int hd, int ffn, int nq, float eps, int* cnt, int* err, long long timeout_ticks,
                                int nwg, int nbo, int nbg, int nbd, int nbq, int cw, long long* stamps, hipStream_t s) {
  if (B < 1 || B > 64 || d % 32 || hd % 32 || ffn % 32 || (wq && nq % 16) || nwg < 1) return -1;
  if ((d / 16) % nbo || (2 * ffn / 16) % nbg || nbg % 2 || (d / 16) % nbd || (wq && (nq / 16) % nbq)) return -3;
  DbArgs a{reinterpret_cast<const uint16_t*>(attn), reinterpret_cast<const uint4*>(wo), h,
           reinterpret_cast<uint16_t*>(x), ss1, ss2, reinterpret_cast<const uint4*>(wgu),
           reinterpret_cast<uint16_t*>(act), reinterpret_cast<const uint4*>(wd), reinterpret_cast<const uint4*>(wq),
           qout, B, d, hd, ffn, nq, eps, cnt, err, timeout_ticks, stamps, 0};
  return db_launch(a, nwg, nbo, nbg, nbd, nbq, cw, s);
}

// One residual GEMM on the ring engine (the block's PO phase alone): h[B][N] += X @ W^T, xout = bf16(h)
// (fragment-major, MT row tiles), ss[m] += sum_n h^2 (Q24) -- no split-K slabs, no arrival tickets, no norm
// launch: every workgroup owns whole 16-column n-blocks over the full K, streamed by its loader wave.
// X: fragment-major [K / 32][MT][64][8] bf16; W: fragment-major [N / 16][K / 32][64].
extern "C" int lsa_res_gemm(const void* X, const void* W, float* h, void* xout, long long* ss, int B, int N, int K,
                            int* err, long long timeout_ticks, int nwg, int cw, long long* stamps, hipStream_t s) {
  if (B < 1 || B > 64 || N % 16 || K % 32 || nwg < 1) return -1;
  DbArgs a{reinterpret_cast<const uint16_t*>(X), reinterpret_cast<const uint4*>(W), h,
           reinterpret_cast<uint16_t*>(xout), ss, ss, reinterpret_cast<const uint4*>(W),
           reinterpret_cast<uint16_t*>(xout), reinterpret_cast<const uint4*>(W), nullptr,
           nullptr, B, N, K, 32, 0, 0.f, nullptr, err, timeout_ticks, stamps, 1};
  return db_launch(a, nwg, 1, 2, 1, 1, cw, s);
}

static int db_launch(const DbArgs& a, int nwg, int nbo, int nbg, int nbd, int nbq, int cw, hipStream_t s) {
  const int mt = a.B <= 16 ? 1 : (a.B <= 32 ? 2 : 4);
#define DB_L(MTV, O, G, D_, Q, CW)                                                                                \
  if (mt == MTV && nbo == O && nbg == G && nbd == D_ && nbq == Q && cw == CW) {                                     \
    static const int cap = db_capacity(reinterpret_cast<const void*>(decode_block_kernel<MTV, O, G, D_, Q, CW>), \
                                       64 * (CW + 1));                                                            \
    hipLaunchKernelGGL((decode_block_kernel<MTV, O, G, D_, Q, CW>), dim3(nwg < cap ? nwg : cap),                 \
                       dim3(64 * (CW + 1)), 0, s, a);                                                             \
    return (int)hipGetLastError();                                                                                \
  }
  DB_L(1, 1, 2, 1, 1, 4) DB_L(2, 1, 2, 1, 1, 4) DB_L(4, 1, 2, 1, 1, 4)
  DB_L(1, 1, 2, 1, 1, 8) DB_L(2, 1, 2, 1, 1, 8)
#undef DB_L
  return -4;
}
