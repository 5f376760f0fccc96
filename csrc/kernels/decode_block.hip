// Persistent post-attention decode block (TP = 1, decode batch <= 64, fragment-major activations), gfx950.
//
// ONE launch per layer runs, in order,
//   PO  o projection + residual   attn (xf) @ Wo: h += o; x = bf16(h) (xf); ss1[m] += sum h^2
//   PG  gate_up                   x @ Wgu, rows scaled by rsqrt(ss1 / d + eps), SiLU(gate) * up -> act (xf)
//   PD  down + residual           act @ Wd: h += y; x = bf16(h) (xf); ss2[m] += sum h^2
//   PQ  next qkv (optional)       x @ Wqkv, rows scaled by rsqrt(ss2 / d + eps) -> qout [B][nq] f32
// in place of six launches (o GEMM, add_rmsnorm, gate_up, down, add_rmsnorm, next qkv); the RMSNorm gammas are
// folded into Wgu / Wqkv at load time (models/llama.py), so a norm is a row scale in the consumer's epilogue.
//
// Why one launch: at decode batch <= 64 each projection is a 2-30 us weight stream that pays ~2-3 us of launch
// boundary, ramp-up and tail (profiles/roofline_b32_decode.md).  Here the weight stream runs through the seams:
//   * every work item is a group of NB 16-column n-blocks over the FULL k range (no split-K: o and down finish
//     their columns' residual in the epilogue, no slab round trip, no residual phase);
//   * workgroup i owns item i of every phase (no claim at a seam); the remaining items are claimed dynamically,
//     a workgroup claiming its NEXT item while computing the current one (the round trip hides behind the
//     k-loop) and issuing the next item's first weight chunks before the current item's epilogue;
//   * at a phase seam it issues its first item of the next phase's weights BEFORE it waits for the current phase
//     to complete (weights never depend on activations: MI355X_MICROARCH.md 'prefetch-credit');
//   * a workgroup publishes its phase work once (one add of its item count to its XCD's done slot), not per item.
//
// The grid is clamped to the co-resident capacity (occupancy x CUs), so every statically owned item belongs to a
// workgroup that is resident, or becomes resident as soon as another stream's kernels drain (they never wait on
// this one): no grid barrier, no deadlock.  Every wait is bounded: on timeout the kernel sets *err and returns.
//
// Hand-offs follow MI355X_MICROARCH.md 'Valid forms' row 1: every byte another workgroup reads inside the launch
// (h, the bf16 activations x / act) is stored write-through (sc1) and loaded with sc1 loads; each storing wave
// drains its stores (s_waitcnt vmcnt(0)), the workgroup barrier follows, then one lane adds to the phase's done
// counter (agent scope); a consumer polls that counter from one lane (relaxed agent loads, s_sleep between
// polls), then joins a workgroup barrier before any wave loads.  Claim and done counters sit on their own 128-B
// lines.  Row sums of squares are int64 Q24 agent-scope atomics (exact and order-independent, as in the
// residual GEMM epilogue: batched decoding stays bit-reproducible; every item reduces its k range in a fixed
// order whichever workgroup runs it).
#include "common.h"

#define DB_THREADS 512
#define DB_WAVES 8
#define DB_SC1 16   // buffer aux: sc1 (write-through store / L1-bypassing load)
#define DB_LINE 32  // ints per counter line (128 B)
#define DB_SLOTS 8  // done counters per phase: one per XCD (workgroup i runs on XCD i % 8)
// per-layer counter block, one 128-B line each: phase p's claim counter at line 9p, its done slots at lines
// 9p + 1 .. 9p + 8
#define DB_CNT_INTS (4 * (1 + DB_SLOTS) * DB_LINE)

namespace {

typedef __attribute__((address_space(1))) int db_g_i32;
typedef __attribute__((address_space(1))) long long db_g_i64;
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
};

__device__ __forceinline__ u32x4_t ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, DB_SC1);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ db_g_i32* claim_ctr(const DbArgs& a, int p) {
  return (db_g_i32*)a.cnt + p * (1 + DB_SLOTS) * DB_LINE;
}
__device__ __forceinline__ db_g_i32* done_ctr(const DbArgs& a, int p, int slot) {
  return (db_g_i32*)a.cnt + (p * (1 + DB_SLOTS) + 1 + slot) * DB_LINE;
}
// dynamic items start after the static ones: workgroup i owns item i of every phase, the rest are claimed
__device__ __forceinline__ int claim_issue(const DbArgs& a, int p) {
  return (int)gridDim.x + __hip_atomic_fetch_add(claim_ctr(a, p), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// end of phase p: every storing wave drains its write-through stores, then one lane adds the workgroup's item
// count to its XCD's done slot (8 slots: no 256-way same-address atomic storm at a seam)
__device__ __forceinline__ void publish(const DbArgs& a, int p, int ndone) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && ndone)
    __hip_atomic_fetch_add(done_ctr(a, p, blockIdx.x % DB_SLOTS), ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait until phase p has n items done (bounded); false on timeout (err set).  Lanes 0-7 of wave 0 poll one slot
// each; the sum is broadcast from lane 0 so the loop stays wave-uniform.
__device__ __forceinline__ bool wait_done(const DbArgs& a, int p, int n, int* s_flag) {
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    int ok = 1;
    const long long t0 = wall_clock64();
    while (true) {
      int v = l < DB_SLOTS ? __hip_atomic_load(done_ctr(a, p, l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (__shfl(v, 0, 64) >= n) break;
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > a.timeout_ticks) {
        if (l == 0) __hip_atomic_store((db_g_i32*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    if (l == 0) *s_flag = ok;
  }
  __syncthreads();
  return *s_flag != 0;
}

__device__ __forceinline__ void stamp(const DbArgs& a, int k, long long v = -1) {
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 16 + k] = v < 0 ? wall_clock64() : v;
}

__device__ __forceinline__ float row_scale(const long long* ss, int m, float inv_d, float eps) {
  const long long v = __hip_atomic_load((db_g_i64*)(ss + m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return rsqrtf((float)v * (1.0f / LSA_Q24) * inv_d + eps);
}

// ------------------------------------------------------------------------------------------------------------
// One GEMM work item: NB n-blocks (16 columns each) x all KB k-blocks.  Wave w owns the contiguous k-blocks
// [w KB / 8, (w + 1) KB / 8) (balanced to one k-block for any KB) and streams them in chunks of U k-blocks with a
// two-deep register pipeline.  load_w() issues the first two chunks' weights (the prefetch), run() continues.
// Chunks past the wave's range re-read its last k-block (an L2 hit) and are masked.
// (A D-deep register ring was measured slower: 7B b32 110 -> 123 us per block, scripts/bench_decode_block.py.)
// ------------------------------------------------------------------------------------------------------------
template <int MT, int NB, int U>
struct GemmItem {
  const uint4* wp[NB];
  int kb0, kb1, n_it;
  uint4 wA[U][NB], wB[U][NB];

  __device__ __forceinline__ void setup(const uint4* W, int KB, int nb0, int w, int lane) {
#pragma unroll
    for (int i = 0; i < NB; ++i) wp[i] = W + (size_t)(nb0 + i) * KB * 64 + lane;
    kb0 = (w * KB) / DB_WAVES;
    kb1 = ((w + 1) * KB) / DB_WAVES;
    n_it = (kb1 - kb0 + U - 1) / U;
  }
  __device__ __forceinline__ int kblk(int c, int u) const { return min(kb0 + c * U + u, kb1 - 1); }
  __device__ __forceinline__ void wload(uint4 (&wr)[U][NB], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = kblk(c, u);
#pragma unroll
      for (int i = 0; i < NB; ++i) wr[u][i] = ldg_nt(wp[i] + (size_t)kk * 64);
    }
  }
  __device__ __forceinline__ void load_w(int) {
    if (n_it > 0) wload(wA, 0);
    if (n_it > 1) wload(wB, 1);
  }
  // activations: xf layout, sc1 loads (handed off inside the launch)
  __device__ __forceinline__ void xload(uint4 (&xr)[U][MT], __amdgpu_buffer_rsrc_t xr_rs, int c, int lane) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = kblk(c, u);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const u32x4_t v = ld_sc1(xr_rs, (uint32_t)((((size_t)kk * MT + j) * 64 + lane) * 16));
        xr[u][j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  __device__ __forceinline__ void comp(f32x4_t (&acc)[NB][MT], const uint4 (&wr)[U][NB], const uint4 (&xr)[U][MT], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = kb0 + c * U + u < kb1;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        uint4 xv = xr[u][j];
        xv.x = live ? xv.x : 0u; xv.y = live ? xv.y : 0u; xv.z = live ? xv.z : 0u; xv.w = live ? xv.w : 0u;
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i][j] = mfma16x16x32(wr[u][i], xv, acc[i][j]);
      }
    }
  }
  __device__ __forceinline__ void run(f32x4_t (&acc)[NB][MT], __amdgpu_buffer_rsrc_t xr_rs, int, int lane) {
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (n_it <= 0) return;
    uint4 xA[U][MT], xB[U][MT];
    xload(xA, xr_rs, 0, lane);
    int i = 0;
    for (; i + 1 < n_it; i += 2) {
      xload(xB, xr_rs, i + 1, lane);
      __builtin_amdgcn_sched_barrier(0);
      comp(acc, wA, xA, i);
      __builtin_amdgcn_sched_barrier(0);
      const int c2 = min(i + 2, n_it - 1);  // clamped: the tail re-reads a cached chunk
      wload(wA, c2);
      xload(xA, xr_rs, c2, lane);
      __builtin_amdgcn_sched_barrier(0);
      comp(acc, wB, xB, i + 1);
      __builtin_amdgcn_sched_barrier(0);
      if (i + 3 < n_it) wload(wB, i + 3);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(acc, wA, xA, i);
  }
};

template <int NB, int MT>
__device__ __forceinline__ f32x4_t lds_sum(const f32x4_t* red, int t, int l) {
  f32x4_t s = red[t * 64 + l];
#pragma unroll
  for (int ww = 1; ww < DB_WAVES; ++ww) s += red[(ww * NB * MT + t) * 64 + l];
  return s;
}

// One GEMM phase: run items until the claim counter is exhausted.  `item` is this workgroup's first item (its
// weights already issued by g.load_w); returns the number of items this workgroup completed.
template <int MT, int NB, int U, typename Epi>
__device__ __forceinline__ int gemm_phase(const DbArgs& a, int p, int n, const uint4* W, int KB,
                                          __amdgpu_buffer_rsrc_t xr, GemmItem<MT, NB, U>& g, int item,
                                          f32x4_t* red, int* s_item, int w, int lane, Epi epi) {
  int done = 0;
  while (item < n) {
    int tk = 0;
    if (threadIdx.x == 0) tk = claim_issue(a, p);  // next item: the round trip hides behind the k-loop
    f32x4_t acc[NB][MT];
    g.run(acc, xr, w, lane);
    __syncthreads();  // the previous item's epilogue is done reading red
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) red[((w * NB + i) * MT + j) * 64 + lane] = acc[i][j];
    if (threadIdx.x == 0) *s_item = tk;
    __syncthreads();
    const int nxt = *s_item;
    if (nxt < n) {  // the next item's weights stream while this one's epilogue runs
      g.setup(W, KB, nxt * NB, w, lane);
      g.load_w(w);
    }
    epi(item * NB, red);
    ++done;
    item = nxt;
  }
  return done;
}

// residual epilogue of o / down for n-blocks nb0 .. nb0 + NB - 1: h += y; x = bf16(h) (xf); ss[m] += sum h^2
template <int NB, int MT>
__device__ __forceinline__ void residual_epi(const DbArgs& a, const f32x4_t* red, int nb0, long long* ss) {
  const __amdgpu_buffer_rsrc_t rh = rsrc(a.h), rx = rsrc(a.x);
  for (int idx = threadIdx.x; idx < NB * MT * 64; idx += DB_THREADS) {
    const int l = idx & 63, t = idx >> 6;
    const int j = t % MT, i = t / MT;
    const int m = j * 16 + (l & 15);
    const int n = (nb0 + i) * 16 + 4 * (l >> 4);
    float hs = 0.f;
    if (m < a.B) {
      const f32x4_t s = lds_sum<NB, MT>(red, t, l);
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

// k-blocks per chunk for MT row tiles x NB n-blocks: as deep as the VGPRs allow without spilling (two chunks of
// weights + two of activations per wave; one workgroup per CU leaves 256 VGPRs per wave)
constexpr int db_chunk(int mt, int nb) {
  return nb == 1 ? (mt == 1 ? 8 : (mt == 2 ? 6 : 4)) : (nb == 2 ? (mt == 4 ? 2 : 4) : (mt == 4 ? 1 : 2));
}

}  // namespace

// NBx: n-blocks per work item of each phase (NBG counts gate + up blocks: even); MT: 16-row tiles (B <= 16 MT)
template <int MT, int NBO, int NBG, int NBD, int NBQ>
__global__ __launch_bounds__(DB_THREADS) void decode_block_kernel(DbArgs a) {
  constexpr int NBMAX = (NBO > NBG ? NBO : NBG) > (NBD > NBQ ? NBD : NBQ) ? (NBO > NBG ? NBO : NBG) : (NBD > NBQ ? NBD : NBQ);
  constexpr int UO = db_chunk(MT, NBO), UG = db_chunk(MT, NBG), UD = db_chunk(MT, NBD), UQ = db_chunk(MT, NBQ);
  __shared__ __attribute__((aligned(16))) f32x4_t red[DB_WAVES * NBMAX * MT * 64];
  __shared__ int s_item, s_flag;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const float inv_d = 1.0f / (float)a.d;
  const int KBo = a.hd / 32, KBg = a.d / 32, KBd = a.ffn / 32, KBq = a.d / 32;
  const int nO = a.d / 16 / NBO, nG = (2 * a.ffn / 16) / NBG, nD = a.d / 16 / NBD;
  const int nQ = a.wq ? (a.nq / 16) / NBQ : 0;

  // ---------------- PO: o projection + residual (ss1)
  int ndone;
  stamp(a, 0);
  {
    GemmItem<MT, NBO, UO> g;
    const int it = blockIdx.x < nO ? (int)blockIdx.x : nO;
    stamp(a, 1);
    if (it < nO) {
      g.setup(a.wo, KBo, it * NBO, w, lane);
      g.load_w(w);
    }
    ndone = gemm_phase<MT, NBO, UO>(a, 0, nO, a.wo, KBo, rsrc(a.attn), g, it, red, &s_item, w, lane,
                                    [&](int nb0, const f32x4_t* r) { residual_epi<NBO, MT>(a, r, nb0, a.ss1); });
    stamp(a, 2);
    stamp(a, 9, ndone);
  }
  // ---------------- PG: gate_up (rows scaled by ss1, SiLU * up -> act); first item's weights before the seam
  {
    GemmItem<MT, NBG, UG> g;
    publish(a, 0, ndone);
    const int it = blockIdx.x < nG ? (int)blockIdx.x : nG;
    if (it < nG) {
      g.setup(a.wgu, KBg, it * NBG, w, lane);
      g.load_w(w);
    }
    if (!wait_done(a, 0, nO, &s_flag)) return;
    stamp(a, 3);
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.act);
    ndone = gemm_phase<MT, NBG, UG>(a, 1, nG, a.wgu, KBg, rsrc(a.x), g, it, red, &s_item, w, lane,
                                    [&](int nb0, const f32x4_t* r) {
      for (int idx = threadIdx.x; idx < (NBG / 2) * MT * 64; idx += DB_THREADS) {
        const int l = idx & 63, t = idx >> 6;
        const int j = t % MT, pr = t / MT;
        const int m = j * 16 + (l & 15);
        if (m >= a.B) continue;
        const f32x4_t gs = lds_sum<NBG, MT>(r, (2 * pr) * MT + j, l);
        const f32x4_t us = lds_sum<NBG, MT>(r, (2 * pr + 1) * MT + j, l);
        const float sc = row_scale(a.ss1, m, inv_d, a.eps);
        const int n = ((nb0 + 2 * pr) >> 1) * 16 + 4 * (l >> 4);
        const u32x2_t pk = {pack2bf(silu(gs[0] * sc) * (us[0] * sc), silu(gs[1] * sc) * (us[1] * sc)),
                            pack2bf(silu(gs[2] * sc) * (us[2] * sc), silu(gs[3] * sc) * (us[3] * sc))};
        __builtin_amdgcn_raw_buffer_store_b64(pk, ra, (int)(xf_off(m, n, MT) * 2), 0, DB_SC1);
      }
    });
    stamp(a, 4);
    stamp(a, 10, ndone);
  }
  // ---------------- PD: down + residual (ss2)
  {
    GemmItem<MT, NBD, UD> g;
    publish(a, 1, ndone);
    const int it = blockIdx.x < nD ? (int)blockIdx.x : nD;
    if (it < nD) {
      g.setup(a.wd, KBd, it * NBD, w, lane);
      g.load_w(w);
    }
    if (!wait_done(a, 1, nG, &s_flag)) return;
    stamp(a, 5);
    ndone = gemm_phase<MT, NBD, UD>(a, 2, nD, a.wd, KBd, rsrc(a.act), g, it, red, &s_item, w, lane,
                                    [&](int nb0, const f32x4_t* r) { residual_epi<NBD, MT>(a, r, nb0, a.ss2); });
    stamp(a, 6);
    stamp(a, 11, ndone);
  }
  if (!nQ) return;
  // ---------------- PQ: next layer's qkv (rows scaled by ss2) -> f32 [B][nq] for the fused-RoPE attention
  {
    GemmItem<MT, NBQ, UQ> g;
    publish(a, 2, ndone);
    const int it = blockIdx.x < nQ ? (int)blockIdx.x : nQ;
    if (it < nQ) {
      g.setup(a.wq, KBq, it * NBQ, w, lane);
      g.load_w(w);
    }
    if (!wait_done(a, 2, nD, &s_flag)) return;
    stamp(a, 7);
    const __amdgpu_buffer_rsrc_t rq = rsrc(a.qout);
    ndone = gemm_phase<MT, NBQ, UQ>(a, 3, nQ, a.wq, KBq, rsrc(a.x), g, it, red, &s_item, w, lane,
                            [&](int nb0, const f32x4_t* r) {
      for (int idx = threadIdx.x; idx < NBQ * MT * 64; idx += DB_THREADS) {
        const int l = idx & 63, t = idx >> 6;
        const int j = t % MT, i = t / MT;
        const int m = j * 16 + (l & 15);
        if (m >= a.B) continue;
        const f32x4_t s = lds_sum<NBQ, MT>(r, t, l) * row_scale(a.ss2, m, inv_d, a.eps);
        const int n = (nb0 + i) * 16 + 4 * (l >> 4);
        const u32x4_t u = {__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])};
        __builtin_amdgcn_raw_buffer_store_b128(u, rq, (int)(((size_t)m * a.nq + n) * 4), 0, 0);
      }
    });
    stamp(a, 8);
    stamp(a, 12, ndone);
  }
}

extern "C" int lsa_decode_block_cnt_ints() { return DB_CNT_INTS; }

// co-resident workgroups of a kernel on this device: occupancy per CU x CUs
static int db_capacity(const void* kernel) {
  int per_cu = 0, dev = 0, ncu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, DB_THREADS, 0) != hipSuccess) per_cu = 1;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 1;
  return (per_cu > 0 ? per_cu : 1) * (ncu > 0 ? ncu : 1);
}

extern "C" int lsa_decode_block(const void* attn, const void* wo, float* h, void* x, long long* ss1, long long* ss2,
                                const void* wgu, void* act, const void* wd, const void* wq, float* qout, int B, int d,
                                int hd, int ffn, int nq, float eps, int* cnt, int* err, long long timeout_ticks,
                                int nwg, int nbo, int nbg, int nbd, int nbq, long long* stamps, hipStream_t s) {
  if (B < 1 || B > 64 || d % 32 || hd % 32 || ffn % 32 || (wq && nq % 16) || nwg < 1) return -1;
  if ((d / 16) % nbo || (2 * ffn / 16) % nbg || nbg % 2 || (d / 16) % nbd || (wq && (nq / 16) % nbq)) return -3;
  const int mt = B <= 16 ? 1 : (B <= 32 ? 2 : 4);
  DbArgs a{reinterpret_cast<const uint16_t*>(attn), reinterpret_cast<const uint4*>(wo), h,
           reinterpret_cast<uint16_t*>(x), ss1, ss2, reinterpret_cast<const uint4*>(wgu),
           reinterpret_cast<uint16_t*>(act), reinterpret_cast<const uint4*>(wd), reinterpret_cast<const uint4*>(wq),
           qout, B, d, hd, ffn, nq, eps, cnt, err, timeout_ticks, stamps};
#define DB_L(MTV, O, G, D_, Q)                                                                              \
  if (mt == MTV && nbo == O && nbg == G && nbd == D_ && nbq == Q) {                                          \
    static const int cap = db_capacity(reinterpret_cast<const void*>(decode_block_kernel<MTV, O, G, D_, Q>)); \
    hipLaunchKernelGGL((decode_block_kernel<MTV, O, G, D_, Q>), dim3(nwg < cap ? nwg : cap), dim3(DB_THREADS), \
                       0, s, a);                                                                            \
    return (int)hipGetLastError();                                                                          \
  }
#define DB_MT(MTV) DB_L(MTV, 1, 2, 1, 1) DB_L(MTV, 1, 2, 1, 2) DB_L(MTV, 2, 2, 2, 2) DB_L(MTV, 1, 4, 1, 1)
  DB_MT(1) DB_MT(2) DB_MT(4)
#undef DB_MT
#undef DB_L
  return -4;
}
