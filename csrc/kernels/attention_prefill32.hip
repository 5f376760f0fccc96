// Causal prefill attention on 32 x 32 x 16 bf16 MFMA tiles (paged KV cache, head_dim 128, packed
// variable-length sequences): 32 query rows per wave, 4 waves (128 rows) per workgroup, K / V tiles of 64
// keys staged through LDS by register staging (the next tile's loads in flight during this tile's MFMAs).
//
// Why 32-row waves: a 16-row wave (attn_prefill_kernel, attention.hip) reads every K / V fragment from LDS
// for 16 query rows only and is LDS-read bound (256 B/clk/CU at one wave per SIMD).  With 32 x 32 tiles
// every fragment read feeds twice the MFMA work: 32 KiB of LDS reads per 32 MFMAs of 32 cycles per wave
// and 64-key tile, half the LDS bandwidth at two waves per SIMD, so the loop is MFMA-paced.
//
//   S^T = K Q^T : A = K (32 keys x 16 dims, ds_read_b128 of a row-swizzled image), B = Q^T (registers)
//                 -> accumulator: column = query row (lane & 31), rows = keys in the registers
//   softmax     : per query row over its registers + one xor-32 exchange (online, exp2 domain)
//   O += P V    : P re-used from the S^T accumulator as the A operand with no lane movement
//                 (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand": element j
//                 of lane half h of k-step s is key 16 s + 8 (j >> 2) + 4 h + (j & 3)); B = V fragments
//                 gathered in that same key order with ds_read_b64_tr_b16 (a 16-lane group reads 4 key
//                 rows x 16 dims and lane i receives dim i's 4 keys) from an XOR-swizzled V image.
#include "common.h"

#define LSA_NEG_P (-1.0e30f)
#ifndef LSA_P32_NBUF1
#define LSA_P32_NBUF1 2  // K / V tile buffers of the single-group (NG = 1) kernel: the DMA runs NBUF - 1 tiles
                         // ahead.  4 (128 KiB, 3 tiles ahead) measured slower: one workgroup per CU instead of two
                         // (3B 2k single 86.5 -> 127.7 us, 4 x 1k 78.3 -> 109.2; profiles/attn_prefill_nbuf_ab_mi355x.jsonl)
#endif

typedef short s16x4p_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4p_t* lds_s4p_ptr;
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x2p_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_u16_ptr;

namespace {

__device__ __forceinline__ uint2 ds_read_tr16p(const uint16_t* p) {
  s16x4p_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p_ptr)(p));
  return __builtin_bit_cast(uint2, v);
}

// LDS-DMA of 16 B per lane into [lds_base + 16 * lane] (lds_base wave-uniform, in M0).  Inline asm on purpose:
// with the builtin, hipcc cannot tell the DMA's destination buffer from the one the MFMAs are reading and
// puts a vmcnt(0) in front of every LDS read, i.e. it serialises the prefetch with the tile it should hide
// under.  The kernel counts these loads itself (s_waitcnt before the barrier that publishes a tile).
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}
// the same DMA from a wave-uniform base (SGPR pair) + a 32-bit per-lane byte offset (saddr form): no 64-bit
// per-lane address arithmetic on the tile loop's VALU
__device__ __forceinline__ void dma16s(const void* gbase, unsigned voff, unsigned lds_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(gbase), "s"(lds_base)
               : "memory");
}

// wait until at most k later tiles' DMAs (8 wave-instructions each: 4 K + 4 V rows groups) are in flight (k is
// wave-uniform; vmcnt counts this wave's vector-memory instructions in issue order), and for this wave's LDS reads
// The builtin (not inline asm), so hipcc's own wait tracking sees it.  simm16 on gfx9: vmcnt[3:0] bits 3:0,
// expcnt bits 6:4 (7 = no wait), lgkmcnt bits 11:8, vmcnt[5:4] bits 15:14.
__device__ __forceinline__ void wait_dma_tiles(int k) {
  if (k <= 0) __builtin_amdgcn_s_waitcnt(0x0070);       // vmcnt(0) lgkmcnt(0)
  else if (k == 1) __builtin_amdgcn_s_waitcnt(0x0078);  // vmcnt(8) lgkmcnt(0)
  else __builtin_amdgcn_s_waitcnt(0x4070);              // vmcnt(16) lgkmcnt(0)
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(lds_u16_ptr)(p);
}

__device__ __forceinline__ f32x16_t mfma32x32x16(const uint4 a, const uint4 b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// K image: 16 B chunk ch of key row r at chunk (ch ^ (r & 15)): the 32 rows x one chunk of a K fragment read
// land in 16 distinct chunk slots per ds_read_b128 lane group (conflict-free)
__device__ __forceinline__ int kp_off(int r, int ch) { return r * 128 + ((ch ^ (r & 15)) << 3); }
// V image: chunk c of row r at chunk (c ^ ((r & 3) << 2)): the 4 rows x 64 B a half-wave's transposed read
// touches fall in 4 disjoint 64 B bank ranges
__device__ __forceinline__ int vp_off(int r, int col) { return r * 128 + ((((col >> 3) ^ ((r & 3) << 2))) << 3) + (col & 7); }

}  // namespace

// NG independent 4-wave groups per workgroup (NG = 2: the host pairs a heavy causal query block with a
// light one, ops.prefill_work, so every workgroup streams about the same number of key tiles; one pair
// per CU instead of two heavy blocks landing on the same CU).  Each group has its own K / V image and its
// own tile count; the groups only share the workgroup barriers (an idle group keeps passing them).
//
// Work item of a group: (seq, q_start, t0, t1) -- the key tiles [t0, t1) of one 128-row query block (the
// whole causal range: t0 = 0; cutting heavy blocks into KV splits with a merge launch, or into two halves
// merged in LDS, were both measured slower and removed: profiles/attn_prefill_kv_split_mi355x.jsonl,
// profiles/attn_prefill_halves_mi355x.jsonl; round 5's split merged inside the same launch through write-through
// partials and a ticket measured slower too, profiles/r5/attn_prefill_kv_split_inlaunch_ab_mi355x.jsonl, and was
// removed in round 6).
//
// O is accumulated TRANSPOSED, O^T += V^T P^T (A = V^T from the transposed LDS reads, B = P^T straight
// from the S^T accumulator): the accumulator's column is then the query row = the lane, so the online-
// softmax rescale and the final 1 / l are lane-local multiplies (no cross-lane shuffles), and each lane
// stores 4 contiguous dims of its own row per register group.
//
// Diagnostic cycle stamps (STAMP instantiations only, scripts/p32_stamps.py): per wave, the s_memtime cycles of each
// tile-loop segment summed over its tiles -> stamps[((wi * H + h) * NG + gi) * 4 + w][8]:
//   0 DMA issue, 1 QK^T + mask + row max, 2 softmax, 3 PV issue, 4 DMA wait, 5 barrier, 6 tiles | nt_max << 32, 7 whole kernel
__device__ unsigned long long* g_p32_stamps = nullptr;

template <int NG, bool STAMP = false>
__global__ __launch_bounds__(256 * NG, 2) void attn_prefill32_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                                     const uint16_t* __restrict__ vc,
                                                                     const int* __restrict__ block_tables, int max_blocks,
                                                                     const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
                                                                     const int* __restrict__ work, int H, int Hkv,
                                                                     float scale_log2, uint16_t* __restrict__ out,
                                                                     int xf_mt) {
  constexpr int WI = 4;  // ints per work item
  constexpr int D = 128;
  unsigned long long sg[6] = {0, 0, 0, 0, 0, 0}, st_t0 = 0, st_prev = 0;
  unsigned st_tiles = 0;
  auto stamp = [&](int k) {  // close segment k (STAMP builds only)
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long v = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (k >= 0) sg[k] += v - st_prev;
      st_prev = v;
    }
  };
  if constexpr (STAMP) {
    st_t0 = __builtin_amdgcn_s_memtime();
    st_prev = st_t0;
  }
  // K / V tiles, NB buffers per group, filled by LDS-DMA (global_load_lds: no staging registers, and the DMAs of
  // the next NB - 1 tiles run under tile t's MFMAs)
  constexpr int NB = NG == 1 ? LSA_P32_NBUF1 : 2;  // tile buffers per group (NG = 2: 2 x 2 x 32 KiB fills the LDS)
  __shared__ __attribute__((aligned(16))) uint16_t Ks[NG][NB][64 * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[NG][NB][64 * D];
  const int wi = blockIdx.x, h = blockIdx.y;
  // wave and group ids are wave-uniform: readfirstlane lets hipcc keep every per-group work field, block id
  // and DMA base in SGPRs (selected by a VGPR id, the whole tile loop's address math ran on the VALU)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int gi = NG == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 8);
  const int r32 = lane & 31, hh = lane >> 5;
  const int hk = h / (H / Hkv);

  // tiles of every group (the loop runs to the largest; the barriers are workgroup-wide)
  int nt_max = 0, ntiles = 0, seq = 0, qs = 0, t0 = 0, t1 = 0;
  int o_nt = 0, o_seq = 0, o_t0 = 0;  // the partner group's item (HELP)
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int* wk = work + WI * (NG * wi + g);
    const int sq = wk[0];
    const int nt = sq >= 0 ? wk[3] - wk[2] : 0;
    nt_max = max(nt_max, nt);
    if (g == gi) {
      ntiles = nt; seq = sq; qs = wk[1]; t0 = wk[2]; t1 = wk[3];
    } else {
      o_nt = nt; o_seq = sq >= 0 ? sq : 0; o_t0 = wk[2];
    }
  }
  const bool active = seq >= 0;
  const int sqc = active ? seq : 0;
  const int q0 = cu_q[sqc], qlen = cu_q[sqc + 1] - q0;
  const int ctx = ctx_lens[sqc];
  const int pos0 = ctx - qlen;

  // Q^T fragments (B operand of S^T): lane (r, h) holds Q[row r][16 s + 8 h .. + 7] for the 8 k-steps
  const int qrow = qs + w * 32 + r32;
  const int qpos = pos0 + qrow;
  uint4 qf[8];
  {
    const uint16_t* qp = q + ((size_t)(q0 + max(0, min(qrow, qlen - 1))) * H + h) * D + 8 * hh;
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) qf[s2] = *reinterpret_cast<const uint4*>(qp + 16 * s2);
  }
  // keys a wave's rows can see (causal): tiles past the wave's last row are skipped by that wave
  const int wave_last = min(qs + w * 32 + 31, qlen - 1);
  const int wave_tiles = (active && qs + w * 32 < qlen) ? min(t1, (min(ctx, pos0 + wave_last + 1) + 63) >> 6) : 0;

  f32x16_t o[4];  // O^T: register i of o[db] = dim 32 db + (i & 3) + 8 (i >> 2) + 4 hh of query row r32
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mrow = LSA_NEG_P, lrow = 0.f;  // of query row r32 (identical in both lane halves)

  const int* bt = block_tables + (size_t)sqc * max_blocks;
  // LDS-DMA of one 64-key tile: 32 wave-instructions of 1 KiB (4 key rows each), 8 per wave of the group.
  // The DMA writes lane-linearly, so the swizzled images (kp_off / vp_off) are produced by permuting the
  // SOURCE chunk each lane fetches: lane l of instruction j fills row 4 j + (l >> 4), slot l & 15.
  const int drow = lane >> 4, dslot = lane & 15;
  // per-lane byte offsets inside a (block, kv-head) tile (loop-invariant) and the LDS images' wave bases
  unsigned koff[4], voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * (w + 4 * i) + drow;
    koff[i] = (unsigned)(r * D + ((dslot ^ (r & 15)) << 3)) * 2u;
    voff[i] = (unsigned)(r * D + ((dslot ^ ((r & 3) << 2)) << 3)) * 2u;
  }
  const unsigned kl0 = __builtin_amdgcn_readfirstlane(lds_addr(&Ks[gi][0][4 * w * D]));
  const unsigned vl0 = __builtin_amdgcn_readfirstlane(lds_addr(&Vs[gi][0][4 * w * D]));
  // HELP (paired groups): once a group has computed its last tile it issues its partner's K / V DMAs, so
  // the heavy causal block's waves -- the launch's critical path -- stop paying ~420 cycles of LDS-DMA issue per tile
  // (scripts/p32_stamps.py).  Same kv-head, the partner's own block table and LDS images; every wave still drains
  // its DMAs (vmcnt(0), two buffers) before the barrier that publishes the tile.
  constexpr bool HELP = NG == 2;
  const int* bt_o = block_tables + (size_t)o_seq * max_blocks;
  const unsigned kl0_o = __builtin_amdgcn_readfirstlane(lds_addr(&Ks[NG - 1 - gi][0][4 * w * D]));
  const unsigned vl0_o = __builtin_amdgcn_readfirstlane(lds_addr(&Vs[NG - 1 - gi][0][4 * w * D]));
  auto dma_tile_o = [&](int blk, int b) {
    const size_t base = ((size_t)blk * Hkv + hk) * 64 * D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (unsigned)(b * 64 * D + 16 * i * D) * 2u;
      dma16s(kc + base, koff[i], kl0_o + lo);
      dma16s(vc + base, voff[i], vl0_o + lo);
    }
  };
  auto dma_tile = [&](int blk, int b) {
    const size_t base = ((size_t)blk * Hkv + hk) * 64 * D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (unsigned)(b * 64 * D + 16 * i * D) * 2u;  // buffer b, rows 4 (w + 4 i) ..
      dma16s(kc + base, koff[i], kl0 + lo);
      dma16s(vc + base, voff[i], vl0 + lo);
    }
  };
  const int G16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  // ---- one tile's pieces (shared by the two loop forms below)
  // S^T for the two 32-key halves of the tile in LDS image Kg
  auto qk = [&](const uint16_t* Kg, f32x16_t (&st)[2]) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      st[kh] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) {
        const uint4 a = *reinterpret_cast<const uint4*>(&Kg[kp_off(32 * kh + r32, 2 * s2 + hh)]);
        st[kh] = mfma32x32x16(a, qf[s2], st[kh]);
      }
    }
  };
  // mask + row max of absolute key tile t; register i of half kh holds key t*64 + 32 kh + (i & 3) + 8 (i >> 2) + 4 hh.
  // Raw scores: the scale is folded into one packed FMA per key pair in the exponent (v_pk_fma_f32), the row max is
  // taken over raw scores and scaled once, masked keys are -inf (exp2 -> 0 whatever the row max; mrow starts finite,
  // so a row with no visible key yet keeps p = 0, l = 0).  The causal / context mask only runs on the tiles that
  // cross this wave's diagonal or the context end (one wave-uniform branch per tile; inside it branch-free selects --
  // a short-circuit per element made hipcc emit 64 exec-mask branches per tile)
  auto mask_max = [&](f32x16_t (&st)[2], int t) -> float {
    if (t * 64 + 63 > min(pos0 + qs + w * 32, ctx - 1)) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = t * 64 + 32 * kh + (i & 3) + 8 * (i >> 2) + 4 * hh;
          const bool ok = (key <= qpos) & (key < ctx);
          st[kh][i] = ok ? st[kh][i] : -__builtin_inff();
        }
    }
    float tmax = -__builtin_inff();
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, st[kh][i]);
    return lsa_max_x32(tmax) * scale_log2;
  };
  // online softmax; the O / l rescale runs only when some row's max grew (exact: alpha = 1 otherwise), which under
  // the causal mask is the first few tiles of a row
  auto rescale = [&](float tmax) {
    if (__any(tmax > mrow)) {
      const float mnew = fmaxf(mrow, tmax);
      const float alpha = __builtin_amdgcn_exp2f(mrow - mnew);
      mrow = mnew;
      lrow *= alpha;
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] *= alpha;  // lane-local: the accumulator column is this lane's row
    }
  };
  // P = exp2(S * scale - m) as bf16 MFMA operands pa[kh][k-step s'] (registers 8 s' .. 8 s' + 7 of half kh); returns
  // the row sum
  auto softmax = [&](const f32x16_t (&st)[2], uint4 (&pa)[2][2]) -> float {
    const f32x2p_t sc2 = {scale_log2, scale_log2}, mn2 = {-mrow, -mrow};
    f32x2p_t ps2 = {0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      float p[16];
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2p_t x = __builtin_elementwise_fma(f32x2p_t{st[kh][i], st[kh][i + 1]}, sc2, mn2);
        p[i] = __builtin_amdgcn_exp2f(x.x);
        p[i + 1] = __builtin_amdgcn_exp2f(x.y);
        ps2 += f32x2p_t{p[i], p[i + 1]};
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        pa[kh][s2].x = pack2bf(p[8 * s2 + 0], p[8 * s2 + 1]);
        pa[kh][s2].y = pack2bf(p[8 * s2 + 2], p[8 * s2 + 3]);
        pa[kh][s2].z = pack2bf(p[8 * s2 + 4], p[8 * s2 + 5]);
        pa[kh][s2].w = pack2bf(p[8 * s2 + 6], p[8 * s2 + 7]);
      }
    }
    float psum = ps2.x + ps2.y;
    return lsa_sum_x32(psum);
  };
  // O^T += V^T P^T: k-step (kh, s') covers keys 32 kh + 16 s' + 8 (j >> 2) + 4 hh + (j & 3) in element j
  auto pv = [&](const uint16_t* Vg, const uint4 (&pa)[2][2]) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int r0 = 32 * kh + 16 * s2 + 4 * (G16 >> 1) + qq;  // this lane's supplied key row (j < 4)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int col = 32 * db + 16 * (G16 & 1) + 4 * pp;
          const uint2 v1 = ds_read_tr16p(&Vg[vp_off(r0, col)]);
          const uint2 v2 = ds_read_tr16p(&Vg[vp_off(r0 + 8, col)]);
          uint4 va;
          va.x = v1.x; va.y = v1.y; va.z = v2.x; va.w = v2.y;
          o[db] = mfma32x32x16(va, pa[kh][s2], o[db]);
        }
      }
  };

  {
    // the DMA runs NB - 1 tiles ahead: the prologue issues tiles 0 .. NB - 2, iteration tt issues tile tt + NB - 1
    // into the buffer tile tt - 1 left (its readers passed the previous barrier)
    int bnext = 0;  // block of the next tile to issue (loaded one iteration ahead: no dependent load on the DMA path)
#pragma unroll
    for (int p = 0; p < NB - 1; ++p)
      if (p < ntiles) dma_tile(__builtin_amdgcn_readfirstlane(bt[t0 + p]), p);
    if (NB - 1 < ntiles) bnext = __builtin_amdgcn_readfirstlane(bt[t0 + NB - 1]);
    // everything issued so far has landed (the Q fragments too, so hipcc's own wait tracking starts the loop with
    // no outstanding loads and inserts no vmcnt waits of its own in front of the K reads)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int tt = 0; tt < nt_max; ++tt) {
      const int t = t0 + tt;  // absolute key tile
      int bnn = 0;
      stamp(-1);
      if (tt + NB - 1 < ntiles) {
        // its buffer's last readers (tile t - 1) passed the previous barrier; an idle partner issues it instead
        if (!HELP || tt < o_nt) dma_tile(bnext, (tt + NB - 1) % NB);
        if (tt + NB < ntiles) bnn = __builtin_amdgcn_readfirstlane(bt[t + NB]);
      }
      if (HELP && tt >= ntiles && tt + NB - 1 < o_nt)
        dma_tile_o(__builtin_amdgcn_readfirstlane(bt_o[o_t0 + tt + NB - 1]), (tt + NB - 1) % NB);
      stamp(0);
      if (t < wave_tiles) {  // causal: tiles past the wave's last row are skipped (barriers stay uniform)
        if constexpr (STAMP) ++st_tiles;
        f32x16_t st[2];
        qk(Ks[gi][tt % NB], st);
        const float tmax = mask_max(st, t);
        stamp(1);
        rescale(tmax);
        uint4 pa[2][2];
        lrow += softmax(st, pa);
        stamp(2);
        pv(Vs[gi][tt % NB], pa);
        stamp(3);
      }
      bnext = bnn;
      // tile t + 1's DMA has landed before the barrier publishes it; the tiles issued after it may stay in flight
      if constexpr (HELP) __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): own or helped DMAs (NB = 2)
      else wait_dma_tiles(min(ntiles - 1, tt + NB - 1) - (tt + 1));
      stamp(4);
      __syncthreads();
      stamp(5);
    }
  }
  if constexpr (STAMP) {
    if (g_p32_stamps && lane == 0) {
      unsigned long long* o8 = g_p32_stamps + ((((size_t)wi * H + h) * NG + gi) * 4 + w) * 8;
#pragma unroll
      for (int k = 0; k < 6; ++k) o8[k] = sg[k];
      o8[6] = (unsigned long long)st_tiles | ((unsigned long long)nt_max << 32);
      o8[7] = __builtin_amdgcn_s_memtime() - st_t0;
    }
  }
  // normalise and store: lane = query row r32; register group gq of o[db] = dims 32 db + 8 gq + 4 hh + 0..3
  const int qr = qs + w * 32 + r32;
  if (active && qr < qlen) {
    const float inv = lrow > 0.f ? 1.f / lrow : 0.f;
    // row-major [T][H][128], or (xf_mt) the fragment-major layout the o projection's stream-K GEMM stages whole
    uint16_t* orow = out + ((size_t)(q0 + qr) * H + h) * D + 4 * hh;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 pk;
        pk.x = pack2bf(o[db][4 * gq + 0] * inv, o[db][4 * gq + 1] * inv);
        pk.y = pack2bf(o[db][4 * gq + 2] * inv, o[db][4 * gq + 3] * inv);
        const int dd = 32 * db + 8 * gq + 4 * hh;
        *reinterpret_cast<uint2*>(xf_mt ? out + xf_off(q0 + qr, h * D + dd, xf_mt) : orow + 32 * db + 8 * gq) = pk;
      }
  }
}

static bool g_p32_stamps_on = false;

// stamps: [nwork * H * NG * 4][8] u64 device buffer, or null to switch the diagnostic kernel off
extern "C" int lsa_p32_set_stamps(void* p) {
  unsigned long long* v = reinterpret_cast<unsigned long long*>(p);
  g_p32_stamps_on = v != nullptr;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_p32_stamps), &v, sizeof(v));
}

// work: NG (seq, q_start, t0, t1) items per workgroup (seq < 0: that group idles), nwork workgroups
extern "C" int lsa_attn_prefill32(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                                  const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv,
                                  float scale, void* out, int ng, int xf_mt, hipStream_t s) {
  if (nwork <= 0) return 0;
  if (H % Hkv) return -1;
  if (ng != 1 && ng != 2) return -2;
  dim3 grid(nwork, H);
  const float sl2 = scale * 1.4426950408889634f;
#define LSA_P32_LAUNCH(NGV, STV)                                                                                \
  hipLaunchKernelGGL((attn_prefill32_kernel<NGV, STV>), grid, dim3(256 * NGV), 0, s,                             \
                     reinterpret_cast<const uint16_t*>(q), reinterpret_cast<const uint16_t*>(kc),                 \
                     reinterpret_cast<const uint16_t*>(vc), block_tables, max_blocks, cu_q, ctx_lens, work, H, Hkv, \
                     sl2, reinterpret_cast<uint16_t*>(out), xf_mt)
#define LSA_P32_NG(STV)                  \
  do {                                   \
    if (ng == 2) LSA_P32_LAUNCH(2, STV); \
    else LSA_P32_LAUNCH(1, STV);         \
  } while (0)
  if (g_p32_stamps_on) LSA_P32_NG(true);  // diagnostic build of the kernel (lsa_p32_set_stamps)
  else LSA_P32_NG(false);
#undef LSA_P32_NG
#undef LSA_P32_LAUNCH
  return (int)hipGetLastError();
}
