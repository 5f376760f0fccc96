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
// profiles/attn_prefill_halves_mi355x.jsonl).
//
// O is accumulated TRANSPOSED, O^T += V^T P^T (A = V^T from the transposed LDS reads, B = P^T straight
// from the S^T accumulator): the accumulator's column is then the query row = the lane, so the online-
// softmax rescale and the final 1 / l are lane-local multiplies (no cross-lane shuffles), and each lane
// stores 4 contiguous dims of its own row per register group.
template <int NG>
__global__ __launch_bounds__(256 * NG, 2) void attn_prefill32_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                                     const uint16_t* __restrict__ vc,
                                                                     const int* __restrict__ block_tables, int max_blocks,
                                                                     const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
                                                                     const int* __restrict__ work, int H, int Hkv,
                                                                     float scale_log2, uint16_t* __restrict__ out) {
  constexpr int D = 128;
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
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int* wk = work + 4 * (NG * wi + g);
    const int sq = wk[0];
    const int nt = sq >= 0 ? wk[3] - wk[2] : 0;
    nt_max = max(nt_max, nt);
    if (g == gi) { ntiles = nt; seq = sq; qs = wk[1]; t0 = wk[2]; t1 = wk[3]; }
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
  auto dma_tile = [&](int blk, int b) {
    const size_t base = ((size_t)blk * Hkv + hk) * 64 * D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (unsigned)(b * 64 * D + 16 * i * D) * 2u;  // buffer b, rows 4 (w + 4 i) ..
      dma16s(kc + base, koff[i], kl0 + lo);
      dma16s(vc + base, voff[i], vl0 + lo);
    }
  };
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
  const int G16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  for (int tt = 0; tt < nt_max; ++tt) {
    const int t = t0 + tt;  // absolute key tile
    int bnn = 0;
    if (tt + NB - 1 < ntiles) {
      dma_tile(bnext, (tt + NB - 1) % NB);  // its buffer's last readers (tile t - 1) passed the previous barrier
      if (tt + NB < ntiles) bnn = __builtin_amdgcn_readfirstlane(bt[t + NB]);
    }
    const uint16_t* Kg = Ks[gi][tt % NB];
    const uint16_t* Vg = Vs[gi][tt % NB];
    if (t < wave_tiles) {  // causal: tiles past the wave's last row are skipped (barriers stay uniform)
      // S^T for the two 32-key halves
      f32x16_t st[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        st[kh] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) {
          const uint4 a = *reinterpret_cast<const uint4*>(&Kg[kp_off(32 * kh + r32, 2 * s2 + hh)]);
          st[kh] = mfma32x32x16(a, qf[s2], st[kh]);
        }
      }
      // mask + online softmax; register i of half kh holds key t*64 + 32 kh + (i & 3) + 8 (i >> 2) + 4 hh.
      // Raw scores: the scale is folded into one packed FMA per key pair in the exponent (v_pk_fma_f32), the
      // row max is taken over raw scores and scaled once, masked keys are -inf (exp2 -> 0 whatever the row
      // max; mrow starts finite, so a row with no visible key yet keeps p = 0, l = 0)
      // causal / context mask, only on the tiles that cross this wave's diagonal or the context end (one
      // wave-uniform branch per tile; inside it branch-free selects -- a short-circuit per element made
      // hipcc emit 64 exec-mask branches per tile)
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
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * scale_log2;
      // online softmax; the O / l rescale runs only when some row's max grew (exact: alpha = 1 otherwise),
      // which under the causal mask is the first few tiles of a row
      if (__any(tmax > mrow)) {
        const float mnew = fmaxf(mrow, tmax);
        const float alpha = __builtin_amdgcn_exp2f(mrow - mnew);
        mrow = mnew;
        lrow *= alpha;
  #pragma unroll
        for (int db = 0; db < 4; ++db) o[db] *= alpha;  // lane-local: the accumulator column is this lane's row
      }
      const f32x2p_t sc2 = {scale_log2, scale_log2}, mn2 = {-mrow, -mrow};
      f32x2p_t ps2 = {0.f, 0.f};
      uint4 pa[2][2];  // [kh][k-step s']: registers 8 s' .. 8 s' + 7 of half kh as bf16
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
      psum += __shfl_xor(psum, 32, 64);
      lrow += psum;
      // O^T += V^T P^T: k-step (kh, s') covers keys 32 kh + 16 s' + 8 (j >> 2) + 4 hh + (j & 3) in element j
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
    }
    bnext = bnn;
    // tile t + 1's DMA has landed before the barrier publishes it; the tiles issued after it may stay in flight
    wait_dma_tiles(min(ntiles - 1, tt + NB - 1) - (tt + 1));
    __syncthreads();
  }
  // normalise and store: lane = query row r32; register group gq of o[db] = dims 32 db + 8 gq + 4 hh + 0..3
  const int qr = qs + w * 32 + r32;
  if (active && qr < qlen) {
    const float inv = lrow > 0.f ? 1.f / lrow : 0.f;
    uint16_t* orow = out + ((size_t)(q0 + qr) * H + h) * D + 4 * hh;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 pk;
        pk.x = pack2bf(o[db][4 * gq + 0] * inv, o[db][4 * gq + 1] * inv);
        pk.y = pack2bf(o[db][4 * gq + 2] * inv, o[db][4 * gq + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * db + 8 * gq) = pk;
      }
  }
}

// ------------------------------------------------------------------------------------------------
// Pipelined variant (PIPE): the same work items, tiles and MFMA shapes, with the K fragments of tile t + 1 read
// from LDS into registers while tile t's P V runs, so the S^T MFMAs of every tile start on operands already in
// VGPRs (the loop above waits on an LDS read in front of each of its 16 S^T MFMAs: ~1.3 k cycles of s_waitcnt
// per wave and tile, profiles/attn_prefill_pmc_3b2k_mi355x.txt).  One barrier per tile, between softmax(t) and
// P V(t); buffer lifetimes:
//   K(t) is consumed into registers before the barrier of tile t  -> 2 K buffers, K(t + 2) DMA'd after barrier t;
//   V(t) is read by P V(t) after the barrier of tile t            -> 3 V buffers, V(t + 2) DMA'd after barrier t.
// LDS per group 2 x 16 + 3 x 16 KiB = 80 KiB (NG = 2: the whole 160 KiB; NG = 1: two workgroups per CU).
// Iteration t:  S^T(t) from registers, mask, softmax -> P | wait DMA(t + 1), barrier | DMA K, V (t + 2) |
//               K(t + 1) LDS reads -> registers | P V(t) (V(t) transposed reads + MFMAs).
// ------------------------------------------------------------------------------------------------
template <int NG>
__global__ __launch_bounds__(256 * NG, NG == 1 ? 2 : 1) void attn_prefill32p_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                                      const uint16_t* __restrict__ vc,
                                                                      const int* __restrict__ block_tables, int max_blocks,
                                                                      const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
                                                                      const int* __restrict__ work, int H, int Hkv,
                                                                      float scale_log2, uint16_t* __restrict__ out) {
  constexpr int D = 128;
  constexpr int KT = 64 * D;  // elements of one 64-key tile image
  __shared__ __attribute__((aligned(16))) uint16_t Ks[NG][2][KT];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[NG][3][KT];
  const int wi = blockIdx.x, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int gi = NG == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 8);
  const int r32 = lane & 31, hh = lane >> 5;
  const int hk = h / (H / Hkv);

  int nt_max = 0, ntiles = 0, seq = 0, qs = 0, t0 = 0, t1 = 0;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int* wk = work + 4 * (NG * wi + g);
    const int sq = wk[0];
    const int nt = sq >= 0 ? wk[3] - wk[2] : 0;
    nt_max = max(nt_max, nt);
    if (g == gi) { ntiles = nt; seq = sq; qs = wk[1]; t0 = wk[2]; t1 = wk[3]; }
  }
  const bool active = seq >= 0;
  const int sqc = active ? seq : 0;
  const int q0 = cu_q[sqc], qlen = cu_q[sqc + 1] - q0;
  const int ctx = ctx_lens[sqc];
  const int pos0 = ctx - qlen;

  const int qrow = qs + w * 32 + r32;
  const int qpos = pos0 + qrow;
  uint4 qf[8];
  {
    const uint16_t* qp = q + ((size_t)(q0 + max(0, min(qrow, qlen - 1))) * H + h) * D + 8 * hh;
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) qf[s2] = *reinterpret_cast<const uint4*>(qp + 16 * s2);
  }
  const int wave_last = min(qs + w * 32 + 31, qlen - 1);
  const int wave_tiles = (active && qs + w * 32 < qlen) ? min(t1, (min(ctx, pos0 + wave_last + 1) + 63) >> 6) : 0;

  f32x16_t o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mrow = LSA_NEG_P, lrow = 0.f;

  const int* bt = block_tables + (size_t)sqc * max_blocks;
  const int drow = lane >> 4, dslot = lane & 15;
  unsigned koff[4], voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * (w + 4 * i) + drow;
    koff[i] = (unsigned)(r * D + ((dslot ^ (r & 15)) << 3)) * 2u;
    voff[i] = (unsigned)(r * D + ((dslot ^ ((r & 3) << 2)) << 3)) * 2u;
  }
  const unsigned kl0 = __builtin_amdgcn_readfirstlane(lds_addr(&Ks[gi][0][4 * w * D]));
  const unsigned vl0 = __builtin_amdgcn_readfirstlane(lds_addr(&Vs[gi][0][4 * w * D]));
  // one tile = 8 DMA wave-instructions per wave (4 K + 4 V row groups), into K buffer kb and V buffer vb
  auto dma_tile = [&](int blk, int kb, int vb) {
    const size_t base = ((size_t)blk * Hkv + hk) * 64 * D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned lo = (unsigned)(16 * i * D) * 2u;
      dma16s(kc + base, koff[i], kl0 + (unsigned)(kb * KT) * 2u + lo);
      dma16s(vc + base, voff[i], vl0 + (unsigned)(vb * KT) * 2u + lo);
    }
  };
  // K fragments of one tile for S^T: [kh][s2] = 32 keys (kh) x 16 dims (s2) of the row-swizzled image
  uint4 kf[2][8];
  auto read_k = [&](const uint16_t* Kg) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) kf[kh][s2] = *reinterpret_cast<const uint4*>(&Kg[kp_off(32 * kh + r32, 2 * s2 + hh)]);
  };

  // prologue: tile 0 landed and published with its K fragments in registers, tile 1 in flight.  The full vmcnt(0)
  // after tile 0 also retires the Q loads in hipcc's own wait tracking (it does not see the inline-asm DMAs: a
  // counted vmcnt here left it assuming Q pending and waiting on vmcnt in front of every S^T MFMA of the loop)
  if (0 < ntiles) dma_tile(__builtin_amdgcn_readfirstlane(bt[t0]), 0, 0);
  __builtin_amdgcn_s_waitcnt(0x0070);
  if (1 < ntiles) dma_tile(__builtin_amdgcn_readfirstlane(bt[t0 + 1]), 1, 1);
  int bnext = (2 < ntiles) ? __builtin_amdgcn_readfirstlane(bt[t0 + 2]) : 0;
  __syncthreads();
  if (t0 < wave_tiles) read_k(Ks[gi][0]);

  const int G16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  int vcur = 0;  // V buffer of tile tt (tt % 3)
  for (int tt = 0; tt < nt_max; ++tt) {
    const int t = t0 + tt;
    const bool live = t < wave_tiles;
    uint4 pa[2][2];
    if (live) {
      f32x16_t st[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        st[kh] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) st[kh] = mfma32x32x16(kf[kh][s2], qf[s2], st[kh]);
      }
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
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * scale_log2;
      if (__any(tmax > mrow)) {
        const float mnew = fmaxf(mrow, tmax);
        const float alpha = __builtin_amdgcn_exp2f(mrow - mnew);
        mrow = mnew;
        lrow *= alpha;
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db] *= alpha;
      }
      float psum = 0.f;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        float p[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          p[i] = __builtin_amdgcn_exp2f(fmaf(st[kh][i], scale_log2, -mrow));
          psum += p[i];
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          pa[kh][s2].x = pack2bf(p[8 * s2 + 0], p[8 * s2 + 1]);
          pa[kh][s2].y = pack2bf(p[8 * s2 + 2], p[8 * s2 + 3]);
          pa[kh][s2].z = pack2bf(p[8 * s2 + 4], p[8 * s2 + 5]);
          pa[kh][s2].w = pack2bf(p[8 * s2 + 6], p[8 * s2 + 7]);
        }
      }
      psum += __shfl_xor(psum, 32, 64);
      lrow += psum;
    }
    // tile tt + 1 landed (its DMA, issued one iteration ago, is this wave's only one in flight) and published;
    // every wave is past S^T(tt) and P V(tt - 1), so K buffer tt & 1 and V buffer (tt + 2) % 3 are free
    __builtin_amdgcn_s_waitcnt(0x0070);
    __syncthreads();
    const int vnext2 = vcur == 0 ? 2 : vcur - 1;  // (tt + 2) % 3
    if (tt + 2 < ntiles) {
      dma_tile(bnext, tt & 1, vnext2);
      if (tt + 3 < ntiles) bnext = __builtin_amdgcn_readfirstlane(bt[t + 3]);
    }
    if (t + 1 < wave_tiles && tt + 1 < ntiles) read_k(Ks[gi][(tt + 1) & 1]);
    if (live) {
      // P V(t): four k-steps (kh, s2) of 4 MFMAs; the 8 transposed V reads of k-step j + 1 are issued before
      // k-step j's MFMAs (two named register sets), so each MFMA group waits only for reads issued a group ago
      const uint16_t* Vg = Vs[gi][vcur];
      auto read_v = [&](uint4 (&va)[4], int j) {
        const int r0 = 16 * j + 4 * (G16 >> 1) + qq;  // j = 2 kh + s2
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int col = 32 * db + 16 * (G16 & 1) + 4 * pp;
          const uint2 v1 = ds_read_tr16p(&Vg[vp_off(r0, col)]);
          const uint2 v2 = ds_read_tr16p(&Vg[vp_off(r0 + 8, col)]);
          va[db] = make_uint4(v1.x, v1.y, v2.x, v2.y);
        }
      };
      auto pv = [&](const uint4 (&va)[4], const uint4& p) {
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db] = mfma32x32x16(va[db], p, o[db]);
      };
      uint4 vA[4], vB[4];
      read_v(vA, 0);
      read_v(vB, 1);
      pv(vA, pa[0][0]);
      read_v(vA, 2);
      pv(vB, pa[0][1]);
      read_v(vB, 3);
      pv(vA, pa[1][0]);
      pv(vB, pa[1][1]);
    }
    vcur = vcur == 2 ? 0 : vcur + 1;
  }
  const int qr = qs + w * 32 + r32;
  if (active && qr < qlen) {
    const float inv = lrow > 0.f ? 1.f / lrow : 0.f;
    uint16_t* orow = out + ((size_t)(q0 + qr) * H + h) * D + 4 * hh;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 pk;
        pk.x = pack2bf(o[db][4 * gq + 0] * inv, o[db][4 * gq + 1] * inv);
        pk.y = pack2bf(o[db][4 * gq + 2] * inv, o[db][4 * gq + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * db + 8 * gq) = pk;
      }
  }
}

// work: NG (seq, q_start, t0, t1) items per workgroup (seq < 0: that group idles), nwork workgroups;
// pipe: 1 = the pipelined loop (attn_prefill32p_kernel)
extern "C" int lsa_attn_prefill32(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                                  const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv,
                                  float scale, void* out, int ng, int pipe, hipStream_t s) {
  if (nwork <= 0) return 0;
  if (H % Hkv) return -1;
  dim3 grid(nwork, H);
  const float sl2 = scale * 1.4426950408889634f;
#define LSA_P32_LAUNCH(KERN, NGV)                                                                                \
  hipLaunchKernelGGL(KERN<NGV>, grid, dim3(256 * NGV), 0, s, reinterpret_cast<const uint16_t*>(q),               \
                     reinterpret_cast<const uint16_t*>(kc), reinterpret_cast<const uint16_t*>(vc), block_tables,  \
                     max_blocks, cu_q, ctx_lens, work, H, Hkv, sl2, reinterpret_cast<uint16_t*>(out))
  if (ng != 1 && ng != 2) return -2;
  if (pipe) {
    if (ng == 2) LSA_P32_LAUNCH(attn_prefill32p_kernel, 2);
    else LSA_P32_LAUNCH(attn_prefill32p_kernel, 1);
  } else {
    if (ng == 2) LSA_P32_LAUNCH(attn_prefill32_kernel, 2);
    else LSA_P32_LAUNCH(attn_prefill32_kernel, 1);
  }
#undef LSA_P32_LAUNCH
  return (int)hipGetLastError();
}
