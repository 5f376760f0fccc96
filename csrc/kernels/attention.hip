// Attention over the paged KV cache, head_dim 128, bf16.
//
// Cache layout (one tensor per layer and per K / V):  [num_blocks, Hkv, 64 tokens, 128]  so that one
// (block, kv-head) tile is a contiguous 16 KiB run — a 64-key attention tile is one cache block.
//
//   attn_decode_kernel   one query token per sequence (decode).  Memory-bound split-KV
//                        ("flash-decoding"): grid (splits, Hkv, B), all G = H / Hkv query heads of a kv
//                        head share every K/V load.  A wave reads 4 keys per 1 KiB wave-instruction
//                        straight to VGPRs (no LDS round trip: the guide's decode-attention row),
//                        16-lane dot products + xor-shuffle reductions, online softmax in exp2 domain,
//                        cross-lane-group merge through LDS, and either the final output (1 split) or an
//                        (o, m, l) partial merged in the same launch by the last-arriving split of the
//                        (sequence, kv-head).  Optionally fuses RoPE + the KV-cache append of the new token.
//   attn_prefill_kernel  causal flash attention for (chunked) prefill of packed variable-length
//                        sequences, MFMA 16x16x32 bf16.  4 waves x 16 query rows per workgroup; K/V tiles
//                        of 64 keys staged through LDS (register staging, issue-early / write-late);
//                        S^T = K Q^T so each lane owns one query row (softmax max over 16 values +
//                        2 xor shuffles); P stays in registers and feeds the PV MFMA as the A operand;
//                        V is read as the B operand with ds_read_b64_tr_b16 (hardware transpose) from
//                        an XOR-swizzled image (conflict-free per 32-lane half).
#include "common.h"

#define LSA_NEG (-1.0e30f)
#ifndef LSA_PREFILL_QG
#define LSA_PREFILL_QG 1  // 16-row query groups per wave in prefill attention (work items of 64 * QG rows);
                          // QG = 2 halves LDS reads per FLOP but needs 300 registers -> 1 wave/SIMD: measured
                          // 1.6x slower (3B 2k: 129 -> 205 us), so 1 ships
#endif
#ifndef LSA_ATTN_NT
#define LSA_ATTN_NT 1  // non-temporal K/V loads in decode attention (read once per step: 3-5 % faster at B = 32)
#endif
#define LSA_NT 2    // buffer cache-policy aux bit: nt (streaming)
#define LSA_SC1 16  // buffer cache-policy aux bit: sc1 (write-through store / L1-bypassing load)

typedef __attribute__((address_space(1))) unsigned long long g_u64;
typedef __attribute__((address_space(1))) int g_i32;


// Fused RoPE + KV append (decode): q/k/v of the new token come straight from the QKV projection's f32
// split-K slabs; every workgroup rotates its own G query heads, the workgroup holding the last block
// appends the rotated k and v to the cache, and the new token's key/value are substituted from
// registers where the score loop meets position p (no dependency on the cache write completing).
// timing probe (scripts/attn_stamps.py): when set, thread 0 of every decode-attention workgroup records
// s_memrealtime (100 MHz) at 7 points of its critical path into [wg][8]; null in production
__device__ unsigned long long* g_attn_stamps = nullptr;
#define LSA_STAMP(K)                                                                                  \
  if (stp && tid == 0) stp[((size_t)(split * gridDim.y + b) * gridDim.x + hk) * 8 + (K)] = __builtin_amdgcn_s_memrealtime()

struct RopeArgs {
  const float* parts;  // [nparts][B][(H + 2 Hkv) * 128] f32
  size_t part_stride;
  int nparts;
  const float* cos_t;  // [max_pos][64]
  const float* sin_t;
  uint16_t* kc;        // cache (writable aliases of the kernel's kc / vc)
  uint16_t* vc;
  float* ks;           // fp8 cache: per-(token, kv-head) scales (writable aliases of ksc / vsc)
  float* vs;
  const long long* rowss;  // or null: the slabs are the QKV projection of UN-normalised rows (the residual-reduce
                           // decode step, gemm.hip RR); row b's q / k / v are scaled by rsqrt(rowss[b] inv_k + eps)
  float inv_k;
  float eps;
};

// WV = waves per workgroup: 8 for G <= 3 (two keys per lane group per block -> half the K/V registers,
// so four 4-wave-equivalents fit per CU and a B x Hkv = 1024 grid runs in whole rounds; G = 3: half the
// per-wave score work on the latency-bound small grids, 3B B=32 ctx 200 11.1 -> 10.0 us), else 4 (the
// [NLG][G][128] merge buffer of G >= 4 would not fit 64 KiB of LDS with 32 lane groups)
//
// G = 1 is capped at 80 VGPRs (6 waves per SIMD = three 8-wave workgroups per CU, 64 spills):
// the 7B B x Hkv = 1024 workgroups run in 1.33 rounds instead of two (7B B=32 ctx 200: 23.4 -> 21.0 us).
#ifndef LSA_ATTN_WPE
#define LSA_ATTN_WPE 6
#endif
#ifndef LSA_ATTN_WPE8
#define LSA_ATTN_WPE8 6  // fp8 cache, G = 1 (8 = 64 VGPRs, one grid round at B x Hkv = 1024: spills, 7B b32 ctx 200 17.6 -> 18.2 us)
#endif
#ifndef LSA_ATTN_SB8
#define LSA_ATTN_SB8 1  // the single-buffered G = 1 kernel for the fp8 KV cache too
#endif
#ifndef LSA_ATTN_SB_MIN_WG
#define LSA_ATTN_SB_MIN_WG 512  // grids of at least this many workgroups run the single-buffered G = 1 kernel (SB)
#endif
#ifndef LSA_ATTN_SPEC_MAX_WG
#define LSA_ATTN_SPEC_MAX_WG 512  // grids up to this many workgroups speculate every split's first block (below)
#endif
#ifndef LSA_ATTN_WV23
#define LSA_ATTN_WV23 4  // waves per workgroup for G = 2, 3 on small grids (below)
#endif
#ifndef LSA_ATTN_SMALL23_WG
#define LSA_ATTN_SMALL23_WG 256
#endif
#ifndef LSA_ATTN_BUF_G
#define LSA_ATTN_BUF_G 2
#endif
#ifndef LSA_ATTN_NEWREG_G
#define LSA_ATTN_NEWREG_G 3
#endif
#ifndef LSA_ATTN_DOT2_G
#define LSA_ATTN_DOT2_G 99
#endif
//
// KV8: fp8 cache (ops.KV_FP8) -- kc / vc hold e4m3 bytes, 8 KiB per (block, kv-head) tile in the token-pair
// order of common.h kv8_off, and ksc / vsc the per-(token, kv-head) f32 scales [blocks, Hkv, 64].  Same 16-lane
// groups of 8 dims, but one 16-byte load per lane now carries two keys (half the load instructions and half
// the HBM bytes of the bf16 cache); a K slice is widened to bf16 exactly (v_cvt_scalef32_pk_bf16_fp8) for the
// same dot2 products and its scale multiplies the reduced score; a V slice goes to f32 with its scale in p.
//
// SB (G = 1, bf16 cache, large grids): ONE K/V register set -- each wave waits for its own block, and the 56-VGPR
// kernel runs 8 waves per SIMD (four 8-wave workgroups per CU), so the 7B's B x Hkv = 1024 workgroups at batch 32
// fill the chip in one grid round and the waves of a CU hide each other's load latency: 7B b32 ctx 200
// 22.1 -> 18.6 us, decode step 3.60 -> 3.50 ms (profiles/attn_decode_sb_ab_mi355x.jsonl).  Small grids keep the
// two-set pipeline (7B b1: 6.8 vs 7.1 us).
// Dims d0 .. d0 + 3 of head h of row b: bf16 (row-major [B, H, 128], or fragment-major with xf_mt row tiles), or
// -- s8 set -- e4m3 in the xf8 layout with one E8M0 scale per (row, head) into s8 (common.h xs8_off; the byte of
// each of the head's four 32-dim lane blocks): the W8A8 / W4A8 o projection's input.  The 32 threads finishing a
// head are one aligned half-wave (e = tid + k * NT, NT a multiple of 64), so the head's amax is 5 xor shuffles;
// every thread of the workgroup's loop iteration must call this (no early exits around it).
__device__ __forceinline__ void attn_store4(uint16_t* out, uint8_t* s8, int xf_mt, int b, int H, int h, int d0, float o0,
                                            float o1, float o2, float o3) {
  if (s8 == nullptr) {
    uint2 pk;
    pk.x = pack2bf(o0, o1);
    pk.y = pack2bf(o2, o3);
    *reinterpret_cast<uint2*>(out + (xf_mt ? xf_off(b, h * 128 + d0, xf_mt) : ((size_t)b * H + h) * 128 + d0)) = pk;
    return;
  }
  float a = fmaxf(fmaxf(fabsf(o0), fabsf(o1)), fmaxf(fabsf(o2), fabsf(o3)));
  a = lsa_max_x16(lsa_row16_max(a));  // the head's 32 threads: two whole rows of one half-wave
  const int e = e8m0_for_amax(a);
  const int k = h * 128 + d0;
  *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(out) + xf8_off(b, k, xf_mt)) = pack4_fp8(o0, o1, o2, o3, e8m0_inv(e));
  if ((d0 & 31) == 0) s8[xs8_off(b, k, xf_mt)] = (uint8_t)e;
}

template <int G, int ROPE, int WV, bool KV8 = false, bool SB = false>  // ROPE: 0 = q given; > 0 = that many QKV slabs; < 0 = runtime
__global__ __launch_bounds__(64 * WV)
__attribute__((amdgpu_waves_per_eu(G == 1 && WV == 8 ? (SB ? 8 : (KV8 ? LSA_ATTN_WPE8 : LSA_ATTN_WPE)) : 1))) void attn_decode_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                          const uint16_t* __restrict__ vc,
                                                          const float* __restrict__ ksc, const float* __restrict__ vsc,
                                                          const int* __restrict__ block_tables, int max_blocks,
                                                          const int* __restrict__ pos, int Hkv, float scale_log2,
                                                          int chunk_blocks, int nsplit, int unsplit_max,
                                                          uint16_t* __restrict__ out, float* __restrict__ opart, float* __restrict__ mlpart,
                                                          int* __restrict__ counters, int xf_mt, RopeArgs ra,
                                                          uint8_t* __restrict__ s8) {
  constexpr int D = 128;
  constexpr int NT = 64 * WV;      // threads
  constexpr int NLG = 4 * WV;      // 16-lane groups
  constexpr int TU = 16 / WV;      // 4-key quads per lane group and block
  constexpr int TW = 64 / WV;      // keys per wave and block
  // heads fastest: consecutive workgroups (round-robin over the 8 XCDs) are different (b, kv-head) pairs of
  // the same split, so splits a sequence does not need (eff_split) never leave whole XCDs idle
  const int hk = blockIdx.x, b = blockIdx.y, split = blockIdx.z;
  const int H = Hkv * G;
  const int tid = threadIdx.x;
  unsigned long long* const stp = g_attn_stamps;
  LSA_STAMP(0);
  const __amdgpu_buffer_rsrc_t rs_o = __builtin_amdgcn_make_buffer_rsrc(opart, 0, 0x7fffffff, 0x00020000);
  const int lg = tid >> 4, li = tid & 15, wv = tid >> 6;
  const int* bt = block_tables + (size_t)b * max_blocks;
  // K/V of block blk+1 are in flight while block blk is scored (two register sets, static names)
  // KV8: one 16-byte load carries the lane's 8 dims of a token PAIR (kv8_off), so NL = TU / 2 loads per block
  constexpr int NL = KV8 ? TU / 2 : TU;
  static_assert(!KV8 || TU % 2 == 0, "KV8 pairs keys");
  uint4 kA[NL], vA[NL], kB[NL], vB[NL];
  float2 ksA[NL], vsA[NL], ksB[NL], vsB[NL];  // KV8 only: the pair's key / value row scales
  // keys past the context in the last block re-read the last valid row (a cache hit, not HBM traffic);
  // they are masked in the score
  // G >= LSA_ATTN_BUF_G: one buffer resource per (block, kv-head) slab, built in SGPRs from the uniform
  // block-table entry, the lanes carry 32-bit offsets (3B: 10.3 -> 9.8 us at B = 32); G = 1 keeps 64-bit
  // global loads (buffer loads measured 20.7 -> 22.4 us for the 7B at B = 32)
  constexpr bool BUF = G >= LSA_ATTN_BUF_G;
  auto fetch = [&](uint4 (&kr)[NL], uint4 (&vr)[NL], float2 (&ksr)[NL], float2 (&vsr)[NL], int blk, int last_tok) {
    const size_t rowb = ((size_t)__builtin_amdgcn_readfirstlane(bt[blk]) * Hkv + hk) * 64;
    const size_t base = rowb * D;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      if constexpr (KV8) {  // pair pr = tokens 2 pr, 2 pr + 1 (clamped like single keys)
        const int pr = min(wv * (TW / 2) + u * 4 + (lg & 3), last_tok >> 1);
        const size_t off = base + kv8_off(2 * pr, li * 8);
        kr[u] = ldg_nt(reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(kc) + off));
        vr[u] = ldg_nt(reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(vc) + off));
        ksr[u] = *reinterpret_cast<const float2*>(ksc + rowb + 2 * pr);
        vsr[u] = *reinterpret_cast<const float2*>(vsc + rowb + 2 * pr);
        continue;
      }
      const int tok = min(wv * TW + u * 4 + (lg & 3), last_tok);
      if constexpr (BUF) {
        const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)(kc + base), 0, 64 * D * 2, 0x00020000);
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(vc + base), 0, 64 * D * 2, 0x00020000);
        const int off = (tok * D + li * 8) * 2;
        const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(rk, off, 0, LSA_ATTN_NT ? LSA_NT : 0);
        const u32x4_t c = __builtin_amdgcn_raw_buffer_load_b128(rv, off, 0, LSA_ATTN_NT ? LSA_NT : 0);
        kr[u] = make_uint4(a[0], a[1], a[2], a[3]);
        vr[u] = make_uint4(c[0], c[1], c[2], c[3]);
      } else {
        kr[u] = ldg_nt(reinterpret_cast<const uint4*>(kc + base + tok * D + li * 8));
        vr[u] = ldg_nt(reinterpret_cast<const uint4*>(vc + base + tok * D + li * 8));
      }
    }
  };
  // split 0 always starts at block 0, which every sequence owns (padding rows map it to the scratch
  // block): its first K/V fetch leaves before the context length is even known.  (Speculating the other
  // splits' first blocks too was measured: splits a short sequence does not need then cost a wasted
  // block read each, 23 -> 36 us at B = 32, ctx 200, 4 splits.)
  // Small grids (the latency-bound batch-1 shapes, <= LSA_ATTN_SPEC_MAX_WG workgroups): every other split
  // speculates that its range starts at split * chunk_blocks -- exact whenever the context is longer than the
  // unsplit threshold, because the host plan has nsplit * chunk_blocks >= every context the captured graph
  // serves -- so its first K/V fetch also leaves before pos[b] is read (one dependent round trip off the
  // chain, 3B 2k explain: start->ctx 1.2 us); a mismatch (a short context) re-fetches below.
  const int spec_blk = (split != 0 && (int)(gridDim.x * gridDim.y * gridDim.z) <= LSA_ATTN_SPEC_MAX_WG &&
                        split * chunk_blocks < max_blocks) ? split * chunk_blocks : -1;
  if (split == 0) fetch(kA, vA, ksA, vsA, 0, 63);
  else if (spec_blk >= 0) fetch(kA, vA, ksA, vsA, spec_blk, 63);
  // fused RoPE: the new token's q / k / v rows (sum of the QKV projection's split-K slabs) do not depend on
  // the context length -- their loads leave before pos[b] is read, off the prologue's dependent chain
  float xq[8];
  if constexpr (ROPE != 0) {
    if (lg < G + 2) {
      const float* row = ra.parts + (size_t)b * (H + 2 * Hkv) * D;
      const int off = (lg < G ? (hk * G + lg) * D : (lg == G ? (H + hk) * D : (H + Hkv + hk) * D)) + li * 8;
      const float4 a0 = *reinterpret_cast<const float4*>(row + off);
      const float4 a1 = *reinterpret_cast<const float4*>(row + off + 4);
      xq[0] = a0.x; xq[1] = a0.y; xq[2] = a0.z; xq[3] = a0.w; xq[4] = a1.x; xq[5] = a1.y; xq[6] = a1.z; xq[7] = a1.w;
      const int np = ROPE > 0 ? ROPE : ra.nparts;
      const long long ssq = ra.rowss ? ra.rowss[b] : 0;
#pragma unroll
      for (int sp = 1; sp < np; ++sp) {
        const float* r2 = row + sp * ra.part_stride + off;
        const float4 b0 = *reinterpret_cast<const float4*>(r2);
        const float4 b1 = *reinterpret_cast<const float4*>(r2 + 4);
        xq[0] += b0.x; xq[1] += b0.y; xq[2] += b0.z; xq[3] += b0.w;
        xq[4] += b1.x; xq[5] += b1.y; xq[6] += b1.z; xq[7] += b1.w;
      }
      if (ra.rowss) {  // the RMS row scale of the residual-reduce step (linear: before RoPE, like the GEMM's)
        const float rs = rsqrtf((float)ssq * (1.0f / LSA_Q24) * ra.inv_k + ra.eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) xq[j] *= rs;
      }
    }
  }
  const int ctx = pos[b] + 1;
  const int nblk = (ctx + 63) >> 6;
  int ech, nse;
  eff_split(nblk, chunk_blocks, nsplit, unsplit_max, ech, nse);
  LSA_STAMP(1);
  if (split >= nse) return;  // whole workgroup: this sequence needs fewer splits
  const int blk0 = split * ech;
  const int blk1 = min(nblk, blk0 + ech);

  // the first K/V block is in flight while the query (and, fused, RoPE) is prepared
  if (split != 0 && blk0 < blk1 && blk0 != spec_blk) fetch(kA, vA, ksA, vsA, blk0, ctx - 1 - blk0 * 64);
  __builtin_amdgcn_sched_barrier(0);

  const int tpos = ctx - 1;  // position of the new token
  // q, and the new token's k / v, stay packed bf16 (the dot products run on v_dot2c_f32_bf16 and the
  // softmax scale is applied to the reduced score): 12 VGPRs instead of 24 f32 for G = 1
  uint4 qb[G];
  // the new token's rotated k / v: for G < LSA_ATTN_NEWREG_G they stay in LDS (read back by the one lane
  // group that meets position tpos: 8 VGPRs fewer in the score loop), else in registers (a select instead
  // of a branch around an LDS read)
  constexpr bool NEWREG = G >= LSA_ATTN_NEWREG_G;
  __shared__ uint4 qkv_s[G + 2][16];
  __shared__ uint2 new8_s[KV8 ? 2 : 1][16];  // KV8: the new token's e4m3 key / value row and its scales
  __shared__ float newsc_s[2];
  uint4 knew = make_uint4(0, 0, 0, 0), vnew = make_uint4(0, 0, 0, 0);
  if constexpr (ROPE != 0) {
    // lane group j < G builds query head j, group G the new key, group G + 1 the new value (each lane
    // 8 dims, summed over the split-K slabs, rotated in f32, rounded to bf16 like the unfused path);
    // the results go through LDS to all lane groups
    static_assert(G + 2 <= NLG, "fused rope: one lane group per q head + k + v");
    if (lg < G + 2) {
      const int dd = li * 8;  // own 8 dims; the rotate-half partners live in lane li ^ 8
      const float* x = xq;
      float y[8];
      if (lg <= G) {  // rotate q heads and k
        const float4 c0 = *reinterpret_cast<const float4*>(ra.cos_t + (size_t)tpos * 64 + (dd & 63));
        const float4 c1 = *reinterpret_cast<const float4*>(ra.cos_t + (size_t)tpos * 64 + (dd & 63) + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(ra.sin_t + (size_t)tpos * 64 + (dd & 63));
        const float4 s1 = *reinterpret_cast<const float4*>(ra.sin_t + (size_t)tpos * 64 + (dd & 63) + 4);
        const float sg = li < 8 ? -1.f : 1.f;
        const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = x[j] * cc[j] + sg * lsa_xor8(x[j]) * sn[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = x[j];
      }
      qkv_s[lg][li] = pack8(y);
      if constexpr (KV8) {  // the new key / value row quantised like every cached row (16-lane amax)
        if (lg >= G) {
          float a = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) a = fmaxf(a, fabsf(y[j]));
          a = lsa_row16_max(a);
          new8_s[lg - G][li] = pack8_fp8(y, kv8_inv(a));
          if (li == 0) newsc_s[lg - G] = a * LSA_KV8_RMAX;
        }
      }
    }
    __syncthreads();
    LSA_STAMP(2);
#pragma unroll
    for (int g = 0; g < G; ++g) qb[g] = qkv_s[g][li];
    if constexpr (NEWREG) {
      knew = qkv_s[G][li];
      vnew = qkv_s[G + 1][li];
    }
  } else {
#pragma unroll
    for (int g = 0; g < G; ++g) qb[g] = *reinterpret_cast<const uint4*>(q + ((size_t)(b * H + hk * G + g)) * D + li * 8);
  }
  // G < LSA_ATTN_DOT2_G: scores on v_dot2c_f32_bf16 from the packed q (fewest VGPRs); else q in f32,
  // pre-scaled, and each key unpacked once for all G heads
  constexpr bool DOT2 = G < LSA_ATTN_DOT2_G;
  float qf[DOT2 ? 1 : G][8];
  if constexpr (!DOT2) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      unpack8(qb[g], qf[g]);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[g][j] *= scale_log2;
    }
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = LSA_NEG;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
  }

  // key slot u of this lane group -> its position (KV8: slot u is half u & 1 of load u / 2's token pair)
  auto slot_pos = [&](int blk, int u) {
    return KV8 ? blk * 64 + 2 * (wv * (TW / 2) + (u >> 1) * 4 + (lg & 3)) + (u & 1) : blk * 64 + wv * TW + u * 4 + (lg & 3);
  };
  auto score = [&](const uint4 (&kr)[NL], const uint4 (&vr)[NL], const float2 (&ksr)[NL], const float2 (&vsr)[NL],
                   int blk) {
    float s[TU][G];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      uint4 kq;
      float ksu = 1.f;
      const int tp = slot_pos(blk, u);
      const bool valid = tp < ctx;
      if constexpr (KV8) {
        const uint4 kp = kr[u >> 1];
        uint2 k8 = (u & 1) ? make_uint2(kp.z, kp.w) : make_uint2(kp.x, kp.y);
        ksu = (u & 1) ? ksr[u >> 1].y : ksr[u >> 1].x;
        if constexpr (ROPE != 0) {
          if (tp == tpos) {
            k8 = new8_s[0][li];
            ksu = newsc_s[0];
          }
        }
        kq = fp8x8_to_bf16x8(k8);
        if constexpr (DOT2) ksu *= scale_log2;  // (else q was pre-scaled)
      } else {
        kq = kr[u];
        if constexpr (ROPE != 0) {
          if (tp == tpos) kq = NEWREG ? knew : qkv_s[G][li];
        }
      }
      float kf[8];
      if constexpr (!DOT2) unpack8(kq, kf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d;
        if constexpr (DOT2) {
          d = dot8_bf16(qb[g], kq);
        } else {
          d = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) d = fmaf(qf[g][j], kf[j], d);
        }
        d = lsa_row16_sum(d);
        s[u][g] = valid ? (KV8 ? d * ksu : (DOT2 ? d * scale_log2 : d)) : LSA_NEG;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = s[0][g];
#pragma unroll
      for (int u = 1; u < TU; ++u) mx = fmaxf(mx, s[u][g]);
      const float mn = fmaxf(m[g], mx);
      const float alpha = __builtin_amdgcn_exp2f(m[g] - mn);
      m[g] = mn;
      float p[TU], ps = 0.f;
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        p[u] = __builtin_amdgcn_exp2f(s[u][g] - mn);
        ps += p[u];
      }
      l[g] = l[g] * alpha + ps;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] *= alpha;
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        float vf[8], pu = p[u];
        if constexpr (KV8) {
          const uint4 vp = vr[u >> 1];
          uint2 v8 = (u & 1) ? make_uint2(vp.z, vp.w) : make_uint2(vp.x, vp.y);
          float vsu = (u & 1) ? vsr[u >> 1].y : vsr[u >> 1].x;
          if constexpr (ROPE != 0) {
            if (slot_pos(blk, u) == tpos) {
              v8 = new8_s[1][li];
              vsu = newsc_s[1];
            }
          }
          fp8x8_to_f32(v8, vf);
          pu *= vsu;
        } else {
          uint4 vq = vr[u];
          if constexpr (ROPE != 0) {
            if (blk * 64 + wv * TW + u * 4 + (lg & 3) == tpos) vq = NEWREG ? vnew : qkv_s[G + 1][li];
          }
          unpack8(vq, vf);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) o[g][j] = fmaf(pu, vf[j], o[g][j]);
      }
    }
  };
  static_assert(!SB || G == 1, "SB: G = 1");
  if constexpr (SB) {
    // single register set: each wave waits for its block, the 32 waves of a CU overlap each other's loads
    for (int blk = blk0; blk < blk1; ++blk) {
      if (blk != blk0) fetch(kA, vA, ksA, vsA, blk, ctx - 1 - blk * 64);
      __builtin_amdgcn_sched_barrier(0);
      score(kA, vA, ksA, vsA, blk);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else if (blk0 < blk1) {
    int blk = blk0;
    for (; blk + 1 < blk1; blk += 2) {
      fetch(kB, vB, ksB, vsB, blk + 1, ctx - 1 - (blk + 1) * 64);
      __builtin_amdgcn_sched_barrier(0);
      score(kA, vA, ksA, vsA, blk);
      __builtin_amdgcn_sched_barrier(0);
      fetch(kA, vA, ksA, vsA, min(blk + 2, blk1 - 1), ctx - 1 - min(blk + 2, blk1 - 1) * 64);
      __builtin_amdgcn_sched_barrier(0);
      score(kB, vB, ksB, vsB, blk + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (blk < blk1) score(kA, vA, ksA, vsA, blk);
  }
  LSA_STAMP(3);

  if constexpr (ROPE != 0) {
    // the workgroup covering position tpos appends the new token's k / v to the cache: after its score loop
    // (which substitutes them from LDS / registers where it meets tpos), off the prologue's critical path
    if (lg >= G && lg < G + 2 && blk0 < nblk && blk1 == nblk) {
      const size_t row = ((size_t)block_tables[(size_t)b * max_blocks + (tpos >> 6)] * Hkv + hk) * 64 + (tpos & 63);
      if constexpr (KV8) {
        *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(lg == G ? ra.kc : ra.vc) + (row - (tpos & 63)) * D +
                                  kv8_off(tpos & 63, li * 8)) = new8_s[lg - G][li];
        if (li == 0) (lg == G ? ra.ks : ra.vs)[row] = newsc_s[lg - G];
      } else {
        *reinterpret_cast<uint4*>((lg == G ? ra.kc : ra.vc) + row * D + li * 8) = qkv_s[lg][li];
      }
    }
  }
  // merge the 4 lane groups of each wave in registers (xor-16 / xor-32 lane exchanges), then the WV wave
  // partials through LDS: a quarter of the LDS traffic and merge loop of a lane-group-level merge
  // (7B B=32 ctx ~190: 23.6 -> 22.1 us; 7B B=1: 7.3 -> 6.4 us, rocprofv3)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float mo = lsa_max_x32(lsa_max_x16(m[g]));
    const float a = __builtin_amdgcn_exp2f(m[g] - mo);
    l[g] *= a;
    l[g] = lsa_sum_x32(lsa_sum_x16(l[g]));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[g][j] *= a;
      o[g][j] = lsa_sum_x32(lsa_sum_x16(o[g][j]));
    }
    m[g] = mo;
  }
  __shared__ float sm[WV][G], sl[WV][G];
  __shared__ __attribute__((aligned(16))) float so[WV][G][D];
  if ((tid & 63) < 16) {  // lane group 0 of every wave carries the wave's merged partial
    if (li == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        sm[wv][g] = m[g];
        sl[wv][g] = l[g];
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      *reinterpret_cast<float4*>(&so[wv][g][li * 8]) = make_float4(o[g][0], o[g][1], o[g][2], o[g][3]);
      *reinterpret_cast<float4*>(&so[wv][g][li * 8 + 4]) = make_float4(o[g][4], o[g][5], o[g][6], o[g][7]);
    }
  }
  __syncthreads();
  LSA_STAMP(4);
  // each thread finishes 4 consecutive dims of one head
  for (int e = tid; e < G * 32; e += NT) {
    const int g = e >> 5, d0 = (e & 31) * 4;
    float M = LSA_NEG;
#pragma unroll
    for (int k = 0; k < WV; ++k) M = fmaxf(M, sm[k][g]);
    float L = 0.f, O[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const float wgt = __builtin_amdgcn_exp2f(sm[k][g] - M);
      L += sl[k][g] * wgt;
      const float4 v = *reinterpret_cast<const float4*>(&so[k][g][d0]);
      O[0] += v.x * wgt; O[1] += v.y * wgt; O[2] += v.z * wgt; O[3] += v.w * wgt;
    }
    const int h = hk * G + g;
    if (nse == 1) {
      const float inv = L > 0.f ? 1.f / L : 0.f;
      attn_store4(out, s8, xf_mt, b, H, h, d0, O[0] * inv, O[1] * inv, O[2] * inv, O[3] * inv);
    } else {
      // publish the partial write-through (sc1): the reducing workgroup may sit on another XCD
      const size_t pi = ((size_t)b * H + h) * nsplit + split;
      const u32x4_t v = {__float_as_uint(O[0]), __float_as_uint(O[1]), __float_as_uint(O[2]), __float_as_uint(O[3])};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs_o, (int)((pi * D + d0) * 4), 0, LSA_SC1);
      if (d0 == 0)
        __hip_atomic_store((g_u64*)(mlpart) + pi,
                           ((unsigned long long)__float_as_uint(L) << 32) | __float_as_uint(M), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (nse == 1) return;

  // split-KV combine inside the launch: the last of this (sequence, kv-head)'s nse workgroups to arrive
  // merges all partials (guide §6 G16 counter form: sc1 stores drained -> barrier -> one relaxed agent
  // ticket add; the reducer reads every partial with sc1 loads, no fences).  The ticket word is reset by
  // the reducer for the next layer / replay.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  g_i32* ctr = (g_i32*)(counters) + (size_t)b * Hkv + hk;
  if (tid == 0) s_last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nse - 1;
  __syncthreads();
  LSA_STAMP(5);
  if (!s_last) return;
  if (tid == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the partials are spread over SS thread slices per (head, 4 dims): each slice loads its share of the nse
  // (max, sum) words and partial vectors in one batch (one memory round trip; the maxima are merged online,
  // log-sum-exp style) and the slices are combined through LDS.  Loading all maxima first and then the
  // vectors nse / 4 at a time by one thread per (head, 4 dims) was the tail of the decode-attention
  // latency chain (3B 2k explain: 3.1 us of 11.1, scripts/attn_stamps.py)
  constexpr int NPAIR = G * 32;
  constexpr int SS = (NT / NPAIR) >= 4 ? 4 : (NT / NPAIR);
  __shared__ __attribute__((aligned(16))) float cpo[SS][G][D];
  __shared__ float cpm[SS][G], cpl[SS][G];
  if (tid < SS * NPAIR) {
    const int pair = tid % NPAIR, slice = tid / NPAIR;
    const int g = pair >> 5, d0 = (pair & 31) * 4;
    const size_t pi0 = ((size_t)b * H + hk * G + g) * nsplit;
    float M = LSA_NEG, L = 0.f, O[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int sp = slice; sp < nse; sp += SS) {
      const unsigned long long ml =
          __hip_atomic_load((g_u64*)(mlpart) + pi0 + sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs_o, (int)(((pi0 + sp) * D + d0) * 4), 0, LSA_SC1);
      const float mi = __uint_as_float((uint32_t)ml), li = __uint_as_float((uint32_t)(ml >> 32));
      const float mn = fmaxf(M, mi);
      const float a = __builtin_amdgcn_exp2f(M - mn), wgt = __builtin_amdgcn_exp2f(mi - mn);
      M = mn;
      L = L * a + li * wgt;
      O[0] = O[0] * a + __uint_as_float(v[0]) * wgt; O[1] = O[1] * a + __uint_as_float(v[1]) * wgt;
      O[2] = O[2] * a + __uint_as_float(v[2]) * wgt; O[3] = O[3] * a + __uint_as_float(v[3]) * wgt;
    }
    *reinterpret_cast<float4*>(&cpo[slice][g][d0]) = make_float4(O[0], O[1], O[2], O[3]);
    if (d0 == 0) {
      cpm[slice][g] = M;
      cpl[slice][g] = L;
    }
  }
  __syncthreads();
  for (int e = tid; e < NPAIR; e += NT) {
    const int g = e >> 5, d0 = (e & 31) * 4;
    float M = LSA_NEG;
#pragma unroll
    for (int sl = 0; sl < SS; ++sl) M = fmaxf(M, cpm[sl][g]);
    float L = 0.f, O[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < SS; ++sl) {
      const float wgt = __builtin_amdgcn_exp2f(cpm[sl][g] - M);
      L += cpl[sl][g] * wgt;
      const float4 v = *reinterpret_cast<const float4*>(&cpo[sl][g][d0]);
      O[0] += v.x * wgt; O[1] += v.y * wgt; O[2] += v.z * wgt; O[3] += v.w * wgt;
    }
    const int h = hk * G + g;
    const float inv = L > 0.f ? 1.f / L : 0.f;
    attn_store4(out, s8, xf_mt, b, H, h, d0, O[0] * inv, O[1] * inv, O[2] * inv, O[3] * inv);
  }
  LSA_STAMP(6);
}

extern "C" int lsa_attn_set_stamps(void* p) {
  unsigned long long* v = reinterpret_cast<unsigned long long*>(p);
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), &v, sizeof(v));
}

extern "C" int lsa_attn_decode(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                               const int* pos, int B, int H, int Hkv, float scale, int chunk_blocks, int nsplit,
                               int unsplit_max, void* out, float* opart, float* mlpart, int* counters, int xf_mt,
                               const float* qkv_parts, int nparts,
                               long part_stride, const float* cos_t, const float* sin_t, const float* ks,
                               const float* vs, void* out_s8, const long long* rowss, float inv_k, float eps,
                               hipStream_t s) {
  if (rowss && !qkv_parts) return -7;  // the row scale applies to the fused-RoPE slabs
  if (H % Hkv) return -1;
  if (xf_mt && B > 16 * xf_mt) return -4;
  if (out_s8 && !xf_mt) return -6;  // the e4m3 output lives in the xf8 layout
  if (nsplit > 256) return -3;
  if ((ks == nullptr) != (vs == nullptr)) return -5;
  const int G = H / Hkv;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(Hkv, B, nsplit);
  const uint16_t* qq = reinterpret_cast<const uint16_t*>(q);
  const uint16_t* kk = reinterpret_cast<const uint16_t*>(kc);
  const uint16_t* vv = reinterpret_cast<const uint16_t*>(vc);
  uint16_t* oo = reinterpret_cast<uint16_t*>(out);
  const RopeArgs ra{qkv_parts, (size_t)part_stride, nparts, cos_t, sin_t, const_cast<uint16_t*>(kk),
                    const_cast<uint16_t*>(vv), const_cast<float*>(ks), const_cast<float*>(vs), rowss, inv_k, eps};
#define LSA_ADL(GV, RP, WV, KV8, SB)                                                                              \
  hipLaunchKernelGGL((attn_decode_kernel<GV, RP, WV, KV8, SB>), grid, dim3(64 * (WV)), 0, s, qq, kk, vv, ks, vs,     \
                     block_tables, max_blocks, pos, Hkv, sl2, chunk_blocks, nsplit, unsplit_max, oo, opart, mlpart,  \
                     counters, xf_mt, ra, reinterpret_cast<uint8_t*>(out_s8))
  // waves per workgroup: 8 for G = 1 (single-buffered at >= LSA_ATTN_SB_MIN_WG workgroups); for G = 2, 3 four on
  // grids of <= LSA_ATTN_SMALL23_WG workgroups (3B batch 1, 2k context: 11.34 -> 10.74 us -- half the cross-wave
  // merge, profiles/r3/attn_decode_wv23_ab_mi355x.jsonl) and eight above (3B batch 32: 10.54 vs 11.33 us); else 4
  const long nwg = (long)grid.x * grid.y * grid.z;
  const bool sb = nwg >= LSA_ATTN_SB_MIN_WG, small23 = nwg <= LSA_ATTN_SMALL23_WG;
#define LSA_ADK(GV, RP)                                                                                               \
  do {                                                                                                                 \
    if constexpr (GV == 1) {                                                                                           \
      if (ks && LSA_ATTN_SB8 && sb) LSA_ADL(GV, RP, 8, true, true);                                                    \
      else if (ks) LSA_ADL(GV, RP, 8, true, false);                                                                    \
      else if (sb) LSA_ADL(GV, RP, 8, false, true);                                                                    \
      else LSA_ADL(GV, RP, 8, false, false);                                                                           \
    } else if constexpr (GV <= 3) {                                                                                    \
      if (small23) {                                                                                                   \
        if (ks) LSA_ADL(GV, RP, LSA_ATTN_WV23, true, false);                                                           \
        else LSA_ADL(GV, RP, LSA_ATTN_WV23, false, false);                                                             \
      } else {                                                                                                         \
        if (ks) LSA_ADL(GV, RP, 8, true, false);                                                                       \
        else LSA_ADL(GV, RP, 8, false, false);                                                                         \
      }                                                                                                                \
    } else {                                                                                                           \
      if (ks) LSA_ADL(GV, RP, 4, true, false);                                                                         \
      else LSA_ADL(GV, RP, 4, false, false);                                                                           \
    }                                                                                                                  \
  } while (0)
#define LSA_AD(GV)                                  \
  case GV:                                          \
    if (!qkv_parts) LSA_ADK(GV, 0);                 \
    else if (nparts == 1) LSA_ADK(GV, 1);           \
    else if (nparts == 2) LSA_ADK(GV, 2);           \
    else if (nparts == 4) LSA_ADK(GV, 4);           \
    else if (nparts == 8) LSA_ADK(GV, 8);           \
    else LSA_ADK(GV, -1);                           \
    break;
  switch (G) {
    LSA_AD(1) LSA_AD(2) LSA_AD(3) LSA_AD(4) LSA_AD(8)
    default: return -2;
  }
#undef LSA_ADL
#undef LSA_ADK
#undef LSA_AD
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// prefill
// ------------------------------------------------------------------------------------------------
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t* lds_s4_ptr;

__device__ __forceinline__ uint2 ds_read_tr16(const uint16_t* p) {
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(p));
  return __builtin_bit_cast(uint2, v);
}

// K image: 16 B chunk ch of key row r stored at chunk (ch ^ (r & 15))   (ds_read_b128 row reads)
// V image: chunk ch of row r at chunk (ch ^ ((r & 7) << 1))               (ds_read_b64_tr_b16 reads)
__device__ __forceinline__ int k_off(int r, int ch) { return r * 128 + ((ch ^ (r & 15)) << 3); }
__device__ __forceinline__ int v_off(int r, int col) { return r * 128 + ((((col >> 3) ^ ((r & 7) << 1))) << 3) + (col & 7); }

// QG query groups of 16 rows per wave (WG = 4 waves x 16*QG rows): every K / V fragment read from LDS
// feeds QG MFMAs, so QG = 2 halves the LDS traffic per FLOP (the kernel is LDS-read bound at QG = 1:
// each wave re-reads the whole 64-key K and V tiles for only 16 query rows).
template <int QG>
__global__ __launch_bounds__(256) void attn_prefill_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                           const uint16_t* __restrict__ vc,
                                                           const int* __restrict__ block_tables, int max_blocks,
                                                           const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
                                                           const int* __restrict__ work, int H, int Hkv,
                                                           float scale_log2, uint16_t* __restrict__ out, int xf_mt) {
  constexpr int D = 128;
  constexpr int QW = 16 * QG;   // query rows per wave
  constexpr int QB = 4 * QW;    // query rows per workgroup
  __shared__ __attribute__((aligned(16))) uint16_t Ks[64 * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[64 * D];
  const int wi = blockIdx.x, h = blockIdx.y;
  const int seq = work[2 * wi], qs = work[2 * wi + 1];
  const int hk = h / (H / Hkv);
  const int q0 = cu_q[seq], qlen = cu_q[seq + 1] - q0;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, r = lane & 15;

  uint4 qf[QG][4];
  int qpos[QG];
#pragma unroll
  for (int gi = 0; gi < QG; ++gi) {
    const int qrow = qs + w * QW + gi * 16 + r;
    const int qrow_c = min(qrow, qlen - 1);
    qpos[gi] = pos0 + qrow;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[gi][s] = *reinterpret_cast<const uint4*>(q + ((size_t)(q0 + qrow_c) * H + h) * D + 32 * s + 8 * g);
  }

  const int last_row = min(qs + QB - 1, qlen - 1);
  const int kv_end = min(ctx, pos0 + last_row + 1);
  const int ntiles = (kv_end + 63) >> 6;

  f32x4_t o[QG][8];
  float mrow[QG], lrow[QG];
#pragma unroll
  for (int gi = 0; gi < QG; ++gi) {
    mrow[gi] = LSA_NEG;
    lrow[gi] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[gi][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  const int* bt = block_tables + (size_t)seq * max_blocks;
  // register staging of the next K/V tile: issued unconditionally (tile index clamped) right after the
  // LDS image of the current tile is written, consumed one iteration later, so the global latency hides
  // behind the current tile's MFMAs.  (A conditional refill inside the loop made hipcc keep the staging
  // registers in scratch and wait for every fetch at once: 2x slower, scripts/bench_attn_prefill.py.)
  uint4 kr0, kr1, kr2, kr3, vr0, vr1, vr2, vr3;
#define LSA_PF_FETCH(T)                                                                  \
  {                                                                                      \
    const size_t base_ = ((size_t)bt[(T)] * Hkv + hk) * 64 * D;                          \
    const uint4* kb_ = reinterpret_cast<const uint4*>(kc + base_) + tid;                 \
    const uint4* vb_ = reinterpret_cast<const uint4*>(vc + base_) + tid;                 \
    kr0 = kb_[0]; kr1 = kb_[256]; kr2 = kb_[512]; kr3 = kb_[768];                        \
    vr0 = vb_[0]; vr1 = vb_[256]; vr2 = vb_[512]; vr3 = vb_[768];                        \
  }
  LSA_PF_FETCH(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    {
      const int row = tid >> 4, ch = tid & 15;  // chunk c = tid + 256 i -> row + 16 i, same ch
      *reinterpret_cast<uint4*>(&Ks[k_off(row, ch)]) = kr0;
      *reinterpret_cast<uint4*>(&Ks[k_off(row + 16, ch)]) = kr1;
      *reinterpret_cast<uint4*>(&Ks[k_off(row + 32, ch)]) = kr2;
      *reinterpret_cast<uint4*>(&Ks[k_off(row + 48, ch)]) = kr3;
      *reinterpret_cast<uint4*>(&Vs[v_off(row, ch * 8)]) = vr0;
      *reinterpret_cast<uint4*>(&Vs[v_off(row + 16, ch * 8)]) = vr1;
      *reinterpret_cast<uint4*>(&Vs[v_off(row + 32, ch * 8)]) = vr2;
      *reinterpret_cast<uint4*>(&Vs[v_off(row + 48, ch * 8)]) = vr3;
    }
    __syncthreads();
    LSA_PF_FETCH(min(t + 1, ntiles - 1));

    // S^T[key][q] = K Q^T over 4 subtiles of 16 keys; one K fragment feeds QG MFMAs
    f32x4_t st[QG][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int gi = 0; gi < QG; ++gi) st[gi][kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int krow = 16 * kt + r;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const uint4 a = *reinterpret_cast<const uint4*>(&Ks[k_off(krow, 4 * s + g)]);
#pragma unroll
        for (int gi = 0; gi < QG; ++gi) st[gi][kt] = mfma16x16x32(a, qf[gi][s], st[gi][kt]);
      }
    }
    uint4 pa[QG][2];
#pragma unroll
    for (int gi = 0; gi < QG; ++gi) {
      float tmax = LSA_NEG;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = t * 64 + 16 * kt + 4 * g + i;
          float v = st[gi][kt][i] * scale_log2;
          v = (key > qpos[gi] || key >= ctx) ? LSA_NEG : v;
          st[gi][kt][i] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = lsa_max_x32(lsa_max_x16(tmax));
      const float mnew = fmaxf(mrow[gi], tmax);
      const float alpha = __builtin_amdgcn_exp2f(mrow[gi] - mnew);
      mrow[gi] = mnew;
      float psum = 0.f;
      uint32_t pk[4][2];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p[i] = __builtin_amdgcn_exp2f(st[gi][kt][i] - mnew);
          psum += p[i];
        }
        pk[kt][0] = pack2bf(p[0], p[1]);
        pk[kt][1] = pack2bf(p[2], p[3]);
      }
      lrow[gi] = lrow[gi] * alpha + psum;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float ai = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[gi][dt][i] *= ai;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        pa[gi][s2].x = pk[2 * s2][0]; pa[gi][s2].y = pk[2 * s2][1];
        pa[gi][s2].z = pk[2 * s2 + 1][0]; pa[gi][s2].w = pk[2 * s2 + 1][1];
      }
    }
    // O[q][d] += P[q][key] V[key][d]; one V fragment feeds QG MFMAs
    const int qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int kb1 = 32 * s2 + 4 * g + qq, kb2 = kb1 + 16;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const int col = 16 * dt + 4 * pp;
        const uint2 v1 = ds_read_tr16(&Vs[v_off(kb1, col)]);
        const uint2 v2 = ds_read_tr16(&Vs[v_off(kb2, col)]);
        uint4 vb;
        vb.x = v1.x; vb.y = v1.y; vb.z = v2.x; vb.w = v2.y;
#pragma unroll
        for (int gi = 0; gi < QG; ++gi) o[gi][dt] = mfma16x16x32(pa[gi][s2], vb, o[gi][dt]);
      }
    }
  }
#undef LSA_PF_FETCH
#pragma unroll
  for (int gi = 0; gi < QG; ++gi) {
    const float lt = lsa_sum_x32(lsa_sum_x16(lrow[gi]));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float li = __shfl(lt, 4 * g + i, 64);
      const float inv = li > 0.f ? 1.f / li : 0.f;
      const int qr = qs + w * QW + gi * 16 + 4 * g + i;
      if (qr < qlen) {
        uint16_t* orow = out + ((size_t)(q0 + qr) * H + h) * D;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)  // row-major, or (xf_mt) the o projection's fragment-major input
          (xf_mt ? out[xf_off(q0 + qr, h * D + 16 * dt + r, xf_mt)] : orow[16 * dt + r]) = f2bf(o[gi][dt][i] * inv);
      }
    }
  }
}

extern "C" int lsa_prefill_qblock() { return 64 * LSA_PREFILL_QG; }

extern "C" int lsa_attn_prefill(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                                const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv,
                                float scale, void* out, int xf_mt, hipStream_t s) {
  if (nwork <= 0) return 0;
  if (H % Hkv) return -1;
  dim3 grid(nwork, H);
  hipLaunchKernelGGL(attn_prefill_kernel<LSA_PREFILL_QG>, grid, dim3(256), 0, s, reinterpret_cast<const uint16_t*>(q),
                     reinterpret_cast<const uint16_t*>(kc), reinterpret_cast<const uint16_t*>(vc), block_tables,
                     max_blocks, cu_q, ctx_lens, work, H, Hkv, scale * 1.4426950408889634f,
                     reinterpret_cast<uint16_t*>(out), xf_mt);
  return (int)hipGetLastError();
}
