// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this package.
//
// Everything here is written for wave64 + MFMA 16x16x32 bf16.  Conventions used by every
// kernel in this directory:
//   * bf16 tensors travel as raw uint16 bit patterns (uint16_t / uint4 = 8 bf16);
//   * the MFMA "fragment" of a 16x32 operand tile is 64 lanes x 16 B: lane l holds row (l & 15),
//     k-columns 8*(l >> 4) .. 8*(l >> 4) + 7 (cdna_hip_programming.md §3 operand maps);
//   * the D (accumulator) map of mfma_f32_16x16x32_bf16 is D[row = 4*(l >> 4) + i][col = l & 15].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsa_epi.h"

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// non-temporal 16-byte load (weights streamed once per forward: 'nt-weights' in MI355X_MICROARCH.md)
__device__ __forceinline__ uint4 ldg_nt(const uint4* p) {
  u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

#define LSA_WAVE 64

__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, lowers to v_cvt_pk_bf16_f32 on gfx950
  return __builtin_bit_cast(uint16_t, b);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// ONE v_cvt_pk_bf16_f32 (RNE) for the pair; two scalar f2bf + shift + or cost 4 VALU per pair
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  const bf16x2_t v = __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, v);
}

// 8 bf16 (one uint4) -> 8 floats
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2bf(f[0], f[1]); r.y = pack2bf(f[2], f[3]);
  r.z = pack2bf(f[4], f[5]); r.w = pack2bf(f[6], f[7]);
  return r;
}

// dot product of 8 bf16 pairs on v_dot2c_f32_bf16 (f32 accumulate), no unpacking
__device__ __forceinline__ float dot8_bf16(const uint4 a, const uint4 b) {
  float d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.x), __builtin_bit_cast(bf16x2_t, b.x), 0.f, false);
  d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.y), __builtin_bit_cast(bf16x2_t, b.y), d, false);
  d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.z), __builtin_bit_cast(bf16x2_t, b.z), d, false);
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a.w), __builtin_bit_cast(bf16x2_t, b.w), d, false);
}

__device__ __forceinline__ f32x4_t mfma16x16x32(const uint4 a, const uint4 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// Cross-lane reductions on the VALU.  hipcc lowers every __shfl_xor to ds_bpermute_b32, an LDS-crossbar round trip
// (address VALU + LDS pipe + lgkmcnt wait) per butterfly step of a dependent chain; within a 16-lane row DPP does the
// step as a modifier of the add / max itself, and across rows / halves v_permlane16_swap / v_permlane32_swap exchange
// whole rows in one VALU op.  Every pairing below is symmetric (lane a reads b iff b reads a) and each op is
// commutative, so all lanes of a reduction end bitwise identical, as with the xor butterfly.  Callers run with whole
// 16-lane rows active (whole waves for the x16 / x32 / wave forms): DPP from a disabled lane reads 0.
template <int CTRL>
__device__ __forceinline__ float lsa_dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
// DPP controls: row_mirror (lane i <- 15 - i), row_half_mirror (i <- 7 - i in each 8), quad_perm [1,0,3,2] / [2,3,0,1]
// (xor 1 / xor 2), row_ror:8 (xor 8 within the row)
#define LSA_DPP_ROW_MIRROR 0x140
#define LSA_DPP_HALF_MIRROR 0x141
#define LSA_DPP_XOR1 0xB1
#define LSA_DPP_XOR2 0x4E
#define LSA_DPP_ROR8 0x128
// sum / max over the 16 lanes of each row, in every lane of the row
__device__ __forceinline__ float lsa_row16_sum(float d) {
  d += lsa_dpp<LSA_DPP_ROW_MIRROR>(d);
  d += lsa_dpp<LSA_DPP_HALF_MIRROR>(d);
  d += lsa_dpp<LSA_DPP_XOR1>(d);
  return d + lsa_dpp<LSA_DPP_XOR2>(d);
}
__device__ __forceinline__ float lsa_row16_max(float d) {
  d = fmaxf(d, lsa_dpp<LSA_DPP_ROW_MIRROR>(d));
  d = fmaxf(d, lsa_dpp<LSA_DPP_HALF_MIRROR>(d));
  d = fmaxf(d, lsa_dpp<LSA_DPP_XOR1>(d));
  return fmaxf(d, lsa_dpp<LSA_DPP_XOR2>(d));
}
// the value of lane i ^ 8 (same row)
__device__ __forceinline__ float lsa_xor8(float x) { return lsa_dpp<LSA_DPP_ROR8>(x); }
// lanes i and i ^ 16 / i ^ 32 combined: the swap of x with itself returns {rows [0 0 2 2], rows [1 1 3 3]} (x16) or
// {halves [lo lo], [hi hi]} (x32), so op(r0, r1) pairs each lane with its partner in the same order in both
__device__ __forceinline__ float lsa_sum_x16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float lsa_max_x16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float lsa_sum_x32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float lsa_max_x32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// 64-lane max of a packed 64-bit key (argmax: orderable value << 32 | ~index): each half moved by the same DPP /
// permlane pattern, compared whole
template <int CTRL>
__device__ __forceinline__ unsigned long long lsa_dpp64(unsigned long long x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long lsa_umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  v = lsa_umax64(v, lsa_dpp64<LSA_DPP_ROW_MIRROR>(v));
  v = lsa_umax64(v, lsa_dpp64<LSA_DPP_HALF_MIRROR>(v));
  v = lsa_umax64(v, lsa_dpp64<LSA_DPP_XOR1>(v));
  v = lsa_umax64(v, lsa_dpp64<LSA_DPP_XOR2>(v));
  {
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(v >> 32), (uint32_t)(v >> 32), false, false);
    v = lsa_umax64(((unsigned long long)hi[0] << 32) | lo[0], ((unsigned long long)hi[1] << 32) | lo[1]);
  }
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(v >> 32), (uint32_t)(v >> 32), false, false);
  return lsa_umax64(((unsigned long long)hi[0] << 32) | lo[0], ((unsigned long long)hi[1] << 32) | lo[1]);
}

__device__ __forceinline__ float wave_sum(float v) { return lsa_sum_x32(lsa_sum_x16(lsa_row16_sum(v))); }

__device__ __forceinline__ float wave_max(float v) { return lsa_max_x32(lsa_max_x16(lsa_row16_max(v))); }

// block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  __syncthreads();
  return t;
}

// block-wide max for blockDim.x <= 1024; `red` must hold >= 16 floats
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = red[0];
  for (int i = 1; i < nw; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Byte offset of e4m3 activation (m, k) in the W8A8 / W4A8 decode layout X8[k/128][mt][64 lanes][32 B]: lane (g, r)
// holds row 16 mt + r at k = 128 s + 16 g .. +15 (bytes 0..15) and 128 s + 64 + 16 g .. +15 (bytes 16..31).  That is
// the K order in which v_mfma_scale_f32_16x16x128_f8f6f4 reads an 8-bit operand, so the MFMA's K index is k itself;
// a 4-bit operand lane (g, r) holds K 128 s + 32 g .. +31 (one MX block), and the scale byte of lane group b covers
// K 128 s + 32 b .. +31 for either operand (measured: scripts/probe_mfma_scale.py, profiles/r4/probe_mfma_scale_mi355x.jsonl;
// tests/test_kernels_gpu.py::test_a8_gemm_block_scales).  So activation block scales cover 32 consecutive k, for
// e4m3 and e2m1 weights alike.  8 consecutive k from a multiple of 8 are contiguous.
__device__ __forceinline__ size_t xf8_off(int m, int k, int mt) {
  const int kc = k & 127;
  return (((size_t)(k >> 7) * mt + (m >> 4)) * 64 + 16 * ((kc & 63) >> 4) + (m & 15)) * 32 + 16 * (kc >> 6) + (kc & 15);
}
// Byte offset of the E8M0 scale of k's 32-block in the block-scale array S8[k/128][mt][64 lanes] (lane group b = block b)
__device__ __forceinline__ size_t xs8_off(int m, int k, int mt) {
  return ((size_t)(k >> 7) * mt + (m >> 4)) * 64 + 16 * ((k & 127) >> 5) + (m & 15);
}
// E8M0 exponent of the smallest power of two s with amax / s <= 448 (the e4m3 maximum), clamped to [1, 253];
// e8m0_inv(e) = 1 / s.  ops.e8m0_for_amax is the host twin.
__device__ __forceinline__ int e8m0_for_amax(float amax) {
  const uint32_t b = __float_as_uint(amax * (1.0f / 448.0f));
  const int e = (int)(b >> 23) + ((b & 0x7fffffu) != 0u);
  return e < 1 ? 1 : (e > 253 ? 253 : e);
}
__device__ __forceinline__ float e8m0_inv(int e) { return __uint_as_float((uint32_t)(254 - e) << 23); }
// 4 floats * inv -> 4 OCP e4m3 bytes
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d, float inv) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a * inv, b * inv, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c * inv, d * inv, lo, true);
}

// 8 floats * inv -> 8 OCP e4m3 bytes (v_cvt_pk_fp8_f32: round to nearest even, saturating)
__device__ __forceinline__ uint2 pack8_fp8(const float* f, float inv) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0] * inv, f[1] * inv, 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2] * inv, f[3] * inv, lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4] * inv, f[5] * inv, 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6] * inv, f[7] * inv, hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}

// 8 OCP e4m3 bytes -> 8 bf16 (v_cvt_scalef32_pk_bf16_fp8 at unit scale; exact: every e4m3 value is a bf16 value)
__device__ __forceinline__ uint4 fp8x8_to_bf16x8(const uint2 q) {
  uint4 r;
  r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.x, 1.0f, false));
  r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.x, 1.0f, true));
  r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.y, 1.0f, false));
  r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q.y, 1.0f, true));
  return r;
}

// 8 OCP e4m3 bytes -> 8 floats (v_cvt_pk_f32_fp8)
__device__ __forceinline__ void fp8x8_to_f32(const uint2 q, float* f) {
  const f32x2_t a = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.x, true);
  const f32x2_t c = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)q.y, true);
  f[0] = a[0]; f[1] = a[1]; f[2] = b[0]; f[3] = b[1]; f[4] = c[0]; f[5] = c[1]; f[6] = d[0]; f[7] = d[1];
}

// fp8 KV cache (ops.KV_FP8): every (token, kv-head) row of 128 values is stored as e4m3(x * 448 / amax) with the
// f32 scale amax / 448 beside it (ops/reference.py quant_kv_rows is the host twin of these two formulas)
#define LSA_KV8_RMAX (1.0f / 448.0f)
// Byte offset of (token t, dim d) inside one fp8 (block, kv-head) tile of 64 x 128 bytes: tokens are stored in
// pairs, the 8-byte chunk d / 8 of tokens 2p and 2p + 1 side by side, so one 16-byte lane load carries its 8 dims
// of two keys (ops/reference.py kv8_physical is the host twin)
__device__ __forceinline__ int kv8_off(int t, int d) { return (((t >> 1) * 16 + (d >> 3)) * 2 + (t & 1)) * 8 + (d & 7); }
__device__ __forceinline__ float kv8_inv(float amax) { return amax > 0.f ? 448.0f / amax : 0.f; }

// Element offset of activation (m, k) in the fragment-major decode layout Xf[k/32][mt][64 lanes][8]
// (lane = 16 * ((k % 32) / 8) + m % 16): one MFMA B-fragment per (k-step, 16-row tile) is 1 KiB
// lane-linear.  8 consecutive k starting at a multiple of 8 are contiguous.
__device__ __forceinline__ size_t xf_off(int m, int k, int mt) {
  return ((((size_t)(k >> 5) * mt + (m >> 4)) * 64) + 16 * ((k & 31) >> 3) + (m & 15)) * 8 + (k & 7);
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

// Decode-GEMM epilogue extensions (RMSNorm folded into the GEMMs, no norm launches):
//  * rowss != null: X rows are the UN-normalised residual stream (the norm's gamma is folded into W at
//    load time), so every output row m is scaled by rsqrt(rowss[m] * inv_k + eps) -- rowss[m] = sum_k x^2
//    accumulated by the producing kernel.
//  * EPI_RES (splitk 1): h[m][n] += y (f32 residual, row stride ldh); xout = bf16(h) (fragment-major
//    with xmt row tiles when xmt > 0, else row-major [M][ldh]) for the next GEMM; ss_out[m] += sum over
//    this workgroup's columns of h^2 (one device-scope float atomic per row and workgroup).
#define EPI_RES 3

// Row sums of squares travel as Q24 fixed point in int64: integer atomics add exactly, so the sum (and every
// token decoded from it) is independent of the order in which the workgroups arrive -- float atomics made
// two identical requests in one batch diverge after a few tokens on a near-tied argmax.
#define LSA_Q24 16777216.0f
__device__ __forceinline__ long long ss_to_q24(float v) { return (long long)(v * LSA_Q24); }

__device__ __forceinline__ float epi_row_scale(const LsaEpi& ep, int m) {
  return ep.rowss ? rsqrtf((float)ep.rowss[m] * (1.0f / LSA_Q24) * ep.inv_k + ep.eps) : 1.0f;
}

//    With split-K (grid.y > 1) every split publishes its f32 partial write-through (sc1) into the
//    [splitk][M][N] slab buffer, takes a ticket, and the last arriver of the column sums the slabs with
//    sc1 loads and runs the epilogue (guide §6 G16 / MI355X_MICROARCH "Valid forms" table, row 1).
#define LSA_SC1_AUX 16  // buffer cache-policy aux bit: sc1 (write-through store / L1-bypassing load)

// EPI_RES for 4 consecutive columns n..n+3 of row m; returns sum of the new h^2 over them
__device__ __forceinline__ float epi_residual4(const LsaEpi& ep, int m, int n, f32x4_t v) {
  float* hp = ep.h + (size_t)m * ep.ldh + n;
  float4 hv = *reinterpret_cast<const float4*>(hp);
  hv.x += v[0]; hv.y += v[1]; hv.z += v[2]; hv.w += v[3];
  *reinterpret_cast<float4*>(hp) = hv;
  uint2 pk;
  pk.x = pack2bf(hv.x, hv.y);
  pk.y = pack2bf(hv.z, hv.w);
  *reinterpret_cast<uint2*>(ep.xout + (ep.xmt ? xf_off(m, n, ep.xmt) : (size_t)m * ep.ldh + n)) = pk;
  return hv.x * hv.x + hv.y * hv.y + hv.z * hv.z + hv.w * hv.w;
}

// n-block range of a skinny decode-GEMM workgroup (gemm.hip, gemm_fp4.hip): NB blocks each when NB divides the
// column count NBtot; otherwise (a ragged grid of ceil(NBtot / NB) workgroups) the column units -- P = 2 for the
// interleaved gate/up pairs of a SiLU epilogue -- are dealt as evenly as possible, cnt <= NB (7B gate_up at 32 rows:
// 688 pairs as 2-3 per workgroup on 230 CUs instead of 4 on 172).  Blocks i >= cnt re-load the workgroup's last block
// (an L2 hit, no branch in the weight stream) and are never stored.
template <int NB, int P>
__device__ __forceinline__ void skinny_nblocks(int NBtot, int& nb0, int& cnt) {
  nb0 = blockIdx.x * NB;
  cnt = NB;
  if (NBtot % NB) {
    const int units = NBtot / P, G = gridDim.x, base = units / G, rem = units % G, b = blockIdx.x;
    nb0 = (b * base + min(b, rem)) * P;
    cnt = (base + (b < rem ? 1 : 0)) * P;
  }
}

typedef __attribute__((address_space(1))) int lsa_g_i32;

// Split-K residual epilogue, called by every workgroup of a column with its reduced tile available
// through tile(m_index) -> (m, n, f32x4 partial) enumerations.  Returns true in the one workgroup that
// must finish the column (the last to arrive); the partials are then read back by res_slab_sum.
template <int NT>
__device__ __forceinline__ bool res_publish_and_ticket(const LsaEpi& ep, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 partial stores
  __syncthreads();
  if (threadIdx.x == 0)
    *s_flag = __hip_atomic_fetch_add((lsa_g_i32*)(ep.tickets) + blockIdx.x, 1, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.y - 1;
  __syncthreads();
  if (!*s_flag) return false;
  if (threadIdx.x == 0)
    __hip_atomic_store((lsa_g_i32*)(ep.tickets) + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__device__ __forceinline__ void res_store_partial(__amdgpu_buffer_rsrc_t rs, size_t elem, f32x4_t v) {
  const u32x4_t u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, rs, (int)(elem * 4), 0, LSA_SC1_AUX);
}

__device__ __forceinline__ f32x4_t res_slab_sum(__amdgpu_buffer_rsrc_t rs, size_t elem, size_t slab_elems, int nsplit) {
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  // unrolled so the split loads leave together (one memory round trip, not one per split)
#pragma unroll 8
  for (int sp = 0; sp < nsplit; ++sp) {
    const u32x4_t u = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((elem + sp * slab_elems) * 4), 0, LSA_SC1_AUX);
    s[0] += __uint_as_float(u[0]); s[1] += __uint_as_float(u[1]);
    s[2] += __uint_as_float(u[2]); s[3] += __uint_as_float(u[3]);
  }
  return s;
}

// Per-sequence split of the decode-attention context (attention.hip; the grid is sized for the longest context a
// captured graph can see; each sequence uses what its own length needs): <= unsplit_max blocks run unsplit (a split
// costs a combine pass, measured slower below ~256 keys, scripts/bench_attn.py), longer contexts use splits of
// chunk_blocks blocks, widened when the grid has fewer splits than that needs.
__device__ __forceinline__ void eff_split(int nblk, int chunk_blocks, int nsplit, int unsplit_max, int& ech, int& nse) {
  ech = nblk <= unsplit_max ? max(nblk, 1) : max(chunk_blocks, (nblk + nsplit - 1) / nsplit);
  nse = (nblk + ech - 1) / ech;
}

// Orderable 32-bit key of a float (larger float -> larger unsigned key).
__device__ __forceinline__ uint32_t float_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
  const uint32_t mask = (uint32_t)((int32_t)k >> 31);  // all ones iff the sign bit of the key is set
  return __uint_as_float(k ^ (~mask | 0x80000000u));
}
