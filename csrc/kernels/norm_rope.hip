// Residual-stream kernels (memory-bound, vectorised 16 B / lane everywhere):
//
//   lsa_add_rmsnorm   h[r] (+)= emb[ids[r]] | sum_s parts[s][r];  xn[m] = rmsnorm(h[r]) * w   (bf16 out)
//                     One kernel covers: embedding gather + first input norm, the split-K combine of
//                     the O / down projections (f32 slabs written by gemm EPI_F32) + residual add +
//                     next norm, and the final norm over gathered last-token rows (row_idx).
//   lsa_rope_append   rotary embedding (rotate-half convention, cos/sin table from the host) of the
//                     q and k heads of the fused QKV output + paged KV-cache append of k and v.
//   lsa_silu_mul      standalone silu(g) * u for non-interleaved inputs.
#include "common.h"

// One workgroup per output row, one 8-wide vector per thread and pass (blockDim = D/8 rounded up to a
// wave when D <= 8192).  NP = number of split-K slabs known at compile time, so every slab load of a
// thread is issued before the first add (the kernel is pure latency at decode sizes); NP < 0 = runtime.
template <int NP, int VPT>
__global__ __launch_bounds__(1024) void add_rmsnorm_kernel(float* __restrict__ h, const float* __restrict__ parts,
                                                           int nparts, size_t part_stride, const int* __restrict__ ids,
                                                           const uint16_t* __restrict__ emb,
                                                           const int* __restrict__ row_idx, int write_h,
                                                           const uint16_t* __restrict__ w, float eps,
                                                           uint16_t* __restrict__ xn, int D, int xf_mt,
                                                           long long* __restrict__ ss_out, int ss_ld, int ss_nzero,
                                                           uint8_t* __restrict__ x8, float* __restrict__ sx8) {
  __shared__ float red[16];
  const int m = blockIdx.x;
  const int r = row_idx ? row_idx[m] : m;
  float* hr = h + (size_t)r * D;
  const int nt = blockDim.x;
  float v[VPT][8];
  float ss = 0.f;
  uint4 wq[VPT];  // norm weights: requested up front, they do not depend on the reduction
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int c = (threadIdx.x + q * nt) * 8;
    wq[q] = c < D ? *reinterpret_cast<const uint4*>(w + c) : make_uint4(0u, 0u, 0u, 0u);
  }
  auto add8 = [](float* x, const float* p) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    x[0] += a.x; x[1] += a.y; x[2] += a.z; x[3] += a.w;
    x[4] += b.x; x[5] += b.y; x[6] += b.z; x[7] += b.w;
  };
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int c = (threadIdx.x + q * nt) * 8;
    if (c < D) {
      if (ids) {
        unpack8(*reinterpret_cast<const uint4*>(emb + (size_t)ids[r] * D + c), v[q]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[q][j] = 0.f;
        add8(v[q], hr + c);
      }
      const float* p = parts + (size_t)r * D + c;
      if constexpr (NP >= 0) {
        float t[NP > 0 ? NP : 1][8];
#pragma unroll
        for (int s = 0; s < NP; ++s) {
#pragma unroll
          for (int j = 0; j < 8; ++j) t[s][j] = 0.f;
          add8(t[s], p + s * part_stride);
        }
#pragma unroll
        for (int s = 0; s < NP; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[q][j] += t[s][j];
      } else {
        for (int s = 0; s < nparts; ++s) add8(v[q], p + s * part_stride);
      }
      if (write_h) {
        *reinterpret_cast<float4*>(hr + c) = make_float4(v[q][0], v[q][1], v[q][2], v[q][3]);
        *reinterpret_cast<float4*>(hr + c + 4) = make_float4(v[q][4], v[q][5], v[q][6], v[q][7]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[q][j] * v[q][j];
    }
  }
  const float tot = block_sum(ss, red);
  if (ss_out) {
    // raw mode (norm folded into the next GEMMs): xn = bf16(h) un-normalised, ss_out[m] = sum h^2, and
    // the following ss_nzero accumulators of this row (rows ss_ld apart) are zeroed for their producers
    if (threadIdx.x == 0) ss_out[m] = ss_to_q24(tot);
    for (int k = threadIdx.x; k < ss_nzero; k += nt) ss_out[(size_t)(k + 1) * ss_ld + m] = 0;
  }
  const float inv = ss_out ? 1.0f : rsqrtf(tot / (float)D + eps);
  float amax = 0.f;
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int c = (threadIdx.x + q * nt) * 8;
    if (c < D) {
      float wf[8];
      unpack8(wq[q], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[q][j] = ss_out ? v[q][j] : v[q][j] * inv * wf[j];
        amax = fmaxf(amax, fabsf(v[q][j]));
      }
      if (xn) *reinterpret_cast<uint4*>(xn + (xf_mt ? xf_off(m, c, xf_mt) : (size_t)m * D + c)) = pack8(v[q]);
    }
  }
  if (x8) {
    // W8A8 decode input: the row (as the GEMM will see it) in OCP e4m3 with a per-row scale amax / 448,
    // straight into the xf8 fragment layout of the fp8-activation GEMM (gemm_fp8a.hip)
    amax = block_max(amax, red);
    const float sc = fmaxf(amax, 1e-30f) * (1.0f / 448.f);
    if (threadIdx.x == 0) sx8[m] = sc;
    const float isc = 1.0f / sc;
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int c = (threadIdx.x + q * nt) * 8;
      if (c < D) *reinterpret_cast<uint2*>(x8 + xf8_off(m, c, xf_mt)) = pack8_fp8(v[q], isc);
    }
  }
}

template <int VPT>
static void launch_rmsnorm(int np, int rows, int nt, hipStream_t s, float* h, const float* parts, size_t ps,
                           const int* ids, const uint16_t* e, const int* row_idx, int write_h, const uint16_t* w,
                           float eps, uint16_t* o, int D, int xf_mt, long long* ss_out, int ss_ld, int ss_nzero,
                           uint8_t* x8, float* sx8) {
#define LSA_RN(NP)                                                                                         \
  hipLaunchKernelGGL((add_rmsnorm_kernel<NP, VPT>), dim3(rows), dim3(nt), 0, s, h, parts, np, ps, ids, e, \
                     row_idx, write_h, w, eps, o, D, xf_mt, ss_out, ss_ld, ss_nzero, x8, sx8)
  switch (parts ? np : 0) {
    case 0: LSA_RN(0); break;
    case 1: LSA_RN(1); break;
    case 2: LSA_RN(2); break;
    case 3: LSA_RN(3); break;
    case 4: LSA_RN(4); break;
    case 6: LSA_RN(6); break;
    case 8: LSA_RN(8); break;
    default: LSA_RN(-1); break;
  }
#undef LSA_RN
}

// Prefill RMSNorm of h into the fragment-major layout (the stream-K GEMM's X, ops.PREFILL_XF), D <= 4096: one
// workgroup per 8 rows (half a 16-row tile).  Pass 1: wave w reads row w with whole-line loads, sums its squares
// (DPP / permlane wave sum) and parks the f32 row in LDS.  Pass 2: lane (s, g, r) = (l >> 5, (l >> 3) & 3, l & 7)
// takes row r's columns 32 ks + 8 g .. + 7 of k-step ks = 2 i + s, scales them and stores 16 B at its fragment lane
// 16 g + 8 (tile half) + r: per instruction four 128-B runs in each of two fragments, all whole lines.  The
// row-per-workgroup kernel above writes the layout as 16-B pieces of 64 different lines per instruction (3B 2k rows:
// 18.4 us vs 9.7 row-major); a 16-row-tile kernel with the fragment mapping in both passes ran 16-21 us at every
// size (1024 threads on rows / 16 CUs, half-line loads; scripts/bench_norm_xf.py).
#define LSA_XFN_DMAX 4096
__global__ __launch_bounds__(512) void rmsnorm_xf_kernel(const float* __restrict__ h, const uint16_t* __restrict__ w,
                                                        float eps, uint16_t* __restrict__ xn, int M, int D, int mt) {
  __shared__ __attribute__((aligned(16))) float img[8 * (LSA_XFN_DMAX + 4)];
  __shared__ float rinv[8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x, m = b * 8 + wv, ld = D + 4;
  float ss = 0.f;
  if (m < M) {
    const float4* hr = reinterpret_cast<const float4*>(h + (size_t)m * D);
#pragma unroll 4
    for (int c4 = lane; c4 < D / 4; c4 += 64) {
      const float4 a = hr[c4];
      ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
      *reinterpret_cast<float4*>(&img[wv * ld + 4 * c4]) = a;
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) rinv[wv] = m < M ? rsqrtf(ss / (float)D + eps) : 0.f;
  __syncthreads();
  const int s = lane >> 5, g = (lane >> 3) & 3, r = lane & 7, KS = D >> 5;
  const int rb = b >> 1, fl = 16 * g + 8 * (b & 1) + r;
  const float inv = rinv[r];
  for (int i = wv; 2 * i < KS; i += 8) {
    const int ks = 2 * i + s;
    if (ks < KS) {
      const int c = 32 * ks + 8 * g;
      const float4 a = *reinterpret_cast<const float4*>(&img[r * ld + c]);
      const float4 q = *reinterpret_cast<const float4*>(&img[r * ld + c + 4]);
      float wf[8];
      unpack8(*reinterpret_cast<const uint4*>(w + c), wf);
      float v[8] = {a.x, a.y, a.z, a.w, q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * inv * wf[j];
      *reinterpret_cast<uint4*>(xn + ((size_t)(ks * mt + rb) * 64 + fl) * 8) = pack8(v);
    }
  }
}

// minimum rows for rmsnorm_xf_kernel (below it the row-per-workgroup kernel writes the layout);
// lsa_rmsnorm_xf_tile_min sets it (A/B knob, scripts/bench_norm_xf.py)
static int g_xf_tile_min = 512;
extern "C" void lsa_rmsnorm_xf_tile_min(int rows) { g_xf_tile_min = rows; }

// x8 / sx8 (optional): also write the output rows as fp8 e4m3 in the xf8 layout of xf_mt row tiles with a
// per-row scale (the W8A8 decode GEMM input); xn may then be null (no bf16 copy)
extern "C" int lsa_add_rmsnorm(float* h, const float* parts, int nparts, long part_stride, const int* ids,
                               const void* emb, const int* row_idx, int write_h, const void* w, float eps, void* xn,
                               int rows, int D, int xf_mt, long long* ss_out, int ss_ld, int ss_nzero, void* x8,
                               float* sx8, hipStream_t s) {
  if (D % 8 != 0 || rows <= 0) return -1;
  if (xf_mt && (D % 32 != 0 || rows > 16 * xf_mt)) return -3;
  if (ss_out && (row_idx || ss_ld < rows || ss_nzero < 0)) return -4;
  if (x8 && (!sx8 || !xf_mt || D % 128 != 0 || row_idx)) return -5;
  if (!xn && !x8) return -6;
  if (xf_mt && rows > 64 && rows >= g_xf_tile_min && D <= LSA_XFN_DMAX && !(parts && nparts) && !ids && !row_idx &&
      !ss_out && !x8 && xn) {
    // prefill norm of h alone into the fragment-major layout (write_h is a no-op without parts / ids)
    hipLaunchKernelGGL(rmsnorm_xf_kernel, dim3((rows + 7) / 8), dim3(512), 0, s, h,
                       reinterpret_cast<const uint16_t*>(w), eps, reinterpret_cast<uint16_t*>(xn), rows, D, xf_mt);
    return (int)hipGetLastError();
  }
  const int vec = D / 8;
  const uint16_t* e = reinterpret_cast<const uint16_t*>(emb);
  const uint16_t* ww = reinterpret_cast<const uint16_t*>(w);
  uint16_t* o = reinterpret_cast<uint16_t*>(xn);
  uint8_t* q8 = reinterpret_cast<uint8_t*>(x8);
  if (vec <= 1024) {
    launch_rmsnorm<1>(nparts, rows, (vec + 63) / 64 * 64, s, h, parts, (size_t)part_stride, ids, e, row_idx, write_h,
                      ww, eps, o, D, xf_mt, ss_out, ss_ld, ss_nzero, q8, sx8);
  } else if (vec <= 4096) {
    launch_rmsnorm<4>(nparts, rows, 1024, s, h, parts, (size_t)part_stride, ids, e, row_idx, write_h, ww, eps, o, D, xf_mt,
                      ss_out, ss_ld, ss_nzero, q8, sx8);
  } else {
    return -2;
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Wide raw residual add (decode step with the RMSNorm gammas folded into the next GEMMs, which scale their
// output rows by rsqrt(ss / D + eps)):  h[m] += sum_s parts[s][m];  xn[m] = bf16(h[m]) (fragment-major when
// xf_mt);  ss_out[m] += sum_c h[m][c]^2 (Q24 int64 atomics, so the total does not depend on arrival order).
// ss_out must be zero on entry (the step's embedding launch zeroes every layer's accumulator).
// One WAVE per 512-column slice of a row: grid (D / 512, rows) of one-wave workgroups (7B batch 32: 256; 3B
// batch 1: 6), every lane's slab loads issued before the first add, a shuffle reduction and one atomic per
// wave -- no block-wide reduction, a single dependent memory round trip.  Replaces add_rmsnorm's one
// 512-thread workgroup per row (whose LDS reduction and per-row serial chain are the decode-step norm cost).
template <int NP>
__global__ __launch_bounds__(64) void res_add_ss_kernel(float* __restrict__ h, const float* __restrict__ parts,
                                                        int nparts, size_t part_stride, uint16_t* __restrict__ xn,
                                                        int D, int xf_mt, long long* __restrict__ ss_out) {
  const int m = blockIdx.y;
  const int c = (blockIdx.x * 64 + threadIdx.x) * 8;
  float ss = 0.f;
  if (c < D) {
    float* hr = h + (size_t)m * D + c;
    const float* p = parts + (size_t)m * D + c;
    float v[8];
    {
      const float4 a = *reinterpret_cast<const float4*>(hr);
      const float4 b = *reinterpret_cast<const float4*>(hr + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    if constexpr (NP > 0) {
      float4 t[NP][2];
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        t[s][0] = *reinterpret_cast<const float4*>(p + s * part_stride);
        t[s][1] = *reinterpret_cast<const float4*>(p + s * part_stride + 4);
      }
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        v[0] += t[s][0].x; v[1] += t[s][0].y; v[2] += t[s][0].z; v[3] += t[s][0].w;
        v[4] += t[s][1].x; v[5] += t[s][1].y; v[6] += t[s][1].z; v[7] += t[s][1].w;
      }
    } else {
      for (int s = 0; s < nparts; ++s) {
        const float4 a = *reinterpret_cast<const float4*>(p + s * part_stride);
        const float4 b = *reinterpret_cast<const float4*>(p + s * part_stride + 4);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
    }
    *reinterpret_cast<float4*>(hr) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(hr + 4) = make_float4(v[4], v[5], v[6], v[7]);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    *reinterpret_cast<uint4*>(xn + (xf_mt ? xf_off(m, c, xf_mt) : (size_t)m * D + c)) = pack8(v);
  }
  ss = wave_sum(ss);
  if (threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(ss_out) + m, (unsigned long long)ss_to_q24(ss));
}

extern "C" int lsa_res_add_ss(float* h, const float* parts, int nparts, long part_stride, void* xn, int rows, int D,
                              int xf_mt, long long* ss_out, hipStream_t s) {
  if (D % 8 != 0 || rows <= 0 || nparts < 0 || !ss_out || !xn) return -1;
  if (xf_mt && (D % 32 != 0 || rows > 16 * xf_mt)) return -3;
  const dim3 grid((D / 8 + 63) / 64, rows);
  uint16_t* o = reinterpret_cast<uint16_t*>(xn);
#define LSA_RS(NP) \
  hipLaunchKernelGGL((res_add_ss_kernel<NP>), grid, dim3(64), 0, s, h, parts, nparts, (size_t)part_stride, o, D, xf_mt, ss_out)
  switch (parts ? nparts : 0) {
    case 0: LSA_RS(0); break;
    case 1: LSA_RS(1); break;
    case 2: LSA_RS(2); break;
    case 3: LSA_RS(3); break;
    case 4: LSA_RS(4); break;
    case 6: LSA_RS(6); break;
    case 8: LSA_RS(8); break;
    default: LSA_RS(-1); break;
  }
#undef LSA_RS
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// RoPE + paged KV append.  qkv: [T, (H + 2*Hkv) * 128]; q_out: [T, H, 128];
// cache: [nblk, Hkv, 64, 128]; token t of sequence seq(t) at position pos(t) goes to
// block_tables[seq * max_blocks + pos / 64], slot pos % 64.  cos/sin: [max_pos, 64] f32.
// One workgroup per token; each thread rotates 4 (d, d+64) pairs (8 B loads of both halves).
// ------------------------------------------------------------------------------------------------
// KV8: fp8 cache -- kc / vc are e4m3 bytes and every (token, kv-head) row is stored as e4m3(x * 448 / amax)
// with amax / 448 in ks / vs [nblk, Hkv, 64] (common.h kv8_inv); the 16 threads of a head (aligned lanes)
// reduce the row's amax with xor shuffles.
template <int NP, bool KV8 = false>  // NP = 0: bf16 qkv rows; NP > 0: that many f32 split-K slabs; NP < 0: runtime
__global__ __launch_bounds__(1024) void rope_append_kernel(const uint16_t* __restrict__ qkv, const float* __restrict__ qkv_parts,
                                                          int nparts, size_t part_stride, const int* __restrict__ pos,
                                                          const int* __restrict__ tok_seq,
                                                          const int* __restrict__ block_tables, int max_blocks,
                                                          const float* __restrict__ cos_t,
                                                          const float* __restrict__ sin_t, uint16_t* __restrict__ q_out,
                                                          uint16_t* __restrict__ kc, uint16_t* __restrict__ vc,
                                                          float* __restrict__ ks, float* __restrict__ vs, int H,
                                                          int Hkv) {
  constexpr int D = 128;
  const int t = blockIdx.x;
  const int p = pos[t];
  const int seq = tok_seq ? tok_seq[t] : t;
  const int blk = block_tables[(size_t)seq * max_blocks + (p >> 6)];
  const int off = p & 63;
  const size_t row_off = (size_t)t * (H + 2 * Hkv) * D;
  const uint16_t* row = qkv + row_off;
  const float* prow = qkv_parts + row_off;
  // 4 consecutive values of the fused q|k|v row: bf16 row or the sum of f32 split-K slabs
  auto load4 = [&](int off, float* v) {
    if constexpr (NP > 0) {
      float4 b[NP];
#pragma unroll
      for (int s = 0; s < NP; ++s) b[s] = *reinterpret_cast<const float4*>(prow + s * part_stride + off);
      float4 a = b[0];
#pragma unroll
      for (int s = 1; s < NP; ++s) { a.x += b[s].x; a.y += b[s].y; a.z += b[s].z; a.w += b[s].w; }
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else if constexpr (NP < 0) {
      float4 a = *reinterpret_cast<const float4*>(prow + off);
      for (int s = 1; s < nparts; ++s) {
        const float4 b = *reinterpret_cast<const float4*>(prow + s * part_stride + off);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else {
      const uint2 u = *reinterpret_cast<const uint2*>(row + off);
      v[0] = bf2f(u.x & 0xffff); v[1] = bf2f(u.x >> 16); v[2] = bf2f(u.y & 0xffff); v[3] = bf2f(u.y >> 16);
    }
  };
  const float* cr = cos_t + (size_t)p * (D / 2);
  const float* sr = sin_t + (size_t)p * (D / 2);
  // rotation work items: (head, quad) with quad = 4 consecutive d in [0, 64)
  const int nrot = (H + Hkv) * 16;
  for (int it = threadIdx.x; it < nrot; it += blockDim.x) {
    const int hd = it >> 4, d0 = (it & 15) * 4;
    float x0[4], x1[4];
    load4(hd * D + d0, x0);
    load4(hd * D + d0 + 64, x1);
    const float4 c = *reinterpret_cast<const float4*>(cr + d0);
    const float4 s = *reinterpret_cast<const float4*>(sr + d0);
    const float cc[4] = {c.x, c.y, c.z, c.w}, sn[4] = {s.x, s.y, s.z, s.w};
    float y0[4], y1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      y0[j] = x0[j] * cc[j] - x1[j] * sn[j];
      y1[j] = x1[j] * cc[j] + x0[j] * sn[j];
    }
    if (KV8 && hd >= H) {  // (uniform over the 16 lanes of a head)
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) a = fmaxf(a, fmaxf(fabsf(y0[j]), fabsf(y1[j])));
      a = lsa_row16_max(a);
      const float inv = kv8_inv(a);
      const size_t r8 = ((size_t)blk * Hkv + (hd - H)) * 64 + off;
      uint8_t* tile = reinterpret_cast<uint8_t*>(kc) + (r8 - off) * D;  // token-pair order (common.h kv8_off)
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(y0[0] * inv, y0[1] * inv, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(y0[2] * inv, y0[3] * inv, lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(y1[0] * inv, y1[1] * inv, 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(y1[2] * inv, y1[3] * inv, hi, true);
      *reinterpret_cast<int*>(tile + kv8_off(off, d0)) = lo;
      *reinterpret_cast<int*>(tile + kv8_off(off, d0 + 64)) = hi;
      if (d0 == 0) ks[r8] = a * LSA_KV8_RMAX;
      continue;
    }
    uint2 olo, ohi;
    olo.x = pack2bf(y0[0], y0[1]); olo.y = pack2bf(y0[2], y0[3]);
    ohi.x = pack2bf(y1[0], y1[1]); ohi.y = pack2bf(y1[2], y1[3]);
    uint16_t* dst;
    if (hd < H) {
      dst = q_out + ((size_t)t * H + hd) * D;
    } else {
      dst = kc + (((size_t)blk * Hkv + (hd - H)) * 64 + off) * D;
    }
    *reinterpret_cast<uint2*>(dst + d0) = olo;
    *reinterpret_cast<uint2*>(dst + d0 + 64) = ohi;
  }
  // v copy: Hkv * 16 chunks of 8 bf16
  for (int it = threadIdx.x; it < Hkv * 16; it += blockDim.x) {
    const int hv = it >> 4, c = (it & 15) * 8;
    if constexpr (KV8) {
      float f[8];
      if constexpr (NP != 0) {
        load4((H + Hkv + hv) * D + c, f);
        load4((H + Hkv + hv) * D + c + 4, f + 4);
      } else {
        unpack8(*reinterpret_cast<const uint4*>(row + (H + Hkv + hv) * D + c), f);
      }
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) a = fmaxf(a, fabsf(f[j]));
      a = lsa_row16_max(a);
      const size_t r8 = ((size_t)blk * Hkv + hv) * 64 + off;
      *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(vc) + (r8 - off) * D + kv8_off(off, c)) = pack8_fp8(f, kv8_inv(a));
      if (c == 0) vs[r8] = a * LSA_KV8_RMAX;
      continue;
    }
    uint4 v;
    if constexpr (NP != 0) {
      float f[8];
      load4((H + Hkv + hv) * D + c, f);
      load4((H + Hkv + hv) * D + c + 4, f + 4);
      v = pack8(f);
    } else {
      v = *reinterpret_cast<const uint4*>(row + (H + Hkv + hv) * D + c);
    }
    *reinterpret_cast<uint4*>(vc + (((size_t)blk * Hkv + hv) * 64 + off) * D + c) = v;
  }
}

extern "C" int lsa_rope_append(const void* qkv, const float* qkv_parts, int nparts, long part_stride, const int* pos, const int* tok_seq, const int* block_tables,
                               int max_blocks, const float* cos_t, const float* sin_t, void* q_out, void* kc, void* vc,
                               float* ks, float* vs, int T, int H, int Hkv, hipStream_t s) {
  if (T <= 0) return 0;
  if ((ks == nullptr) != (vs == nullptr)) return -5;
  // one rotation item per thread where possible (the decode case is latency-bound)
  const int items = (H + Hkv) * 16;
  const int nt = items >= 1024 ? 1024 : (items + 63) / 64 * 64;
  const uint16_t* q16 = reinterpret_cast<const uint16_t*>(qkv);
  uint16_t* qo = reinterpret_cast<uint16_t*>(q_out);
  uint16_t* k16 = reinterpret_cast<uint16_t*>(kc);
  uint16_t* v16 = reinterpret_cast<uint16_t*>(vc);
#define LSA_RA(NP)                                                                                                   \
  do {                                                                                                                \
    if (ks)                                                                                                           \
      hipLaunchKernelGGL((rope_append_kernel<NP, true>), dim3(T), dim3(nt), 0, s, q16, qkv_parts, nparts,             \
                         (size_t)part_stride, pos, tok_seq, block_tables, max_blocks, cos_t, sin_t, qo, k16, v16, ks, vs, \
                         H, Hkv);                                                                                     \
    else                                                                                                              \
      hipLaunchKernelGGL((rope_append_kernel<NP>), dim3(T), dim3(nt), 0, s, q16, qkv_parts, nparts,                   \
                         (size_t)part_stride, pos, tok_seq, block_tables, max_blocks, cos_t, sin_t, qo, k16, v16, ks, vs, \
                         H, Hkv);                                                                                     \
  } while (0)
  switch (qkv_parts ? nparts : 0) {
    case 0: LSA_RA(0); break;
    case 1: LSA_RA(1); break;
    case 2: LSA_RA(2); break;
    case 3: LSA_RA(3); break;
    case 4: LSA_RA(4); break;
    case 8: LSA_RA(8); break;
    default: LSA_RA(-1); break;
  }
#undef LSA_RA
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void silu_mul_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u,
                                                       uint16_t* __restrict__ o, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float a[8], b[8], c[8];
    unpack8(reinterpret_cast<const uint4*>(g)[i], a);
    unpack8(reinterpret_cast<const uint4*>(u)[i], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = silu(a[j]) * b[j];
    reinterpret_cast<uint4*>(o)[i] = pack8(c);
  }
}

extern "C" int lsa_silu_mul(const void* g, const void* u, void* o, long n, hipStream_t s) {
  if (n % 8) return -1;
  const long n8 = n / 8;
  const long gl = (n8 + 255) / 256;
  const int grid = (int)(gl < 2048 ? gl : 2048);
  hipLaunchKernelGGL(silu_mul_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(g),
                     reinterpret_cast<const uint16_t*>(u), reinterpret_cast<uint16_t*>(o), n8);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// silu(gate) * up from f32 split-K slabs of the interleaved gate_up projection:
// parts [S][M][2F], column block 2j = gate rows 16j..16j+15, block 2j+1 = up rows 16j..  -> out [M][F] bf16
__global__ __launch_bounds__(256) void silu_parts_kernel(const float* __restrict__ parts, int nparts, size_t stride,
                                                         int M, int F, uint16_t* __restrict__ out) {
  const long total4 = (long)M * F / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 4;
    const int m = (int)(e / F), f = (int)(e - (long)m * F);
    const int blk = f >> 4, off = f & 15;
    const size_t gi = (size_t)m * 2 * F + (size_t)(2 * blk) * 16 + off;
    float4 gs = *reinterpret_cast<const float4*>(parts + gi);
    float4 us = *reinterpret_cast<const float4*>(parts + gi + 16);
    for (int s = 1; s < nparts; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(parts + s * stride + gi);
      const float4 b = *reinterpret_cast<const float4*>(parts + s * stride + gi + 16);
      gs.x += a.x; gs.y += a.y; gs.z += a.z; gs.w += a.w;
      us.x += b.x; us.y += b.y; us.z += b.z; us.w += b.w;
    }
    uint2 pk;
    pk.x = pack2bf(silu(gs.x) * us.x, silu(gs.y) * us.y);
    pk.y = pack2bf(silu(gs.z) * us.z, silu(gs.w) * us.w);
    *reinterpret_cast<uint2*>(out + e) = pk;
  }
}

extern "C" int lsa_silu_parts(const float* parts, int nparts, long part_stride, int M, int F, void* out,
                              hipStream_t s) {
  if (F % 16) return -1;
  const long total4 = (long)M * F / 4;
  const long gl = (total4 + 255) / 256;
  hipLaunchKernelGGL(silu_parts_kernel, dim3((unsigned)(gl < 4096 ? gl : 4096)), dim3(256), 0, s, parts, nparts,
                     (size_t)part_stride, M, F, reinterpret_cast<uint16_t*>(out));
  return (int)hipGetLastError();
}

// Infinity-Cache warm-up: stream up to four byte ranges through the memory hierarchy with plain (allocating)
// loads and no stores, so a later kernel that reads the same lines is served from the 256 MiB die-level cache
// instead of HBM.  Launched on a side stream of the captured decode step, concurrent with latency-bound work
// (attention, residual adds, kernel ramps) during which HBM would otherwise idle.  The loaded values feed an
// empty asm so the loads are kept without writing anything.
struct LsaRanges {
  const uint4* p[4];
  long n[4];  // 16-byte units
};

__global__ __launch_bounds__(256) void prefetch_kernel(LsaRanges r) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const long stride = (long)gridDim.x * 256;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4* p = r.p[k];
    const long n = r.n[k];
    long i = blockIdx.x * 256L + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
      acc.x ^= a.x ^ b.x ^ c.x ^ d.x;
      acc.y ^= a.y ^ b.y ^ c.y ^ d.y;
    }
    for (; i < n; i += stride) acc.x ^= p[i].x;
  }
  asm volatile("" ::"v"(acc.x), "v"(acc.y));
}

extern "C" int lsa_prefetch(const void* const* ptrs, const long* bytes, int nr, int wgs, hipStream_t s) {
  if (nr < 1 || nr > 4 || wgs < 1) return -1;
  LsaRanges r{};
  for (int k = 0; k < nr; ++k) {
    if (reinterpret_cast<uintptr_t>(ptrs[k]) % 16 || bytes[k] < 0) return -2;
    r.p[k] = reinterpret_cast<const uint4*>(ptrs[k]);
    r.n[k] = bytes[k] / 16;
  }
  hipLaunchKernelGGL(prefetch_kernel, dim3(wgs), dim3(256), 0, s, r);
  return (int)hipGetLastError();
}

// silu(gate) * up from the bf16 output of the vendor gate_up GEMM (prefill): y [M][2F] bf16 with gate / up rows
// interleaved per 16 columns as packed -> out [M][F] bf16.  Eight outputs per thread (one 16-byte gate and one
// 16-byte up load), so the pass streams 3 bytes per output at full width.
__global__ __launch_bounds__(256) void silu_bf16_kernel(const uint16_t* __restrict__ y, int M, int F,
                                                        uint16_t* __restrict__ out) {
  const long total8 = (long)M * F / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total8; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    const int m = (int)(e / F), f = (int)(e - (long)m * F);
    const int blk = f >> 4, off = f & 15;
    const size_t gi = (size_t)m * 2 * F + (size_t)(2 * blk) * 16 + off;
    const uint4 g = *reinterpret_cast<const uint4*>(y + gi);
    const uint4 u = *reinterpret_cast<const uint4*>(y + gi + 16);
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, uw[4] = {u.x, u.y, u.z, u.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = pack2bf(silu(bf2f(gw[j] & 0xffffu)) * bf2f(uw[j] & 0xffffu), silu(bf2f(gw[j] >> 16)) * bf2f(uw[j] >> 16));
    *reinterpret_cast<uint4*>(out + e) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

extern "C" int lsa_silu_bf16(const void* y, int M, int F, void* out, hipStream_t s) {
  if (F % 16 || M <= 0) return -1;
  const long total8 = (long)M * F / 8;
  const long gl = (total8 + 255) / 256;
  hipLaunchKernelGGL(silu_bf16_kernel, dim3((unsigned)(gl < 8192 ? gl : 8192)), dim3(256), 0, s,
                     reinterpret_cast<const uint16_t*>(y), M, F, reinterpret_cast<uint16_t*>(out));
  return (int)hipGetLastError();
}
