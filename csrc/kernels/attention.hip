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
//                        (o, m, l) partial merged by attn_combine_kernel.
//   attn_prefill_kernel  causal flash attention for (chunked) prefill of packed variable-length
//                        sequences, MFMA 16x16x32 bf16.  4 waves x 16 query rows per workgroup; K/V tiles
//                        of 64 keys staged through LDS (register staging, issue-early / write-late);
//                        S^T = K Q^T so each lane owns one query row (softmax max over 16 values +
//                        2 xor shuffles); P stays in registers and feeds the PV MFMA as the A operand;
//                        V is read as the B operand with ds_read_b64_tr_b16 (hardware transpose) from
//                        an XOR-swizzled image (conflict-free per 32-lane half).
#include "common.h"

#define LSA_NEG (-1.0e30f)

template <int G>
__global__ __launch_bounds__(256) void attn_decode_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                          const uint16_t* __restrict__ vc,
                                                          const int* __restrict__ block_tables, int max_blocks,
                                                          const int* __restrict__ pos, int Hkv, float scale_log2,
                                                          int chunk_blocks, int nsplit, uint16_t* __restrict__ out,
                                                          float* __restrict__ opart, float* __restrict__ mlpart,
                                                          int xf_mt) {
  constexpr int D = 128;
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int H = Hkv * G;
  const int tid = threadIdx.x;
  const int lg = tid >> 4, li = tid & 15, wv = tid >> 6;
  const int ctx = pos[b] + 1;
  const int nblk = (ctx + 63) >> 6;
  const int blk0 = split * chunk_blocks;
  const int blk1 = min(nblk, blk0 + chunk_blocks);

  float qf[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint4 v = *reinterpret_cast<const uint4*>(q + ((size_t)(b * H + hk * G + g)) * D + li * 8);
    unpack8(v, qf[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[g][j] *= scale_log2;
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = LSA_NEG;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
  }

  const int* bt = block_tables + (size_t)b * max_blocks;
  // K/V of block blk+1 are in flight while block blk is scored (two register sets, static names)
  uint4 kA[4], vA[4], kB[4], vB[4];
  auto fetch = [&](uint4 (&kr)[4], uint4 (&vr)[4], int blk) {
    const size_t base = ((size_t)bt[blk] * Hkv + hk) * 64 * D;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tok = wv * 16 + u * 4 + (lg & 3);
      kr[u] = *reinterpret_cast<const uint4*>(kc + base + tok * D + li * 8);
      vr[u] = *reinterpret_cast<const uint4*>(vc + base + tok * D + li * 8);
    }
  };
  auto score = [&](const uint4 (&kr)[4], const uint4 (&vr)[4], int blk) {
    float s[4][G];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float kf[8];
      unpack8(kr[u], kf);
      const bool valid = (blk * 64 + wv * 16 + u * 4 + (lg & 3)) < ctx;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d = fmaf(qf[g][j], kf[j], d);
        d += __shfl_xor(d, 8, 64);
        d += __shfl_xor(d, 4, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 1, 64);
        s[u][g] = valid ? d : LSA_NEG;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mx = fmaxf(fmaxf(s[0][g], s[1][g]), fmaxf(s[2][g], s[3][g]));
      const float mn = fmaxf(m[g], mx);
      const float alpha = exp2f(m[g] - mn);
      m[g] = mn;
      float p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) p[u] = exp2f(s[u][g] - mn);
      l[g] = l[g] * alpha + (p[0] + p[1]) + (p[2] + p[3]);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] *= alpha;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float vf[8];
        unpack8(vr[u], vf);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[g][j] = fmaf(p[u], vf[j], o[g][j]);
      }
    }
  };
  if (blk0 < blk1) {
    fetch(kA, vA, blk0);
    int blk = blk0;
    for (; blk + 1 < blk1; blk += 2) {
      fetch(kB, vB, blk + 1);
      __builtin_amdgcn_sched_barrier(0);
      score(kA, vA, blk);
      __builtin_amdgcn_sched_barrier(0);
      fetch(kA, vA, min(blk + 2, blk1 - 1));
      __builtin_amdgcn_sched_barrier(0);
      score(kB, vB, blk + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (blk < blk1) score(kA, vA, blk);
  }

  // merge the 16 lane groups
  __shared__ float sm[16][G], sl[16][G];
  __shared__ __attribute__((aligned(16))) float so[16][G][D];
  if (li == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      sm[lg][g] = m[g];
      sl[lg][g] = l[g];
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    *reinterpret_cast<float4*>(&so[lg][g][li * 8]) = make_float4(o[g][0], o[g][1], o[g][2], o[g][3]);
    *reinterpret_cast<float4*>(&so[lg][g][li * 8 + 4]) = make_float4(o[g][4], o[g][5], o[g][6], o[g][7]);
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int g = e / D, d = e % D;
    float M = LSA_NEG;
#pragma unroll
    for (int k = 0; k < 16; ++k) M = fmaxf(M, sm[k][g]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float wgt = exp2f(sm[k][g] - M);
      L += sl[k][g] * wgt;
      O += so[k][g][d] * wgt;
    }
    const int h = hk * G + g;
    if (nsplit == 1) {
      out[xf_mt ? xf_off(b, h * D + d, xf_mt) : ((size_t)b * H + h) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const size_t pi = ((size_t)b * H + h) * nsplit + split;
      opart[pi * D + d] = O;
      if (d == 0) {
        mlpart[pi * 2] = M;
        mlpart[pi * 2 + 1] = L;
      }
    }
  }
}

// merge the split-KV partials of one (sequence, head): the split maxima / weights go through LDS once,
// then every thread sums its output dim over the splits with independent (pipelined) loads
__global__ __launch_bounds__(128) void attn_combine_kernel(const float* __restrict__ opart,
                                                           const float* __restrict__ mlpart, int nsplit,
                                                           uint16_t* __restrict__ out, int H, int xf_mt) {
  __shared__ float wts[256];
  __shared__ float red[2];
  const int bh = blockIdx.x, d = threadIdx.x;
  const float* ml = mlpart + (size_t)bh * nsplit * 2;
  float mloc = LSA_NEG;
  for (int s = d; s < nsplit; s += 128) mloc = fmaxf(mloc, ml[2 * s]);
  mloc = wave_max(mloc);
  if ((d & 63) == 0) red[d >> 6] = mloc;
  __syncthreads();
  const float M = fmaxf(red[0], red[1]);
  float lloc = 0.f;
  for (int s = d; s < nsplit; s += 128) {
    const float w = exp2f(ml[2 * s] - M);
    wts[s] = w;
    lloc += ml[2 * s + 1] * w;
  }
  lloc = wave_sum(lloc);
  __syncthreads();
  if ((d & 63) == 0) red[d >> 6] = lloc;
  __syncthreads();
  const float L = red[0] + red[1];
  const float* op = opart + (size_t)bh * nsplit * 128 + d;
  float O = 0.f;
#pragma unroll 8
  for (int s = 0; s < nsplit; ++s) O = fmaf(op[(size_t)s * 128], wts[s], O);
  const size_t oi = xf_mt ? xf_off(bh / H, (bh % H) * 128 + d, xf_mt) : (size_t)bh * 128 + d;
  out[oi] = f2bf(L > 0.f ? O / L : 0.f);
}

extern "C" int lsa_attn_decode(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                               const int* pos, int B, int H, int Hkv, float scale, int chunk_blocks, int nsplit,
                               void* out, float* opart, float* mlpart, int xf_mt, hipStream_t s) {
  if (H % Hkv) return -1;
  if (xf_mt && B > 16 * xf_mt) return -4;
  if (nsplit > 256) return -3;
  const int G = H / Hkv;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(nsplit, Hkv, B);
  const uint16_t* qq = reinterpret_cast<const uint16_t*>(q);
  const uint16_t* kk = reinterpret_cast<const uint16_t*>(kc);
  const uint16_t* vv = reinterpret_cast<const uint16_t*>(vc);
  uint16_t* oo = reinterpret_cast<uint16_t*>(out);
#define LSA_AD(GV)                                                                                                 \
  case GV:                                                                                                         \
    hipLaunchKernelGGL(attn_decode_kernel<GV>, grid, dim3(256), 0, s, qq, kk, vv, block_tables, max_blocks, pos, Hkv, \
                       sl2, chunk_blocks, nsplit, oo, opart, mlpart, xf_mt);                                      \
    break;
  switch (G) {
    LSA_AD(1) LSA_AD(2) LSA_AD(3) LSA_AD(4) LSA_AD(8)
    default: return -2;
  }
#undef LSA_AD
  if (nsplit > 1) hipLaunchKernelGGL(attn_combine_kernel, dim3(B * H), dim3(128), 0, s, opart, mlpart, nsplit, oo, H,
                                     xf_mt);
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

__global__ __launch_bounds__(256) void attn_prefill_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                           const uint16_t* __restrict__ vc,
                                                           const int* __restrict__ block_tables, int max_blocks,
                                                           const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
                                                           const int* __restrict__ work, int H, int Hkv,
                                                           float scale_log2, uint16_t* __restrict__ out) {
  constexpr int D = 128;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[64 * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[64 * D];
  const int wi = blockIdx.x, h = blockIdx.y;
  const int seq = work[2 * wi], qs = work[2 * wi + 1];
  const int hk = h / (H / Hkv);
  const int q0 = cu_q[seq], qlen = cu_q[seq + 1] - q0;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, r = lane & 15;

  const int qrow = qs + w * 16 + r;
  const int qrow_c = min(qrow, qlen - 1);
  const int qpos = pos0 + qrow;
  uint4 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = *reinterpret_cast<const uint4*>(q + ((size_t)(q0 + qrow_c) * H + h) * D + 32 * s + 8 * g);

  const int last_row = min(qs + 63, qlen - 1);
  const int kv_end = min(ctx, pos0 + last_row + 1);
  const int ntiles = (kv_end + 63) >> 6;

  f32x4_t o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float mrow = LSA_NEG, lrow = 0.f;

  const int* bt = block_tables + (size_t)seq * max_blocks;
  uint4 kr[4], vr[4];
  auto fetch = [&](int t) {
    const size_t base = ((size_t)bt[t] * Hkv + hk) * 64 * D;
    const uint4* kb = reinterpret_cast<const uint4*>(kc + base);
    const uint4* vb = reinterpret_cast<const uint4*>(vc + base);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kr[i] = kb[tid + 256 * i];
      vr[i] = vb[tid + 256 * i];
    }
  };
  if (ntiles > 0) fetch(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int row = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(&Ks[k_off(row, ch)]) = kr[i];
      *reinterpret_cast<uint4*>(&Vs[v_off(row, ch * 8)]) = vr[i];
    }
    __syncthreads();
    if (t + 1 < ntiles) fetch(t + 1);

    // S^T[key][q] = K Q^T over 4 subtiles of 16 keys
    f32x4_t st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      st[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int krow = 16 * kt + r;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const uint4 a = *reinterpret_cast<const uint4*>(&Ks[k_off(krow, 4 * s + g)]);
        st[kt] = mfma16x16x32(a, qf[s], st[kt]);
      }
    }
    float tmax = LSA_NEG;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = t * 64 + 16 * kt + 4 * g + i;
        float v = st[kt][i] * scale_log2;
        v = (key > qpos || key >= ctx) ? LSA_NEG : v;
        st[kt][i] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(mrow, tmax);
    const float alpha = exp2f(mrow - mnew);
    mrow = mnew;
    float psum = 0.f;
    uint32_t pk[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float p[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p[i] = exp2f(st[kt][i] - mnew);
        psum += p[i];
      }
      pk[kt][0] = pack2bf(p[0], p[1]);
      pk[kt][1] = pack2bf(p[2], p[3]);
    }
    lrow = lrow * alpha + psum;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float ai = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) o[dt][i] *= ai;
    }
    // O[q][d] += P[q][key] V[key][d]
    const int qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint4 pa;
      pa.x = pk[2 * s2][0]; pa.y = pk[2 * s2][1];
      pa.z = pk[2 * s2 + 1][0]; pa.w = pk[2 * s2 + 1][1];
      const int kb1 = 32 * s2 + 4 * g + qq, kb2 = kb1 + 16;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const int col = 16 * dt + 4 * pp;
        const uint2 v1 = ds_read_tr16(&Vs[v_off(kb1, col)]);
        const uint2 v2 = ds_read_tr16(&Vs[v_off(kb2, col)]);
        uint4 vb;
        vb.x = v1.x; vb.y = v1.y; vb.z = v2.x; vb.w = v2.y;
        o[dt] = mfma16x16x32(pa, vb, o[dt]);
      }
    }
  }
  float lt = lrow + __shfl_xor(lrow, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float li = __shfl(lt, 4 * g + i, 64);
    const float inv = li > 0.f ? 1.f / li : 0.f;
    const int qr = qs + w * 16 + 4 * g + i;
    if (qr < qlen) {
      uint16_t* orow = out + ((size_t)(q0 + qr) * H + h) * D;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) orow[16 * dt + r] = f2bf(o[dt][i] * inv);
    }
  }
}

extern "C" int lsa_attn_prefill(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                                const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv,
                                float scale, void* out, hipStream_t s) {
  if (nwork <= 0) return 0;
  if (H % Hkv) return -1;
  dim3 grid(nwork, H);
  hipLaunchKernelGGL(attn_prefill_kernel, grid, dim3(256), 0, s, reinterpret_cast<const uint16_t*>(q),
                     reinterpret_cast<const uint16_t*>(kc), reinterpret_cast<const uint16_t*>(vc), block_tables,
                     max_blocks, cu_q, ctx_lens, work, H, Hkv, scale * 1.4426950408889634f,
                     reinterpret_cast<uint16_t*>(out));
  return (int)hipGetLastError();
}
