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

typedef short s16x4p_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4p_t* lds_s4p_ptr;
typedef float f32x16_t __attribute__((ext_vector_type(16)));

namespace {

__device__ __forceinline__ uint2 ds_read_tr16p(const uint16_t* p) {
  s16x4p_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p_ptr)(p));
  return __builtin_bit_cast(uint2, v);
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

__global__ __launch_bounds__(256, 2) void attn_prefill32_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                                const uint16_t* __restrict__ vc,
                                                                const int* __restrict__ block_tables, int max_blocks,
                                                                const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
                                                                const int* __restrict__ work, int H, int Hkv,
                                                                float scale_log2, uint16_t* __restrict__ out) {
  constexpr int D = 128;
  constexpr int QB = 128;  // query rows per workgroup
  __shared__ __attribute__((aligned(16))) uint16_t Ks[64 * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[64 * D];
  const int wi = blockIdx.x, h = blockIdx.y;
  const int seq = work[2 * wi], qs = work[2 * wi + 1];
  const int hk = h / (H / Hkv);
  const int q0 = cu_q[seq], qlen = cu_q[seq + 1] - q0;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;

  // Q^T fragments (B operand): lane (r, h) holds Q[row r][16 s + 8 h .. + 7] for the 8 k-steps of 16 dims
  const int qrow = qs + w * 32 + r32;
  const int qpos = pos0 + qrow;
  uint4 qf[8];
  {
    const uint16_t* qp = q + ((size_t)(q0 + min(qrow, qlen - 1)) * H + h) * D + 8 * hh;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = *reinterpret_cast<const uint4*>(qp + 16 * s);
  }
  const int last_row = min(qs + QB - 1, qlen - 1);
  const int kv_end = min(ctx, pos0 + last_row + 1);
  const int ntiles = (kv_end + 63) >> 6;
  // keys a wave's rows can see (causal): tiles past the wave's last row are skipped by that wave
  const int wave_last = min(qs + w * 32 + 31, qlen - 1);
  const int wave_tiles = (min(ctx, pos0 + wave_last + 1) + 63) >> 6;

  f32x16_t o[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) o[db] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mrow = LSA_NEG_P, lrow = 0.f;  // of query row r32 (identical in both lane halves)

  const int* bt = block_tables + (size_t)seq * max_blocks;
  uint4 kr0, kr1, kr2, kr3, vr0, vr1, vr2, vr3;
#define LSA_P32_FETCH(T)                                                                 \
  {                                                                                      \
    const size_t base_ = ((size_t)bt[(T)] * Hkv + hk) * 64 * D;                          \
    const uint4* kb_ = reinterpret_cast<const uint4*>(kc + base_) + tid;                 \
    const uint4* vb_ = reinterpret_cast<const uint4*>(vc + base_) + tid;                 \
    kr0 = kb_[0]; kr1 = kb_[256]; kr2 = kb_[512]; kr3 = kb_[768];                        \
    vr0 = vb_[0]; vr1 = vb_[256]; vr2 = vb_[512]; vr3 = vb_[768];                        \
  }
  LSA_P32_FETCH(0);
  const int G16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    {
      const int row = tid >> 4, ch = tid & 15;  // 16 B chunk c = tid + 256 i -> row + 16 i, chunk ch
      *reinterpret_cast<uint4*>(&Ks[kp_off(row, ch)]) = kr0;
      *reinterpret_cast<uint4*>(&Ks[kp_off(row + 16, ch)]) = kr1;
      *reinterpret_cast<uint4*>(&Ks[kp_off(row + 32, ch)]) = kr2;
      *reinterpret_cast<uint4*>(&Ks[kp_off(row + 48, ch)]) = kr3;
      *reinterpret_cast<uint4*>(&Vs[vp_off(row, ch * 8)]) = vr0;
      *reinterpret_cast<uint4*>(&Vs[vp_off(row + 16, ch * 8)]) = vr1;
      *reinterpret_cast<uint4*>(&Vs[vp_off(row + 32, ch * 8)]) = vr2;
      *reinterpret_cast<uint4*>(&Vs[vp_off(row + 48, ch * 8)]) = vr3;
    }
    __syncthreads();
    LSA_P32_FETCH(min(t + 1, ntiles - 1));
    if (t >= wave_tiles) continue;  // causal: nothing this wave's rows can see (barriers stay uniform)

    // S^T for the two 32-key halves
    f32x16_t st[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      st[kh] = f32x16_t{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const uint4 a = *reinterpret_cast<const uint4*>(&Ks[kp_off(32 * kh + r32, 2 * s + hh)]);
        st[kh] = mfma32x32x16(a, qf[s], st[kh]);
      }
    }
    // mask + online softmax; register i of half kh holds key t*64 + 32 kh + (i & 3) + 8 (i >> 2) + 4 hh
    float tmax = LSA_NEG_P;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = t * 64 + 32 * kh + (i & 3) + 8 * (i >> 2) + 4 * hh;
        float v = st[kh][i] * scale_log2;
        v = (key > qpos || key >= ctx) ? LSA_NEG_P : v;
        st[kh][i] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(mrow, tmax);
    const float alpha = exp2f(mrow - mnew);
    mrow = mnew;
    float psum = 0.f;
    uint4 pa[2][2];  // [kh][k-step s']: registers 8 s' .. 8 s' + 7 of half kh as bf16
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      float p[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        p[i] = exp2f(st[kh][i] - mnew);
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
    lrow = lrow * alpha + psum;
    // rescale O: register i of o[db] is query row (i & 3) + 8 (i >> 2) + 4 hh (alpha lives on lane = row)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float ai = __shfl(alpha, (i & 3) + 8 * (i >> 2) + 4 * hh, 64);
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db][i] *= ai;
    }
    // O += P V: k-step (kh, s') covers keys 32 kh + 16 s' + 8 (j >> 2) + 4 hh + (j & 3) in element j
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int r0 = 32 * kh + 16 * s2 + 4 * (G16 >> 1) + qq;  // this lane's supplied key row (j < 4)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int col = 32 * db + 16 * (G16 & 1) + 4 * pp;
          const uint2 v1 = ds_read_tr16p(&Vs[vp_off(r0, col)]);
          const uint2 v2 = ds_read_tr16p(&Vs[vp_off(r0 + 8, col)]);
          uint4 vb;
          vb.x = v1.x; vb.y = v1.y; vb.z = v2.x; vb.w = v2.y;
          o[db] = mfma32x32x16(pa[kh][s2], vb, o[db]);
        }
      }
  }
#undef LSA_P32_FETCH
  // normalise and store: register i of o[db] = O[row (i & 3) + 8 (i >> 2) + 4 hh][dim 32 db + r32]
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int rr = (i & 3) + 8 * (i >> 2) + 4 * hh;
    const float li = __shfl(lrow, rr, 64);
    const float inv = li > 0.f ? 1.f / li : 0.f;
    const int qr = qs + w * 32 + rr;
    if (qr < qlen) {
      uint16_t* orow = out + ((size_t)(q0 + qr) * H + h) * D;
#pragma unroll
      for (int db = 0; db < 4; ++db) orow[32 * db + r32] = f2bf(o[db][i] * inv);
    }
  }
}

extern "C" int lsa_attn_prefill32(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                                  const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv,
                                  float scale, void* out, hipStream_t s) {
  if (nwork <= 0) return 0;
  if (H % Hkv) return -1;
  dim3 grid(nwork, H);
  hipLaunchKernelGGL(attn_prefill32_kernel, grid, dim3(256), 0, s, reinterpret_cast<const uint16_t*>(q),
                     reinterpret_cast<const uint16_t*>(kc), reinterpret_cast<const uint16_t*>(vc), block_tables,
                     max_blocks, cu_q, ctx_lens, work, H, Hkv, scale * 1.4426950408889634f,
                     reinterpret_cast<uint16_t*>(out));
  return (int)hipGetLastError();
}
