// Batch-1 decode: attention + O projection + residual in ONE launch (MHA models, short contexts).
//
// At batch 1 the decode step is a chain of latency-bound launches; attention (~6 us for 32 heads x 4 blocks)
// and the O projection (33.6 MB of weights, ~9 us with its residual epilogue) are two of them.  Here the grid
// is heads x CS column slices: workgroup (h, c) computes head h's attention output o_h (fused RoPE of the
// new token from the QKV split-K slabs, paged K/V, online softmax; the 8 column-slice workgroups of a head
// compute it redundantly -- they sit on one XCD, so the K/V come from L2 after the first) and multiplies it
// into its slice of Wo: rows c * 512 .. +511, columns h * 128 .. +127.  Those 128 KiB of weights are loaded
// into registers at kernel start, independent of the attention, so the weight stream overlaps the whole
// attention critical path.  The 32 per-head partial rows are summed by the last-arriving head of each
// column slice (sc1 write-through partials + one relaxed agent-scope ticket per slice, as the split-K
// residual epilogue of the GEMMs), which also does the residual update h += y, writes bf16(h) for the next
// GEMM and adds the slice's sum of squares (Q24 fixed point) for the next GEMM's RMS row scale.
//
// Replaces attn_decode + the residual O GEMM of the norm-free batch-1 step (engine/runner.py) when the
// context is at most 8 blocks; G = 1 only (duckdb-nsql / Mistral-style MHA; GQA models keep the two launches).
#include "common.h"

#define LSA_AO_NEG (-1.0e30f)

namespace {
typedef __attribute__((address_space(1))) int ao_g_i32;
}

// timing probe (scripts/attn_stamps.py --ao): s_memrealtime at 6 points of each workgroup's path, [wg][8]
__device__ unsigned long long* g_ao_stamps = nullptr;
#define LSA_AO_STAMP(K) \
  if (stp && tid == 0) stp[(size_t)blockIdx.x * 8 + (K)] = __builtin_amdgcn_s_memrealtime()

template <int NP>
__global__ __launch_bounds__(512) void attn_o_b1_kernel(const float* __restrict__ qkv_parts, size_t part_stride,
                                                        const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                        const int* __restrict__ pos, uint16_t* __restrict__ kc,
                                                        uint16_t* __restrict__ vc, const int* __restrict__ bt, int H,
                                                        float scale_log2, const uint4* __restrict__ Wo, int N,
                                                        float* __restrict__ slabs, int* __restrict__ tickets, LsaEpi ep) {
  constexpr int D = 128, NT = 512, WV = 8, TU = 2, TW = 8;
  const int H_ = H;
  const int h = blockIdx.x % H_, c = blockIdx.x / H_;  // heads fastest: a head's slices share an XCD (H % 8 == 0)
  const int tid = threadIdx.x, lg = tid >> 4, li = tid & 15, wv = tid >> 6;
  const int n = c * NT + tid;  // this thread's output column of the O projection
  unsigned long long* const stp = g_ao_stamps;
  LSA_AO_STAMP(0);
  const int KB = H_ * 4;       // k-blocks (32 wide) of Wo's K = H * 128

  // 2) the new token's q / k / v for head h (sum of the QKV slabs), rotated, through LDS
  const int tpos = pos[0];
  const int ctx = tpos + 1;
  const int nblk = (ctx + 63) >> 6;
  __shared__ uint4 qkv_s[3][16];
  float xq[8];
  if (lg < 3) {
    const int off = (lg == 0 ? h : (lg == 1 ? H_ + h : 2 * H_ + h)) * D + li * 8;
    const float4 a0 = *reinterpret_cast<const float4*>(qkv_parts + off);
    const float4 a1 = *reinterpret_cast<const float4*>(qkv_parts + off + 4);
    xq[0] = a0.x; xq[1] = a0.y; xq[2] = a0.z; xq[3] = a0.w; xq[4] = a1.x; xq[5] = a1.y; xq[6] = a1.z; xq[7] = a1.w;
#pragma unroll
    for (int sp = 1; sp < NP; ++sp) {
      const float* r2 = qkv_parts + sp * part_stride + off;
      const float4 b0 = *reinterpret_cast<const float4*>(r2);
      const float4 b1 = *reinterpret_cast<const float4*>(r2 + 4);
      xq[0] += b0.x; xq[1] += b0.y; xq[2] += b0.z; xq[3] += b0.w; xq[4] += b1.x; xq[5] += b1.y; xq[6] += b1.z; xq[7] += b1.w;
    }
    float y[8];
    if (lg <= 1) {  // rotate-half RoPE of q and k (the partner dims live in lane li ^ 8)
      const int dd = li * 8;
      const float4 c0 = *reinterpret_cast<const float4*>(cos_t + (size_t)tpos * 64 + (dd & 63));
      const float4 c1 = *reinterpret_cast<const float4*>(cos_t + (size_t)tpos * 64 + (dd & 63) + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(sin_t + (size_t)tpos * 64 + (dd & 63));
      const float4 s1 = *reinterpret_cast<const float4*>(sin_t + (size_t)tpos * 64 + (dd & 63) + 4);
      const float sg = li < 8 ? -1.f : 1.f;
      const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = xq[j] * cc[j] + sg * __shfl_xor(xq[j], 8, 64) * sn[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = xq[j];
    }
    qkv_s[lg][li] = pack8(y);
  }
  __syncthreads();
  LSA_AO_STAMP(1);
  const uint4 qb = qkv_s[0][li];

  // 3) attention over the paged cache: lane group lg scores keys wv * 8 + u * 4 + (lg & 3) of each block
  //    (16 lanes x 8 dims per key), K / V of block b + 1 in flight while block b is scored
  uint4 kA[TU], vA[TU], kB[TU], vB[TU];
  auto fetch = [&](uint4 (&kr)[TU], uint4 (&vr)[TU], int blk) {
    const size_t base = ((size_t)__builtin_amdgcn_readfirstlane(bt[blk]) * H_ + h) * 64 * D;
    const int last = ctx - 1 - blk * 64;
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int tok = min(wv * TW + u * 4 + (lg & 3), last);
      kr[u] = ldg_nt(reinterpret_cast<const uint4*>(kc + base + tok * D + li * 8));
      vr[u] = ldg_nt(reinterpret_cast<const uint4*>(vc + base + tok * D + li * 8));
    }
  };
  float m = LSA_AO_NEG, l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto score = [&](const uint4 (&kr)[TU], const uint4 (&vr)[TU], int blk) {
    float s[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int tp = blk * 64 + wv * TW + u * 4 + (lg & 3);
      const uint4 kq = tp == tpos ? qkv_s[1][li] : kr[u];  // the new token's key is not in the cache yet
      float d = dot8_bf16(qb, kq);
      d += __shfl_xor(d, 8, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 1, 64);
      s[u] = tp < ctx ? d * scale_log2 : LSA_AO_NEG;
    }
    const float mn = fmaxf(m, fmaxf(s[0], s[1]));
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    float p[TU], ps = 0.f;
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      p[u] = __builtin_amdgcn_exp2f(s[u] - mn);
      ps += p[u];
    }
    l = l * alpha + ps;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] *= alpha;
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int tp = blk * 64 + wv * TW + u * 4 + (lg & 3);
      const uint4 vq = tp == tpos ? qkv_s[2][li] : vr[u];
      float vf[8];
      unpack8(vq, vf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf(p[u], vf[j], o[j]);
    }
  };
  fetch(kA, vA, 0);
  // the weight slice: 16 fragments' worth (8 bf16 each) of row n, columns h * 128 .. +127 -- issued after the
  // attention's first K / V block (queued ahead of it they delayed the latency-critical loads: the probe
  // measured start -> RoPE 1.1 -> 2.2 us) and still in flight under the whole score loop
  uint4 w[16];
  {
    const uint4* wp = Wo + ((size_t)(n >> 4) * KB + h * 4) * 64 + (n & 15);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int k8 = 0; k8 < 4; ++k8) w[kb * 4 + k8] = ldg_nt(wp + (size_t)kb * 64 + 16 * k8);
  }
  const float h_old = ep.h[n];  // the residual row (the last-arriving head updates it)
  int blk = 0;
  for (; blk + 1 < nblk; blk += 2) {
    fetch(kB, vB, blk + 1);
    __builtin_amdgcn_sched_barrier(0);
    score(kA, vA, blk);
    __builtin_amdgcn_sched_barrier(0);
    fetch(kA, vA, min(blk + 2, nblk - 1));
    __builtin_amdgcn_sched_barrier(0);
    score(kB, vB, blk + 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (blk < nblk) score(kA, vA, blk);
  LSA_AO_STAMP(2);

  // the slice-0 workgroup appends the new token's k / v to the cache
  if (c == 0 && (lg == 1 || lg == 2)) {
    const size_t co = (((size_t)bt[tpos >> 6] * H_ + h) * 64 + (tpos & 63)) * D + li * 8;
    *reinterpret_cast<uint4*>((lg == 1 ? kc : vc) + co) = qkv_s[lg][li];
  }

  // 4) merge the 32 lane groups: the 4 of a wave in registers, the 8 waves through LDS
  {
    float mo = fmaxf(m, __shfl_xor(m, 16, 64));
    mo = fmaxf(mo, __shfl_xor(mo, 32, 64));
    const float a = __builtin_amdgcn_exp2f(m - mo);
    l *= a;
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] *= a;
      o[j] += __shfl_xor(o[j], 16, 64);
      o[j] += __shfl_xor(o[j], 32, 64);
    }
    m = mo;
  }
  __shared__ float sm[WV], sl[WV];
  __shared__ __attribute__((aligned(16))) float so[WV][D];
  __shared__ __attribute__((aligned(16))) uint16_t oh[D];  // o_h rounded to bf16, like the unfused path
  if ((tid & 63) < 16) {
    if (li == 0) {
      sm[wv] = m;
      sl[wv] = l;
    }
    *reinterpret_cast<float4*>(&so[wv][li * 8]) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(&so[wv][li * 8 + 4]) = make_float4(o[4], o[5], o[6], o[7]);
  }
  __syncthreads();
  if (tid < D) {
    float M = LSA_AO_NEG;
#pragma unroll
    for (int k = 0; k < WV; ++k) M = fmaxf(M, sm[k]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int k = 0; k < WV; ++k) {
      const float wgt = __builtin_amdgcn_exp2f(sm[k] - M);
      L += sl[k] * wgt;
      O += so[k][tid] * wgt;
    }
    oh[tid] = f2bf(L > 0.f ? O / L : 0.f);
  }
  __syncthreads();
  LSA_AO_STAMP(3);

  // 5) this slice's rows of the O projection for head h: y[n] = sum_k o_h[k] * Wo[n][h * 128 + k]
  float y = 0.f;
  {
    const uint4* ohv = reinterpret_cast<const uint4*>(oh);
#pragma unroll
    for (int f = 0; f < 16; ++f) y += dot8_bf16(w[f], ohv[f]);  // fragment (kb, k8) = columns 32 kb + 8 k8 .. +7
  }

  // 6) head partials -> the last-arriving head of this column slice finishes: residual, bf16 copy, sum of squares
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slabs, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), rs, (int)(((size_t)h * N + n) * 4), 0, LSA_SC1_AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  if (tid == 0)
    s_last = __hip_atomic_fetch_add((ao_g_i32*)(tickets) + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == H_ - 1;
  __syncthreads();
  LSA_AO_STAMP(4);
  if (!s_last) return;
  if (tid == 0) __hip_atomic_store((ao_g_i32*)(tickets) + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float acc = 0.f;
#pragma unroll 8
  for (int hh = 0; hh < H_; ++hh)
    acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(((size_t)hh * N + n) * 4), 0, LSA_SC1_AUX));
  const float hv = h_old + acc;
  ep.h[n] = hv;
  ep.xout[n] = f2bf(hv);
  __shared__ float red[16];
  const float ss = block_sum(hv * hv, red);
  if (tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(ep.ss_out), (unsigned long long)ss_to_q24(ss));
  LSA_AO_STAMP(5);
}

extern "C" int lsa_attn_o_set_stamps(void* p) {
  unsigned long long* v = reinterpret_cast<unsigned long long*>(p);
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ao_stamps), &v, sizeof(v));
}

// B = 1, MHA (H == Hkv), head_dim 128, N = d (a multiple of 512), ctx <= 8 blocks of 64
extern "C" int lsa_attn_o_b1(const float* qkv_parts, int nparts, long part_stride, const float* cos_t, const float* sin_t,
                             const int* pos, void* kc, void* vc, const int* block_table, int H, float scale,
                             const void* Wo, int N, float* slabs, int* tickets, const LsaEpi* ep, hipStream_t s) {
  if (N % 512 || H % 8 || !ep || !ep->h || !ep->xout || !ep->ss_out || ep->xmt) return -1;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(H * (N / 512));
#define LSA_AO(NPV)                                                                                               \
  hipLaunchKernelGGL((attn_o_b1_kernel<NPV>), grid, dim3(512), 0, s, qkv_parts, (size_t)part_stride, cos_t, sin_t, pos, \
                     reinterpret_cast<uint16_t*>(kc), reinterpret_cast<uint16_t*>(vc), block_table, H, sl2,         \
                     reinterpret_cast<const uint4*>(Wo), N, slabs, tickets, *ep)
  switch (nparts) {
    case 1: LSA_AO(1); break;
    case 2: LSA_AO(2); break;
    case 4: LSA_AO(4); break;
    case 8: LSA_AO(8); break;
    default: return -2;
  }
#undef LSA_AO
  return (int)hipGetLastError();
}
