// Decode layer on the LATENCY path: batch <= 4, bf16 weights, TP = 1 -- BASELINE configs 2 and 3 (duckdb-nsql-7B
// NL->SQL and Llama-3.2-3B /explain_error at batch 1; /root/reference/FastAPI/app.py:85-90,105-109 serve one request
// per call).  At one row a decode layer is ~200-400 MB of weights over five to seven launches, and each launch that
// only moves a few KB (a residual add + RMSNorm, a split-KV combine) costs 4-5 us of dependent round trips.  This
// path removes them:
//
//   per layer:  qkv GEMV -> attention (partials only) -> o GEMV -> gate_up GEMV -> down GEMV      (5 launches)
//
// * The residual stream h lives as Q32 fixed point in int64 ([M][d], value x 2^32).  The row-parallel o / down
//   projections ADD their split-K partials into it with 64-bit integer atomics (fire-and-forget, executed at the
//   memory side): no f32 slabs, no last-arriver ticket, no residual-add launch -- and integer adds make the sum
//   independent of arrival order, so decoding stays bit-reproducible.
// * The RMSNorm of the next projection is folded: its gamma lives in the weights (models/llama.py norms_folded) and
//   the GEMV scales its output rows by rsqrt(sum h^2 / d + eps).  Each workgroup converts its own K-range of h to
//   bf16 (the MFMA B operand, staged in LDS) and sums its squares on the way; the workgroups of n-group 0 (one per
//   K split, the first dispatched) publish their partial sums into ONE packed word per row, (Q16 sum << 8) |
//   publishers, by an agent-scope atomic add; every workgroup reads the complete sum at its epilogue -- long after
//   the publishers ran -- with a relaxed sc1 poll (MI355X_MICROARCH.md "Valid forms" row 1), bounded: a poll that
//   times out computes the row sums itself from h (always correct, counted in stats[0]).
// * Decode attention leaves every split's unnormalised (o, m, l) partial (attention.hip part_only) and the o
//   projection, split by whole heads, merges the partials of its heads in its prologue while its first weight
//   chunk is in flight -- no in-attention combine (ticket + write-through drain + re-read: ~3.6 us of the 3B 2k
//   attention chain, profiles/attn_decode_stamps_after_mi355x.jsonl).
//
// GEMV body: the skinny decode GEMM's weight stream (gemm.hip: fragment-major 1 KiB lane-linear loads, a two-deep
// register pipeline of U x NB fragments per wave, chunks dealt round-robin to the waves), with the activation
// B-fragments read from the LDS-staged K-range instead of global memory.
#include "common.h"
#include "lsa_lat.h"

#define LAT_MMAX 4
#define LAT_SRC_ACT 0   // bf16 row-major activations [M][ldx] (the down projection's SiLU output)
#define LAT_SRC_HQ 1    // the Q32 residual stream [M][K] (+ row sums of squares -> folded RMSNorm)
#define LAT_SRC_PART 2  // split-KV attention partials of the K-range's heads (the o projection)
#define LAT_EPI_F32 0   // f32 split-K slabs [splitk][M][N] (qkv: summed by the fused RoPE attention)
#define LAT_EPI_SILU 1  // silu(gate) * up -> bf16 [M][N / 2] (gate / up rows interleaved per 16)
#define LAT_EPI_ATOM 2  // Q32 integer atomics into the residual stream [M][N]

typedef __attribute__((address_space(1))) unsigned long long lat_g_u64;
typedef __attribute__((address_space(1))) int lat_g_i32;


#define LAT_Q32 4294967296.0f
#define LAT_Q16 65536.0f
__device__ __forceinline__ long long lat_q32(float v) { return (long long)(v * LAT_Q32); }
__device__ __forceinline__ float lat_f32(long long q) { return (float)q * (1.0f / LAT_Q32); }

template <int NB, int SRC, int EPI, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void gemv_lat_kernel(const LatArgs a) {
  constexpr int NT = 64 * WAVES;
  constexpr int U = NB >= 8 ? 1 : (NB >= 4 ? 2 : 4);  // k-steps per chunk: U x NB weight fragments per stage
  extern __shared__ __attribute__((aligned(16))) uint4 lat_lds[];
  uint16_t* xs = reinterpret_cast<uint16_t*>(lat_lds);  // staged activations [M][LDX] bf16
  __shared__ float s_red[WAVES][LAT_MMAX];
  __shared__ float s_scale[LAT_MMAX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int split = blockIdx.x, ng = blockIdx.y;
  const int M = a.M;
  const int kbA = split * a.kb_per_split;
  const int kbB = min(a.KB, kbA + a.kb_per_split);
  const int nk = kbB - kbA;
  const int LDX = a.kb_per_split * 32;
  const int nb0 = ng * NB;

  const uint4* wp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wp[i] = reinterpret_cast<const uint4*>(a.W) + ((size_t)(nb0 + i) * a.KB + kbA) * 64 + lane;
  const int nch = (nk + U - 1) / U;
  const int n_it = nch > w ? (nch - w + WAVES - 1) / WAVES : 0;
  const int last_c = w + WAVES * (n_it - 1);
  auto wload = [&](uint4 (&wr)[U][NB], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(c * U + u, nk - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) wr[u][i] = ldg_nt(wp[i] + (size_t)kk * 64);
    }
  };
  uint4 wA[U][NB], wB[U][NB];
  // the first weight chunk leaves before the prologue: its HBM latency covers the activation staging
  if (n_it > 0) wload(wA, w);
  __builtin_amdgcn_sched_barrier(0);

  // ---------------------------------------------------------------- prologue: this split's activations -> LDS
  if constexpr (SRC == LAT_SRC_ACT) {
    const int per = nk * 4;  // 16-byte chunks per row
    for (int c = tid; c < M * per; c += NT) {
      const int m = c / per, k8 = c - m * per;
      *reinterpret_cast<uint4*>(xs + m * LDX + k8 * 8) =
          *reinterpret_cast<const uint4*>(a.X + (size_t)m * a.ldx + (size_t)kbA * 32 + k8 * 8);
    }
  } else if constexpr (SRC == LAT_SRC_HQ) {
    float ssr[LAT_MMAX];
#pragma unroll
    for (int q = 0; q < LAT_MMAX; ++q) ssr[q] = 0.f;
    const int per = nk * 4;
    for (int c = tid; c < M * per; c += NT) {
      const int m = c / per, k8 = c - m * per;
      const longlong2* hp = reinterpret_cast<const longlong2*>(a.hq + (size_t)m * a.ldh + (size_t)kbA * 32 + k8 * 8);
      float f[8];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const longlong2 v = hp[j];
        f[2 * j] = lat_f32(v.x);
        f[2 * j + 1] = lat_f32(v.y);
        s += f[2 * j] * f[2 * j] + f[2 * j + 1] * f[2 * j + 1];
      }
#pragma unroll
      for (int q = 0; q < LAT_MMAX; ++q) ssr[q] += q == m ? s : 0.f;  // static register index
      *reinterpret_cast<uint4*>(xs + m * LDX + k8 * 8) = pack8(f);
    }
    // fixed-order reduction (lanes, then waves): the published partial is deterministic
#pragma unroll
    for (int q = 0; q < LAT_MMAX; ++q) {
      const float v = wave_sum(ssr[q]);
      if (lane == 0) s_red[w][q] = v;
    }
    __syncthreads();
    if (ng == 0 && tid < M) {
      float t = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) t += s_red[ww][tid];
      const unsigned long long word = ((unsigned long long)(t * LAT_Q16) << 8) | 1ull;
      __hip_atomic_fetch_add((lat_g_u64*)(a.ss_acc) + tid, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {  // LAT_SRC_PART: merge the attention splits of every (row, head) of this K-range
    constexpr int NG = NT / 128;  // split groups per (row, head): thread = (group, dim)
    __shared__ float s_pm[NG], s_pl[NG];
    __shared__ __attribute__((aligned(16))) float s_po[NG][128];
    const int nh = (nk * 32) >> 7, h0 = (kbA * 32) >> 7;
    const int d = tid & 127, grp = tid >> 7;
    for (int q = 0; q < M * nh; ++q) {
      const int m = q / nh, hh = h0 + (q - m * nh);
      const int nblk = (a.pos[m] + 1 + 63) >> 6;
      int ech, nse;
      eff_split(nblk, a.chunk_blocks, a.nsplit, a.unsplit_max, ech, nse);
      const size_t base = ((size_t)m * a.H + hh) * a.nsplit;
      float Mx = -1.0e30f, L = 0.f, O = 0.f;
#pragma unroll 8
      for (int sp = grp; sp < nse; sp += NG) {
        const unsigned long long ml = a.mlpart[base + sp];
        const float o = a.opart[(base + sp) * 128 + d];
        const float mi = __uint_as_float((uint32_t)ml), li = __uint_as_float((uint32_t)(ml >> 32));
        const float mn = fmaxf(Mx, mi);
        const float al = __builtin_amdgcn_exp2f(Mx - mn), wt = __builtin_amdgcn_exp2f(mi - mn);
        Mx = mn;
        L = L * al + li * wt;
        O = O * al + o * wt;
      }
      if (d == 0) {
        s_pm[grp] = Mx;
        s_pl[grp] = L;
      }
      s_po[grp][d] = O;
      __syncthreads();
      if (grp == 0) {
        float Mt = -1.0e30f;
#pragma unroll
        for (int k = 0; k < NG; ++k) Mt = fmaxf(Mt, s_pm[k]);
        float Lt = 0.f, Ot = 0.f;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
          const float wt = __builtin_amdgcn_exp2f(s_pm[k] - Mt);
          Lt += s_pl[k] * wt;
          Ot += s_po[k][d] * wt;
        }
        xs[m * LDX + (hh - h0) * 128 + d] = f2bf(Lt > 0.f ? Ot / Lt : 0.f);
      }
      __syncthreads();
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- main loop (B operand from LDS)
  f32x4_t acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int xrow = (r < M ? r : 0) * LDX + g * 8;
  auto comp = [&](const uint4 (&wr)[U][NB], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = c * U + u;
      uint4 xv = *reinterpret_cast<const uint4*>(xs + xrow + min(kk, nk - 1) * 32);
      const bool ok = kk < nk && r < M;
      xv.x = ok ? xv.x : 0u; xv.y = ok ? xv.y : 0u; xv.z = ok ? xv.z : 0u; xv.w = ok ? xv.w : 0u;
#pragma unroll
      for (int i = 0; i < NB; ++i) acc[i] = mfma16x16x32(wr[u][i], xv, acc[i]);
    }
  };
  if (n_it > 0) {
    int i = 0;
    for (; i + 1 < n_it; i += 2) {
      wload(wB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
      comp(wA, w + WAVES * i);
      __builtin_amdgcn_sched_barrier(0);
      wload(wA, min(w + WAVES * (i + 2), last_c));
      __builtin_amdgcn_sched_barrier(0);
      comp(wB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(wA, w + WAVES * i);
  }

  // ---------------------------------------------------------------- cross-wave reduction (reuses the staging LDS)
  __syncthreads();
  f32x4_t* red = reinterpret_cast<f32x4_t*>(lat_lds);  // [WAVES][NB][64]
#pragma unroll
  for (int i = 0; i < NB; ++i) red[(w * NB + i) * 64 + lane] = acc[i];

  // folded RMSNorm: the complete row sums of squares (published by n-group 0 of every K split)
  if constexpr (SRC == LAT_SRC_HQ) {
    if (tid < M) {
      const long long t0 = wall_clock64();
      unsigned long long v;
      float sc = -1.f;
      while (true) {
        v = __hip_atomic_load((lat_g_u64*)(a.ss_acc) + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int)(v & 255ull) >= (int)gridDim.x) {
          sc = rsqrtf((float)(v >> 8) * (1.0f / LAT_Q16) * a.inv_k + a.eps);
          break;
        }
        if (wall_clock64() - t0 > a.timeout) break;
        __builtin_amdgcn_s_sleep(1);
      }
      s_scale[tid] = sc;
    }
  }
  __syncthreads();
  if constexpr (SRC == LAT_SRC_HQ) {
    // fallback (a publisher was not scheduled in time): the workgroup sums the rows' squares itself from h
    for (int m = 0; m < M; ++m) {
      if (s_scale[m] >= 0.f) continue;  // uniform over the workgroup
      float s = 0.f;
      for (int k = tid; k < a.ldh; k += NT) {
        const float v = lat_f32(a.hq[(size_t)m * a.ldh + k]);
        s += v * v;
      }
      s = wave_sum(s);
      if (lane == 0) s_red[w][0] = s;
      __syncthreads();
      if (tid == 0) {
        float t = 0.f;
        for (int ww = 0; ww < WAVES; ++ww) t += s_red[ww][0];
        s_scale[m] = rsqrtf(t * a.inv_k + a.eps);
        if (a.stats) atomicAdd(a.stats, 1);
      }
      __syncthreads();
    }
  }

  // ---------------------------------------------------------------- epilogues
  if constexpr (EPI == LAT_EPI_SILU) {
    for (int idx = tid; idx < (NB / 2) * 64; idx += NT) {
      const int p = idx >> 6, l = idx & 63;
      const int m = l & 15;
      if (m >= M) continue;
      f32x4_t gs = red[(2 * p) * 64 + l], us = red[(2 * p + 1) * 64 + l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) {
        gs += red[(ww * NB + 2 * p) * 64 + l];
        us += red[(ww * NB + 2 * p + 1) * 64 + l];
      }
      const float sc = SRC == LAT_SRC_HQ ? s_scale[m] : 1.f;
      const int f = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
      uint2 pk;
      pk.x = pack2bf(silu(gs[0] * sc) * (us[0] * sc), silu(gs[1] * sc) * (us[1] * sc));
      pk.y = pack2bf(silu(gs[2] * sc) * (us[2] * sc), silu(gs[3] * sc) * (us[3] * sc));
      *reinterpret_cast<uint2*>(a.act + (size_t)m * (a.N >> 1) + f) = pk;
    }
  } else {
    for (int idx = tid; idx < NB * 64; idx += NT) {
      const int i = idx >> 6, l = idx & 63;
      const int m = l & 15;
      if (m >= M) continue;
      f32x4_t s = red[i * 64 + l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) s += red[(ww * NB + i) * 64 + l];
      const int n = (nb0 + i) * 16 + 4 * (l >> 4);
      if constexpr (EPI == LAT_EPI_F32) {
        const float sc = SRC == LAT_SRC_HQ ? s_scale[m] : 1.f;
        *reinterpret_cast<float4*>(a.out + ((size_t)split * M + m) * a.N + n) =
            make_float4(s[0] * sc, s[1] * sc, s[2] * sc, s[3] * sc);
      } else {  // LAT_EPI_ATOM
        lat_g_u64* hp = (lat_g_u64*)(a.hq_out + (size_t)m * a.N + n);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          __hip_atomic_fetch_add(hp + q, (unsigned long long)lat_q32(s[q]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// h[m] = Q32(emb[ids[m]]); the step's row-sum words ss[k * ss_ld + m] (k < nzero) are zeroed for their publishers
__global__ __launch_bounds__(256) void lat_embed_kernel(const int* __restrict__ ids, const uint16_t* __restrict__ emb,
                                                        int D, long long* __restrict__ hq,
                                                        unsigned long long* __restrict__ ss, int ss_ld, int nzero) {
  const int m = blockIdx.x;
  const uint16_t* er = emb + (size_t)ids[m] * D;
  for (int c = threadIdx.x * 8; c < D; c += blockDim.x * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(er + c), f);
    longlong2* o = reinterpret_cast<longlong2*>(hq + (size_t)m * D + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = make_longlong2(lat_q32(f[2 * j]), lat_q32(f[2 * j + 1]));
  }
  for (int k = threadIdx.x; k < nzero; k += blockDim.x) ss[(size_t)k * ss_ld + m] = 0ull;
}

// final RMSNorm of the Q32 stream: xn[m] = bf16(h[m] * rsqrt(mean h^2 + eps) * w)   (the lm_head input)
__global__ __launch_bounds__(512) void lat_final_norm_kernel(const long long* __restrict__ hq,
                                                             const uint16_t* __restrict__ w, float eps,
                                                             uint16_t* __restrict__ xn, int D) {
  __shared__ float red[16];
  const int m = blockIdx.x;
  const int c = threadIdx.x * 8;
  float f[8];
  float s = 0.f;
  if (c < D) {
    const longlong2* hp = reinterpret_cast<const longlong2*>(hq + (size_t)m * D + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const longlong2 v = hp[j];
      f[2 * j] = lat_f32(v.x);
      f[2 * j + 1] = lat_f32(v.y);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[j] * f[j];
  }
  const float inv = rsqrtf(block_sum(s, red) / (float)D + eps);
  if (c < D) {
    float wf[8];
    unpack8(*reinterpret_cast<const uint4*>(w + c), wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= inv * wf[j];
    *reinterpret_cast<uint4*>(xn + (size_t)m * D + c) = pack8(f);
  }
}

extern "C" {

int lsa_lat_embed(const int* ids, const void* emb, int M, int D, long long* hq, unsigned long long* ss, int ss_ld,
                  int nzero, hipStream_t s) {
  if (M < 1 || M > LAT_MMAX || D % 8 || ss_ld < M) return -1;
  hipLaunchKernelGGL(lat_embed_kernel, dim3(M), dim3(256), 0, s, ids, reinterpret_cast<const uint16_t*>(emb), D, hq,
                     ss, ss_ld, nzero);
  return (int)hipGetLastError();
}

int lsa_lat_final_norm(const long long* hq, const void* w, float eps, void* xn, int M, int D, hipStream_t s) {
  if (M < 1 || D % 8 || D / 8 > 512) return -1;
  hipLaunchKernelGGL(lat_final_norm_kernel, dim3(M), dim3((D / 8 + 63) / 64 * 64), 0, s, hq,
                     reinterpret_cast<const uint16_t*>(w), eps, reinterpret_cast<uint16_t*>(xn), D);
  return (int)hipGetLastError();
}

// src / epi: LAT_SRC_* / LAT_EPI_*; grid = (splitk, N / 16 / nb): the first splitk workgroups are n-group 0 (the row-sum
// publishers of LAT_SRC_HQ)
int lsa_lat_gemv(const LatArgs* args, int src, int epi, int nb, int waves, int splitk, hipStream_t s) {
  LatArgs a = *args;
  if (a.M < 1 || a.M > LAT_MMAX || a.N % 16 || a.KB < 1 || splitk < 1) return -1;
  if (nb != 1 && nb != 2 && nb != 4 && nb != 8) return -2;
  if ((a.N / 16) % nb) return -2;
  if (waves != 4 && waves != 8) return -3;
  a.kb_per_split = (a.KB + splitk - 1) / splitk;
  if ((a.KB + a.kb_per_split - 1) / a.kb_per_split != splitk) return -4;  // every split owns >= 1 k-block
  if (epi == LAT_EPI_SILU && (nb % 2 || splitk != 1)) return -5;
  if (src == LAT_SRC_PART && (a.kb_per_split % 4 || a.KB % a.kb_per_split || !a.opart || !a.mlpart || !a.pos)) return -6;
  if (src == LAT_SRC_HQ && (!a.hq || !a.ss_acc || splitk > 255)) return -7;
  if (src == LAT_SRC_ACT && !a.X) return -8;
  if ((epi == LAT_EPI_F32 && !a.out) || (epi == LAT_EPI_SILU && !a.act) || (epi == LAT_EPI_ATOM && !a.hq_out)) return -9;
  const size_t xb = (size_t)a.M * a.kb_per_split * 32 * 2, rb = (size_t)waves * nb * 1024;
  const size_t lds = xb > rb ? xb : rb;
  if (lds > 64 * 1024) return -10;
  const dim3 grid(splitk, a.N / 16 / nb);
#define LAT_L(NBV, S, E, WV) \
  hipLaunchKernelGGL((gemv_lat_kernel<NBV, S, E, WV>), grid, dim3(64 * (WV)), lds, s, a)
#define LAT_W(NBV, S, E) \
  do {                                 \
    if (waves == 8) LAT_L(NBV, S, E, 8); \
    else LAT_L(NBV, S, E, 4);          \
  } while (0)
#define LAT_NB(S, E)                                    \
  do {                                                  \
    switch (nb) {                                       \
      case 1: LAT_W(1, S, E); break;                    \
      case 2: LAT_W(2, S, E); break;                    \
      case 4: LAT_W(4, S, E); break;                    \
      default: LAT_W(8, S, E); break;                   \
    }                                                   \
  } while (0)
  if (src == LAT_SRC_HQ && epi == LAT_EPI_F32) LAT_NB(LAT_SRC_HQ, LAT_EPI_F32);
  else if (src == LAT_SRC_HQ && epi == LAT_EPI_SILU) {
    switch (nb) {  // SiLU pairs: nb even
      case 2: LAT_W(2, LAT_SRC_HQ, LAT_EPI_SILU); break;
      case 4: LAT_W(4, LAT_SRC_HQ, LAT_EPI_SILU); break;
      default: LAT_W(8, LAT_SRC_HQ, LAT_EPI_SILU); break;
    }
  } else if (src == LAT_SRC_PART && epi == LAT_EPI_ATOM) LAT_NB(LAT_SRC_PART, LAT_EPI_ATOM);
  else if (src == LAT_SRC_ACT && epi == LAT_EPI_ATOM) LAT_NB(LAT_SRC_ACT, LAT_EPI_ATOM);
  else return -11;
#undef LAT_NB
#undef LAT_W
#undef LAT_L
  return (int)hipGetLastError();
}

}  // extern "C"
