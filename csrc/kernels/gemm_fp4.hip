// MXFP4 (OCP MX: FP4 e2m1 elements, one E8M0 power-of-two scale per 32 consecutive k) weight-only linear layers:
//   out = X[M, K] @ dequant(Wq, S)^T     (bf16 activations, f32 accumulate on MFMA 16x16x32 bf16)
//
// The 4-bit weight class the reference actually served (Ollama's default tags are 4-bit GGUF quants):
// a quarter of the bf16 weight bytes, half of fp8's, so decode -- a weight stream -- moves 3.7x fewer bytes.
//
// Weight layout (ops.pack_mxfp4): Wq[nb][kb128][lane][16 B], lane = 16 g + r holds W[16 nb + r][128 kb + 32 g ..
// + 31] as 32 e2m1 nibbles (element 2i in the low nibble of byte i) -- exactly one MX block per lane and 128-k
// step, so one 16-B load per lane (1 KiB per wave-instruction) feeds FOUR mfma_f32_16x16x32_bf16 k-steps:
// step s uses the lane's elements 8 s .. 8 s + 7 (the k order inside an MFMA step only has to agree between A
// and B, so lane (m, g)'s activations for step s are x[m][128 kb + 32 g + 8 s .. + 7]).
// Scales: S[nb][kb128 / 4][lane][4 B] -- the lane's E8M0 byte of four consecutive 128-k steps in one word.
// Dequantisation in registers: v_cvt_scalef32_pk_bf16_fp4 (2 nibbles -> 2 bf16, times the block's 2^(e - 127),
// exact: an e2m1 value times a power of two is a bf16 value), one VALU op per 2 weights.
// Epilogues as gemm.hip / gemm_fp8.hip: bf16, f32 split-K slabs, SiLU * up (gate / up rows interleaved per 16),
// the norm-free decode extensions (LsaEpi row scale / residual).  Prefill (M > 64) dequantises the layer into a
// bf16 fragment-layout scratch (lsa_fp4_dequant) for the 256^2 tile GEMM.
#include "common.h"

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2

namespace {

__device__ __forceinline__ float e8m0_f32(uint32_t e) { return __uint_as_float(e << 23); }  // 2^(e - 127), e >= 1

template <int B>
__device__ __forceinline__ uint32_t cvt4(uint32_t w, float sc) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(w, sc, B));
}
// 8 e2m1 (one 32-bit word) -> one bf16 MFMA fragment (8 values), scaled
__device__ __forceinline__ uint4 fp4x8_to_bf16(uint32_t w, float sc) {
  return make_uint4(cvt4<0>(w, sc), cvt4<1>(w, sc), cvt4<2>(w, sc), cvt4<3>(w, sc));
}

}  // namespace

// XF: X in the fragment-major decode layout (common.h xf_off): lane (r, g)'s 8 activations of step s,
// k = 128 kb + 32 g + 8 s .. + 7, are lane (16 s + r) of bf16 k-step 4 kb + g
template <int MT, int NB, int EPI, int WAVES, int U, bool XF = false>
__global__ __launch_bounds__(64 * WAVES) void gemm_fp4_skinny_kernel(const uint16_t* __restrict__ X, int ldx, int M,
                                                                     int KB128, const uint4* __restrict__ Wq,
                                                                     const uint32_t* __restrict__ Sw,
                                                                     void* __restrict__ out, int ldo, int kb_per_split,
                                                                     LsaEpi ep) {
  // chunks of U 128-k steps round-robin over the waves, two-deep register pipeline pinned with sched_barrier(0)
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  int nb0, cnt;  // this workgroup's n-blocks (ragged grids: common.h skinny_nblocks)
  skinny_nblocks<NB, EPI == EPI_SILU ? 2 : 1>(EPI == EPI_SILU ? ldo / 8 : ldo / 16, nb0, cnt);
  const int kbA = blockIdx.y * kb_per_split;
  const int kbB = min(KB128, kbA + kb_per_split);
  const int nk = kbB - kbA;
  const int nch = (nk + U - 1) / U;
  const int n_it = nch > w ? (nch - w + WAVES - 1) / WAVES : 0;
  const int last_c = w + WAVES * (n_it - 1);
  const int KB4 = (KB128 + 3) >> 2;

  f32x4_t acc[NB][MT];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bool xvalid[MT];
  // row-major X: padding rows (>= M) read zeros from past the buffer range, no memory request (gemm.hip)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, XF ? 0x7fffffff : M * ldx * 2, 0x00020000);
  uint32_t xoff[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = j * 16 + r;
    xvalid[j] = m < M;
    xoff[j] = XF ? (uint32_t)((((size_t)g * MT + j) * 64 + r) * 16)
                 : (xvalid[j] ? (uint32_t)(((size_t)m * ldx + 32 * g) * 2) : 0x80000000u);
  }
  const uint4* wp[NB];
  const uint32_t* sp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    wp[i] = Wq + (size_t)(nb0 + min(i, cnt - 1)) * KB128 * 64 + lane;
    sp[i] = Sw + (size_t)(nb0 + min(i, cnt - 1)) * KB4 * 64 + lane;
  }

  auto load = [&](uint4 (&wr)[U][NB], uint32_t (&sr)[U][NB], uint4 (&xr)[U][MT][4], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        wr[u][i] = ldg_nt(wp[i] + (size_t)kk * 64);
        sr[u][i] = (sp[i][(size_t)(kk >> 2) * 64] >> (8 * (kk & 3))) & 0xffu;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          // XF: bf16 k-step 4 kk + g, lane 16 s + r; row-major: x[m][128 kk + 32 g + 8 s]
          const uint32_t o = XF ? xoff[j] + (uint32_t)(((size_t)kk * 4 * MT * 64 + 16 * s) * 16)
                                : xoff[j] + (uint32_t)kk * 256u + 16u * s;
          const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
          xr[u][j][s] = make_uint4(a[0], a[1], a[2], a[3]);
        }
      }
    }
  };
  auto comp = [&](const uint4 (&wr)[U][NB], const uint32_t (&sr)[U][NB], const uint4 (&xr)[U][MT][4], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = (kb + u) < kbB;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const float sc = live ? e8m0_f32(sr[u][i]) : 0.f;  // a dead (clamped) step contributes zeros
        const uint32_t q[4] = {wr[u][i].x, wr[u][i].y, wr[u][i].z, wr[u][i].w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const uint4 a = fp4x8_to_bf16(q[s], sc);
#pragma unroll
          for (int j = 0; j < MT; ++j) acc[i][j] = mfma16x16x32(a, xr[u][j][s], acc[i][j]);  // padding rows:
          // their own (discarded) output rows only
        }
      }
    }
  };
  if (n_it > 0) {
    uint4 wA[U][NB], xA[U][MT][4], wB[U][NB], xB[U][MT][4];
    uint32_t sA[U][NB], sB[U][NB];
    load(wA, sA, xA, w);
    int i = 0;
    for (; i + 1 < n_it; i += 2) {
      load(wB, sB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
      comp(wA, sA, xA, w + WAVES * i);
      __builtin_amdgcn_sched_barrier(0);
      load(wA, sA, xA, min(w + WAVES * (i + 2), last_c));
      __builtin_amdgcn_sched_barrier(0);
      comp(wB, sB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(wA, sA, xA, w + WAVES * i);
  }

  __shared__ __attribute__((aligned(16))) f32x4_t red[WAVES][NB * MT][64];
  __shared__ unsigned long long ssw[16 * MT];  // EPI_RES: per-row sum of h^2 over this workgroup's columns (Q24)
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) red[w][i * MT + j][lane] = acc[i][j];
  if constexpr (EPI == EPI_RES) {
    if (threadIdx.x < 16 * MT) ssw[threadIdx.x] = 0ull;
  }
  __syncthreads();

  if constexpr (EPI == EPI_SILU) {
    for (int idx = threadIdx.x; idx < (NB / 2) * MT * 64; idx += 64 * WAVES) {
      const int l = idx & 63, t = idx >> 6;
      const int j = t % MT, p = t / MT;
      f32x4_t gs = red[0][(2 * p) * MT + j][l], us = red[0][(2 * p + 1) * MT + j][l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) {
        gs += red[ww][(2 * p) * MT + j][l];
        us += red[ww][(2 * p + 1) * MT + j][l];
      }
      const int m = j * 16 + (l & 15);
      if (m < M && 2 * p < cnt) {
        const int n = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
        const float sc = epi_row_scale(ep, m);
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(gs[q] * sc) * (us[q] * sc);
        uint2 pk;
        pk.x = pack2bf(v[0], v[1]);
        pk.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (XF ? xf_off(m, n, MT) : (size_t)m * ldo + n)) = pk;
      }
    }
  } else {
    const size_t slab = (size_t)blockIdx.y * M * ldo;
    if constexpr (EPI == EPI_RES) {
      if (gridDim.y > 1) {  // split-K: publish, ticket, the last split finishes the column (gemm.hip)
        const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
          const int l = idx & 63, t = idx >> 6;
          const int j = t % MT, i = t / MT;
          f32x4_t s = red[0][t][l];
#pragma unroll
          for (int ww = 1; ww < WAVES; ++ww) s += red[ww][t][l];
          const int m = j * 16 + (l & 15);
          if (m < M && i < cnt) res_store_partial(rsc, slab + (size_t)m * ldo + (nb0 + i) * 16 + 4 * (l >> 4), s);
        }
        __shared__ int s_last;
        if (!res_publish_and_ticket<64 * WAVES>(ep, &s_last)) return;
        for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
          const int l = idx & 63, t = idx >> 6;
          const int j = t % MT, i = t / MT;
          const int m = j * 16 + (l & 15);
          if (m < M && i < cnt) {
            const int n = (nb0 + i) * 16 + 4 * (l >> 4);
            atomicAdd(&ssw[m], (unsigned long long)ss_to_q24(
                epi_residual4(ep, m, n, res_slab_sum(rsc, (size_t)m * ldo + n, (size_t)M * ldo, gridDim.y) *
                                        epi_row_scale(ep, m))));
          }
        }
        __syncthreads();
        if (threadIdx.x < M) atomicAdd(reinterpret_cast<unsigned long long*>(ep.ss_out) + threadIdx.x, ssw[threadIdx.x]);
        return;
      }
    }
    for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
      const int l = idx & 63, t = idx >> 6;
      const int j = t % MT, i = t / MT;
      f32x4_t s = red[0][t][l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) s += red[ww][t][l];
      const int m = j * 16 + (l & 15);
      if (m >= M || i >= cnt) continue;
      const int n = (nb0 + i) * 16 + 4 * (l >> 4);
      s *= epi_row_scale(ep, m);
      if constexpr (EPI == EPI_RES) {
        atomicAdd(&ssw[m], (unsigned long long)ss_to_q24(epi_residual4(ep, m, n, s)));
      } else if constexpr (EPI == EPI_F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + slab + (size_t)m * ldo + n) =
            make_float4(s[0], s[1], s[2], s[3]);
      } else {
        uint2 pk;
        pk.x = pack2bf(s[0], s[1]);
        pk.y = pack2bf(s[2], s[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + n) = pk;
      }
    }
    if constexpr (EPI == EPI_RES) {
      __syncthreads();
      if (threadIdx.x < M) atomicAdd(reinterpret_cast<unsigned long long*>(ep.ss_out) + threadIdx.x, ssw[threadIdx.x]);
    }
  }
}

// mxfp4 [nb][kb128][lane][16 B] + scales -> bf16 fragment layout [nb][kb32][lane][8] (ops.shuffle_weight)
__global__ __launch_bounds__(256) void fp4_dequant_kernel(const uint4* __restrict__ Wq, const uint32_t* __restrict__ Sw,
                                                          int KB128, long nfrag, uint4* __restrict__ Wf) {
  const int KB4 = (KB128 + 3) >> 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nfrag * 64; i += (long)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const long f = i >> 6;  // (nb, kb128)
    const long nb = f / KB128;
    const int kb = (int)(f % KB128);
    const int r = lane & 15, g = lane >> 4;
    const float sc = e8m0_f32((Sw[(nb * KB4 + (kb >> 2)) * 64 + lane] >> (8 * (kb & 3))) & 0xffu);
    const uint4 q = Wq[i];
    const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
    // element k = 128 kb + 32 g + 8 s + e -> bf16 fragment kb32 = 4 kb + g, lane' = 16 s + r
#pragma unroll
    for (int s = 0; s < 4; ++s) Wf[((nb * 4L * KB128) + 4L * kb + g) * 64 + 16 * s + r] = fp4x8_to_bf16(qw[s], sc);
  }
}

static thread_local int g_fp4_xfrag = 0;
static thread_local LsaEpi g_fp4_epi = {};

template <int MT, int NB, int EPI, int WV, int U>
static void launch_fx(const uint16_t* X, int ldx, int M, int KB128, const uint4* Wq, const uint32_t* S, int NBtot,
                      void* out, int ldo, int kbps, int splitk, hipStream_t s) {
  if (g_fp4_xfrag)
    hipLaunchKernelGGL((gemm_fp4_skinny_kernel<MT, NB, EPI, WV, U, true>), dim3((NBtot + NB - 1) / NB, splitk), dim3(64 * WV), 0,
                       s, X, ldx, M, KB128, Wq, S, out, ldo, kbps, g_fp4_epi);
  else
    hipLaunchKernelGGL((gemm_fp4_skinny_kernel<MT, NB, EPI, WV, U, false>), dim3((NBtot + NB - 1) / NB, splitk), dim3(64 * WV), 0,
                       s, X, ldx, M, KB128, Wq, S, out, ldo, kbps, g_fp4_epi);
}

template <int EPI>
static void launch_fe(const uint16_t* X, int ldx, int M, int KB128, const uint4* Wq, const uint32_t* S, int NBtot,
                      void* out, int ldo, int nb, int splitk, int waves, hipStream_t s) {
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int kbps = (KB128 + splitk - 1) / splitk;
  // U = 2 128-k steps per chunk (one 16-B weight load feeds 4 k-steps of MFMA work: the shallow point); wide
  // n-groups (NB 8: one set of activation pieces feeds 8 weight fragments -- at 32 rows the activation loads are
  // 4 x MT / NB of the weight bytes) one step per chunk (registers)
#define LSA_F4(MTV, NBV)                                                                                           \
  if (mt == MTV && nb == NBV) {                                                                                    \
    constexpr int U4 = NBV >= 8 ? 1 : 2; /* 4 at one row tile measured slower at batch 1 (7B 1.57 -> 1.69 ms) */ \
    constexpr int U8 = (MTV >= 4 || NBV >= 4) ? 1 : U4; /* 8 waves: 256 VGPRs per wave, no spills */             \
    if (waves == 8) launch_fx<MTV, NBV, EPI, 8, U8>(X, ldx, M, KB128, Wq, S, NBtot, out, ldo, kbps, splitk, s);   \
    else launch_fx<MTV, NBV, EPI, 4, U4>(X, ldx, M, KB128, Wq, S, NBtot, out, ldo, kbps, splitk, s);              \
    return;                                                                                                        \
  }
  LSA_F4(1, 2) LSA_F4(1, 4) LSA_F4(2, 2) LSA_F4(2, 4) LSA_F4(4, 2) LSA_F4(1, 8) LSA_F4(2, 8) LSA_F4(2, 6)
  if constexpr (EPI != EPI_SILU) { LSA_F4(1, 1) LSA_F4(2, 1) LSA_F4(4, 1) }
#undef LSA_F4
  // unsupported nb: nb = 2 at the same row-tile count
  if (mt == 1) launch_fx<1, 2, EPI, 4, 2>(X, ldx, M, KB128, Wq, S, NBtot, out, ldo, kbps, splitk, s);
  else if (mt == 2) launch_fx<2, 2, EPI, 4, 2>(X, ldx, M, KB128, Wq, S, NBtot, out, ldo, kbps, splitk, s);
  else launch_fx<4, 2, EPI, 4, 2>(X, ldx, M, KB128, Wq, S, NBtot, out, ldo, kbps, splitk, s);
}

extern "C" int lsa_fp4_dequant(const void* Wq, const void* S, int N, int K, void* Wf, hipStream_t s) {
  if (K % 128 || N % 16) return -1;
  const int KB128 = K / 128;
  const long nfrag = (long)(N / 16) * KB128;
  const long gl = (nfrag * 64 + 255) / 256;
  hipLaunchKernelGGL(fp4_dequant_kernel, dim3((unsigned)(gl < 8192 ? gl : 8192)), dim3(256), 0, s,
                     reinterpret_cast<const uint4*>(Wq), reinterpret_cast<const uint32_t*>(S), KB128, nfrag,
                     reinterpret_cast<uint4*>(Wf));
  return (int)hipGetLastError();
}

// M <= 64 decode GEMM.  xfrag = 1: X in the fragment-major decode layout (a SiLU output is written in it too);
// ep (nullable): decode epilogue extensions (common.h LsaEpi)
extern "C" int lsa_fp4_gemm_ex(const void* X, int ldx, int M, int K, const void* Wq, const void* S, int N, void* out,
                               int epi, int nb, int splitk, int waves, int xfrag, const LsaEpi* ep, hipStream_t stream) {
  g_fp4_epi = ep ? *ep : LsaEpi{};
  if ((ep || epi == EPI_RES) && (M > 64 || (splitk > 1 && epi != EPI_F32 && epi != EPI_RES))) return -7;
  if (epi == EPI_RES && (!ep || !ep->h || !ep->xout || !ep->ss_out || ep->ldh != N || (splitk > 1 && !ep->tickets)))
    return -8;
  if (K % 128 != 0 || N % 16 != 0 || M <= 0 || M > 64) return -1;
  g_fp4_xfrag = xfrag ? 1 : 0;
  const int KB128 = K / 128, NBtot = N / 16;
  const int ldo = (epi == EPI_SILU) ? N / 2 : N;
  if (nb <= 0) nb = 1;
  if (epi == EPI_SILU && nb < 2) nb = 2;
  // a ragged grid (nb not dividing the n-blocks) needs >= 1 column unit per workgroup; SiLU units are pairs
  if (NBtot % nb != 0 && (epi == EPI_SILU ? (nb % 2 || NBtot % 2 || NBtot / 2 < (NBtot + nb - 1) / nb)
                                            : NBtot < (NBtot + nb - 1) / nb))
    return -2;
  if (splitk < 1) splitk = 1;
  if (epi != EPI_F32 && epi != EPI_RES && splitk != 1) return -3;
  if (M > 32 && nb > 2) nb = 2;
  const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
  const uint4* w = reinterpret_cast<const uint4*>(Wq);
  const uint32_t* sc = reinterpret_cast<const uint32_t*>(S);
  switch (epi) {
    case EPI_BF16: launch_fe<EPI_BF16>(x, ldx, M, KB128, w, sc, NBtot, out, ldo, nb, splitk, waves, stream); break;
    case EPI_F32: launch_fe<EPI_F32>(x, ldx, M, KB128, w, sc, NBtot, out, ldo, nb, splitk, waves, stream); break;
    case EPI_SILU: launch_fe<EPI_SILU>(x, ldx, M, KB128, w, sc, NBtot, out, ldo, nb, splitk, waves, stream); break;
    case EPI_RES: launch_fe<EPI_RES>(x, ldx, M, KB128, w, sc, NBtot, out, ldo, nb, splitk, waves, stream); break;
    default: return -4;
  }
  return (int)hipGetLastError();
}
