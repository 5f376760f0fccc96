// W8A8 decode linear layers (M <= 64) on the gfx950 fp8 MFMA:  out = (X8 * sx[m]) @ (Wq * wscale[n])^T
//
// The W8A16 decode kernel (gemm_fp8.hip) converts every weight to bf16 on the VALU and reads bf16
// activation fragments: at M = 32 it moves 2 * MT / NB bytes of activations per weight byte through L2 and
// streams the weights at ~4 TB/s (profiles/bench_fp8_decode_wide_nb_mi355x.jsonl).  Here the activations
// are fp8 too (per-row scale sx, quantised by the producing add_rmsnorm launch straight into the fragment
// layout below), so one v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales) consumes a 2 KiB weight
// slab and a 2 KiB activation slab per 16 x 16 x 128 step: half the activation bytes, no conversion VALU,
// a quarter of the MFMA issues.  Same work split as the skinny kernels: chunks of U k128-steps dealt
// round-robin to the waves, split-K over blockIdx.y, a two-deep register pipeline pinned with
// sched_barrier, cross-wave reduction through LDS.
//
// Weights: the fp8 decode layout Wq[nb][kb64][lane][16 B] (lane = 16 g + r holds W[16 nb + r][64 kb64 +
// 16 g .. +15]); one MFMA A operand = fragments kb64 = 2 s and 2 s + 1 of lane l, i.e. the k-set
// {128 s + 16 g .. +15} u {128 s + 64 + 16 g .. +15}.
// Activations ("xf8"): X8[kb128][MT][lane][32 B], lane (g, r) holds row 16 mt + r over the same k-set
// (ops.to_xf8 / the add_rmsnorm fp8 output), rows >= M masked here.
//
// Epilogues: EPI_F32 -> f32 split-K slabs [splitk][M][N];  EPI_SILU -> bf16 silu(gate) * up, gate / up rows
// interleaved per 16, written in the bf16 fragment-major layout (xf_off) for the W8A16 down projection.
// The rownorm extension (LsaEpi.rowss) multiplies a row scale in like the other decode GEMMs.
#include "common.h"

#define EPI_F32 1
#define EPI_SILU 2

typedef int a8_i32x8_t __attribute__((ext_vector_type(8)));

namespace {

__device__ __forceinline__ f32x4_t mfma_a8(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1, f32x4_t c) {
  const a8_i32x8_t a = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
  const a8_i32x8_t b = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  // formats 0 / 0 = e4m3 x e4m3; block scales 0x7f = 2^0 (the real scales are applied in the epilogue)
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}

}  // namespace

template <int MT, int NB, int EPI, int WAVES, int U, bool XFO>
__global__ __launch_bounds__(64 * WAVES) void gemm_a8_skinny_kernel(const uint4* __restrict__ X8, const float* __restrict__ sx,
                                                                    int M, int KB128, const uint4* __restrict__ Wq,
                                                                    const float* __restrict__ wscale, void* __restrict__ out,
                                                                    int ldo, int kb_per_split, LsaEpi ep) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15;
  int nb0, cnt;  // this workgroup's n-blocks (ragged grids: common.h skinny_nblocks)
  skinny_nblocks<NB, EPI == EPI_SILU ? 2 : 1>(EPI == EPI_SILU ? ldo / 8 : ldo / 16, nb0, cnt);
  const int kbA = blockIdx.y * kb_per_split;
  const int kbB = min(KB128, kbA + kb_per_split);
  const int nk = kbB - kbA;
  const int nch = (nk + U - 1) / U;
  const int n_it = nch > w ? (nch - w + WAVES - 1) / WAVES : 0;
  const int last_c = w + WAVES * (n_it - 1);

  f32x4_t acc[NB][MT];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bool xvalid[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) xvalid[j] = j * 16 + r < M;
  const uint4* wp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wp[i] = Wq + (size_t)(nb0 + min(i, cnt - 1)) * (2 * KB128) * 64 + lane;
  const uint4* xp = X8 + 2 * lane;

  auto load = [&](uint4 (&wr)[U][NB][2], uint4 (&xr)[U][MT][2], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        wr[u][i][0] = ldg_nt(wp[i] + (size_t)(2 * kk) * 64);
        wr[u][i][1] = ldg_nt(wp[i] + (size_t)(2 * kk + 1) * 64);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const uint4* px = xp + (size_t)(kk * MT + j) * 128;
        xr[u][j][0] = px[0];
        xr[u][j][1] = px[1];
      }
    }
  };
  auto comp = [&](const uint4 (&wr)[U][NB][2], const uint4 (&xr)[U][MT][2], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = (kb + u) < kbB;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const bool ok = live && xvalid[j];
        uint4 x0 = xr[u][j][0], x1 = xr[u][j][1];
        x0.x = ok ? x0.x : 0u; x0.y = ok ? x0.y : 0u; x0.z = ok ? x0.z : 0u; x0.w = ok ? x0.w : 0u;
        x1.x = ok ? x1.x : 0u; x1.y = ok ? x1.y : 0u; x1.z = ok ? x1.z : 0u; x1.w = ok ? x1.w : 0u;
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i][j] = mfma_a8(wr[u][i][0], wr[u][i][1], x0, x1, acc[i][j]);
      }
    }
  };
  if (n_it > 0) {
    uint4 wA[U][NB][2], xA[U][MT][2], wB[U][NB][2], xB[U][MT][2];
    load(wA, xA, w);
    int i = 0;
    for (; i + 1 < n_it; i += 2) {
      load(wB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
      comp(wA, xA, w + WAVES * i);
      __builtin_amdgcn_sched_barrier(0);
      load(wA, xA, min(w + WAVES * (i + 2), last_c));
      __builtin_amdgcn_sched_barrier(0);
      comp(wB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(wA, xA, w + WAVES * i);
  }

  __shared__ __attribute__((aligned(16))) f32x4_t red[WAVES][NB * MT][64];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) red[w][i * MT + j][lane] = acc[i][j];
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
        const int nrow_g = (nb0 + 2 * p) * 16 + 4 * (l >> 4);
        const int nrow_u = nrow_g + 16;
        const int n = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
        const float sc = sx[m] * epi_row_scale(ep, m);
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(gs[q] * (sc * wscale[nrow_g + q])) * (us[q] * (sc * wscale[nrow_u + q]));
        uint2 pk;
        pk.x = pack2bf(v[0], v[1]);
        pk.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (XFO ? xf_off(m, n, MT) : (size_t)m * ldo + n)) = pk;
      }
    }
  } else {
    const size_t slab = (size_t)blockIdx.y * M * ldo;
    for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
      const int l = idx & 63, t = idx >> 6;
      const int j = t % MT, i = t / MT;
      f32x4_t s = red[0][t][l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) s += red[ww][t][l];
      const int m = j * 16 + (l & 15);
      if (m >= M || i >= cnt) continue;
      const int n = (nb0 + i) * 16 + 4 * (l >> 4);
      const float4 sc = *reinterpret_cast<const float4*>(wscale + n);
      const float rs = sx[m] * epi_row_scale(ep, m);
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + slab + (size_t)m * ldo + n) =
          make_float4(s[0] * sc.x * rs, s[1] * sc.y * rs, s[2] * sc.z * rs, s[3] * sc.w * rs);
    }
  }
}

static thread_local LsaEpi g_a8_epi = {};
static thread_local int g_a8_waves = 4, g_a8_depth = 1, g_a8_xfo = 1;

template <int MT, int NB, int EPI, int WV, int U>
static void launch_a8_x(const uint4* X8, const float* sx, int M, int KB128, const uint4* Wq, const float* sc, int NBtot,
                        void* out, int ldo, int splitk, hipStream_t s) {
  const int kbps = (KB128 + splitk - 1) / splitk;
  if (g_a8_xfo)
    hipLaunchKernelGGL((gemm_a8_skinny_kernel<MT, NB, EPI, WV, U, true>), dim3((NBtot + NB - 1) / NB, splitk), dim3(64 * WV), 0, s,
                       X8, sx, M, KB128, Wq, sc, out, ldo, kbps, g_a8_epi);
  else
    hipLaunchKernelGGL((gemm_a8_skinny_kernel<MT, NB, EPI, WV, U, false>), dim3((NBtot + NB - 1) / NB, splitk), dim3(64 * WV), 0, s,
                       X8, sx, M, KB128, Wq, sc, out, ldo, kbps, g_a8_epi);
}

template <int MT, int NB, int EPI>
static void launch_a8_t(const uint4* X8, const float* sx, int M, int KB128, const uint4* Wq, const float* sc, int NBtot,
                        void* out, int ldo, int splitk, hipStream_t s) {
  // U0 k128-steps per chunk: 2 for one n-block, else 1 (a chunk is NB * U 2 KiB weight slabs per wave);
  // depth 2 doubles it
  // (8 waves and depth 2 only where the registers allow: the wide / 4-tile variants would spill)
  constexpr int U = NB == 1 ? 2 : 1;
  if constexpr (NB <= 4 && MT <= 2) {
    if (g_a8_waves == 8) {
      if (g_a8_depth == 2) launch_a8_x<MT, NB, EPI, 8, 2 * U>(X8, sx, M, KB128, Wq, sc, NBtot, out, ldo, splitk, s);
      else launch_a8_x<MT, NB, EPI, 8, U>(X8, sx, M, KB128, Wq, sc, NBtot, out, ldo, splitk, s);
      return;
    }
    if (g_a8_depth == 2) {
      launch_a8_x<MT, NB, EPI, 4, 2 * U>(X8, sx, M, KB128, Wq, sc, NBtot, out, ldo, splitk, s);
      return;
    }
  }
  launch_a8_x<MT, NB, EPI, 4, U>(X8, sx, M, KB128, Wq, sc, NBtot, out, ldo, splitk, s);
}

template <int EPI>
static int launch_a8_e(const uint4* X8, const float* sx, int M, int KB128, const uint4* Wq, const float* sc, int NBtot,
                       void* out, int ldo, int nb, int splitk, hipStream_t s) {
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_A8(MTV, NBV)                                                             \
  if (mt == MTV && nb == NBV) {                                                      \
    launch_a8_t<MTV, NBV, EPI>(X8, sx, M, KB128, Wq, sc, NBtot, out, ldo, splitk, s); \
    return 0;                                                                        \
  }
  LSA_A8(1, 2) LSA_A8(1, 4) LSA_A8(2, 2) LSA_A8(2, 4) LSA_A8(2, 6) LSA_A8(2, 8) LSA_A8(4, 2)
  if constexpr (EPI != EPI_SILU) { LSA_A8(1, 1) LSA_A8(2, 1) LSA_A8(4, 1) }
#undef LSA_A8
  return -6;  // unsupported (mt, nb)
}

// xfo: the SiLU output in the bf16 fragment-major layout (16 < M <= 64 decode) or row-major [M, N / 2]
extern "C" int lsa_fp8a_gemm(const void* X8, const float* sx, int M, int K, const void* Wq, const float* wscale, int N,
                             void* out, int epi, int nb, int splitk, int waves, int depth, int xfo, const LsaEpi* ep,
                             hipStream_t stream) {
  if (M <= 0 || M > 64 || K % 128 != 0 || N % 16 != 0) return -1;
  if (epi != EPI_F32 && epi != EPI_SILU) return -4;
  g_a8_epi = ep ? *ep : LsaEpi{};
  g_a8_waves = waves == 8 ? 8 : 4;
  g_a8_depth = depth == 2 ? 2 : 1;
  g_a8_xfo = xfo ? 1 : 0;
  const int KB128 = K / 128, NBtot = N / 16;
  if (nb <= 0) nb = 2;
  if (epi == EPI_SILU && nb < 2) nb = 2;
  if (M > 32 && nb > 2) nb = 2;
  // a ragged grid (nb not dividing the n-blocks) needs >= 1 column unit per workgroup; SiLU units are pairs
  if (NBtot % nb != 0 && (epi == EPI_SILU ? (nb % 2 || NBtot % 2 || NBtot / 2 < (NBtot + nb - 1) / nb)
                                            : NBtot < (NBtot + nb - 1) / nb))
    return -2;
  if (splitk < 1) splitk = 1;
  if (epi == EPI_SILU && splitk != 1) return -3;
  if ((KB128 + ((KB128 + splitk - 1) / splitk) - 1) / ((KB128 + splitk - 1) / splitk) != splitk) return -3;
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  const uint4* x8 = reinterpret_cast<const uint4*>(X8);
  const uint4* w = reinterpret_cast<const uint4*>(Wq);
  const int rc = epi == EPI_F32 ? launch_a8_e<EPI_F32>(x8, sx, M, KB128, w, wscale, NBtot, out, ldo, nb, splitk, stream)
                                : launch_a8_e<EPI_SILU>(x8, sx, M, KB128, w, wscale, NBtot, out, ldo, nb, splitk, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// x [M, K] bf16 -> xf8 fragment layout (rows of the mt tiles past M zeroed) + per-row scale amax / 448:
// the standalone form of the add_rmsnorm fp8 output (tests, benches, prefill-free callers)
__global__ __launch_bounds__(256) void quant_xf8_kernel(const uint16_t* __restrict__ x, int ldx, int M, int K, int MT,
                                                        uint8_t* __restrict__ x8, float* __restrict__ sx) {
  __shared__ float red[8];
  const int m = blockIdx.x;  // one workgroup per row of the MT tiles
  float amax = 0.f;
  if (m < M)
    for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * ldx + c), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
    }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-30f) / 448.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0 && m < M) sx[m] = s;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    uint2 q = make_uint2(0u, 0u);
    if (m < M) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * ldx + c), f);
      q = pack8_fp8(f, inv);
    }
    *reinterpret_cast<uint2*>(x8 + xf8_off(m, c, MT)) = q;
  }
}

extern "C" int lsa_quant_xf8(const void* x, int ldx, int M, int K, int MT, void* x8, float* sx, hipStream_t s) {
  if (M <= 0 || M > 16 * MT || K % 128 != 0) return -1;
  hipLaunchKernelGGL(quant_xf8_kernel, dim3(16 * MT), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x), ldx, M, K, MT,
                     reinterpret_cast<uint8_t*>(x8), sx);
  return (int)hipGetLastError();
}
