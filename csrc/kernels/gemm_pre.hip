// Decode GEMM with the residual add + RMSNorm folded into its activation prologue (batch <= 4):
//
//   x[m] = h[m] + sum_s parts[s][m]            (f32 residual stream + the previous row-parallel GEMM's split-K slabs)
//   hout[m] = x[m]                             (workgroup (0, 0) only: the residual stream's next value)
//   out[m] = rsqrt(mean(x[m]^2) + eps) * (bf16(x[m]) @ W^T)     with the RMSNorm gamma folded into W (models/llama.py)
//
// so the decode step needs no norm launch and no split-K last-arriver tail: qkv and gate_up read the previous
// projection's f32 slabs themselves.  Every workgroup loads the whole (M x K) row block -- at M <= 4 that is
// <= 64 KiB of L2 / MALL reads per workgroup -- sums it in f32, computes the row sums of squares itself (a fixed
// reduction order, so every workgroup derives bitwise the same scale) and stages bf16(x) in LDS; the first TWO
// weight chunks of every wave are issued before that prologue, so the HBM weight stream is already in flight
// while the activation row is being built (the earlier prologue form, which normalised before issuing any weight
// load, measured slower than the norm launch it replaced -- profiles/fuse_norm_mi355x.txt).
//
// Main loop: the skinny decode GEMM of gemm.hip (MT = 1: one 16-row MFMA tile, rows >= M masked), weights in
// the fragment-major layout, NB n-blocks per workgroup, split-K over grid.y (f32 slabs, each split scaled by the
// same full-row RMS), activation fragments read from LDS.  Epilogues: bf16, f32 slab, SiLU(gate) * up.
#include "common.h"

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2
#define LSA_PRE_MAXP 8  // split-K slabs of the previous projection the prologue can sum

namespace {

template <int NB, int DIV>
struct PreCfg {
  static constexpr int U0 = (16 / (NB > 2 ? NB : 2)) < 2 ? 2 : (16 / (NB > 2 ? NB : 2));
  static constexpr int U = (U0 / DIV) < 1 ? 1 : (U0 / DIV);
};

}  // namespace

template <int NB, int EPI, int WAVES, int DIV>
__global__ __launch_bounds__(64 * WAVES) void gemm_pre_kernel(const float* __restrict__ H, const float* __restrict__ parts,
                                                              int np, size_t pstride, float* __restrict__ Hout, int M,
                                                              int KB, const uint4* __restrict__ Wf, void* __restrict__ out,
                                                              int ldo, int kb_per_split, float eps) {
  constexpr int U = PreCfg<NB, DIV>::U;
  constexpr int NT = 64 * WAVES;
  extern __shared__ __attribute__((aligned(16))) uint4 xs[];  // [K / 8][M] bf16 x 8
  __shared__ float ssr[WAVES][4];
  __shared__ float rscale[4];
  const int K = KB * 32;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nb0 = blockIdx.x * NB;
  const int kbA = blockIdx.y * kb_per_split;
  const int kbB = min(KB, kbA + kb_per_split);
  const int nk = kbB - kbA;
  const int nch = (nk + U - 1) / U;
  const int n_it = nch > w ? (nch - w + WAVES - 1) / WAVES : 0;
  const int last_c = w + WAVES * (n_it - 1);

  const uint4* wp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wp[i] = Wf + (size_t)(nb0 + i) * KB * 64 + lane;
  auto wload = [&](uint4 (&wr)[U][NB], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) wr[u][i] = ldg_nt(wp[i] + (size_t)kk * 64);
    }
  };
  const int rr = min(r, M - 1);
  const bool rvalid = r < M;
  auto xload = [&](uint4 (&xr)[U], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
      xr[u] = xs[(size_t)(kk * 4 + g) * M + rr];
    }
  };
  f32x4_t acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto comp = [&](const uint4 (&wr)[U][NB], const uint4 (&xr)[U], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = (kb + u) < kbB && rvalid;
      uint4 xv = xr[u];
      xv.x = ok ? xv.x : 0u; xv.y = ok ? xv.y : 0u; xv.z = ok ? xv.z : 0u; xv.w = ok ? xv.w : 0u;
#pragma unroll
      for (int i = 0; i < NB; ++i) acc[i] = mfma16x16x32(wr[u][i], xv, acc[i]);
    }
  };

  uint4 wA[U][NB], wB[U][NB], xA[U], xB[U];
  // the first two weight chunks leave before the activation prologue (their latency overlaps it)
  if (n_it > 0) wload(wA, w);
  if (n_it > 1) wload(wB, w + WAVES);
  __builtin_amdgcn_sched_barrier(0);

  // ---- prologue: x = h + sum parts over the whole M x K block, bf16(x) -> LDS, row sums of squares
  float ss[4] = {0.f, 0.f, 0.f, 0.f};
  const bool writer = Hout != nullptr && blockIdx.x == 0 && blockIdx.y == 0;
  const int nvec = M * K / 4;
#pragma unroll 2
  for (int v = threadIdx.x; v < nvec; v += NT) {
    const size_t e = (size_t)v * 4;
    float4 a = *reinterpret_cast<const float4*>(H + e);
    float4 b[LSA_PRE_MAXP];  // every slab load of this vector leaves before the first add
#pragma unroll
    for (int s = 0; s < LSA_PRE_MAXP; ++s)
      if (s < np) b[s] = *reinterpret_cast<const float4*>(parts + s * pstride + e);
#pragma unroll
    for (int s = 0; s < LSA_PRE_MAXP; ++s)
      if (s < np) {
        a.x += b[s].x; a.y += b[s].y; a.z += b[s].z; a.w += b[s].w;
      }
    if (writer) *reinterpret_cast<float4*>(Hout + e) = a;
    const int m = (int)(e / K), k = (int)(e - (size_t)m * K);
    const float q = a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
#pragma unroll
    for (int j = 0; j < 4; ++j) ss[j] += (m == j) ? q : 0.f;
    uint2 pk;
    pk.x = pack2bf(a.x, a.y);
    pk.y = pack2bf(a.z, a.w);
    *reinterpret_cast<uint2*>(reinterpret_cast<char*>(xs) + ((size_t)(k >> 3) * M + m) * 16 + (k & 7) * 2) = pk;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float t = ss[j];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) ssr[w][j] = t;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float t = 0.f;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) t += ssr[ww][threadIdx.x];
    rscale[threadIdx.x] = rsqrtf(t / (float)K + eps);
  }
  // (rscale is read after the reduction barrier below)

  if (n_it > 0) {
    xload(xA, w);
    if (n_it > 1) xload(xB, w + WAVES);
    int i = 0;
    for (; i + 1 < n_it; i += 2) {
      comp(wA, xA, w + WAVES * i);
      __builtin_amdgcn_sched_barrier(0);
      if (i + 2 < n_it) {
        wload(wA, w + WAVES * (i + 2));
        xload(xA, w + WAVES * (i + 2));
      }
      __builtin_amdgcn_sched_barrier(0);
      comp(wB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
      if (i + 3 < n_it) {
        wload(wB, min(w + WAVES * (i + 3), last_c));
        xload(xB, min(w + WAVES * (i + 3), last_c));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(wA, xA, w + WAVES * i);
  }

  // cross-wave reduction
  __shared__ __attribute__((aligned(16))) f32x4_t red[WAVES][NB][64];
#pragma unroll
  for (int i = 0; i < NB; ++i) red[w][i][lane] = acc[i];
  __syncthreads();
  if constexpr (EPI == EPI_SILU) {
    for (int idx = threadIdx.x; idx < (NB / 2) * 64; idx += NT) {
      const int l = idx & 63, p = idx >> 6;
      f32x4_t gs = red[0][2 * p][l], us = red[0][2 * p + 1][l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) {
        gs += red[ww][2 * p][l];
        us += red[ww][2 * p + 1][l];
      }
      const int m = l & 15;
      if (m < M) {
        const int n = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
        const float sc = rscale[m];
        uint2 pk;
        pk.x = pack2bf(silu(gs[0] * sc) * (us[0] * sc), silu(gs[1] * sc) * (us[1] * sc));
        pk.y = pack2bf(silu(gs[2] * sc) * (us[2] * sc), silu(gs[3] * sc) * (us[3] * sc));
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + n) = pk;
      }
    }
  } else {
    const size_t slab = (size_t)blockIdx.y * M * ldo;
    for (int idx = threadIdx.x; idx < NB * 64; idx += NT) {
      const int l = idx & 63, i = idx >> 6;
      f32x4_t s = red[0][i][l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) s += red[ww][i][l];
      const int m = l & 15;
      if (m < M) {
        s *= rscale[m];
        const int n = (nb0 + i) * 16 + 4 * (l >> 4);
        if constexpr (EPI == EPI_F32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + slab + (size_t)m * ldo + n) =
              make_float4(s[0], s[1], s[2], s[3]);
        } else {
          uint2 pk;
          pk.x = pack2bf(s[0], s[1]);
          pk.y = pack2bf(s[2], s[3]);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + n) = pk;
        }
      }
    }
  }
}

// M <= 4 rows; K % 32 == 0; N % 16 == 0 (EPI_SILU: gate/up rows interleaved per 16, N % 32 == 0); parts: np f32
// slabs [np][M][K] pstride elements apart (np = 0: none); hout (nullable): receives h + sum parts (must not alias h:
// every workgroup reads h while workgroup (0, 0) writes hout).  nb 1 | 2 | 4 | 8, waves 4 | 8, div 1 | 2 | 4.
extern "C" int lsa_gemm_pre(const float* h, const float* parts, int np, long pstride, float* hout, int M, int K,
                            const void* Wf, int N, void* out, int epi, int nb, int splitk, int waves, int div, float eps,
                            hipStream_t stream) {
  if (M < 1 || M > 4 || K % 32 != 0 || N % 16 != 0 || np < 0 || np > LSA_PRE_MAXP || (np > 0 && !parts)) return -1;
  if (hout && hout == h) return -9;
  const int KB = K / 32, NBtot = N / 16;
  if (nb <= 0) nb = 1;
  if (epi == EPI_SILU && (nb < 2 || nb % 2)) return -2;
  if (NBtot % nb != 0) return -2;
  if (splitk < 1) splitk = 1;
  if (epi != EPI_F32 && splitk != 1) return -3;
  const int kbps = (KB + splitk - 1) / splitk;
  if ((KB + kbps - 1) / kbps != splitk) return -3;
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  const size_t lds = (size_t)M * K * 2;
  if (lds > 64 * 1024) return -6;
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
  dim3 grid(NBtot / nb, splitk);
  waves = waves == 8 ? 8 : 4;
  div = (div == 1 || div == 2) ? div : 4;
#define LSA_PRE(NBV, EPIV, WV, DV)                                                                               \
  if (nb == NBV && epi == EPIV && waves == WV && div == DV) {                                                   \
    hipLaunchKernelGGL((gemm_pre_kernel<NBV, EPIV, WV, DV>), grid, dim3(64 * WV), lds, stream, h, parts, np,    \
                       (size_t)pstride, hout, M, KB, w, out, ldo, kbps, eps);                                   \
    return (int)hipGetLastError();                                                                             \
  }
#define LSA_PRE_D(NBV, EPIV, WV) LSA_PRE(NBV, EPIV, WV, 1) LSA_PRE(NBV, EPIV, WV, 2) LSA_PRE(NBV, EPIV, WV, 4)
#define LSA_PRE_W(NBV, EPIV) LSA_PRE_D(NBV, EPIV, 4) LSA_PRE_D(NBV, EPIV, 8)
  LSA_PRE_W(1, EPI_F32) LSA_PRE_W(2, EPI_F32) LSA_PRE_W(4, EPI_F32)
  LSA_PRE_W(1, EPI_BF16) LSA_PRE_W(2, EPI_BF16)
  LSA_PRE_W(2, EPI_SILU) LSA_PRE_W(4, EPI_SILU) LSA_PRE_W(8, EPI_SILU)
#undef LSA_PRE_W
#undef LSA_PRE_D
#undef LSA_PRE
  return -4;
}
