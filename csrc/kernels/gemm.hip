// Linear layers on MFMA for gfx950:  out[M, N] = X[M, K] @ W[N, K]^T   (bf16 in, f32 accumulate)
//
// Weights live in the "fragment-major" layout produced by ops.shuffle_weight():
//     Wf[nb][kb][lane][8 bf16]  with  nb = n / 16, kb = k / 32, lane = 16 * ((k % 32) / 8) + n % 16
// i.e. one 1 KiB MFMA A-fragment (16 rows x 32 k) per (nb, kb), lane-linear.  Every weight load
// is therefore a fully coalesced 1 KiB wave-instruction (global_load_dwordx4) and, in the tiled
// kernel, a lane-linear global_load_lds_dwordx4 whose LDS image is read back with conflict-free
// ds_read_b128 at lane*16 (no swizzle needed: cdna_hip_programming.md §5 Caveat / rule 21).
//
// Two kernels:
//   * gemm_skinny  — decode (M <= 64).  Memory-bound weight stream: 8 waves/WG split K, each wave
//     keeps 16 x 1 KiB weight fragments in flight straight into VGPRs (no LDS round trip, the
//     'GEMV / M <= 16 decode weights' row of the guide), non-temporal weight loads, cross-wave
//     reduction through LDS, fused epilogues (bf16 store, f32 split-K slab for the following
//     residual+RMSNorm kernel, SiLU(gate)*up for the interleaved gate_up projection).
//   * gemm_tile    — prefill (M > 64) when the 256^2 kernel (gemm_tile256.hip) would under-fill the
//     chip.  128x128x64 LDS tile, both operands staged by global_load_lds (16 B), double-buffered,
//     4 waves of 64x64.
//
// Epilogue modes: EPI_BF16 -> bf16 [M, N];  EPI_F32 -> f32 [splitk][M][N];
//                 EPI_SILU -> bf16 [M, N/2] = silu(gate) * up, gate/up rows interleaved per 16.
#include "common.h"

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2


template <int EPI>
__device__ __forceinline__ void store4(void* out, int ldo, size_t slab, int m, int n, f32x4_t v) {
  if constexpr (EPI == EPI_F32) {
    float* o = reinterpret_cast<float*>(out) + slab + (size_t)m * ldo + n;
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint16_t* o = reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + n;
    uint2 p;
    p.x = pack2bf(v[0], v[1]);
    p.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(o) = p;
  }
}


// ------------------------------------------------------------------------------------------------
// decode / small-M kernel
//
// Work split: workgroup = 8 waves over NB n-blocks (16 rows each) and one split-K range; the range is
// cut into chunks of U k-steps dealt round-robin to the waves.  Each wave streams its chunks with a
// two-deep register pipeline: chunk i+1's NB*U weight fragments (+ the activation fragments) are in
// flight while chunk i's MFMAs run, so the memory pipe never drains between chunks.  Out-of-range
// k-steps are clamped (duplicate L2 hits) and masked by zeroing the activation fragment, never by a
// per-load branch (which would force vmcnt(0) per element).
// ------------------------------------------------------------------------------------------------
template <int MT, int NB, int DIV = 1>
struct SkinnyCfg {
  static constexpr int U0 = (16 / (NB > 2 * MT ? NB : 2 * MT)) < 2 ? 2 : (16 / (NB > 2 * MT ? NB : 2 * MT));
  static constexpr int U = (U0 / DIV) < 1 ? 1 : (U0 / DIV);
};

// XF: X is in the fragment-major activation layout Xf[k/32][MT][64 lanes][8 bf16] (ops.to_xfrag,
// written directly by the producing kernels in the decode path), so an activation fragment is one
// lane-linear 1 KiB load (8 full lines) instead of 16 half-used row segments.
//
// RR > 0 (batch 1, MT = 1): the residual-reduce prologue of lsa_epi.h LsaRr, RR = the most split-K slabs it sums
// (the loads are clamped to slab np - 1 and masked, so every slab load of a lane leaves before the first add).
// The workgroup's X slice (<= RR_KMAX values) is formed once into LDS as bf16 and the k-step fragments are read
// back from there (16 lanes of a row group read one address: broadcast, conflict-free).  Replaces the residual-add
// launch between the row-parallel projection and this GEMM (one kernel boundary less per layer side).
#define RR_KMAX 8192
template <int MT, int NB, int EPI, int WAVES, int DIV = 1, bool XF = false, int RR = 0>
__global__ __launch_bounds__(64 * WAVES) void gemm_skinny_kernel(const uint16_t* __restrict__ X, int ldx, int M,
                                                                 int KB, const uint4* __restrict__ Wf,
                                                                 void* __restrict__ out, int ldo,
                                                                 int kb_per_split, LsaEpi ep, LsaRr rr) {
  static_assert(RR == 0 || (MT == 1 && !XF && EPI != EPI_RES), "residual-reduce prologue: batch 1, row-major");
  constexpr int U = SkinnyCfg<MT, NB, DIV>::U;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  int nb0, cnt;  // this workgroup's n-blocks (ragged grids: common.h skinny_nblocks)
  skinny_nblocks<NB, EPI == EPI_SILU ? 2 : 1>(EPI == EPI_SILU ? ldo / 8 : ldo / 16, nb0, cnt);
  const int kbA = blockIdx.y * kb_per_split;
  const int kbB = min(KB, kbA + kb_per_split);
  const int nk = kbB - kbA;
  const int nch = (nk + U - 1) / U;                     // chunks in this split
  const int n_it = nch > w ? (nch - w + WAVES - 1) / WAVES : 0;  // chunks of this wave
  const int last_c = w + WAVES * (n_it - 1);

  f32x4_t acc[NB][MT];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const uint16_t* xp[MT];
  bool xvalid[MT];
  // row-major X: rows >= M are read through a buffer resource at an offset past its range, so the hardware
  // returns zeros without a memory request (at batch 1 the 15 padding rows of the 16-row MFMA tile were 15/16
  // of the activation loads, every one re-reading row 0's lines)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, XF ? 0 : M * ldx * 2, 0x00020000);
  uint32_t xoff[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = j * 16 + r;
    xvalid[j] = m < M;
    xp[j] = XF ? X + ((size_t)j * 64 + lane) * 8 : X + (size_t)(xvalid[j] ? m : 0) * ldx + 8 * g;
    xoff[j] = xvalid[j] ? (uint32_t)(((size_t)m * ldx + 8 * g) * 2) : 0x80000000u;
  }
  const uint4* wp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wp[i] = Wf + (size_t)(nb0 + min(i, cnt - 1)) * KB * 64 + lane;

  auto wload = [&](uint4 (&wr)[U][NB], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) wr[u][i] = ldg_nt(wp[i] + (size_t)kk * 64);
    }
  };
  // RR: the workgroup's X slice as bf16 (k - kbA * 32), filled by the prologue below
  __shared__ __attribute__((aligned(16))) uint4 xs[RR ? RR_KMAX / 8 : 1];
  auto xload = [&](uint4 (&xr)[U][MT], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if constexpr (RR > 0) {
          xr[u][j] = xs[(kk - kbA) * 4 + g];
        } else if constexpr (XF) {
          xr[u][j] = *reinterpret_cast<const uint4*>(xp[j] + (size_t)kk * MT * 512);
        } else {
          const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff[j] + (uint32_t)kk * 64u, 0, 0);
          xr[u][j] = make_uint4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };
  auto load = [&](uint4 (&wr)[U][NB], uint4 (&xr)[U][MT], int c) {
    wload(wr, c);
    xload(xr, c);
  };
  auto comp = [&](const uint4 (&wr)[U][NB], const uint4 (&xr)[U][MT], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = (kb + u) < kbB;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const bool ok = live && xvalid[j];
        uint4 xv = xr[u][j];
        xv.x = ok ? xv.x : 0u; xv.y = ok ? xv.y : 0u; xv.z = ok ? xv.z : 0u; xv.w = ok ? xv.w : 0u;
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i][j] = mfma16x16x32(wr[u][i], xv, acc[i][j]);
      }
    }
  };

  // RR prologue: X = h + sum_s parts[s] over this split's K slice -> LDS (bf16) and, from the f32 values, the
  // slice's sum of squares.  The first weight chunk is requested before it (it does not depend on X), so the
  // prologue's L2 round trip overlaps the weight stream's HBM latency.
  float rr_scale = 1.f;
  uint4 wA[U][NB], xA[U][MT], wB[U][NB], xB[U][MT];
  if constexpr (RR > 0) {
    if (n_it > 0) wload(wA, w);
    __shared__ float rr_red[WAVES];
    const int k0 = kbA * 32, n8 = nk * 4;  // 8-value groups of the slice
    const bool wr_h = blockIdx.x == 0;
    float ssl = 0.f;
    for (int i = threadIdx.x; i < n8; i += 64 * WAVES) {
      const size_t e = (size_t)k0 + 8 * i;
      float4 a[RR + 1][2];
      a[0][0] = *reinterpret_cast<const float4*>(rr.h + e);
      a[0][1] = *reinterpret_cast<const float4*>(rr.h + e + 4);
#pragma unroll
      for (int s = 0; s < RR; ++s) {
        const float* p = rr.parts + (size_t)min(s, rr.np - 1) * rr.pstride + e;
        a[s + 1][0] = *reinterpret_cast<const float4*>(p);
        a[s + 1][1] = *reinterpret_cast<const float4*>(p + 4);
      }
      float v[8] = {a[0][0].x, a[0][0].y, a[0][0].z, a[0][0].w, a[0][1].x, a[0][1].y, a[0][1].z, a[0][1].w};
#pragma unroll
      for (int s = 0; s < RR; ++s) {
        const float on = s < rr.np ? 1.f : 0.f;
        v[0] += on * a[s + 1][0].x; v[1] += on * a[s + 1][0].y; v[2] += on * a[s + 1][0].z; v[3] += on * a[s + 1][0].w;
        v[4] += on * a[s + 1][1].x; v[5] += on * a[s + 1][1].y; v[6] += on * a[s + 1][1].z; v[7] += on * a[s + 1][1].w;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ssl += v[j] * v[j];
      if (wr_h) {
        *reinterpret_cast<float4*>(rr.h_out + e) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(rr.h_out + e + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
      xs[i] = pack8(v);
    }
    ssl = wave_sum(ssl);
    if (lane == 0) rr_red[w] = ssl;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) tot += rr_red[ww];
    if (rr.local) rr_scale = rsqrtf(tot * rr.inv_k + rr.eps);
    else if (wr_h && threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(rr.ss_out), (unsigned long long)ss_to_q24(tot));
    if (n_it > 0) xload(xA, w);
  } else {
    if (n_it > 0) load(wA, xA, w);
  }
  if (n_it > 0) {
    int i = 0;
    // sched_barrier(0) pins the issue order: the next chunk's loads all leave before this chunk's
    // MFMAs (hipcc otherwise interleaves them and keeps only ~8 loads in flight)
    for (; i + 1 < n_it; i += 2) {
      load(wB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
      comp(wA, xA, w + WAVES * i);
      __builtin_amdgcn_sched_barrier(0);
      load(wA, xA, min(w + WAVES * (i + 2), last_c));  // clamped: the tail re-reads a cached chunk
      __builtin_amdgcn_sched_barrier(0);
      comp(wB, xB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(wA, xA, w + WAVES * i);
  }

  // cross-wave reduction: red[w][tile][lane]
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
      const int l = idx & 63;
      const int t = idx >> 6;
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
        const float sc = epi_row_scale(ep, m) * rr_scale;
        f32x4_t v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(gs[q] * sc) * (us[q] * sc);
        if constexpr (XF) {  // fragment-major in -> fragment-major out (the down projection's input)
          uint2 pk;
          pk.x = pack2bf(v[0], v[1]);
          pk.y = pack2bf(v[2], v[3]);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + xf_off(m, n, MT)) = pk;
        } else {
          store4<EPI_SILU>(out, ldo, 0, m, n, v);
        }
      }
    }
  } else {
    const size_t slab = (size_t)blockIdx.y * M * ldo;
    if constexpr (EPI == EPI_RES) {
      if (gridDim.y > 1) {  // split-K: publish, ticket, the last split finishes the column
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
          const int l = idx & 63, t = idx >> 6;
          const int j = t % MT, i = t / MT;
          f32x4_t s = red[0][t][l];
#pragma unroll
          for (int ww = 1; ww < WAVES; ++ww) s += red[ww][t][l];
          const int m = j * 16 + (l & 15);
          if (m < M && i < cnt) res_store_partial(rs, slab + (size_t)m * ldo + (nb0 + i) * 16 + 4 * (l >> 4), s);
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
                epi_residual4(ep, m, n, res_slab_sum(rs, (size_t)m * ldo + n, (size_t)M * ldo, gridDim.y) *
                                        epi_row_scale(ep, m))));
          }
        }
        __syncthreads();
        if (threadIdx.x < M) atomicAdd(reinterpret_cast<unsigned long long*>(ep.ss_out) + threadIdx.x, ssw[threadIdx.x]);
        return;
      }
    }
    for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
      const int l = idx & 63;
      const int t = idx >> 6;
      const int j = t % MT, i = t / MT;
      f32x4_t s = red[0][t][l];
#pragma unroll
      for (int ww = 1; ww < WAVES; ++ww) s += red[ww][t][l];
      const int m = j * 16 + (l & 15);
      if (m < M && i < cnt) {
        s *= epi_row_scale(ep, m) * rr_scale;
        const int n = (nb0 + i) * 16 + 4 * (l >> 4);
        if constexpr (EPI == EPI_RES) atomicAdd(&ssw[m], (unsigned long long)ss_to_q24(epi_residual4(ep, m, n, s)));
        else store4<EPI>(out, ldo, slab, m, n, s);
      }
    }
    if constexpr (EPI == EPI_RES) {
      __syncthreads();
      if (threadIdx.x < M) atomicAdd(reinterpret_cast<unsigned long long*>(ep.ss_out) + threadIdx.x, ssw[threadIdx.x]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
// Per-call tuning knobs (chosen by ops.pick_gemm_config from the measured table):
//   waves 4|8 per workgroup (a 16-wave variant for one 16-row tile never won a sweep: removed in round 4); div 1|2|4 divides the chunk depth U (fewer VGPRs -> more resident waves;
//   on MI355X div 4 won most decode shapes, scripts/bench_gemm.py).
static thread_local int g_skinny_waves = 4;
static thread_local int g_skinny_div = 4;

static thread_local LsaEpi g_epi = {};
static thread_local LsaRr g_rr = {};

template <int MT, int NB, int EPI, bool XF, int RR = 0>
static void launch_skinny_x(const uint16_t* X, int ldx, int M, int KB, const uint4* Wf, int NBtot, void* out,
                            int ldo, int splitk, hipStream_t s) {
  const int kbps = (KB + splitk - 1) / splitk;
  dim3 grid((NBtot + NB - 1) / NB, splitk);  // ragged when NB does not divide NBtot (kernel deals the blocks)
#define LSA_SKL(WV, DV) \
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NB, EPI, WV, DV, XF, RR>), grid, dim3(64 * WV), 0, s, X, \
                     ldx, M, KB, Wf, out, ldo, kbps, g_epi, g_rr)
  if constexpr (NB >= 6) {
    // wide n-groups (one activation fragment feeds NB weight fragments): 4 waves only, the cross-wave
    // reduction buffer is WAVES * NB * MT KiB
    if (g_skinny_div == 1) LSA_SKL(4, 1);
    else LSA_SKL(4, 2);
  } else if (g_skinny_div == 2) {
    if (g_skinny_waves == 8) LSA_SKL(8, 2);
    else LSA_SKL(4, 2);
  } else if (g_skinny_div == 4) {
    LSA_SKL(4, 4);
  } else {
    if (g_skinny_waves == 8) LSA_SKL(8, 1);
    else LSA_SKL(4, 1);
  }
#undef LSA_SKL
}

static thread_local int g_xfrag = 0;

template <int MT, int NB, int EPI>
static void launch_skinny_t(const uint16_t* X, int ldx, int M, int KB, const uint4* Wf, int NBtot, void* out,
                            int ldo, int splitk, hipStream_t s) {
  if (g_xfrag) launch_skinny_x<MT, NB, EPI, true>(X, ldx, M, KB, Wf, NBtot, out, ldo, splitk, s);
  else launch_skinny_x<MT, NB, EPI, false>(X, ldx, M, KB, Wf, NBtot, out, ldo, splitk, s);
}

template <int EPI>
static void launch_skinny_e(const uint16_t* X, int ldx, int M, int KB, const uint4* Wf, int NBtot, void* out,
                            int ldo, int nb, int splitk, hipStream_t s) {
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_SK(MTV, NBV)                                                                         \
  if (mt == MTV && nb == NBV) {                                                                  \
    launch_skinny_t<MTV, NBV, EPI>(X, ldx, M, KB, Wf, NBtot, out, ldo, splitk, s);               \
    return;                                                                                      \
  }
  LSA_SK(1, 2) LSA_SK(1, 4) LSA_SK(2, 2) LSA_SK(2, 4) LSA_SK(4, 2) LSA_SK(2, 6) LSA_SK(2, 8) LSA_SK(1, 8)
  if constexpr (EPI != EPI_SILU) { LSA_SK(1, 1) LSA_SK(2, 1) LSA_SK(4, 1) }
#undef LSA_SK
  // fallback (nb=4 with mt=4 or unsupported): nb=2 at the same row-tile count
  if (mt == 1) launch_skinny_t<1, 2, EPI>(X, ldx, M, KB, Wf, NBtot, out, ldo, splitk, s);
  else if (mt == 2) launch_skinny_t<2, 2, EPI>(X, ldx, M, KB, Wf, NBtot, out, ldo, splitk, s);
  else launch_skinny_t<4, 2, EPI>(X, ldx, M, KB, Wf, NBtot, out, ldo, splitk, s);
}

extern "C" int lsa_gemm_cfg(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb,
                            int splitk, int waves, int div, int xlds, hipStream_t stream);

extern "C" int lsa_gemm(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb,
                        int splitk, hipStream_t stream) {
  return lsa_gemm_cfg(X, ldx, M, K, Wf, N, out, epi, nb, splitk, 4, 4, 0, stream);
}

extern "C" int lsa_gemm_ex(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb,
                           int splitk, int waves, int div, int xlds, const LsaEpi* ep, hipStream_t stream);

extern "C" int lsa_gemm_cfg(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb,
                            int splitk, int waves, int div, int xlds, hipStream_t stream) {
  return lsa_gemm_ex(X, ldx, M, K, Wf, N, out, epi, nb, splitk, waves, div, xlds, nullptr, stream);
}

// ep (nullable): decode epilogue extensions (common.h LsaEpi): row scale and/or epi == EPI_RES; M <= 64 only
extern "C" int lsa_gemm_ex(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb,
                           int splitk, int waves, int div, int xlds, const LsaEpi* ep, hipStream_t stream) {
  g_epi = ep ? *ep : LsaEpi{};
  if ((ep || epi == EPI_RES) && (M > 64 || (splitk > 1 && epi != EPI_F32 && epi != EPI_RES))) return -7;
  if (epi == EPI_RES && (!ep || !ep->h || !ep->xout || !ep->ss_out || ep->ldh != N || (splitk > 1 && !ep->tickets)))
    return -8;
  g_skinny_waves = waves == 8 ? 8 : 4;
  g_skinny_div = (div == 1 || div == 2) ? div : 4;
  // xlds: 0 = row-major X, 2 = fragment-major X (ops.to_xfrag); the LDS-staged variant (1) was removed in
  // round 4 (measured slower than the register pipeline on every decode shape, ARCHITECTURE.md §4)
  if (xlds != 0 && xlds != 2) return -6;
  g_xfrag = xlds == 2 ? 1 : 0;
  if (K % 32 != 0 || N % 16 != 0 || M <= 0) return -1;
  if (g_xfrag && M > 64) return -5;
  const int KB = K / 32, NBtot = N / 16;
  const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
  const int ldo = (epi == EPI_SILU) ? N / 2 : N;
  if (M <= 64) {
    if (nb <= 0) nb = 1;
    if (epi == EPI_SILU && nb < 2) nb = 2;
    // a ragged grid (nb not dividing the n-blocks) needs >= 1 column unit per workgroup; SiLU units are pairs
    if (NBtot % nb != 0 && (epi == EPI_SILU ? (nb % 2 || NBtot % 2 || NBtot / 2 < (NBtot + nb - 1) / nb)
                                              : NBtot < (NBtot + nb - 1) / nb))
      return -2;
    if (splitk < 1) splitk = 1;
    if (epi != EPI_F32 && epi != EPI_RES && splitk != 1) return -3;
    if (M > 32 && nb > 2) nb = 2;
    switch (epi) {
      case EPI_BF16: launch_skinny_e<EPI_BF16>(x, ldx, M, KB, w, NBtot, out, ldo, nb, splitk, stream); break;
      case EPI_F32: launch_skinny_e<EPI_F32>(x, ldx, M, KB, w, NBtot, out, ldo, nb, splitk, stream); break;
      case EPI_SILU: launch_skinny_e<EPI_SILU>(x, ldx, M, KB, w, NBtot, out, ldo, nb, splitk, stream); break;
      case EPI_RES: launch_skinny_e<EPI_RES>(x, ldx, M, KB, w, NBtot, out, ldo, nb, splitk, stream); break;
      default: return -4;
    }
  } else {
    return -9;  // M > 64: the stream-K prefill kernel (gemm_tile256.hip lsa_gemm_sk)
  }
  return (int)hipGetLastError();
}

// Batch-1 decode GEMM with the residual-reduce prologue (lsa_epi.h LsaRr; kernel template RR): X = rr.h + sum of
// rr.np f32 slabs, formed per split K slice in LDS.  epi: EPI_F32 (split-K slabs, rr.local = 0: the row scale is
// left to the slab consumer, which reads rr.ss_out) or EPI_SILU (splitk 1, rr.local = 1: the workgroup's full-row
// sum of squares scales the gate / up rows before SiLU).
template <int NB, int EPI, int RR>
static void launch_rr_nb(int KB, const uint4* Wf, int NBtot, void* out, int ldo, int splitk, hipStream_t s) {
  launch_skinny_x<1, NB, EPI, false, RR>(nullptr, 0, 1, KB, Wf, NBtot, out, ldo, splitk, s);
}

template <int EPI, int RR>
static int launch_rr_e(int KB, const uint4* Wf, int NBtot, void* out, int ldo, int nb, int splitk, hipStream_t s) {
  if constexpr (EPI != EPI_SILU) {
    if (nb == 1) {
      launch_rr_nb<1, EPI, RR>(KB, Wf, NBtot, out, ldo, splitk, s);
      return 0;
    }
  }
  if (nb == 2) launch_rr_nb<2, EPI, RR>(KB, Wf, NBtot, out, ldo, splitk, s);
  else if (nb == 4) launch_rr_nb<4, EPI, RR>(KB, Wf, NBtot, out, ldo, splitk, s);
  else return -2;
  return 0;
}

extern "C" int lsa_gemm_rr(int K, const void* Wf, int N, void* out, int epi, int nb, int splitk, int waves, int div,
                           const LsaRr* rr, hipStream_t stream) {
  if (!rr || !rr->h || !rr->h_out || rr->h == rr->h_out || rr->np < 1 || rr->np > 4 || !rr->parts)
    return -1;
  if (K % 32 != 0 || N % 16 != 0) return -1;
  if (splitk < 1) splitk = 1;
  const int KB = K / 32, NBtot = N / 16;
  if ((KB + splitk - 1) / splitk * 32 > RR_KMAX) return -3;  // the K slice must fit the LDS image
  if (epi == EPI_SILU ? (splitk != 1 || !rr->local || nb < 2) : (epi != EPI_F32 || rr->local || !rr->ss_out)) return -4;
  if (NBtot % nb) return -2;
  g_epi = LsaEpi{};
  g_rr = *rr;
  g_skinny_waves = waves == 8 ? 8 : 4;
  g_skinny_div = (div == 1 || div == 2) ? div : 4;
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  int rc;
  if (epi == EPI_SILU)
    rc = rr->np <= 2 ? launch_rr_e<EPI_SILU, 2>(KB, w, NBtot, out, ldo, nb, 1, stream)
                     : launch_rr_e<EPI_SILU, 4>(KB, w, NBtot, out, ldo, nb, 1, stream);
  else
    rc = rr->np <= 2 ? launch_rr_e<EPI_F32, 2>(KB, w, NBtot, out, ldo, nb, splitk, stream)
                     : launch_rr_e<EPI_F32, 4>(KB, w, NBtot, out, ldo, nb, splitk, stream);
  g_rr = LsaRr{};
  if (rc) return rc;
  return (int)hipGetLastError();
}
