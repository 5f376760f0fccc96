// fp8 (OCP e4m3fn, gfx950-native) weight-only linear layers:  out = X[M,K] @ (Wq[N,K] * scale[n])^T
//
// Weight layout (ops.shuffle_weight_fp8): Wq[nb][kb64][lane][16 B], lane = 16*g + r holds
// W[16*nb + r][64*kb64 + 16*g + 0..15].  One 16 B load per lane = 1 KiB per wave-instruction feeds TWO
// mfma_f32_16x16x32_bf16 k-steps: step 0 uses k-slots 16g + 0..7, step 1 uses 16g + 8..15 (the k order
// inside an MFMA step only has to agree between A and B, so the activation fragment of lane (m, g) is
// simply x[m][64*kb64 + 16g .. +15] as two uint4).  fp8 -> bf16 with v_cvt_scalef32_pk_bf16_fp8
// (one VALU op per 2 weights, far below the HBM-bound budget), per-output-channel scale in the epilogue.
// Decode therefore streams half the bytes of the bf16 path.  For prefill (M > 64) the layer is
// dequantised (lsa_fp8_dequant) into a bf16 fragment-layout scratch buffer owned by the caller
// and run through gemm_tile.
#include "common.h"

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

template <bool HI>
__device__ __forceinline__ uint32_t cvt2(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w, 1.0f, HI));
}
// 16 fp8 -> two bf16 fragments (k-slots 0..7 and 8..15)
__device__ __forceinline__ void fp8x16_to_bf16(const uint4 q, uint4& a, uint4& b) {
  a.x = cvt2<false>(q.x); a.y = cvt2<true>(q.x); a.z = cvt2<false>(q.y); a.w = cvt2<true>(q.y);
  b.x = cvt2<false>(q.z); b.y = cvt2<true>(q.z); b.z = cvt2<false>(q.w); b.w = cvt2<true>(q.w);
}

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2

// XF: X in the fragment-major decode layout (common.h xf_off): lane (r, g)'s 16 activations
// k = 64 kb64 + 16 g .. +15 are the two 16-B pieces (g' = 2 (g & 1), g' + 1) of bf16 k-step 2 kb64 + g / 2
template <int MT, int NB, int EPI, int WAVES, int U, bool XF = false>
__global__ __launch_bounds__(64 * WAVES) void gemm_fp8_skinny_kernel(const uint16_t* __restrict__ X, int ldx, int M,
                                                                     int KB64, const uint4* __restrict__ Wq,
                                                                     const float* __restrict__ wscale,
                                                                     void* __restrict__ out, int ldo, int kb_per_split,
                                                                     LsaEpi ep) {
  // same work split as gemm_skinny_kernel: chunks of U k64-steps round-robin over the waves, two-deep
  // register pipeline pinned with sched_barrier(0)
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nb0 = blockIdx.x * NB;
  const int kbA = blockIdx.y * kb_per_split;
  const int kbB = min(KB64, kbA + kb_per_split);
  const int nk = kbB - kbA;
  const int nch = (nk + U - 1) / U;
  const int n_it = nch > w ? (nch - w + WAVES - 1) / WAVES : 0;
  const int last_c = w + WAVES * (n_it - 1);

  f32x4_t acc[NB][MT];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint16_t* xp[MT];
  bool xvalid[MT];
  // row-major X: padding rows (>= M) read zeros from past the buffer range, no memory request (gemm.hip)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, XF ? 0 : M * ldx * 2, 0x00020000);
  uint32_t xoff[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = j * 16 + r;
    xvalid[j] = m < M;
    xp[j] = XF ? X + (((size_t)(g >> 1) * MT + j) * 64 + 32 * (g & 1) + r) * 8
               : X + (size_t)(xvalid[j] ? m : 0) * ldx + 16 * g;
    xoff[j] = xvalid[j] ? (uint32_t)(((size_t)m * ldx + 16 * g) * 2) : 0x80000000u;
  }
  const uint4* wp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wp[i] = Wq + (size_t)(nb0 + i) * KB64 * 64 + lane;

  auto load = [&](uint4 (&wr)[U][NB], uint4 (&xr)[U][MT][2], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) wr[u][i] = ldg_nt(wp[i] + (size_t)kk * 64);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if constexpr (XF) {
          const uint4* px = reinterpret_cast<const uint4*>(xp[j] + (size_t)kk * 2 * MT * 512);
          xr[u][j][0] = px[0];
          xr[u][j][1] = px[16];
        } else {
          const uint32_t o = xoff[j] + (uint32_t)kk * 128u;
          const u32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
          const u32x4_t b = __builtin_amdgcn_raw_buffer_load_b128(xrs, o + 16u, 0, 0);
          xr[u][j][0] = make_uint4(a[0], a[1], a[2], a[3]);
          xr[u][j][1] = make_uint4(b[0], b[1], b[2], b[3]);
        }
      }
    }
  };
  auto comp = [&](const uint4 (&wr)[U][NB], const uint4 (&xr)[U][MT][2], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = (kb + u) < kbB;
      uint4 x0[MT], x1[MT];
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const bool ok = live && xvalid[j];
        x0[j] = xr[u][j][0];
        x1[j] = xr[u][j][1];
        x0[j].x = ok ? x0[j].x : 0u; x0[j].y = ok ? x0[j].y : 0u; x0[j].z = ok ? x0[j].z : 0u; x0[j].w = ok ? x0[j].w : 0u;
        x1[j].x = ok ? x1[j].x : 0u; x1[j].y = ok ? x1[j].y : 0u; x1[j].z = ok ? x1[j].z : 0u; x1[j].w = ok ? x1[j].w : 0u;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        uint4 a0, a1;
        fp8x16_to_bf16(wr[u][i], a0, a1);
#pragma unroll
        for (int j = 0; j < MT; ++j) {
          acc[i][j] = mfma16x16x32(a0, x0[j], acc[i][j]);
          acc[i][j] = mfma16x16x32(a1, x1[j], acc[i][j]);
        }
      }
    }
  };
  if (n_it > 0) {
    uint4 wA[U][NB], xA[U][MT][2], wB[U][NB], xB[U][MT][2];
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
      if (m < M) {
        const int nrow_g = (nb0 + 2 * p) * 16 + 4 * (l >> 4);
        const int nrow_u = nrow_g + 16;
        const int n = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
        uint2 pk;
        float v[4];
        const float sc = epi_row_scale(ep, m);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(gs[q] * (sc * wscale[nrow_g + q])) * (us[q] * (sc * wscale[nrow_u + q]));
        pk.x = pack2bf(v[0], v[1]);
        pk.y = pack2bf(v[2], v[3]);
        // fragment-major in -> fragment-major out (the down projection's input)
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (XF ? xf_off(m, n, MT) : (size_t)m * ldo + n)) = pk;
      }
    }
  } else {
    const size_t slab = (size_t)blockIdx.y * M * ldo;
    if constexpr (EPI == EPI_RES) {
      if (gridDim.y > 1) {  // split-K: publish (channel-scaled), ticket, the last split finishes the column
        const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
        for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
          const int l = idx & 63, t = idx >> 6;
          const int j = t % MT, i = t / MT;
          f32x4_t s = red[0][t][l];
#pragma unroll
          for (int ww = 1; ww < WAVES; ++ww) s += red[ww][t][l];
          const int m = j * 16 + (l & 15);
          if (m >= M) continue;
          const int n = (nb0 + i) * 16 + 4 * (l >> 4);
          const float4 sc = *reinterpret_cast<const float4*>(wscale + n);
          s[0] *= sc.x; s[1] *= sc.y; s[2] *= sc.z; s[3] *= sc.w;
          res_store_partial(rsc, slab + (size_t)m * ldo + n, s);
        }
        __shared__ int s_last;
        if (!res_publish_and_ticket<64 * WAVES>(ep, &s_last)) return;
        for (int idx = threadIdx.x; idx < NB * MT * 64; idx += 64 * WAVES) {
          const int l = idx & 63, t = idx >> 6;
          const int j = t % MT, i = t / MT;
          const int m = j * 16 + (l & 15);
          if (m < M) {
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
      if (m >= M) continue;
      const int n = (nb0 + i) * 16 + 4 * (l >> 4);
      const float4 sc = *reinterpret_cast<const float4*>(wscale + n);
      const float rs = epi_row_scale(ep, m);
      s[0] *= sc.x * rs; s[1] *= sc.y * rs; s[2] *= sc.z * rs; s[3] *= sc.w * rs;
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

// fp8 [nb][kb64][lane][16] -> bf16 fragment layout [nb][kb32][lane][8] with the channel scale applied
__global__ __launch_bounds__(256) void fp8_dequant_kernel(const uint4* __restrict__ Wq, const float* __restrict__ wscale,
                                                          int KB64, long nfrag, uint4* __restrict__ Wf) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nfrag * 64; i += (long)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const long f = i >> 6;  // (nb, kb64)
    const long nb = f / KB64;
    const int kb64 = (int)(f % KB64);
    const int r = lane & 15, g = lane >> 4;
    const float sc = wscale[nb * 16 + r];
    uint4 a0, a1;
    fp8x16_to_bf16(Wq[i], a0, a1);
    // elements k = 64*kb64 + 16g + e  (e = 0..15) -> bf16 fragment kb32 = 2*kb64 + (16g + e) / 32,
    // lane' = 16 * (((16g + e) % 32) / 8) + r
    float f0[8], f1[8];
    unpack8(a0, f0);
    unpack8(a1, f1);
#pragma unroll
    for (int j = 0; j < 8; ++j) { f0[j] *= sc; f1[j] *= sc; }
    const int k0 = 16 * g;  // e = 0..7 -> k0 .. k0+7 ; e = 8..15 -> k0+8 ..
    const long kb32 = 2 * kb64 + (k0 >> 5);
    const int lane0 = 16 * ((k0 & 31) >> 3) + r;
    const int lane1 = 16 * (((k0 + 8) & 31) >> 3) + r;
    Wf[((nb * (2L * KB64)) + kb32) * 64 + lane0] = pack8(f0);
    Wf[((nb * (2L * KB64)) + kb32) * 64 + lane1] = pack8(f1);
  }
}

static thread_local int g_fp8_xfrag = 0;
static thread_local LsaEpi g_fp8_epi = {};

// Per-call knobs (ops.pick_gemm_config, fp8 tuning entries): waves 4 | 8 per workgroup; depth 1 | 2
// multiplies the chunk of k64-steps each wave keeps in flight (U0 = 4 / NB fragments per chunk: the
// shallow point; depth 2 doubles the weight bytes in flight per wave for grids with few waves per CU).
static thread_local int g_fp8_waves = 4;
static thread_local int g_fp8_depth = 1;

template <int MT, int NB, int EPI, int WV, int U>
static void launch_tx(const uint16_t* X, int ldx, int M, int KB64, const uint4* Wq, const float* sc, int NBtot,
                      void* out, int ldo, int kbps, int splitk, hipStream_t s) {
  if (g_fp8_xfrag)
    hipLaunchKernelGGL((gemm_fp8_skinny_kernel<MT, NB, EPI, WV, U, true>), dim3(NBtot / NB, splitk), dim3(64 * WV), 0,
                       s, X, ldx, M, KB64, Wq, sc, out, ldo, kbps, g_fp8_epi);
  else
    hipLaunchKernelGGL((gemm_fp8_skinny_kernel<MT, NB, EPI, WV, U, false>), dim3(NBtot / NB, splitk), dim3(64 * WV), 0,
                       s, X, ldx, M, KB64, Wq, sc, out, ldo, kbps, g_fp8_epi);
}

template <int MT, int NB, int EPI>
static void launch_t(const uint16_t* X, int ldx, int M, int KB64, const uint4* Wq, const float* sc, int NBtot, void* out,
                     int ldo, int splitk, hipStream_t s) {
  // default: 4 waves, 4 fragments (NB * U) per chunk (the shallow-chunk / high-occupancy point that won the
  // bf16 sweeps: each fp8 fragment feeds twice the MFMA work of a bf16 one)
  constexpr int U = (4 / NB) < 1 ? 1 : (4 / NB);
  const int kbps = (KB64 + splitk - 1) / splitk;
  if constexpr (EPI == EPI_BF16 || NB >= 6) {
    // bf16 out: not on the decode hot path, one configuration.  Wide n-groups (NB 6 / 8: one pair of
    // activation fragments feeds 6-8 weight fragments, the activation traffic is 2 * MT / NB of the weight
    // bytes): 4 waves only (the reduction buffer is WAVES * NB * MT KiB), depth 1 | 2
    if (EPI != EPI_BF16 && g_fp8_depth == 2) launch_tx<MT, NB, EPI, 4, 2 * U>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, kbps, splitk, s);
    else launch_tx<MT, NB, EPI, 4, U>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, kbps, splitk, s);
  } else {
    if (g_fp8_waves == 8) {
      if (g_fp8_depth == 2) launch_tx<MT, NB, EPI, 8, 2 * U>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, kbps, splitk, s);
      else launch_tx<MT, NB, EPI, 8, U>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, kbps, splitk, s);
    } else {
      if (g_fp8_depth == 2) launch_tx<MT, NB, EPI, 4, 2 * U>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, kbps, splitk, s);
      else launch_tx<MT, NB, EPI, 4, U>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, kbps, splitk, s);
    }
  }
}

template <int EPI>
static void launch_e(const uint16_t* X, int ldx, int M, int KB64, const uint4* Wq, const float* sc, int NBtot, void* out,
                     int ldo, int nb, int splitk, hipStream_t s) {
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_F8(MTV, NBV)                                                       \
  if (mt == MTV && nb == NBV) {                                                \
    launch_t<MTV, NBV, EPI>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, splitk, s); \
    return;                                                                    \
  }
  LSA_F8(1, 2) LSA_F8(1, 4) LSA_F8(2, 2) LSA_F8(2, 4) LSA_F8(4, 2) LSA_F8(2, 6) LSA_F8(2, 8) LSA_F8(1, 8)
  if constexpr (EPI != EPI_SILU) { LSA_F8(1, 1) LSA_F8(2, 1) LSA_F8(4, 1) }
#undef LSA_F8
  // fallback (unsupported nb): nb = 2 at the same row-tile count
  if (mt == 1) launch_t<1, 2, EPI>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, splitk, s);
  else if (mt == 2) launch_t<2, 2, EPI>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, splitk, s);
  else launch_t<4, 2, EPI>(X, ldx, M, KB64, Wq, sc, NBtot, out, ldo, splitk, s);
}

extern "C" int lsa_fp8_dequant(const void* Wq, const float* wscale, int N, int K, void* Wf, hipStream_t s) {
  if (K % 64 || N % 16) return -1;
  const int KB64 = K / 64;
  const long nfrag = (long)(N / 16) * KB64;
  const long tot = nfrag * 64;
  const long gl = (tot + 255) / 256;
  hipLaunchKernelGGL(fp8_dequant_kernel, dim3((unsigned)(gl < 8192 ? gl : 8192)), dim3(256), 0, s,
                     reinterpret_cast<const uint4*>(Wq), wscale, KB64, nfrag, reinterpret_cast<uint4*>(Wf));
  return (int)hipGetLastError();
}

extern "C" int lsa_fp8_gemm_cfg(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N,
                                void* out, int epi, int nb, int splitk, int xfrag, hipStream_t stream);

extern "C" int lsa_fp8_gemm(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N, void* out,
                            int epi, int nb, int splitk, hipStream_t stream) {
  return lsa_fp8_gemm_cfg(X, ldx, M, K, Wq, wscale, N, out, epi, nb, splitk, 0, stream);
}

// xfrag = 1: X in the fragment-major decode layout (M <= 64); a SiLU output is written in it too
extern "C" int lsa_fp8_gemm_ex(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N,
                               void* out, int epi, int nb, int splitk, int xfrag, const LsaEpi* ep, hipStream_t stream);

extern "C" void lsa_fp8_gemm_knobs(int waves, int depth) {
  g_fp8_waves = waves == 8 ? 8 : 4;
  g_fp8_depth = depth == 2 ? 2 : 1;
}

extern "C" int lsa_fp8_gemm_cfg(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N,
                                void* out, int epi, int nb, int splitk, int xfrag, hipStream_t stream) {
  return lsa_fp8_gemm_ex(X, ldx, M, K, Wq, wscale, N, out, epi, nb, splitk, xfrag, nullptr, stream);
}

// ep (nullable): decode epilogue extensions (common.h LsaEpi), M <= 64
extern "C" int lsa_fp8_gemm_ex(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N,
                               void* out, int epi, int nb, int splitk, int xfrag, const LsaEpi* ep, hipStream_t stream) {
  g_fp8_epi = ep ? *ep : LsaEpi{};
  if ((ep || epi == EPI_RES) && (M > 64 || (splitk > 1 && epi != EPI_F32 && epi != EPI_RES))) return -7;
  if (epi == EPI_RES && (!ep || !ep->h || !ep->xout || !ep->ss_out || ep->ldh != N || (splitk > 1 && !ep->tickets)))
    return -8;
  if (K % 64 != 0 || N % 16 != 0 || M <= 0) return -1;
  if (xfrag && M > 64) return -5;
  g_fp8_xfrag = xfrag ? 1 : 0;
  const int KB64 = K / 64, NBtot = N / 16;
  const int ldo = (epi == EPI_SILU) ? N / 2 : N;
  if (M <= 64) {
    if (nb <= 0) nb = 1;
    if (epi == EPI_SILU && nb < 2) nb = 2;
    if (NBtot % nb != 0) return -2;
    if (splitk < 1) splitk = 1;
    if (epi != EPI_F32 && epi != EPI_RES && splitk != 1) return -3;
    if (M > 32 && nb > 2) nb = 2;
    const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
    const uint4* w = reinterpret_cast<const uint4*>(Wq);
    switch (epi) {
      case EPI_BF16: launch_e<EPI_BF16>(x, ldx, M, KB64, w, wscale, NBtot, out, ldo, nb, splitk, stream); break;
      case EPI_F32: launch_e<EPI_F32>(x, ldx, M, KB64, w, wscale, NBtot, out, ldo, nb, splitk, stream); break;
      case EPI_SILU: launch_e<EPI_SILU>(x, ldx, M, KB64, w, wscale, NBtot, out, ldo, nb, splitk, stream); break;
      case EPI_RES: launch_e<EPI_RES>(x, ldx, M, KB64, w, wscale, NBtot, out, ldo, nb, splitk, stream); break;
      default: return -4;
    }
    return (int)hipGetLastError();
  }
  return -6;  // M > 64: caller dequantises (lsa_fp8_dequant) and runs the bf16 tile GEMM
}
