// W8A8 / W4A8 decode linear layers (M <= 64) on the gfx950 block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4:
//   out = (X8 . act scales) @ (W . weight scales)^T
//
// The W8A16 / W4A16 decode kernels (gemm_fp8.hip, gemm_fp4.hip) widen every weight to bf16 on the VALU and read
// bf16 activation fragments: at M = 32 they move 2 * MT / NB bytes of activations per fp8 weight byte (4 * MT / NB
// per fp4 byte) through L2 and the VALU conversion sits in every k-step.  Here the activations are e4m3 and the
// weights go to the matrix core in their stored format -- e4m3 (WK 0) or MXFP4 e2m1 (WK 1, the weight's own E8M0
// block scales as the MFMA's A scale operand) -- so one MFMA consumes a 16 x 128 weight slab and a 16 x 128
// activation slab: half the activation bytes, no conversion VALU, a quarter of the MFMA issues.  Same work split as
// the skinny kernels: chunks of U k128-steps dealt round-robin to the waves, split-K over blockIdx.y, a two-deep
// register pipeline pinned with sched_barrier, cross-wave reduction through LDS.
//
// Activations ("xf8", common.h xf8_off): X8[kb128][MT][lane][32 B], lane (g, r) holds row 16 mt + r at k = 128 s + 16 g
// .. +15 and 128 s + 64 + 16 g .. +15 -- the K order the matrix core reads an 8-bit operand in (measured,
// scripts/probe_mfma_scale.py), so the MFMA's K index is k itself.  Two scalings:
//   * per-row f32 sx (the RMSNorm launch quantises its output rows by amax / 448; ops.quantize_xf8), and/or
//   * ASC: per-32-k-block E8M0 bytes S8[kb128][MT][lane] (common.h xs8_off: lane group b = k 128 s + 32 b .. +31)
//     fed to the MFMA's B scale operand -- what the decode attention (o input: one scale per (row, head)) and this
//     kernel's own SiLU epilogue (down input: one per (row, 32 columns)) produce without a whole-row reduction.
// Weights: WK 0 -- the fp8 decode layout Wq[nb][kb64][lane][16 B] (lane 16 g + r = W[16 nb + r][64 kb64 + 16 g ..
//   +15]); an MFMA step kk takes the lane's fragments of k64 blocks 2 kk and 2 kk + 1 (the 8-bit K order above), the
//   per-output-channel f32 scale applies in the epilogue.
//   WK 1 -- MXFP4 Wq[nb][kb128][lane][16 B] (lane (g, r) = W[16 nb + r][128 kb + 32 g .. +31] as e2m1 nibbles: the
//   4-bit K order, one MX block per lane) + S[nb][kb128 / 4][lane][4 B] E8M0 (gemm_fp4.hip's layout: the W4A16 path
//   reads the same bytes), the lane's byte as the MFMA's A scale operand.
//
// Epilogues: EPI_F32 -> f32 split-K slabs [splitk][M][N];  EPI_SILU -> silu(gate) * up, gate / up rows interleaved
// per 16, written as bf16 (row-major, XFO 0, or fragment-major, XFO 1, for a 16-bit down projection) or -- XFO 2 --
// as e4m3 in the xf8 layout with one E8M0 scale per (row, 32 columns) for a W8A8 / W4A8 down projection (NB a
// multiple of 4: a workgroup's column pairs (2 c, 2 c + 1) are exactly one 32-column block; the block amax
// through LDS).  The rownorm extension (LsaEpi.rowss) multiplies a row scale in like the other decode GEMMs.
#include "common.h"

#define EPI_F32 1
#define EPI_SILU 2

typedef int a8_i32x8_t __attribute__((ext_vector_type(8)));

namespace {

// one 16 x 16 x 128 step: A = weights (WK 0: e4m3, unit scale; WK 1: e2m1 in the low 4 dwords, E8M0 scale sa),
// B = e4m3 activations with E8M0 scale sb (0x7f = 2^0)
template <int WK>
__device__ __forceinline__ f32x4_t mfma_blk(const uint4 a0, const uint4 a1, int sa, const uint4 b0, const uint4 b1, int sb,
                                            f32x4_t c) {
  const a8_i32x8_t b = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  if constexpr (WK == 0) {
    const a8_i32x8_t a = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0x7f, 0, sb);
  } else {
    const a8_i32x8_t a = {(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 0, 0, sa, 0, sb);
  }
}

}  // namespace

// RR > 0 (batch 1): the residual-reduce prologue of lsa_epi.h LsaRr (gemm.hip has the 16-bit form): X = h + sum of the
// previous projection's f32 split-K slabs over this split's K slice, quantised in the prologue to e4m3 with one E8M0
// scale per 32 k (the MFMA's B scale operand) into an LDS image of row 0's xf8 bytes (128 B + 4 scale bytes per k128
// step; the 16 lanes of a row group read one address), so no quantising norm launch precedes the GEMM.  RR = the most
// slabs summed (loads clamped to slab np - 1 and masked).  The row's RMS scale: rr.local (splitk 1) from the
// workgroup's own full-row sum in the epilogue, else the column-0 workgroups add the slice's sum of squares to
// rr.ss_out for the slab consumer.
#define A8_RR_KMAX 8192
template <int MT, int NB, int EPI, int WAVES, int U, int XFO, int WK, bool ASC, int RR = 0>
__global__ __launch_bounds__(64 * WAVES) void gemm_a8_skinny_kernel(const uint4* __restrict__ X8, const uint8_t* __restrict__ S8,
                                                                    const float* __restrict__ sx, int M, int KB128,
                                                                    const uint4* __restrict__ Wq, const float* __restrict__ wscale,
                                                                    const uint32_t* __restrict__ Sw, void* __restrict__ out,
                                                                    uint8_t* __restrict__ out_s8, int ldo, int kb_per_split,
                                                                    LsaEpi ep, LsaRr rr) {
  static_assert(RR == 0 || (MT == 1 && ASC), "residual-reduce prologue: batch 1, block-scaled activations");
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
#pragma unroll
  for (int j = 0; j < MT; ++j) xvalid[j] = j * 16 + r < M;
  const uint4* wp[NB];
  const uint32_t* sp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const size_t nbi = (size_t)(nb0 + min(i, cnt - 1));
    if constexpr (WK == 0) {
      wp[i] = Wq + nbi * (2 * KB128) * 64 + lane;
      sp[i] = nullptr;
    } else {
      wp[i] = Wq + nbi * KB128 * 64 + lane;
      sp[i] = Sw + nbi * KB4 * 64 + lane;
    }
  }
  const uint4* xp = X8 + 2 * lane;
  // RR: row 0's xf8 bytes of the slice (lane group g of k128-step s at [s][g][32 B]) and its E8M0 bytes [s][g]
  __shared__ __attribute__((aligned(16))) uint4 x8s[RR ? A8_RR_KMAX / 16 : 1];
  __shared__ uint8_t s8s[RR ? A8_RR_KMAX / 32 : 1];

  auto wload = [&](uint4 (&wr)[U][NB][2], int (&sa)[U][NB], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        if constexpr (WK == 0) {
          wr[u][i][0] = ldg_nt(wp[i] + (size_t)(2 * kk) * 64);
          wr[u][i][1] = ldg_nt(wp[i] + (size_t)(2 * kk + 1) * 64);
          sa[u][i] = 0x7f;
        } else {
          wr[u][i][0] = ldg_nt(wp[i] + (size_t)kk * 64);
          wr[u][i][1] = make_uint4(0u, 0u, 0u, 0u);
          sa[u][i] = (int)((sp[i][(size_t)(kk >> 2) * 64] >> (8 * (kk & 3))) & 0xffu);
        }
      }
    }
  };
  auto xload = [&](uint4 (&xr)[U][MT][2], int (&sb)[U][MT], int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = min(kb + u, kbB - 1);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        if constexpr (RR > 0) {
          xr[u][j][0] = x8s[(kk - kbA) * 8 + 2 * g];
          xr[u][j][1] = x8s[(kk - kbA) * 8 + 2 * g + 1];
          sb[u][j] = (int)s8s[(kk - kbA) * 4 + g];
        } else {
          const uint4* px = xp + (size_t)(kk * MT + j) * 128;
          xr[u][j][0] = px[0];
          xr[u][j][1] = px[1];
          sb[u][j] = ASC ? (int)S8[(size_t)(kk * MT + j) * 64 + lane] : 0x7f;
        }
      }
    }
  };
  auto load = [&](uint4 (&wr)[U][NB][2], int (&sa)[U][NB], uint4 (&xr)[U][MT][2], int (&sb)[U][MT], int c) {
    wload(wr, sa, c);
    xload(xr, sb, c);
  };
  auto comp = [&](const uint4 (&wr)[U][NB][2], const int (&sa)[U][NB], const uint4 (&xr)[U][MT][2], const int (&sb)[U][MT],
                  int c) {
    const int kb = kbA + c * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = (kb + u) < kbB;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        // a dead (clamped) step or a padding row contributes zeros (and a unit scale: an unwritten byte could be the
        // E8M0 NaN code)
        const bool ok = live && xvalid[j];
        uint4 x0 = xr[u][j][0], x1 = xr[u][j][1];
        x0.x = ok ? x0.x : 0u; x0.y = ok ? x0.y : 0u; x0.z = ok ? x0.z : 0u; x0.w = ok ? x0.w : 0u;
        x1.x = ok ? x1.x : 0u; x1.y = ok ? x1.y : 0u; x1.z = ok ? x1.z : 0u; x1.w = ok ? x1.w : 0u;
        const int s = ok ? sb[u][j] : 0x7f;
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i][j] = mfma_blk<WK>(wr[u][i][0], wr[u][i][1], sa[u][i], x0, x1, s, acc[i][j]);
      }
    }
  };
  uint4 wA[U][NB][2], xA[U][MT][2], wB[U][NB][2], xB[U][MT][2];
  int saA[U][NB], sbA[U][MT], saB[U][NB], sbB[U][MT];
  float rr_scale = 1.f;
  if constexpr (RR > 0) {
    if (n_it > 0) wload(wA, saA, w);  // the first weight chunk does not depend on X: in flight during the prologue
    __shared__ float rr_red[WAVES];
    const int k0 = kbA * 128, n8 = nk * 16;  // 8-value groups of the slice; 4 consecutive groups = one 32-k block
    const bool wr_h = blockIdx.x == 0;
    float ssl = 0.f;
    for (int i = threadIdx.x; i < n8; i += 64 * WAVES) {
      const size_t e = (size_t)k0 + 8 * i;
      float4 a[RR + 1][2];
      a[0][0] = *reinterpret_cast<const float4*>(rr.h + e);
      a[0][1] = *reinterpret_cast<const float4*>(rr.h + e + 4);
#pragma unroll
      for (int s2 = 0; s2 < RR; ++s2) {
        const float* p = rr.parts + (size_t)min(s2, rr.np - 1) * rr.pstride + e;
        a[s2 + 1][0] = *reinterpret_cast<const float4*>(p);
        a[s2 + 1][1] = *reinterpret_cast<const float4*>(p + 4);
      }
      float v[8] = {a[0][0].x, a[0][0].y, a[0][0].z, a[0][0].w, a[0][1].x, a[0][1].y, a[0][1].z, a[0][1].w};
#pragma unroll
      for (int s2 = 0; s2 < RR; ++s2) {
        const float on = s2 < rr.np ? 1.f : 0.f;
        v[0] += on * a[s2 + 1][0].x; v[1] += on * a[s2 + 1][0].y; v[2] += on * a[s2 + 1][0].z; v[3] += on * a[s2 + 1][0].w;
        v[4] += on * a[s2 + 1][1].x; v[5] += on * a[s2 + 1][1].y; v[6] += on * a[s2 + 1][1].z; v[7] += on * a[s2 + 1][1].w;
      }
      float am = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ssl += v[j] * v[j];
        am = fmaxf(am, fabsf(v[j]));
      }
      if (wr_h) {
        *reinterpret_cast<float4*>(rr.h_out + e) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(rr.h_out + e + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
      // the 32-k block's amax over its 4 threads (a quad of lanes, whole quads active: n8 % 16 == 0)
      am = fmaxf(am, lsa_dpp<LSA_DPP_XOR1>(am));
      am = fmaxf(am, lsa_dpp<LSA_DPP_XOR2>(am));
      const int eb = e8m0_for_amax(am);
      const int kl = 8 * i, st = kl >> 7, kc = kl & 127;  // k128-step of the slice, k within it
      *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(x8s) + st * 128 + ((kc & 63) >> 4) * 32 + 16 * (kc >> 6) +
                                (kc & 15)) = pack8_fp8(v, e8m0_inv(eb));
      if ((i & 3) == 0) s8s[st * 4 + (kc >> 5)] = (uint8_t)eb;
    }
    ssl = wave_sum(ssl);
    if (lane == 0) rr_red[w] = ssl;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) tot += rr_red[ww];
    if (rr.local) rr_scale = rsqrtf(tot * rr.inv_k + rr.eps);
    else if (wr_h && threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(rr.ss_out), (unsigned long long)ss_to_q24(tot));
    if (n_it > 0) xload(xA, sbA, w);
  } else {
    if (n_it > 0) load(wA, saA, xA, sbA, w);
  }
  if (n_it > 0) {
    int i = 0;
    for (; i + 1 < n_it; i += 2) {
      load(wB, saB, xB, sbB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
      comp(wA, saA, xA, sbA, w + WAVES * i);
      __builtin_amdgcn_sched_barrier(0);
      load(wA, saA, xA, sbA, min(w + WAVES * (i + 2), last_c));
      __builtin_amdgcn_sched_barrier(0);
      comp(wB, saB, xB, sbB, w + WAVES * (i + 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < n_it) comp(wA, saA, xA, sbA, w + WAVES * i);
  }

  __shared__ __attribute__((aligned(16))) f32x4_t red[WAVES][NB * MT][64];
  constexpr int NBLK = (XFO == 2 && NB >= 4) ? NB / 4 : 1;  // 32-column blocks of a SiLU workgroup
  __shared__ uint32_t bmax[16 * MT][NBLK];                   // their per-row amax (float bits, >= 0)
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) red[w][i * MT + j][lane] = acc[i][j];
  if constexpr (XFO == 2) {
    for (int t = threadIdx.x; t < 16 * MT * NBLK; t += 64 * WAVES) (&bmax[0][0])[t] = 0u;
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
        const int nrow_g = (nb0 + 2 * p) * 16 + 4 * (l >> 4);
        const int nrow_u = nrow_g + 16;
        const int n = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
        const float sc = (sx ? sx[m] : 1.f) * epi_row_scale(ep, m) * rr_scale;
        f32x4_t v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float cg = WK == 0 ? wscale[nrow_g + q] : 1.f, cu = WK == 0 ? wscale[nrow_u + q] : 1.f;
          v[q] = silu(gs[q] * (sc * cg)) * (us[q] * (sc * cu));
        }
        if constexpr (XFO == 2) {
          // pass 1: the value stays in this thread's own reduction slot, the block amax goes to LDS
          red[0][(2 * p) * MT + j][l] = v;
          const float a = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
          atomicMax(&bmax[m & (16 * MT - 1)][(p >> 1) % NBLK], __float_as_uint(a));
        } else {
          uint2 pk;
          pk.x = pack2bf(v[0], v[1]);
          pk.y = pack2bf(v[2], v[3]);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (XFO ? xf_off(m, n, MT) : (size_t)m * ldo + n)) = pk;
        }
      }
    }
    if constexpr (XFO == 2) {
      // pass 2: e4m3 with the block's E8M0 scale (xf8 layout), one scale byte per (row, block)
      __syncthreads();
      for (int idx = threadIdx.x; idx < (NB / 2) * MT * 64; idx += 64 * WAVES) {
        const int l = idx & 63, t = idx >> 6;
        const int j = t % MT, p = t / MT;
        const int m = j * 16 + (l & 15);
        if (m < M && 2 * p < cnt) {
          const int n = ((nb0 + 2 * p) >> 1) * 16 + 4 * (l >> 4);
          const f32x4_t v = red[0][(2 * p) * MT + j][l];
          const int e = e8m0_for_amax(__uint_as_float(bmax[m][(p >> 1) % NBLK]));
          *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(out) + xf8_off(m, n, MT)) =
              pack4_fp8(v[0], v[1], v[2], v[3], e8m0_inv(e));
          if ((l >> 4) == 0 && (p & 1) == 0) out_s8[xs8_off(m, n, MT)] = (uint8_t)e;
        }
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
      const float4 sc = WK == 0 ? *reinterpret_cast<const float4*>(wscale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float rs = (sx ? sx[m] : 1.f) * epi_row_scale(ep, m) * rr_scale;
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + slab + (size_t)m * ldo + n) =
          make_float4(s[0] * sc.x * rs, s[1] * sc.y * rs, s[2] * sc.z * rs, s[3] * sc.w * rs);
    }
  }
}

namespace {

struct A8Call {
  const uint4* X8;
  const uint8_t* S8;
  const float* sx;
  int M, KB128;
  const uint4* Wq;
  const float* wscale;
  const uint32_t* Sw;
  void* out;
  uint8_t* out_s8;
  int ldo, splitk, NBtot;
  int waves, depth, xfo, wk;
  LsaEpi ep;
  LsaRr rr;  // rr.h set: the residual-reduce prologue (M = 1; f32 slabs or the e4m3 SiLU output)
};

template <int MT, int NB, int EPI, int WV, int U, int XFO, int WK>
void launch_a8_x(const A8Call& c, hipStream_t s) {
  const int kbps = (c.KB128 + c.splitk - 1) / c.splitk;
  const dim3 grid((c.NBtot + NB - 1) / NB, c.splitk);
  if constexpr (MT == 1 && ((EPI == EPI_F32 && XFO == 0) || (EPI == EPI_SILU && XFO == 2))) {
    if (c.rr.h) {
      if (c.rr.np == 1)
        hipLaunchKernelGGL((gemm_a8_skinny_kernel<MT, NB, EPI, WV, U, XFO, WK, true, 1>), grid, dim3(64 * WV), 0, s,
                           c.X8, c.S8, c.sx, c.M, c.KB128, c.Wq, c.wscale, c.Sw, c.out, c.out_s8, c.ldo, kbps, c.ep, c.rr);
      else
        hipLaunchKernelGGL((gemm_a8_skinny_kernel<MT, NB, EPI, WV, U, XFO, WK, true, 4>), grid, dim3(64 * WV), 0, s,
                           c.X8, c.S8, c.sx, c.M, c.KB128, c.Wq, c.wscale, c.Sw, c.out, c.out_s8, c.ldo, kbps, c.ep, c.rr);
      return;
    }
  }
  if (c.S8)
    hipLaunchKernelGGL((gemm_a8_skinny_kernel<MT, NB, EPI, WV, U, XFO, WK, true>), grid, dim3(64 * WV), 0, s, c.X8, c.S8,
                       c.sx, c.M, c.KB128, c.Wq, c.wscale, c.Sw, c.out, c.out_s8, c.ldo, kbps, c.ep, LsaRr{});
  else
    hipLaunchKernelGGL((gemm_a8_skinny_kernel<MT, NB, EPI, WV, U, XFO, WK, false>), grid, dim3(64 * WV), 0, s, c.X8, c.S8,
                       c.sx, c.M, c.KB128, c.Wq, c.wscale, c.Sw, c.out, c.out_s8, c.ldo, kbps, c.ep, LsaRr{});
}

template <int MT, int NB, int EPI, int WV, int U>
void launch_a8_o(const A8Call& c, hipStream_t s) {
  // output layout x weight format; the e4m3 SiLU output only at whole 32-column blocks per workgroup
  constexpr bool F8O = EPI == EPI_SILU && NB % 4 == 0;
  if (c.wk == 0) {
    if (F8O && c.xfo == 2) launch_a8_x<MT, NB, EPI, WV, U, (F8O ? 2 : 1), 0>(c, s);
    else if (c.xfo) launch_a8_x<MT, NB, EPI, WV, U, 1, 0>(c, s);
    else launch_a8_x<MT, NB, EPI, WV, U, 0, 0>(c, s);
  } else {
    if (F8O && c.xfo == 2) launch_a8_x<MT, NB, EPI, WV, U, (F8O ? 2 : 1), 1>(c, s);
    else if (c.xfo) launch_a8_x<MT, NB, EPI, WV, U, 1, 1>(c, s);
    else launch_a8_x<MT, NB, EPI, WV, U, 0, 1>(c, s);
  }
}

template <int MT, int NB, int EPI>
void launch_a8_t(const A8Call& c, hipStream_t s) {
  // U0 k128-steps per chunk: 2 for one n-block, else 1 (a chunk is NB * U 2 KiB weight slabs per wave for fp8, 1 KiB
  // for fp4); depth 2 doubles it (8 waves and depth 2 only where the registers allow: the wide / 4-tile variants
  // would spill)
  constexpr int U = NB == 1 ? 2 : 1;
  if constexpr (NB <= 4 && MT <= 2) {
    if (c.waves == 8) {
      // 8 waves = 256 VGPRs per lane: the two pipeline stages hold 2 U (NB + MT) x 2 uint4, so depth 2 only where
      // 2 U (NB + MT) <= 8 (the wider ones spill)
      if constexpr (2 * U * (NB + MT) <= 8) {
        if (c.depth == 2) {
          launch_a8_o<MT, NB, EPI, 8, 2 * U>(c, s);
          return;
        }
      }
      launch_a8_o<MT, NB, EPI, 8, U>(c, s);
      return;
    }
    if (c.depth == 2) {
      launch_a8_o<MT, NB, EPI, 4, 2 * U>(c, s);
      return;
    }
  }
  launch_a8_o<MT, NB, EPI, 4, U>(c, s);
}

template <int EPI>
int launch_a8_e(const A8Call& c, int nb, hipStream_t s) {
  const int mt = c.M <= 16 ? 1 : (c.M <= 32 ? 2 : 4);
#define LSA_A8(MTV, NBV)              \
  if (mt == MTV && nb == NBV) {       \
    launch_a8_t<MTV, NBV, EPI>(c, s); \
    return 0;                         \
  }
  LSA_A8(1, 2) LSA_A8(1, 4) LSA_A8(2, 2) LSA_A8(2, 4) LSA_A8(2, 6) LSA_A8(2, 8) LSA_A8(4, 2) LSA_A8(1, 8)
  if constexpr (EPI == EPI_SILU) { LSA_A8(4, 4) }
  if constexpr (EPI != EPI_SILU) { LSA_A8(1, 1) LSA_A8(2, 1) LSA_A8(4, 1) }
#undef LSA_A8
  return -6;  // unsupported (mt, nb)
}

}  // namespace

// wk 0: fp8 weights (wscale per output channel); wk 1: MXFP4 weights + E8M0 block scales Sw (wscale unused).
// s8 (nullable): per-lane-block E8M0 activation scales; sx (nullable when s8 is given): per-row f32 scales.
// xfo: SiLU output 0 bf16 row-major [M, N / 2], 1 bf16 fragment-major, 2 e4m3 xf8 + E8M0 blocks into out_s8.
extern "C" int lsa_a8_gemm(const void* X8, const void* s8, const float* sx, int M, int K, const void* Wq,
                           const float* wscale, const void* Sw, int wk, int N, void* out, void* out_s8, int epi, int nb,
                           int splitk, int waves, int depth, int xfo, const LsaEpi* ep, hipStream_t stream) {
  if (M <= 0 || M > 64 || K % 128 != 0 || N % 16 != 0) return -1;
  if (epi != EPI_F32 && epi != EPI_SILU) return -4;
  if ((wk == 0 && !wscale) || (wk == 1 && !Sw) || (wk != 0 && wk != 1)) return -8;
  if (!sx && !s8) return -8;
  const int KB128 = K / 128, NBtot = N / 16;
  if (nb <= 0) nb = 2;
  if (epi == EPI_SILU && nb < 2) nb = 2;
  if (M > 32 && nb > 2 && !(epi == EPI_SILU && xfo == 2 && nb == 4)) nb = 2;
  // a ragged grid (nb not dividing the n-blocks) needs >= 1 column unit per workgroup; SiLU units are pairs
  if (NBtot % nb != 0 && (epi == EPI_SILU ? (nb % 2 || NBtot % 2 || NBtot / 2 < (NBtot + nb - 1) / nb)
                                            : NBtot < (NBtot + nb - 1) / nb))
    return -2;
  // the e4m3 SiLU output: every workgroup holds whole 32-column blocks (nb a multiple of 4, no ragged tail)
  if (epi == EPI_SILU && xfo == 2 && (nb % 4 || NBtot % nb || !out_s8)) return -9;
  if (splitk < 1) splitk = 1;
  if (epi == EPI_SILU && splitk != 1) return -3;
  if ((KB128 + ((KB128 + splitk - 1) / splitk) - 1) / ((KB128 + splitk - 1) / splitk) != splitk) return -3;
  A8Call c{reinterpret_cast<const uint4*>(X8), reinterpret_cast<const uint8_t*>(s8), sx, M, KB128,
           reinterpret_cast<const uint4*>(Wq), wscale, reinterpret_cast<const uint32_t*>(Sw), out,
           reinterpret_cast<uint8_t*>(out_s8), epi == EPI_SILU ? N / 2 : N, splitk, NBtot,
           waves == 8 ? 8 : 4, depth == 2 ? 2 : 1, xfo, wk, ep ? *ep : LsaEpi{}, LsaRr{}};
  const int rc = epi == EPI_F32 ? launch_a8_e<EPI_F32>(c, nb, stream) : launch_a8_e<EPI_SILU>(c, nb, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// The same GEMM at batch 1 with the residual-reduce prologue (kernel template RR, lsa_epi.h LsaRr): no X8 / scales
// in memory -- the prologue forms X from rr.h + rr.parts and quantises it itself.  epi EPI_F32 (f32 slabs, rr.local 0,
// rr.ss_out accumulates sum X^2) or EPI_SILU with the e4m3 output (xfo 2, out_s8; splitk 1, rr.local 1).
extern "C" int lsa_a8_gemm_rr(int K, const void* Wq, const float* wscale, const void* Sw, int wk, int N, void* out,
                              void* out_s8, int epi, int nb, int splitk, int waves, int depth, const LsaRr* rr,
                              hipStream_t stream) {
  if (!rr || !rr->h || !rr->h_out || rr->h == rr->h_out || rr->np < 1 || rr->np > 4 || !rr->parts) return -1;
  if (K % 128 != 0 || N % 16 != 0) return -1;
  if ((wk == 0 && !wscale) || (wk == 1 && !Sw) || (wk != 0 && wk != 1)) return -8;
  if (splitk < 1) splitk = 1;
  const int KB128 = K / 128, NBtot = N / 16;
  if ((KB128 + splitk - 1) / splitk * 128 > A8_RR_KMAX) return -3;
  if ((KB128 + ((KB128 + splitk - 1) / splitk) - 1) / ((KB128 + splitk - 1) / splitk) != splitk) return -3;
  if (epi == EPI_SILU ? (splitk != 1 || !rr->local || nb % 4 || NBtot % nb || !out_s8) : (epi != EPI_F32 || rr->local || !rr->ss_out))
    return -4;
  if (epi == EPI_F32 && NBtot % nb) return -2;
  A8Call c{nullptr, nullptr, nullptr, 1, KB128, reinterpret_cast<const uint4*>(Wq), wscale,
           reinterpret_cast<const uint32_t*>(Sw), out, reinterpret_cast<uint8_t*>(out_s8), epi == EPI_SILU ? N / 2 : N,
           splitk, NBtot, waves == 8 ? 8 : 4, depth == 2 ? 2 : 1, epi == EPI_SILU ? 2 : 0, wk, LsaEpi{}, *rr};
  const int rc = epi == EPI_F32 ? launch_a8_e<EPI_F32>(c, nb, stream) : launch_a8_e<EPI_SILU>(c, nb, stream);
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

// x [M, K] bf16 -> xf8 e4m3 with one E8M0 scale per (row, block of `blk` = 32 | 128 consecutive k) into s8
// (common.h xs8_off; a 128-block's byte repeated for its 4 lanes): the standalone form of the attention / SiLU
// e4m3 outputs (tests, benches)
__global__ __launch_bounds__(256) void quant_xf8_blocks_kernel(const uint16_t* __restrict__ x, int ldx, int M, int K,
                                                               int MT, int blk, uint8_t* __restrict__ x8,
                                                               uint8_t* __restrict__ s8) {
  // one thread per (row of the mt tiles, 32-column block)
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const int nb32 = K / 32;
  if (t >= (long)16 * MT * nb32) return;
  const int m = (int)(t / nb32), c0 = (int)(t % nb32) * 32;
  const int b0 = c0 / blk * blk;
  float amax = 0.f;
  if (m < M)
    for (int c = b0; c < b0 + blk; c += 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * ldx + c), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
    }
  const int e = e8m0_for_amax(amax);
  const float inv = e8m0_inv(e);
  for (int c = c0; c < c0 + 32; c += 8) {
    uint2 q = make_uint2(0u, 0u);
    if (m < M) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)m * ldx + c), f);
      q = pack8_fp8(f, inv);
    }
    *reinterpret_cast<uint2*>(x8 + xf8_off(m, c, MT)) = q;
  }
  s8[xs8_off(m, c0, MT)] = (uint8_t)e;
}

extern "C" int lsa_quant_xf8_blocks(const void* x, int ldx, int M, int K, int MT, int blk, void* x8, void* s8,
                                    hipStream_t s) {
  if (M <= 0 || M > 16 * MT || K % 128 != 0 || (blk != 32 && blk != 128)) return -1;
  const long n = (long)16 * MT * (K / 32);
  hipLaunchKernelGGL(quant_xf8_blocks_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const uint16_t*>(x), ldx, M, K, MT, blk, reinterpret_cast<uint8_t*>(x8),
                     reinterpret_cast<uint8_t*>(s8));
  return (int)hipGetLastError();
}
