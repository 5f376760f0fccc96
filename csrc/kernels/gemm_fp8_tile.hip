// fp8 x fp8 (W8A8) prefill / large-M linear layers on the CDNA4 block-scaled MFMA:
//     out[M, N] = (X8[M, K] * sx[m]) @ (W8[N, K] * sw[n])^T      (OCP e4m3fn operands, f32 accumulate)
//
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (E8M0 127 in every byte) runs a 16 x 16 x 128
// fp8 product in twice the cycles of a 16 x 16 x 32 bf16 MFMA: twice the bf16 FLOP rate
// (MI355X_MICROARCH.md § Matrix cores), and every staged byte carries twice the K of a bf16 byte.  The
// per-token activation scale sx (ops.quantize_rows_fp8 / the fp8 prefill norm) and the per-channel weight
// scale sw are applied to the f32 accumulators in the epilogue, so no weight is ever dequantised (the
// weight-only path dequantised a whole layer into a bf16 scratch per call, gemm_fp8.hip).
//
// Operand images: W keeps the decode layout of ops.quantize_fp8 — fragment (nb, kb64) = 1 KiB, lane
// 16 g + r holds W[16 nb + r][64 kb64 + 16 g .. + 15]; X fragments are gathered lane-wise by the DMA
// addresses into the same shape (lane 16 g + r <- X[row r][64 kb64 + 16 g .. + 15]).  One MFMA consumes
// the two fragments ks = 0, 1 of a 128-wide K-tile as its 32 bytes per lane.  The k slot a byte lands in
// only has to agree between A and B: both are loaded with the same lane -> k map, so the contraction pairs
// W[n][k] with X[m][k] whatever the hardware's internal k order (checked with exact integers,
// tests/test_kernels_gpu.py::test_fp8_tile_gemm_exact_integers).
//
// Structure = gemm_tile256.hip's 256 x 256 8-phase template (8 waves, 2 x 4 of 128 x 64, LDS-DMA staging
// of quarter tiles, counted vmcnt, raw barriers, ping-pong wave groups, XCD-aware tile remap) with
// split-K over grid.y for grids that would under-fill the chip (f32 slab epilogue only).
#include "common.h"

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2

typedef __attribute__((address_space(3))) void* lds_ptr_f8_t;
typedef int i32x8_t __attribute__((ext_vector_type(8)));

namespace {

__device__ __forceinline__ void glds16_f8(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_f8_t)l, 16, 0, 0);
}

__device__ __forceinline__ u32x4_t ds_read16_f8(const void* p) {
  u32x4_t v;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_ptr_f8_t)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

__device__ __forceinline__ f32x4_t mfma_f8_128(const u32x4_t a0, const u32x4_t a1, const u32x4_t b0, const u32x4_t b1,
                                               f32x4_t c) {
  const i32x8_t a = {(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3], (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]};
  const i32x8_t b = {(int)b0[0], (int)b0[1], (int)b0[2], (int)b0[3], (int)b1[0], (int)b1[1], (int)b1[2], (int)b1[3]};
  // formats 0/0 = fp8 e4m3 x fp8 e4m3; block scales 0x7f = 2^0 in every byte (no MX scaling)
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}

}  // namespace

// LDS: [buffer][half][fragment][lane] exactly as gemm_t256_kernel (halves XQ0, XQ1, WQ0, WQ1), 128 KiB.
template <int EPI>
__global__ __launch_bounds__(512) void gemm_fp8_t256_kernel(const uint8_t* __restrict__ X, int ldx, const float* __restrict__ sx,
                                                            int M, int KB64, const uint4* __restrict__ Wq,
                                                            const float* __restrict__ sw, int NBtot,
                                                            void* __restrict__ out, int ldo, int ntm, int tiles_per_split) {
  __shared__ __attribute__((aligned(16))) uint4 lds[2][4][16][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;

  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tm = wgid % ntm, tn = wgid / ntm;
  const int mbase = tm * 256, nbase = tn * 16;

  const int KT = KB64 >> 1;  // 128-wide K-tiles (KB64 is even)
  const int t0 = blockIdx.y * tiles_per_split;
  const int T = min(KT - t0, tiles_per_split);
  const int r16 = lane & 15, c16 = 16 * (lane >> 4);
  auto stage = [&](int h, int t) {
    const int tc = t0 + min(t, T - 1);
    const int buf = t & 1;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int f = 2 * w + e;
      const int kstep = 2 * tc + (f & 1);  // 64-wide k block
      const char* g;
      if (h < 2) {
        const int wi = f >> 1, wr = wi >> 2, i = wi & 3;
        const int row = min(mbase + wr * 128 + h * 64 + i * 16 + r16, M - 1);
        g = reinterpret_cast<const char*>(X + (size_t)row * ldx + kstep * 64 + c16);
      } else {
        const int wj = f >> 1, wc = wj >> 1, j = wj & 1;
        const int nb = min(nbase + wc * 4 + (h - 2) * 2 + j, NBtot - 1);
        g = reinterpret_cast<const char*>(Wq + ((size_t)nb * KB64 + kstep) * 64) + lane * 16;
      }
      glds16_f8(g, &lds[buf][h][f][0]);
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  u32x4_t xr[4][2], wr[2][2];
  auto read_x = [&](int buf, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xr[i][ks] = ds_read16_f8(&lds[buf][qm][(wm * 4 + i) * 2 + ks][lane]);
  };
  auto read_w = [&](int buf, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wr[j][ks] = ds_read16_f8(&lds[buf][2 + qn][((wn * 2 + j) * 2) + ks][lane]);
  };
  auto mma = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[qm * 4 + i][qn * 2 + j] = mfma_f8_128(wr[j][0], wr[j][1], xr[i][0], xr[i][1], acc[qm * 4 + i][qn * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
#define LSA_F8PHASE(READS, STAGE_H, STAGE_T, WAIT, QM, QN) \
  do {                                                     \
    READS;                                                 \
    stage(STAGE_H, STAGE_T);                               \
    WAIT;                                                  \
    __builtin_amdgcn_s_barrier();                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0);                     \
    mma(QM, QN);                                           \
    __builtin_amdgcn_sched_barrier(0);                     \
    __builtin_amdgcn_s_barrier();                          \
  } while (0)

  if (T > 0) {
    stage(0, 0);
    stage(3, 0);
    stage(1, 0);
    stage(2, 0);
    stage(0, 1);
    stage(3, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();
    for (int t = 0; t < T; ++t) {
      const int b = t & 1;
      LSA_F8PHASE((read_x(b, 0), read_w(b, 0)), 1, t + 1, (void)0, 0, 0);
      LSA_F8PHASE(read_w(b, 1), 2, t + 1, (void)0, 0, 1);
      LSA_F8PHASE(read_x(b, 1), 0, t + 2, (void)0, 1, 1);
      LSA_F8PHASE(read_w(b, 0), 3, t + 2, asm volatile("s_waitcnt vmcnt(4)" ::: "memory"), 1, 0);
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef LSA_F8PHASE

  // epilogue: acc[i][j] = D[n = nb_j * 16 + 4 g + q][m = mb_i * 16 + (lane & 15)] * sx[m] * sw[n]
  const int g = lane >> 4;
  const size_t slab = (size_t)blockIdx.y * M * ldo;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + (wm * 8 + i) * 16 + (lane & 15);
    if (m >= M) continue;
    const float xs = sx[m];
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int nb = nbase + wn * 4 + j;  // even: gate block, nb + 1: up block
        if (nb + 1 >= NBtot) continue;
        const float4 sg = *reinterpret_cast<const float4*>(sw + nb * 16 + 4 * g);
        const float4 su = *reinterpret_cast<const float4*>(sw + (nb + 1) * 16 + 4 * g);
        const float gsc[4] = {sg.x, sg.y, sg.z, sg.w}, usc[4] = {su.x, su.y, su.z, su.w};
        uint2 p;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(acc[i][j][q] * xs * gsc[q]) * (acc[i][j + 1][q] * xs * usc[q]);
        p.x = pack2bf(v[0], v[1]);
        p.y = pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + (nb >> 1) * 16 + 4 * g) = p;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nb = nbase + wn * 4 + j;
        if (nb >= NBtot) continue;
        const int n = nb * 16 + 4 * g;
        const float4 s4 = *reinterpret_cast<const float4*>(sw + n);
        const float v0 = acc[i][j][0] * xs * s4.x, v1 = acc[i][j][1] * xs * s4.y;
        const float v2 = acc[i][j][2] * xs * s4.z, v3 = acc[i][j][3] * xs * s4.w;
        if constexpr (EPI == EPI_F32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + slab + (size_t)m * ldo + n) = make_float4(v0, v1, v2, v3);
        } else {
          uint2 p;
          p.x = pack2bf(v0, v1);
          p.y = pack2bf(v2, v3);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + n) = p;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Per-row (per-token) fp8 quantisation of bf16 activations: sx[m] = amax(|x[m]|) / 448 (OCP e4m3fn max),
// x8[m][k] = e4m3(x[m][k] / sx[m]) with v_cvt_pk_fp8_f32 (round to nearest even, saturating in range).
// One workgroup per row, 16 B of input per thread and pass.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const uint16_t* __restrict__ x, int ldx, int K,
                                                             uint8_t* __restrict__ x8, int ld8, float* __restrict__ sx) {
  __shared__ float red[16];
  const int m = blockIdx.x;
  const uint16_t* row = x + (size_t)m * ldx;
  float amax = 0.f;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(row + c), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.0f : 1.0f;
  const float inv = 1.0f / s;
  if (threadIdx.x == 0) sx[m] = s;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(row + c), f);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0] * inv, f[1] * inv, 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2] * inv, f[3] * inv, lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4] * inv, f[5] * inv, 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6] * inv, f[7] * inv, hi, true);
    *reinterpret_cast<uint2*>(x8 + (size_t)m * ld8 + c) = make_uint2((uint32_t)lo, (uint32_t)hi);
  }
}

extern "C" int lsa_quant_rows_fp8(const void* x, int ldx, int M, int K, void* x8, int ld8, float* sx, hipStream_t s) {
  if (K % 8 != 0 || M <= 0) return -1;
  hipLaunchKernelGGL(quant_rows_fp8_kernel, dim3(M), dim3(256), 0, s, reinterpret_cast<const uint16_t*>(x), ldx, K,
                     reinterpret_cast<uint8_t*>(x8), ld8, sx);
  return (int)hipGetLastError();
}

// M > 64 W8A8 linear layer.  K % 128 == 0, N % 16 == 0 (EPI_SILU: N % 32 == 0).  splitk > 1: EPI_F32 only,
// out = [splitk][M][N] f32 slabs (each already scaled by sx * sw; the consumer sums them).
extern "C" int lsa_fp8_gemm_t256(const void* X8, int ldx, const float* sx, int M, int K, const void* Wq,
                                 const float* sw, int N, void* out, int epi, int splitk, hipStream_t stream) {
  if (K % 128 != 0 || N % 16 != 0 || M <= 0) return -1;
  if (splitk < 1) splitk = 1;
  if (splitk > 1 && epi != EPI_F32) return -3;
  const int KB64 = K / 64, NBtot = N / 16;
  const int KT = KB64 / 2;
  const int tps = (KT + splitk - 1) / splitk;
  if ((KT + tps - 1) / tps != splitk) return -3;  // every slab owns >= 1 K-tile
  const int ntm = (M + 255) / 256, ntn = (NBtot + 15) / 16;
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  const dim3 grid(ntm * ntn, splitk);
  const uint8_t* x = reinterpret_cast<const uint8_t*>(X8);
  const uint4* w = reinterpret_cast<const uint4*>(Wq);
  switch (epi) {
    case EPI_BF16:
      hipLaunchKernelGGL(gemm_fp8_t256_kernel<EPI_BF16>, grid, dim3(512), 0, stream, x, ldx, sx, M, KB64, w, sw, NBtot, out,
                         ldo, ntm, tps);
      break;
    case EPI_F32:
      hipLaunchKernelGGL(gemm_fp8_t256_kernel<EPI_F32>, grid, dim3(512), 0, stream, x, ldx, sx, M, KB64, w, sw, NBtot, out,
                         ldo, ntm, tps);
      break;
    case EPI_SILU:
      if (NBtot % 2) return -2;
      hipLaunchKernelGGL(gemm_fp8_t256_kernel<EPI_SILU>, grid, dim3(512), 0, stream, x, ldx, sx, M, KB64, w, sw, NBtot, out,
                         ldo, ntm, tps);
      break;
    default:
      return -4;
  }
  return (int)hipGetLastError();
}
