// Prefill / large-M linear layers, one wave per SIMD:  out[M, N] = X[M, K] @ W[N, K]^T   (bf16 in, f32 accumulate)
//
// 256 x 256 output tile per workgroup of FOUR waves (2 along M x 2 along N, 128 x 128 each: 64 accumulator tiles =
// 256 registers per lane, held in AGPRs), one workgroup per CU.  The 8-wave 256^2 kernel (gemm_tile256.hip) re-reads
// each wave's 128 x 64 operand panel from LDS for a quarter of the MFMA work; here a wave reads 128 rows of X and 128
// n of W per 32-deep k-step for 64 MFMAs, 2 / 3 of the LDS read traffic per flop, and there is no ping-pong partner
// wave whose barrier skew idles a SIMD.
//
// K is consumed in 32-deep slices (one MFMA k-step): a slice is 32 KiB of LDS (16 X fragments of 16 rows + 16 W
// fragments of 16 n, 1 KiB each, lane-linear -- the weights' own fragment-major layout, X gathered lane-wise by the
// DMA addresses), staged by global_load_lds (16 B per lane, 8 per wave per slice) into a ring of R slots.
// Per iteration s (one slice, 64 MFMAs per wave):
//     s_waitcnt vmcnt(8 (R - 3))  -> this wave's part of slice s + 1 has landed
//     s_barrier                   -> every wave's part has, and every wave has finished reading slice s - 1
//     stage slice s + R - 1 into slice s - 1's slot
//     ds_read slice s + 1 into the second register set     (16 x ds_read_b128, in flight under the MFMAs)
//     64 MFMAs on slice s's register set, s_waitcnt lgkmcnt(0)
// so R - 2 slices of global loads (R = 5: 3 slices = 3 x 64 MFMAs of latency cover) and one slice of LDS reads are
// always in flight; one raw s_barrier per slice, never vmcnt(0) in the loop.  LDS reads are inline asm (hipcc would
// drain vmcnt(0) before a compiler-visible LDS read while a DMA is in flight, gemm_tile256.hip).
// XCD-aware bijective tile remap and split-K (f32 slabs) as gemm_tile256.hip.
#include "common.h"

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2

typedef __attribute__((address_space(3))) void* w4_lds_ptr_t;

namespace {

__device__ __forceinline__ void w4_glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (w4_lds_ptr_t)l, 16, 0, 0);
}

__device__ __forceinline__ u32x4_t w4_ds_read16(const void* p) {
  u32x4_t v;
  const uint32_t a = (uint32_t)(uintptr_t)(w4_lds_ptr_t)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

template <int EPI>
__device__ __forceinline__ void w4_store(void* out, int ldo, int m, int n, const f32x4_t& v) {
  if constexpr (EPI == EPI_F32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (size_t)m * ldo + n) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 p;
    p.x = pack2bf(v[0], v[1]);
    p.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + (size_t)m * ldo + n) = p;
  }
}

}  // namespace

template <int EPI, int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4_kernel(
    const uint16_t* __restrict__ X, int ldx, int M, int KB, const uint4* __restrict__ Wf, int NBtot,
    void* __restrict__ out, int ldo, int ntm, int kts) {
  __shared__ __attribute__((aligned(16))) uint4 lds[R][32][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;  // 0..3
  const int wm = w >> 1, wn = w & 1;

  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int ntiles = ntm * ((NBtot + 15) >> 4);
  const int split = kts > 0 ? wgid0 / ntiles : 0;
  const int wgid = kts > 0 ? wgid0 - split * ntiles : wgid0;
  const int tm = wgid % ntm, tn = wgid / ntm;
  const int mbase = tm * 256, nbase = tn * 16;
  const int ks0 = kts > 0 ? split * kts : 0;
  const int S = kts > 0 ? min(KB, ks0 + kts) - ks0 : KB;  // this workgroup's k-steps (>= 1: host-checked)

  // staging: wave w moves fragments 8 w .. 8 w + 7 of a slice -- waves 0, 1 the 16 X row tiles, waves 2, 3 the 16 W
  // n-blocks; per lane the global source address, the LDS destination is the wave-uniform fragment base + lane * 16
  const int r16 = lane & 15, c16 = 8 * (lane >> 4);
  const char* src[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int f = 8 * w + e;
    if (f < 16) {
      const int row = min(mbase + 16 * f + r16, M - 1);
      src[e] = reinterpret_cast<const char*>(X + (size_t)row * ldx + c16);
    } else {
      const int nb = min(nbase + (f - 16), NBtot - 1);
      src[e] = reinterpret_cast<const char*>(Wf + (size_t)nb * KB * 64) + lane * 16;
    }
  }
  auto stage = [&](int t) {  // slice t (clamped to the last: the counted waits stay exact) into slot t % R
    const int ks = ks0 + min(t, S - 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = 8 * w + e;
      const size_t off = f < 16 ? (size_t)ks * 64 : (size_t)ks * 1024;  // X: 32 bf16 of k; W: one 1 KiB fragment
      w4_glds16(src[e] + off, &lds[t % R][f][0]);
    }
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  u32x4_t xa[8], wa[8], xb[8], wb[8];
  auto read = [&](u32x4_t (&xr)[8], u32x4_t (&wr)[8], int t) {
    const int sl = t % R;
#pragma unroll
    for (int j = 0; j < 8; ++j) wr[j] = w4_ds_read16(&lds[sl][16 + wn * 8 + j][lane]);
#pragma unroll
    for (int i = 0; i < 8; ++i) xr[i] = w4_ds_read16(&lds[sl][wm * 8 + i][lane]);
  };
  auto mma = [&](const u32x4_t (&xr)[8], const u32x4_t (&wr)[8]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wr[j]),
                                                            __builtin_bit_cast(bf16x8_t, xr[i]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // one iteration: slice t computed from (xc, wc), slice t + 1 read into (xn, wn_)
#define LSA_W4_ITER(XC, WC, XN, WN, T)                                                  \
  do {                                                                                  \
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (R - 3)) : "memory");                  \
    __builtin_amdgcn_s_barrier();                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    stage((T) + R - 1);                                                                 \
    if ((T) + 1 < S) read(XN, WN, (T) + 1);                                             \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    mma(XC, WC);                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)

  // prologue: slices 0 .. R - 2 in flight, slice 0 landed everywhere, read into set a
#pragma unroll
  for (int t = 0; t < R - 1; ++t) stage(t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (R - 2)) : "memory");
  __builtin_amdgcn_s_barrier();
  read(xa, wa, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int t = 0;
  for (; t + 1 < S; t += 2) {
    LSA_W4_ITER(xa, wa, xb, wb, t);
    LSA_W4_ITER(xb, wb, xa, wa, t + 1);
  }
  if (t < S) LSA_W4_ITER(xa, wa, xb, wb, t);
#undef LSA_W4_ITER
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup

  // epilogue: acc[i][j] = D[n = (nbase + wn * 8 + j) * 16 + 4 g + q][m = mbase + (wm * 8 + i) * 16 + (lane & 15)]
  const int g = lane >> 4;
  void* o = EPI == EPI_F32 ? reinterpret_cast<void*>(reinterpret_cast<float*>(out) + (size_t)split * M * ldo) : out;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + (wm * 8 + i) * 16 + (lane & 15);
    if (m >= M) continue;
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const int nb = nbase + wn * 8 + j;  // even: gate block, nb + 1: up block
        if (nb + 1 >= NBtot) continue;
        f32x4_t v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(acc[i][j][q]) * acc[i][j + 1][q];
        w4_store<EPI_SILU>(o, ldo, m, (nb >> 1) * 16 + 4 * g, v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int nb = nbase + wn * 8 + j;
        if (nb >= NBtot) continue;
        w4_store<EPI>(o, ldo, m, nb * 16 + 4 * g, acc[i][j]);
      }
    }
  }
}

// M > 64 linear layer on the 4-wave 256^2 tile (K % 32 == 0, N % 16 == 0; EPI_SILU needs N % 32 == 0).  splitk > 1
// (EPI_F32 only): the k-steps are cut into splitk pieces of ceil(KB / splitk), one workgroup per (tile, piece), f32
// slab per piece in out[splitk][M][N].  ring: LDS slots of 32 KiB (4 | 5).
extern "C" int lsa_gemm_w4(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int splitk,
                           int ring, hipStream_t stream) {
  if (K % 32 != 0 || N % 16 != 0 || M <= 0) return -1;
  if (ring != 4 && ring != 5) return -2;
  const int KB = K / 32, NBtot = N / 16;
  const int ntm = (M + 255) / 256, ntn = (NBtot + 15) / 16;
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  if (epi == EPI_SILU && NBtot % 2) return -1;
  if (splitk < 1) splitk = 1;
  if (splitk > 1 && epi != EPI_F32) return -3;
  const int kts = splitk > 1 ? (KB + splitk - 1) / splitk : 0;
  if (splitk > 1 && (KB + kts - 1) / kts != splitk) return -3;  // every piece owns >= 1 k-step
  const dim3 grid(ntm * ntn * splitk);
  const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
#define LSA_W4(E, RR) \
  hipLaunchKernelGGL((gemm_w4_kernel<E, RR>), grid, dim3(256), 0, stream, x, ldx, M, KB, w, NBtot, out, ldo, ntm, kts)
  switch (epi) {
    case EPI_BF16: if (ring == 5) LSA_W4(EPI_BF16, 5); else LSA_W4(EPI_BF16, 4); break;
    case EPI_F32: if (ring == 5) LSA_W4(EPI_F32, 5); else LSA_W4(EPI_F32, 4); break;
    case EPI_SILU: if (ring == 5) LSA_W4(EPI_SILU, 5); else LSA_W4(EPI_SILU, 4); break;
    default: return -4;
  }
#undef LSA_W4
  return (int)hipGetLastError();
}
