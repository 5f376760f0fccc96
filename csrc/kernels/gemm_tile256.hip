// Prefill / large-M linear layers on MFMA:  out[M, N] = X[M, K] @ W[N, K]^T   (bf16 in, f32 accumulate)
//
// 256 x 256 output tile per workgroup, 8 waves (2 along M x 4 along N, 128 x 64 each), BK = 64, one
// workgroup per CU (128 KiB of LDS), on the MI355X guide's recipe for breaking the ~900 TF ceiling of
// the 128^2 two-barrier structure (cdna_hip_programming.md §5 "The 256^2 8-phase template"):
//   * both operands staged with global_load_lds (16 B per lane, 1 KiB per wave-instruction) into ONE
//     __shared__ array; fragment reads are inline-asm ds_read_b128 (hipcc would otherwise drain vmcnt(0)
//     before every compiler-visible LDS read while a DMA is in flight);
//   * four phases per K-tile, each: a quadrant's fragment reads, one half-tile of prefetch, raw
//     s_barrier, 16 MFMAs under s_setprio(1), s_barrier; one counted `s_waitcnt vmcnt(4)` per K-tile,
//     never vmcnt(0) inside the loop, so two half-tiles stay in flight across every barrier;
//   * LDS images are fragment-major (W is already stored that way, ops.shuffle_weight; X fragments are
//     gathered lane-wise by the DMA addresses), so every ds_read_b128 is lane-linear and conflict-free
//     without a swizzle;
//   * XCD-aware bijective tile remap: each XCD gets a contiguous run of tiles, M fastest, so the tiles
//     that share a W column panel run on the same L2.
// Epilogues as gemm.hip: EPI_BF16, EPI_F32 (one slab), EPI_SILU (gate/up rows interleaved per 16).
#include "common.h"

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2

typedef __attribute__((address_space(3))) void* lds_ptr_t;

namespace {

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)l, 16, 0, 0);
}

// ds_read_b128 as inline asm: hipcc treats an LDS-DMA in flight as a pending write to every LDS
// location and would drain vmcnt(0) before each compiler-visible ds_read, serialising the prefetch
// with the compute.  The asm read is ordered by the explicit counted waits + raw barriers instead.
__device__ __forceinline__ u32x4_t ds_read16(const void* p) {
  u32x4_t v;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_ptr_t)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

template <int EPI>
__device__ __forceinline__ void store_out(void* out, int ldo, int m, int n, const f32x4_t& v) {
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

// LDS: [buffer][half][fragment][lane].  Halves are cut by the C-quadrant that reads them, so each one
// falls free at a different phase and can be restaged while the rest of its tile is still in use:
//   half 0 = XQ0: X rows {0-63, 128-191} of the tile   (read in phase 1)
//   half 1 = XQ1: X rows {64-127, 192-255}              (read in phase 3)
//   half 2 = WQ0: W n-blocks {0,1, 4,5, 8,9, 12,13}     (read in phases 1 and 4)
//   half 3 = WQ1: W n-blocks {2,3, 6,7, 10,11, 14,15}   (read in phase 2)
// fragment within an X half: (wr * 4 + i) * 2 + ks;  within a W half: (wc * 2 + j) * 2 + ks.
//
// Four phases per K-tile t (quadrant (qm, qn) of each wave's 128 x 64 output, 16 MFMAs each):
//   P1 (0,0): read XQ0 + WQ0 (12 x ds_read_b128)   stage XQ1(t+1)
//   P2 (0,1): read WQ1 (4)                           stage WQ0(t+1)
//   P3 (1,1): read XQ1 (8)                           stage XQ0(t+2)
//   P4 (1,0): read WQ0 (4)                           stage WQ1(t+2), then s_waitcnt vmcnt(4): tile t+1 landed
// Every restage comes >= 2 phases after the last read of that half (WAR); every read comes a phase after
// the wait that retired it (RAW) - cdna_hip_programming.md §5, 8-phase template rules.  Tiles past the
// end are staged from clamped addresses (never read) so the counted wait stays exact.
// XF: X is fragment-major too, Xf[K / 32][mtt][64 lanes][8] (ops.to_xfrag layout with mtt 16-row tiles): every
// X staging DMA then reads one contiguous 1 KiB fragment (8 full 128-B lines) instead of 16 rows x 64 B
template <int EPI, bool XF = false>
__global__ __launch_bounds__(512) void gemm_t256_kernel(const uint16_t* __restrict__ X, int ldx, int M, int KB,
                                                        const uint4* __restrict__ Wf, int NBtot,
                                                        void* __restrict__ out, int ldo, int ntm, int kts) {
  __shared__ __attribute__((aligned(16))) uint4 lds[2][4][16][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;  // 0..7
  const int wm = w >> 2, wn = w & 3;

  // XCD-aware bijective remap (consecutive ids go round-robin over the 8 XCDs)
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  // split-K (EPI_F32 only, kts > 0): workgroup = (output tile, K split); split s covers K-tiles [s*kts, (s+1)*kts)
  // and writes f32 slab s (the consumer sums the slabs)
  const int ntiles = ntm * ((NBtot + 15) >> 4);
  const int split = kts > 0 ? wgid0 / ntiles : 0;
  const int wgid = kts > 0 ? wgid0 - split * ntiles : wgid0;
  const int tm = wgid % ntm, tn = wgid / ntm;
  const int mbase = tm * 256, nbase = tn * 16;  // first row / first n-block

  const int T = (KB + 1) >> 1;  // K-tiles of the whole product
  const int kt0 = kts > 0 ? split * kts : 0;
  const int Tl = kts > 0 ? min(T, kt0 + kts) - kt0 : T;  // this workgroup's K-tiles (>= 1: host-checked)
  const bool odd_tail = KB & 1;  // the last K-tile has one k-step (its second fragments re-read the first)
  const int r16 = lane & 15, c16 = 8 * (lane >> 4);
  // stage half h of K-tile t (clamped to the last tile) into buffer t & 1: this wave moves fragments
  // 2w and 2w + 1 of the half, one global_load_lds (1 KiB) each
  auto stage = [&](int h, int t) {
    const int tc = kt0 + min(t, Tl - 1);  // global K-tile (clamped to this split's last)
    const int buf = t & 1;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int f = 2 * w + e;  // fragment index in the half
      const int ks = (odd_tail && tc == T - 1) ? 0 : (f & 1);
      const int kstep = 2 * tc + ks;
      const char* g;
      if (h < 2) {  // X half h (qm = h): fragment (wr * 4 + i) * 2 + ks
        const int wi = f >> 1, wr = wi >> 2, i = wi & 3;
        if constexpr (XF) {  // ldx = row tiles of the fragment-major X
          const int rt = min((mbase + wr * 128 + h * 64 + i * 16) >> 4, ldx - 1);
          g = reinterpret_cast<const char*>(X + (((size_t)kstep * ldx + rt) * 64 + lane) * 8);
        } else {
          const int row = min(mbase + wr * 128 + h * 64 + i * 16 + r16, M - 1);
          g = reinterpret_cast<const char*>(X + (size_t)row * ldx + kstep * 32 + c16);
        }
      } else {      // W half h - 2 (qn): fragment (wc * 2 + j) * 2 + ks -> n-block wc * 4 + qn * 2 + j
        const int wj = f >> 1, wc = wj >> 1, j = wj & 1;
        const int nb = min(nbase + wc * 4 + (h - 2) * 2 + j, NBtot - 1);
        g = reinterpret_cast<const char*>(Wf + ((size_t)nb * KB + kstep) * 64) + lane * 16;
      }
      glds16(g, &lds[buf][h][f][0]);
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  u32x4_t xr[4][2], wr[2][2];  // X fragments of one M quadrant, W fragments of one N quadrant
  auto read_x = [&](int buf, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) xr[i][ks] = ds_read16(&lds[buf][qm][(wm * 4 + i) * 2 + ks][lane]);
  };
  auto read_w = [&](int buf, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) wr[j][ks] = ds_read16(&lds[buf][2 + qn][((wn * 2 + j) * 2) + ks][lane]);
  };
  auto mma = [&](int qm, int qn, int nks) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks < nks) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qm * 4 + i][qn * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, wr[j][ks]), __builtin_bit_cast(bf16x8_t, xr[i][ks]),
                acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // one phase: fragment reads, one half-tile of prefetch, [counted wait], barrier, MFMAs, barrier
#define LSA_PHASE(READS, STAGE_H, STAGE_T, WAIT, QM, QN)        \
  do {                                                          \
    READS;                                                      \
    stage(STAGE_H, STAGE_T);                                    \
    WAIT;                                                       \
    __builtin_amdgcn_s_barrier();                               \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          \
    __builtin_amdgcn_sched_barrier(0);                          \
    mma(QM, QN, nks);                                           \
    __builtin_amdgcn_sched_barrier(0);                          \
    __builtin_amdgcn_s_barrier();                               \
  } while (0)

  // prologue: all of tile 0, and XQ0 / WQ1 of tile 1
  stage(0, 0);
  stage(3, 0);
  stage(1, 0);
  stage(2, 0);
  stage(0, 1);
  stage(3, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // ping-pong: the second M wave group runs one barrier behind, so one group's MFMA section overlaps the
  // other's fragment reads + prefetch issue (the >= 2-phase WAR/RAW slack above covers the offset)
  if (wm == 1) __builtin_amdgcn_s_barrier();
  for (int t = 0; t < Tl; ++t) {
    const int b = t & 1;
    const int nks = (odd_tail && kt0 + t == T - 1) ? 1 : 2;
    LSA_PHASE((read_x(b, 0), read_w(b, 0)), 1, t + 1, (void)0, 0, 0);
    LSA_PHASE(read_w(b, 1), 2, t + 1, (void)0, 0, 1);
    LSA_PHASE(read_x(b, 1), 0, t + 2, (void)0, 1, 1);
    LSA_PHASE(read_w(b, 0), 3, t + 2, asm volatile("s_waitcnt vmcnt(4)" ::: "memory"), 1, 0);
  }
#undef LSA_PHASE
  if (wm == 0) __builtin_amdgcn_s_barrier();  // rebalance the barrier count
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup

  // epilogue: acc[i][j] = D[n = nb_j * 16 + 4 g + q][m = mb_i * 16 + (lane & 15)]
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + (wm * 8 + i) * 16 + (lane & 15);
    if (m >= M) continue;
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int nb = nbase + wn * 4 + j;  // even: gate block, nb + 1: up block
        if (nb + 1 >= NBtot) continue;
        f32x4_t v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = silu(acc[i][j][q]) * acc[i][j + 1][q];
        store_out<EPI_SILU>(out, ldo, m, (nb >> 1) * 16 + 4 * g, v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nb = nbase + wn * 4 + j;
        if (nb >= NBtot) continue;
        store_out<EPI>(EPI == EPI_F32 ? reinterpret_cast<void*>(reinterpret_cast<float*>(out) + (size_t)split * M * ldo)
                                      : out,
                       ldo, m, nb * 16 + 4 * g, acc[i][j]);
      }
    }
  }
}

// M > 64 linear layer on the 256^2 tile (K % 32 == 0, N % 16 == 0; EPI_SILU needs N % 32 == 0)
// xf_tiles > 0: X is fragment-major with that many 16-row tiles (>= ceil(M / 16))
extern "C" int lsa_gemm_t256x(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi,
                              int xf_tiles, hipStream_t stream) {
  if (K % 32 != 0 || N % 16 != 0 || M <= 0 || (xf_tiles > 0 && xf_tiles * 16 < M)) return -1;
  const int KB = K / 32, NBtot = N / 16;
  const int ntm = (M + 255) / 256, ntn = (NBtot + 15) / 16;
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  const dim3 grid(ntm * ntn);
  const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
  if (xf_tiles <= 0) return -5;
  switch (epi) {
    case EPI_BF16:
      hipLaunchKernelGGL((gemm_t256_kernel<EPI_BF16, true>), grid, dim3(512), 0, stream, x, xf_tiles, M, KB, w, NBtot, out, ldo, ntm, 0);
      break;
    case EPI_F32:
      hipLaunchKernelGGL((gemm_t256_kernel<EPI_F32, true>), grid, dim3(512), 0, stream, x, xf_tiles, M, KB, w, NBtot, out, ldo, ntm, 0);
      break;
    case EPI_SILU:
      hipLaunchKernelGGL((gemm_t256_kernel<EPI_SILU, true>), grid, dim3(512), 0, stream, x, xf_tiles, M, KB, w, NBtot, out, ldo, ntm, 0);
      break;
    default:
      return -4;
  }
  return (int)hipGetLastError();
}

// splitk > 1 (EPI_F32 only): the K range is cut into splitk pieces of ceil(K-tiles / splitk) 64-deep tiles, one
// workgroup per (output tile, piece), f32 slab per piece in out[splitk][M][N] -- fills the chip when the 256^2 tile
// grid alone would not (3B 2k prefill o / down: 96 tiles -> x3)
extern "C" int lsa_gemm_t256(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi,
                             int splitk, hipStream_t stream) {
  if (K % 32 != 0 || N % 16 != 0 || M <= 0) return -1;
  const int KB = K / 32, NBtot = N / 16;
  const int ntm = (M + 255) / 256, ntn = (NBtot + 15) / 16;
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  if (splitk < 1) splitk = 1;
  if (splitk > 1 && epi != EPI_F32) return -3;
  const int T = (KB + 1) / 2, kts = splitk > 1 ? (T + splitk - 1) / splitk : 0;
  if (splitk > 1 && (T + kts - 1) / kts != splitk) return -3;  // every piece owns >= 1 K-tile
  const dim3 grid(ntm * ntn * splitk);
  const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
  switch (epi) {
    case EPI_BF16:
      hipLaunchKernelGGL(gemm_t256_kernel<EPI_BF16>, grid, dim3(512), 0, stream, x, ldx, M, KB, w, NBtot, out, ldo, ntm, 0);
      break;
    case EPI_F32:
      hipLaunchKernelGGL(gemm_t256_kernel<EPI_F32>, grid, dim3(512), 0, stream, x, ldx, M, KB, w, NBtot, out, ldo, ntm, kts);
      break;
    case EPI_SILU:
      hipLaunchKernelGGL(gemm_t256_kernel<EPI_SILU>, grid, dim3(512), 0, stream, x, ldx, M, KB, w, NBtot, out, ldo, ntm, 0);
      break;
    default:
      return -4;
  }
  return (int)hipGetLastError();
}
