// Prefill / large-M linear layers on MFMA:  out[M, N] = X[M, K] @ W[N, K]^T   (bf16 in, f32 accumulate),
// stream-K over 256 x 256 output tiles.
//
// Tile body (unchanged from round 3): 8 waves (2 along M x 4 along N, 128 x 64 each), BK = 64, one workgroup per CU
// (128 KiB of LDS), the MI355X guide's recipe for breaking the ~900 TF ceiling of the 128^2 two-barrier structure
// (cdna_hip_programming.md §5 "The 256^2 8-phase template"):
//   * both operands staged with global_load_lds (16 B per lane, 1 KiB per wave-instruction) into ONE __shared__
//     array; fragment reads are inline-asm ds_read_b128 (hipcc would otherwise drain vmcnt(0) before every
//     compiler-visible LDS read while a DMA is in flight);
//   * four phases per K-tile, each: a quadrant's fragment reads, one half-tile of prefetch, raw s_barrier, 16 MFMAs
//     under s_setprio(1), s_barrier; one counted `s_waitcnt vmcnt(4)` per K-tile, never vmcnt(0) inside the loop;
//   * LDS images are fragment-major (W is stored that way, ops.shuffle_weight; X fragments are gathered lane-wise by
//     the DMA addresses), so every ds_read_b128 is lane-linear and conflict-free without a swizzle.
//
// Decomposition (round 5): a persistent grid of one workgroup per CU walks the (tile, K-tile) iteration space.
//   * Data-parallel part: whole tiles, one per workgroup per round.
//   * Stream-K part: the last (tiles mod CUs) + CUs tiles (all of them when the grid has fewer tiles than CUs) are
//     cut by K-tile ranges, every workgroup taking an equal share of their iterations, so no CU idles in a partial
//     last round (3B 2k prefill: 96 / 160 tiles on 256 CUs; 7B gate_up at 4096 rows: 1376 tiles = 5.4 rounds).
//     A workgroup that covers only part of a tile publishes its f32 partial write-through (sc1), takes the tile's
//     ticket, and the last to arrive sums every contributor's partial in contributor order (so the rounding does
//     not depend on who arrives last) and runs the epilogue -- the counter hand-off of MI355X_MICROARCH.md "Valid
//     forms", row 1; nothing ever waits on another workgroup, so the kernel cannot deadlock whatever the residency.
//   * Virtual CU index: consecutive indices share an XCD (blocks b and b + 8 do), so a run of consecutive tiles
//     (one W column panel, neighbouring X row tiles) meets in one L2.
// Epilogues: EPI_BF16, EPI_F32 (plain f32 store), EPI_SILU (gate / up rows interleaved per 16, bf16 SiLU(g) * u),
// EPI_RES (h[M][N] f32 += acc: the o / down projections accumulate into the residual stream, the norm after them
// reads h alone).
#include "common.h"
#include "gemm_sk.h"

#include <type_traits>

#define EPI_BF16 0
#define EPI_F32 1
#define EPI_SILU 2

typedef __attribute__((address_space(3))) void* lds_ptr_t;

namespace {

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)l, 16, 0, 0);
}

// ds_read_b128 as inline asm: hipcc treats an LDS-DMA in flight as a pending write to every LDS location and would
// drain vmcnt(0) before each compiler-visible ds_read, serialising the prefetch with the compute.  The asm read is
// ordered by the explicit counted waits + raw barriers instead.
__device__ __forceinline__ u32x4_t ds_read16(const void* p) {
  u32x4_t v;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_ptr_t)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

// the same with a compile-time byte offset in the instruction's 16-bit immediate field (no address VALU)
template <int OFF>
__device__ __forceinline__ u32x4_t ds_read16_off(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds_read offset field");
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}

// N consecutive fragments (1 KiB apart) starting at fragment OFF of the wave's base address
template <int OFF, int... Is>
__device__ __forceinline__ void ds_read_frags(u32x4_t* r, uint32_t base, std::integer_sequence<int, Is...>) {
  ((r[Is] = ds_read16_off<(OFF + Is) * 1024>(base)), ...);
}


// first stream-K iteration of virtual CU c
__device__ __forceinline__ int sk_start(int c, int iters, int P) { return (int)((unsigned)(c * iters) / (unsigned)P); }
// virtual CU whose range holds iteration g: the largest c with sk_start(c) <= g
__device__ __forceinline__ int sk_owner(int g, int iters, int P) {
  return (int)((unsigned)((g + 1) * P + iters - 1) / (unsigned)iters) - 1;
}
// partial slot of virtual CU c's segment in tile t: 2c for the segment that opens c's range, 2c + 1 for the one
// that closes it (a range meets at most two partial tiles: its first and its last)
__device__ __forceinline__ int sk_slot(int c, int t, int iters, int P, int T) {
  return 2 * c + (t == sk_start(c, iters, P) / T ? 0 : 1);
}

}  // namespace

// stream-K plan of a launch (external linkage: the kernel templates take it by value)
struct SkPlan {
  int ntm;              // row tiles
  int gm;               // row tiles per raster group (grouped tile order, below)
  int ntiles;           // output tiles (row tile fastest)
  int T;                // K-tiles of 64 per output tile
  int sk_tiles;         // tiles [0, sk_tiles) are stream-K, the rest data-parallel
  int sk_iters;         // sk_tiles * T (host-checked: sk_iters * (grid + 1) < 2^31, so 32-bit index math)
  int epl;              // epilogue: 0 = straight from the accumulators, 1 = through an LDS image (full-row stores)
  int xf;               // fragment-major operands (common.h xf_off, ceil(M / 16) row tiles): +1 X, +2 the SiLU output
};

// EPI_ROPE (prefill qkv projection, bf16 KV cache): the GEMM's output row t is token t's q | k | v; the epilogue
// rotates q and k (RoPE, rotate-half, from the f32 accumulators), writes q to q_out [T][H][128] and appends k / v
// to the paged cache at (block_tables[tok_seq[t]][pos[t] / 64], kv-head, pos[t] % 64) -- the qkv activation never
// makes a round trip through HBM and the rope_append launch is gone.  Tiles of 128 / 256 columns hold whole heads.
#define EPI_ROPE 4
struct RopeEpi {
  const int* pos;
  const int* tok_seq;
  const int* bt;
  int max_blocks;
  const float* cos_t;  // [max_pos][64]
  const float* sin_t;
  uint16_t* q_out;
  uint16_t* kc;
  uint16_t* vc;
  int H, Hkv;
};


// Tile geometry: BM rows (128 | 256) x WN * 64 columns (WN n-blocks of 16 per wave: 2 | 3 | 4), 8 waves as 2 (M) x 4
// (N), each wave owning (BM / 2) x (WN * 16).  A wave's output splits into quadrants (qm, qn): qm halves its rows,
// qn its n-blocks (NQ0 = ceil(WN / 2), NQ1 = WN / 2).  The operands are staged as four LDS halves, each falling free
// at a different phase so it can be restaged while the rest of its K-tile is still in use:
//   half 0 = XQ0: every wave row-group's first BM / 4 rows   (read in phase 1)
//   half 1 = XQ1: the other BM / 4 rows                       (read in phase 3)
//   half 2 = WQ0: every wave's first NQ0 n-blocks            (read in phases 1 and 4)
//   half 3 = WQ1: every wave's last NQ1 n-blocks             (read in phase 2)
// fragment (1 KiB, one 16 x 32 MFMA operand) within an X half: (wr * MI + i) * KS + ks; within a W half
// (wc * NQ + j) * KS + ks.  Each wave moves (half fragments) / 8 of them per half-stage, one global_load_lds each.
// KS = k-steps of 32 per K-tile (2: BK = 64; the kernel body also takes 4, BK = 128 -- measured no faster, see kSkCfgs).
// NW = waves per workgroup: 8 (2 M x 4 N, one workgroup per CU) or 4 (2 M x 2 N with twice the columns per wave, two
// workgroups per CU: 30 % fewer LDS fragment bytes per MFMA for the 128-row tiles, whose 64 x 48 per-wave tiles are
// bound by the LDS reads, profiles/r5/prefill_gemm_bk128_ab_cold_mi355x.jsonl).
template <int BM, int WN, int KS = 2, int NW = 8>
struct TileCfg {
  static constexpr int WGN = NW / 2;                      // wave columns
  static constexpr int MI = BM / 64;                      // 16-row fragments per M quadrant of a wave
  static constexpr int NQ0 = (WN + 1) / 2, NQ1 = WN / 2;  // n-blocks per N quadrant of a wave
  static constexpr int XF = 2 * MI * KS;                  // fragments per X half
  static constexpr int WF0 = WGN * NQ0 * KS, WF1 = WGN * NQ1 * KS;  // fragments per W half
  static constexpr int GX = XF / NW, GW0 = WF0 / NW, GW1 = WF1 / NW;  // glds per wave per half-stage
  static constexpr int WAIT = GX + GW1;  // the K-tile-(t+2) loads a wave has in flight after phase 4's stage
  static constexpr int NBT = WGN * WN;   // n-blocks per tile
  // LDS: one K-tile buffer = the four halves back to back (fragment offsets HOFF), NBUF buffers
  static constexpr int BUFF = 2 * XF + WF0 + WF1;            // fragments (KiB) per K-tile buffer
  static constexpr int HOFF[4] = {0, XF, 2 * XF, 2 * XF + WF0};
  static constexpr bool CAN3 = 3 * BUFF * (NW == 4 ? 2 : 1) <= 160;  // three buffers fit (per CU: 1 or 2 workgroups)
  static constexpr bool CAN4 = 4 * BUFF <= 160 && NW == 8;            // the one-phase schedule's four (128-row tiles)
  static constexpr int WAIT3 = 2 * GX + GW0 + GW1;           // a whole K-tile's loads per wave (3-buffer wait)
};

// timing probe (scripts/sk_stamps.py): when set, thread 0 of every workgroup records s_memrealtime (100 MHz) at
// entry [0], after its first segment's pipeline fill [1], after its last segment's K loop [2] and at exit [3], its
// K-tile [4] and segment [5] counts, and s_memtime (shader clock) at [1] / [2] as [6] / [7]; null in production
__device__ unsigned long long* g_sk_stamps = nullptr;
extern "C" int lsa_sk_set_stamps(unsigned long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sk_stamps), &p, sizeof(p));
}
// (compiled in only with -DLSA_SK_STAMPS: its live scalars cost the 256 x 256 kernels SGPR / VGPR spills)
#ifdef LSA_SK_STAMPS
#define LSA_SK_STAMP(K, V) \
  if (stp && threadIdx.x == 0) stp[(size_t)blockIdx.x * 8 + (K)] = (V)
#else
#define LSA_SK_STAMP(K, V) (void)0
#endif

// The kernel body is a __device__ function template behind a thin __global__ wrapper: hipcc's host pass does not
// emit the launch stub of a kernel template whose own body holds generic (integral_constant) lambdas.
template <int BM, int WN, int EPI, int NBUF, int KS, int NW>
__device__ __forceinline__ void gemm_sk_body(const uint16_t* __restrict__ X, int ldx, int M, int KB,
                                             const uint4* __restrict__ Wf, int NBtot, void* __restrict__ out, int ldo,
                                             const SkPlan& pl, float* __restrict__ ws, int* __restrict__ tickets,
                                             const RopeEpi& re) {
  using C = TileCfg<BM, WN, KS, NW>;
  constexpr int SLOT = BM * C::NBT * 16;  // floats of one partial-tile slot
#ifdef LSA_SK_STAMPS
  unsigned long long* const stp = g_sk_stamps;
  int st_seg = 0, st_kt = 0;
#endif
#ifdef LSA_SK_PHASE
  // (diagnostic LSA_SK_PHASE build, scripts/sk_phase.py) per-wave s_memtime cycles of the one-phase K-tile's parts,
  // summed over the wave's K-tiles: [0] fragment reads + DMA issue + counted waits, [1] barrier 1, [2] MFMA issue,
  // [3] barrier 2, [4] K-tiles -> g_sk_stamps[(block * 8 + wave) * 8 + k]
  // sub-stamps of [0]: [5] fragment reads issued and returned (the stamp waits lgkmcnt), [6] LDS-DMA issue; the
  // counted waits are the rest of [0]
  unsigned long long ph_acc[7] = {0, 0, 0, 0, 0, 0, 0}, ph_t = 0, ph_t0 = 0;
#define LSA_SK_PH(K)                                                             \
  do {                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                           \
    const unsigned long long ph_now = __builtin_amdgcn_s_memtime();              \
    __builtin_amdgcn_sched_barrier(0);                                           \
    if ((K) >= 5) {                                                              \
      ph_acc[(K)] += ph_now - ph_t0;                                             \
      ph_t0 = ph_now;                                                            \
    } else {                                                                     \
      if ((K) > 0) ph_acc[(K) - 1] += ph_now - ph_t;                             \
      if ((K) == 4) ++ph_acc[4];                                                 \
      ph_t = ph_now;                                                             \
      ph_t0 = ph_now;                                                            \
    }                                                                            \
  } while (0)
#else
#define LSA_SK_PH(K) (void)0
#endif
  LSA_SK_STAMP(0, __builtin_amdgcn_s_memrealtime());
  constexpr int MI = C::MI, NQ0 = C::NQ0, NQ1 = C::NQ1;
  constexpr bool BIG = 2 * MI * WN >= 24;  // >= 96 accumulator VGPRs (256 x 256, 4-wave 128 x 192): smaller epilogue load batches
  static_assert(C::GX >= 1 && C::GW1 >= 1 && C::XF % NW == 0 && C::WF0 % NW == 0 && C::WF1 % NW == 0 &&
                    C::XF <= 32 && C::WF0 <= 32 && NBUF * C::BUFF * (NW == 4 ? 2 : 1) <= 160, "tile geometry");
  static_assert(EPI != EPI_SILU || WN % 2 == 0, "SiLU pairs (gate, up) n-blocks inside one wave");
  static_assert(EPI != EPI_ROPE || C::NBT % 8 == 0, "RoPE tiles hold whole 128-column heads");
  static_assert(NBUF == 2 || (NBUF == 3 && C::CAN3) || (NBUF == 4 && C::CAN4), "K-tile buffers");
  __shared__ __attribute__((aligned(16))) uint4 lds[NBUF * C::BUFF * 64];
  const int lane = threadIdx.x & 63;
  // wave ids through readfirstlane: provably uniform, so every per-wave address term lives in SGPRs
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 0..7
  const int wm = w / C::WGN, wn = w % C::WGN;
  const int P = gridDim.x, b = blockIdx.x, xcd = b & 7;
  const int q8 = P >> 3, r8 = P & 7;
  const int vc = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int T = pl.T;
  const int r16 = lane & 15, c16 = 8 * (lane >> 4);

  // operand staging by buffer_load ... lds: the per-lane byte offset of each staged fragment is fixed for a segment
  // (one VGPR each), the K-tile's offset rides in the SGPR soffset -- no VALU per load in the K loop
  // (byte-exact ranges: an odd K's missing last k-step is staged from past the end, which the buffer unit reads as
  // zeros, so the MFMAs of that k-step add nothing and the K loop has no odd-tail branch)
  // fragment-major X (pl.xf & 1, the prefill activation layout): each staged fragment is one contiguous 1 KiB piece
  // (16 rows x 32 k) at (k-step * xmt + row tile) KiB, where the row-major gather reads 16 rows x 64 B, half of each
  // of 16 cache lines -- the ablation with contiguous pieces ran the 128-row tiles' K-tiles 17 % faster
  // (profiles/r6/prefill_gemm_stamps.txt); the K-tile step is then KS * xmt KiB
  const bool xfx = pl.xf & 1;
  const int xmt = (M + 15) >> 4;
  const int xstep = xfx ? KS * xmt * 1024 : KS * 64;
  const int xbytes = xfx ? KB * xmt * 1024 : ((M - 1) * ldx + KB * 32) * 2, wbytes = NBtot * KB * 1024;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)Wf, 0, wbytes, 0x00020000);
  int vx[2][C::GX], vw0[C::GW0], vw1[C::GW1];
  int kt0 = 0, Tl = 1;  // the segment's K-tiles [kt0, kt0 + Tl)
  int mbase = 0, nbase = 0;

  // fragment f of a half: X (wr * MI + i) * KS + ks, W (wc * NQ + j) * KS + ks; this wave stages f = per * w + e
  auto setup = [&](int tile) {
    // grouped raster order: consecutive tile ids walk gm row tiles, then the next column, so the P / 8 consecutive
    // tiles of one XCD's CUs form a gm x (P / 8 / gm) block and its L2 holds gm X panels + that many W panels
    // (the plain column-major order gave each XCD every X panel: 3B down at 2048 rows 345 MB of L2 misses vs 281 MB
    // for hipBLASLt, rocprofv3 TCC_MISS_sum)
    const int ntn = pl.ntiles / pl.ntm, gsz = pl.gm * ntn, grp = tile / gsz, fm = grp * pl.gm;
    const int gmr = min(pl.gm, pl.ntm - fm), loc = tile - grp * gsz;
    const int tm = fm + loc % gmr, tn = loc / gmr;
    mbase = tm * BM;
    nbase = tn * C::NBT;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < C::GX; ++e) {
        const int f = C::GX * w + e, wi = f / KS, ks = f % KS, wr_ = wi / MI, i = wi % MI;
        const int row0 = mbase + wr_ * (BM / 2) + h * (BM / 4) + i * 16;
        if (xfx) {
          vx[h][e] = (ks * xmt + min(row0 >> 4, xmt - 1)) * 1024 + lane * 16;
        } else {
          const int row = min(row0 + r16, M - 1);
          vx[h][e] = (row * ldx + c16) * 2 + ks * 64;
        }
      }
#pragma unroll
    for (int e = 0; e < C::GW0; ++e) {
      const int f = C::GW0 * w + e, wj = f / KS, ks = f % KS, wc = wj / NQ0, j = wj % NQ0;
      const int nb = min(nbase + wc * WN + j, NBtot - 1);
      vw0[e] = (nb * KB + ks) * 1024 + lane * 16;
    }
#pragma unroll
    for (int e = 0; e < C::GW1; ++e) {
      const int f = C::GW1 * w + e, wj = f / KS, ks = f % KS, wc = wj / NQ1, j = wj % NQ1;
      const int nb = min(nbase + wc * WN + NQ0 + j, NBtot - 1);
      vw1[e] = (nb * KB + ks) * 1024 + lane * 16;
    }
  };
  // stage half H of segment K-tile t (clamped to the segment's last) into buffer B
  auto stage = [&](auto Hc, auto Bc, int t) {
    constexpr int H = decltype(Hc)::value, B = decltype(Bc)::value;
    const int tc = kt0 + min(t, Tl - 1);
    constexpr int per = H < 2 ? C::GX : (H == 2 ? C::GW0 : C::GW1);
#pragma unroll
    for (int e = 0; e < per; ++e) {
      const int f = per * w + e;
      const bool oob = tc * KS + f % KS >= KB;  // a k-step past K (the last K-tile's tail): staged as zeros
      void* dst = &lds[(B * C::BUFF + C::HOFF[H] + f) * 64];
      if constexpr (H < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)dst, 16, vx[H][e], oob ? xbytes : tc * xstep, 0, 0);
      else if constexpr (H == 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)dst, 16, vw0[e], oob ? wbytes : tc * (KS * 1024), 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)dst, 16, vw1[e], oob ? wbytes : tc * (KS * 1024), 0, 0);
    }
  };

  f32x4_t acc[2 * MI][WN];
  // X fragments of one M quadrant, W fragments of one N quadrant: [i or j][ks] flattened as i * KS + ks
  u32x4_t xr[MI * KS], wr[NQ0 * KS];
  // fragment reads: one base VGPR per (operand, buffer), the half / fragment offset as the ds_read immediate
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)&lds[0] + lane * 16;
  auto xb = [&](int B) { return lds0 + (B * C::BUFF + wm * MI * KS) * 1024; };
  auto wb0 = [&](int B) { return lds0 + (B * C::BUFF + wn * NQ0 * KS) * 1024; };
  auto wb1 = [&](int B) { return lds0 + (B * C::BUFF + wn * NQ1 * KS) * 1024; };
  // the half's offset rides in the ds_read immediate while it fits the 16-bit field, else in the base VGPR
  auto rd = [&](auto Hc, u32x4_t* r, uint32_t base, auto Nc) {
    constexpr int H = decltype(Hc)::value, N = decltype(Nc)::value;
    if constexpr ((C::HOFF[H] + N) * 1024 <= 65536)
      ds_read_frags<C::HOFF[H]>(r, base, std::make_integer_sequence<int, N>{});
    else
      ds_read_frags<0>(r, base + C::HOFF[H] * 1024, std::make_integer_sequence<int, N>{});
  };
  auto read_x = [&](auto Bc, auto QMc) {
    constexpr int B = decltype(Bc)::value, QM = decltype(QMc)::value;
    rd(std::integral_constant<int, QM>{}, xr, xb(B), std::integral_constant<int, MI * KS>{});
  };
  auto read_w = [&](auto Bc, auto QNc) {
    constexpr int B = decltype(Bc)::value, QN = decltype(QNc)::value;
    if constexpr (QN == 0)
      rd(std::integral_constant<int, 2>{}, wr, wb0(B), std::integral_constant<int, NQ0 * KS>{});
    else
      rd(std::integral_constant<int, 3>{}, wr, wb1(B), std::integral_constant<int, NQ1 * KS>{});
  };
  // one-phase schedule (NBUF 4): the whole K-tile's fragments at once
  u32x4_t xa[2][MI * KS], wa0[NQ0 * KS], wa1[(NQ1 > 0 ? NQ1 : 1) * KS];
  auto read_all = [&](auto Bc) {
    constexpr int B = decltype(Bc)::value;
    rd(std::integral_constant<int, 0>{}, xa[0], xb(B), std::integral_constant<int, MI * KS>{});
    rd(std::integral_constant<int, 1>{}, xa[1], xb(B), std::integral_constant<int, MI * KS>{});
    rd(std::integral_constant<int, 2>{}, wa0, wb0(B), std::integral_constant<int, NQ0 * KS>{});
    if constexpr (NQ1 > 0) rd(std::integral_constant<int, 3>{}, wa1, wb1(B), std::integral_constant<int, NQ1 * KS>{});
  };
  auto mma_all = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[qm * MI + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8_t, j < NQ0 ? wa0[j * KS + ks] : wa1[(j - NQ0) * KS + ks]),
                __builtin_bit_cast(bf16x8_t, xa[qm][i * KS + ks]), acc[qm * MI + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto mma = [&](auto QMc, auto QNc) {
    constexpr int QM = decltype(QMc)::value, QN = decltype(QNc)::value;
    constexpr int nq = QN ? NQ1 : NQ0;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < nq; ++j)
          acc[QM * MI + i][QN * NQ0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, wr[j * KS + ks]), __builtin_bit_cast(bf16x8_t, xr[i * KS + ks]),
              acc[QM * MI + i][QN * NQ0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // one tile segment: acc = X[tile rows] @ W[tile cols]^T over K-tiles [k0, k1).  Four phases per K-tile t
  // (buffer t & 1, the loop unrolled by two so every LDS address is an immediate):
  //   P1 (0,0): read XQ0 + WQ0   stage XQ1(t+1)
  //   P2 (0,1): read WQ1         stage WQ0(t+1)
  //   P3 (1,1): read XQ1         stage XQ0(t+2)
  //   P4 (1,0): read WQ0         stage WQ1(t+2), then s_waitcnt vmcnt(GX + GW1): tile t+1 landed
  // Every restage comes >= 2 phases after the last read of that half (WAR); every read comes a phase after the wait
  // that retired it (RAW) - cdna_hip_programming.md §5, 8-phase template rules.  K-tiles past the segment's end are
  // staged from clamped addresses (never read) so the counted wait stays exact.
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  auto segment = [&](int tile, int k0, int k1) {
    setup(tile);
    kt0 = k0;
    Tl = k1 - k0;
#pragma unroll
    for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    __syncthreads();  // the previous segment's LDS reads (and flag word) are done before the DMA overwrites them
#define LSA_WAITV(N) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory")
#define LSA_PHASE(READS, STAGE, WAIT, QM, QN)                   \
  do {                                                          \
    READS;                                                      \
    STAGE;                                                      \
    WAIT;                                                       \
    __builtin_amdgcn_s_barrier();                               \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          \
    __builtin_amdgcn_sched_barrier(0);                          \
    mma(QM{}, QN{});                                            \
    __builtin_amdgcn_sched_barrier(0);                          \
    __builtin_amdgcn_s_barrier();                               \
  } while (0)
#define LSA_KTILE(B, NB, t)                                                                        \
  do {                                                                                             \
    LSA_PHASE((read_x(B{}, I0{}), read_w(B{}, I0{})), stage(I1{}, NB{}, (t) + 1), (void)0, I0, I0); \
    LSA_PHASE(read_w(B{}, I1{}), stage(I2{}, NB{}, (t) + 1), (void)0, I0, I1);                     \
    LSA_PHASE(read_x(B{}, I1{}), stage(I0{}, B{}, (t) + 2), (void)0, I1, I1);                      \
    LSA_PHASE(read_w(B{}, I0{}), stage(I3{}, B{}, (t) + 2), LSA_WAITV(C::WAIT), I1, I0);           \
  } while (0)
  // Three buffers (NBUF 3, the tiles whose three K-tile buffers fit the LDS): K-tile t in buffer t % 3, and during
  // it every half of K-tile t + 2 goes into buffer (t + 2) % 3 (= t - 1's, each half restaged >= 2 phases after its
  // last read there, as above):
  //   P1 (0,0): read XQ0 + WQ0   stage XQ0, XQ1 (t+2)
  //   P2 (0,1): read WQ1         stage WQ0, WQ1 (t+2)
  //   P3 (1,1): read XQ1
  //   P4 (1,0): read WQ0         s_waitcnt vmcnt(one K-tile's loads): tile t+1 landed
  // so every half is issued 7-10 phases ahead of its first read (the two-buffer order gives WQ0 three): the
  // weight stream's HBM latency hides behind ~2 K-tiles instead of ~0.75 (in-engine, cold-cache prefill GEMMs).
#define LSA_KTILE3(B, B2, t)                                                                                  \
  do {                                                                                                        \
    LSA_PHASE((read_x(B{}, I0{}), read_w(B{}, I0{})), (stage(I0{}, B2{}, (t) + 2), stage(I1{}, B2{}, (t) + 2)), \
              (void)0, I0, I0);                                                                               \
    LSA_PHASE(read_w(B{}, I1{}), (stage(I2{}, B2{}, (t) + 2), stage(I3{}, B2{}, (t) + 2)), (void)0, I0, I1);  \
    LSA_PHASE(read_x(B{}, I1{}), (void)0, (void)0, I1, I1);                                                  \
    LSA_PHASE(read_w(B{}, I0{}), (void)0, LSA_WAITV(C::WAIT3), I1, I0);                                      \
  } while (0)
  // One phase per K-tile (NBUF 4, the 128-row tiles, whose four-phase split left 4-8 MFMAs between barriers): K-tile t
  // in buffer t % 4; read all its fragments, stage all of K-tile t + 3 into buffer (t + 3) % 4 (= t - 1's), wait for
  // the own DMAs of t + 1 and the own reads of t, barrier, then the K-tile's MFMAs in one cluster, barrier.  With the
  // ping-pong offset one group's MFMA cluster runs under the other group's reads.  RAW: t + 1's DMAs (issued two
  // K-tiles ahead) are waited by every wave before the barrier that precedes their reads; WAR: every wave's reads of
  // t - 1 completed (lgkmcnt) before a barrier that precedes the restage of its buffer.
#define LSA_KTILE4(B, BS, t)                                                      \
  do {                                                                            \
    LSA_SK_PH(0);                                                                 \
    read_all(B{});                                                                \
    LSA_SK_PH(5);                                                                 \
    stage(I0{}, BS{}, (t) + 3);                                                   \
    stage(I1{}, BS{}, (t) + 3);                                                   \
    stage(I2{}, BS{}, (t) + 3);                                                   \
    stage(I3{}, BS{}, (t) + 3);                                                   \
    LSA_SK_PH(6);                                                                 \
    LSA_WAITV(2 * C::WAIT3);                                                      \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                            \
    LSA_SK_PH(1);                                                                 \
    __builtin_amdgcn_s_barrier();                                                 \
    LSA_SK_PH(2);                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                            \
    mma_all();                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                            \
    LSA_SK_PH(3);                                                                 \
    __builtin_amdgcn_s_barrier();                                                 \
    LSA_SK_PH(4);                                                                 \
  } while (0)
    if constexpr (NBUF == 4) {
      stage(I0{}, I0{}, 0);
      stage(I1{}, I0{}, 0);
      stage(I2{}, I0{}, 0);
      stage(I3{}, I0{}, 0);
      stage(I0{}, I1{}, 1);
      stage(I1{}, I1{}, 1);
      stage(I2{}, I1{}, 1);
      stage(I3{}, I1{}, 1);
      stage(I0{}, I2{}, 2);
      stage(I1{}, I2{}, 2);
      stage(I2{}, I2{}, 2);
      stage(I3{}, I2{}, 2);
      LSA_WAITV(2 * C::WAIT3);
    } else if constexpr (NBUF == 3) {
      stage(I0{}, I0{}, 0);
      stage(I1{}, I0{}, 0);
      stage(I2{}, I0{}, 0);
      stage(I3{}, I0{}, 0);
      stage(I0{}, I1{}, 1);
      stage(I1{}, I1{}, 1);
      stage(I2{}, I1{}, 1);
      stage(I3{}, I1{}, 1);
      LSA_WAITV(C::WAIT3);
    } else {
      stage(I0{}, I0{}, 0);
      stage(I3{}, I0{}, 0);
      stage(I1{}, I0{}, 0);
      stage(I2{}, I0{}, 0);
      stage(I0{}, I1{}, 1);
      stage(I3{}, I1{}, 1);
      LSA_WAITV(C::WAIT);
    }
    __builtin_amdgcn_s_barrier();
#ifdef LSA_SK_STAMPS
    if (st_seg == 0) {
      LSA_SK_STAMP(1, __builtin_amdgcn_s_memrealtime());
      LSA_SK_STAMP(6, __builtin_amdgcn_s_memtime());
    }
    ++st_seg;
    st_kt += Tl;
#endif
    // ping-pong: the second M wave group runs one barrier behind, so one group's MFMA section overlaps the other's
    // fragment reads + prefetch issue (the >= 2-phase WAR/RAW slack above covers the offset)
    if (wm == 1) __builtin_amdgcn_s_barrier();
    int t = 0;
    if constexpr (NBUF == 4) {
      for (; t + 3 < Tl; t += 4) {
        LSA_KTILE4(I0, I3, t);
        LSA_KTILE4(I1, I0, t + 1);
        LSA_KTILE4(I2, I1, t + 2);
        LSA_KTILE4(I3, I2, t + 3);
      }
      if (t < Tl) LSA_KTILE4(I0, I3, t);
      if (t + 1 < Tl) LSA_KTILE4(I1, I0, t + 1);
      if (t + 2 < Tl) LSA_KTILE4(I2, I1, t + 2);
    } else if constexpr (NBUF == 3) {
      for (; t + 2 < Tl; t += 3) {
        LSA_KTILE3(I0, I2, t);
        LSA_KTILE3(I1, I0, t + 1);
        LSA_KTILE3(I2, I1, t + 2);
      }
      if (t < Tl) LSA_KTILE3(I0, I2, t);
      if (t + 1 < Tl) LSA_KTILE3(I1, I0, t + 1);
    } else {
      for (; t + 1 < Tl; t += 2) {
        LSA_KTILE(I0, I1, t);
        LSA_KTILE(I1, I0, t + 1);
      }
      if (t < Tl) LSA_KTILE(I0, I1, t);
    }
#undef LSA_KTILE4
#undef LSA_KTILE3
#undef LSA_KTILE
#undef LSA_PHASE
#undef LSA_WAITV
    if (wm == 0) __builtin_amdgcn_s_barrier();  // rebalance the barrier count
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the segment
    LSA_SK_STAMP(2, __builtin_amdgcn_s_memrealtime());
    LSA_SK_STAMP(7, __builtin_amdgcn_s_memtime());
  };

  // epilogue of a finished tile: acc[i][j] = D[n = nb_j * 16 + 4 g + q][m = mb_i * 16 + (lane & 15)]
  const int g = lane >> 4;
  auto store_tile = [&]() {
    if constexpr (EPI == EPI_ROPE) return;  // the RoPE epilogue always runs through the LDS image
    if constexpr (EPI == EPI_RES) {
      // h += acc: the h loads of IB fragment rows x WN leave together before their first store (a load after a store
      // through the same pointer is not hoisted, which made this a chain of 2 MI WN dependent round trips)
      constexpr int IB = BIG ? 1 : 2;  // fragment rows per batch of h loads (IB x WN float4 in flight per lane)
#pragma unroll
      for (int hf = 0; hf < 2 * MI / IB; ++hf) {
        float4 hv[IB][WN];
#pragma unroll
        for (int ii = 0; ii < IB; ++ii)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            const int m = mbase + wm * (BM / 2) + (hf * IB + ii) * 16 + (lane & 15);
            const int nb = nbase + wn * WN + j;
            if (m < M && nb < NBtot)
              hv[ii][j] = *reinterpret_cast<const float4*>(reinterpret_cast<float*>(out) + (size_t)m * ldo + nb * 16 + 4 * g);
          }
#pragma unroll
        for (int ii = 0; ii < IB; ++ii) {
          const int i = hf * IB + ii;
          const int m = mbase + wm * (BM / 2) + i * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            const int nb = nbase + wn * WN + j;
            if (m >= M || nb >= NBtot) continue;
            float4 h = hv[ii][j];
            h.x += acc[i][j][0]; h.y += acc[i][j][1]; h.z += acc[i][j][2]; h.w += acc[i][j][3];
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (size_t)m * ldo + nb * 16 + 4 * g) = h;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2 * MI; ++i) {
      const int m = mbase + wm * (BM / 2) + i * 16 + (lane & 15);
      if (m >= M) continue;
      if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < WN; j += 2) {
          const int nb = nbase + wn * WN + j;  // even: gate block, nb + 1: up block
          if (nb + 1 >= NBtot) continue;
          uint2 p;
          p.x = pack2bf(silu(acc[i][j][0]) * acc[i][j + 1][0], silu(acc[i][j][1]) * acc[i][j + 1][1]);
          p.y = pack2bf(silu(acc[i][j][2]) * acc[i][j + 1][2], silu(acc[i][j][3]) * acc[i][j + 1][3]);
          const int c = (nb >> 1) * 16 + 4 * g;
          // fragment-major (pl.xf & 2): a wave-instruction's 16 rows x 16 columns fill 512 contiguous bytes
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) +
                                    ((pl.xf & 2) ? xf_off(m, c, (M + 15) >> 4) : (size_t)m * ldo + c)) = p;
        }
      } else {
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const int nb = nbase + wn * WN + j;
          if (nb >= NBtot) continue;
          const size_t o = (size_t)m * ldo + nb * 16 + 4 * g;
          if constexpr (EPI == EPI_BF16) {
            uint2 p;
            p.x = pack2bf(acc[i][j][0], acc[i][j][1]);
            p.y = pack2bf(acc[i][j][2], acc[i][j][3]);
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + o) = p;
          } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + o) =
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
          }
        }
      }
    }
  };

  // The same epilogue through LDS: the accumulators hold 4 consecutive columns of one row per lane, so a direct
  // store instruction covers 16 rows x 64 B (f32) / 32 B (bf16).  Here each half of the tile's rows (one M wave
  // group) is written to an f32 LDS image [BM / 2][OC] (16-B chunk ch of row r at ch ^ (r & 15): conflict-free
  // writes of 16 rows and reads of one row) and read back one full row per wave-instruction, so the global stores
  // (and the residual's h reads) are whole 128-B lines.
  auto store_tile_lds = [&]() {
    constexpr int OC0 = EPI == EPI_SILU ? C::NBT * 8 : C::NBT * 16;  // output columns of the tile
    constexpr int CH = OC0 / 4;                                      // 16-B f32 chunks per image row
    constexpr int OC = (CH + 15) / 16 * 64;  // image row stride: whole 16-chunk swizzle groups (SiLU of 192: 96 -> 128)
    static_assert(OC * (BM / 2) * 4 <= NBUF * C::BUFF * 1024, "the image fits the K-tile buffers");
    float* img = reinterpret_cast<float*>(&lds[0]);
    const int ncol_out = EPI == EPI_SILU ? NBtot * 8 : NBtot * 16;
    const int col0 = EPI == EPI_SILU ? nbase * 8 : nbase * 16;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      __syncthreads();  // the previous readers (main loop or the other pass) are done with the image
      if (wm == pass) {
#pragma unroll
        for (int i = 0; i < 2 * MI; ++i) {
          const int r = i * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            f32x4_t v = acc[i][j];
            int ch;
            if constexpr (EPI == EPI_SILU) {
              if (j & 1) continue;
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] = silu(acc[i][j][q]) * acc[i][j + 1][q];
              ch = ((wn * WN + j) >> 1) * 4 + (lane >> 4);
            } else {
              ch = (wn * WN + j) * 4 + (lane >> 4);
            }
            *reinterpret_cast<f32x4_t*>(img + r * OC + ((ch ^ (r & 15)) << 2)) = v;
          }
        }
      }
      __syncthreads();
      // this wave's rows of the pass: r = w + NW k, k < RPW (one row per wave-instruction, lanes = 16-B column chunks).
      // Every global load of those rows is issued before the first store: a load after a store through the same
      // output pointer cannot be hoisted by the compiler, so a row-by-row loop paid one full load latency per row
      // (16 rows per wave and pass at BM = 256)
      constexpr int RPW = BM / 2 / NW;
      const bool live_ch = lane < CH && col0 + lane * 4 < ncol_out;
      if constexpr (EPI == EPI_ROPE) {
        // per-row metadata once per pass, lane k for row k: the token's position and its paged-cache block
        int my_pos = 0, my_blk = 0;
        if (lane < RPW) {
          const int m = mbase + pass * (BM / 2) + w + NW * lane;
          if (m < M) {
            my_pos = re.pos[m];
            const int seq = re.tok_seq ? re.tok_seq[m] : m;
            my_blk = re.bt[(size_t)seq * re.max_blocks + (my_pos >> 6)];
          }
        }
        const int ch = lane;
        const int c = col0 + ch * 4, head = c >> 7, d = c & 127, d0 = d & 63;
        const bool rot = head < re.H + re.Hkv;  // q and k heads rotate (rotate-half, partner 64 dims away)
        const int pch = d < 64 ? ch + 16 : ch - 16;
        const float sg = d < 64 ? -1.f : 1.f;
        const int hk = head < re.H + re.Hkv ? head - re.H : head - re.H - re.Hkv;
        uint16_t* cache = head < re.H + re.Hkv ? re.kc : re.vc;
        constexpr int RG = BIG ? 2 : 4;  // rows whose cos / sin loads leave together
#pragma unroll 1
        for (int k0 = 0; k0 < RPW; k0 += RG) {
          float4 cs[RG], sn[RG];
          int pk_[RG];
#pragma unroll
          for (int u = 0; u < RG; ++u) {
            pk_[u] = __builtin_amdgcn_readlane(my_pos, k0 + u);
            cs[u] = *reinterpret_cast<const float4*>(re.cos_t + (size_t)pk_[u] * 64 + d0);
            sn[u] = *reinterpret_cast<const float4*>(re.sin_t + (size_t)pk_[u] * 64 + d0);
          }
#pragma unroll
          for (int u = 0; u < RG; ++u) {
            const int r = w + NW * (k0 + u);
            const int m = mbase + pass * (BM / 2) + r;
            if (m >= M || !live_ch) continue;
            const f32x4_t v = *reinterpret_cast<const f32x4_t*>(img + r * OC + ((ch ^ (r & 15)) << 2));
            f32x4_t y = v;
            if (rot) {
              const f32x4_t pv = *reinterpret_cast<const f32x4_t*>(img + r * OC + ((pch ^ (r & 15)) << 2));
              y[0] = v[0] * cs[u].x + sg * pv[0] * sn[u].x;
              y[1] = v[1] * cs[u].y + sg * pv[1] * sn[u].y;
              y[2] = v[2] * cs[u].z + sg * pv[2] * sn[u].z;
              y[3] = v[3] * cs[u].w + sg * pv[3] * sn[u].w;
            }
            const uint2 pk = make_uint2(pack2bf(y[0], y[1]), pack2bf(y[2], y[3]));
            if (head < re.H) {
              *reinterpret_cast<uint2*>(re.q_out + ((size_t)m * re.H + head) * 128 + d) = pk;
            } else {
              const int p = pk_[u], blk = __builtin_amdgcn_readlane(my_blk, k0 + u);
              *reinterpret_cast<uint2*>(cache + (((size_t)blk * re.Hkv + hk) * 64 + (p & 63)) * 128 + d) = pk;
            }
          }
        }
        continue;
      }
      if constexpr (EPI == EPI_RES) {
        constexpr int RB = BIG ? 2 : 8;  // rows whose h loads leave together
#pragma unroll 1
        for (int k0 = 0; k0 < RPW; k0 += RB) {
        float4 hv[RB];
#pragma unroll
        for (int u = 0; u < RB; ++u) {
          const int m = mbase + pass * (BM / 2) + w + NW * (k0 + u);
          if (m < M && live_ch) hv[u] = *reinterpret_cast<const float4*>(reinterpret_cast<float*>(out) + (size_t)m * ldo + col0 + lane * 4);
        }
#pragma unroll
        for (int u = 0; u < RB; ++u) {
          const int r = w + NW * (k0 + u);
          const int m = mbase + pass * (BM / 2) + r;
          if (m < M && live_ch) {
            const f32x4_t v = *reinterpret_cast<const f32x4_t*>(img + r * OC + ((lane ^ (r & 15)) << 2));
            float4 h = hv[u];
            h.x += v[0]; h.y += v[1]; h.z += v[2]; h.w += v[3];
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (size_t)m * ldo + col0 + lane * 4) = h;
          }
        }
        }
        continue;
      }
#pragma unroll 4
      for (int k = 0; k < RPW; ++k) {
        const int r = w + NW * k;
        const int m = mbase + pass * (BM / 2) + r;
        const int ch = lane;
        if (live_ch && m < M) {
          const f32x4_t v = *reinterpret_cast<const f32x4_t*>(img + r * OC + ((ch ^ (r & 15)) << 2));
          const size_t o = (size_t)m * ldo + col0 + ch * 4;
          if constexpr (EPI == EPI_BF16 || EPI == EPI_SILU) {
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + o) =
                make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
          } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + o) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    }
  };
  auto finish_tile = [&]() {
    // (a fragment-major SiLU output goes straight from the accumulators: their stores are already whole lines)
    if (EPI == EPI_ROPE || (pl.epl && !(EPI == EPI_SILU && (pl.xf & 2)))) store_tile_lds();
    else if constexpr (EPI != EPI_ROPE) store_tile();
  };

  // stream-K part: this virtual CU's iterations [s0, s1) of the first sk_tiles tiles
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
  int* flag = reinterpret_cast<int*>(&lds[0]);
  const int iters = pl.sk_iters;
  const int s1 = iters > 0 ? sk_start(vc + 1, iters, P) : 0;
  constexpr int WSTRIDE = 2 * MI * WN * 64 * 4;  // floats of one wave's accumulators in a partial slot
  for (int gi = iters > 0 ? sk_start(vc, iters, P) : 0; gi < s1;) {
    const int tile = gi / T;
    const int k0 = gi - tile * T;
    const int k1 = min(T, k0 + (s1 - gi));
    segment(tile, k0, k1);
    gi += k1 - k0;
    if (k0 == 0 && k1 == T) {
      finish_tile();
      continue;
    }
    // partial tile: publish (sc1 stores, 1 KiB per wave-instruction), ticket, the last arriver finishes
    const int cf = sk_owner(tile * T, iters, P), cl = sk_owner(tile * T + T - 1, iters, P);
    {
      // this lane's byte offset in its slot (one VGPR); the fragment's 1 KiB step rides in the SGPR offset
      const int voff = (sk_slot(vc, tile, iters, P, T) * SLOT + w * WSTRIDE + lane * 4) * 4;
#pragma unroll
      for (int i = 0; i < 2 * MI; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          const u32x4_t u = {__float_as_uint(acc[i][j][0]), __float_as_uint(acc[i][j][1]),
                             __float_as_uint(acc[i][j][2]), __float_as_uint(acc[i][j][3])};
          __builtin_amdgcn_raw_buffer_store_b128(u, rs, voff, (i * WN + j) * 1024, LSA_SC1_AUX);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 partial stores
    __syncthreads();
    if (threadIdx.x == 0)
      *flag = __hip_atomic_fetch_add((lsa_g_i32*)tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              cl - cf;
    __syncthreads();
    if (!*flag) continue;
    if (threadIdx.x == 0)
      __hip_atomic_store((lsa_g_i32*)tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // sum the contributors' partials in contributor order (cf .. cl), two fragment rows at a time
#pragma unroll
    for (int hh = 0; hh < MI; ++hh) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[2 * hh + i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      for (int c = cf; c <= cl; ++c) {
        const int voff = (sk_slot(c, tile, iters, P, T) * SLOT + w * WSTRIDE + lane * 4) * 4;
        u32x4_t v[2][WN];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            v[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, ((2 * hh + i) * WN + j) * 1024, LSA_SC1_AUX);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[2 * hh + i][j][q] += __uint_as_float(v[i][j][q]);
      }
    }
    finish_tile();
  }

  // data-parallel part: whole tiles sk_tiles + vc, + P, ...
  for (int tile = pl.sk_tiles + vc; tile < pl.ntiles; tile += P) {
    segment(tile, 0, T);
    finish_tile();
  }
  LSA_SK_STAMP(3, __builtin_amdgcn_s_memrealtime());
  LSA_SK_STAMP(4, (unsigned long long)st_kt);
  LSA_SK_STAMP(5, (unsigned long long)st_seg);
#ifdef LSA_SK_PHASE
  if (g_sk_stamps && lane == 0) {
    unsigned long long* o = g_sk_stamps + ((size_t)blockIdx.x * 8 + w) * 8;
#pragma unroll
    for (int k = 0; k < 7; ++k) o[k] = ph_acc[k];
  }
#endif
}

template <int BM, int WN, int EPI, int NBUF, int KS, int NW>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void gemm_sk_kernel(const uint16_t* __restrict__ X, int ldx, int M, int KB,
                                                      const uint4* __restrict__ Wf, int NBtot,
                                                      void* __restrict__ out, int ldo, SkPlan pl,
                                                      float* __restrict__ ws, int* __restrict__ tickets,
                                                      RopeEpi re) {
  gemm_sk_body<BM, WN, EPI, NBUF, KS, NW>(X, ldx, M, KB, Wf, NBtot, out, ldo, pl, ws, tickets, re);
}

// Plan for a grid of (at most) ncu workgroups over BM x (NBT * 16) tiles: the data-parallel rounds keep whole tiles;
// the remainder round plus one full round (or every tile, when there are fewer tiles than CUs) is split by K-tile
// ranges.  min_share: the fewest K-tiles a workgroup's stream-K range may hold (a shorter range gives up parallelism
// for fewer partial tiles: the grid shrinks instead).  sk = false: whole tiles only (ceil(tiles / ncu) rounds).
static SkPlan sk_plan(int M, int KB, int NBtot, int BM, int NBT, int KS, int ncu, int min_share, bool sk, int* grid) {
  SkPlan pl;
  pl.epl = 0;
  pl.ntm = (M + BM - 1) / BM;
  pl.ntiles = pl.ntm * ((NBtot + NBT - 1) / NBT);
  // raster group: the power-of-two row count a of an XCD's block of tiles (ncu / 8 of them) that minimises the L2
  // footprint a * BM + (ncu / 8 / a) * BN (an X panel is BM x K, a W panel BN x K)
  {
    const int per_xcd = ncu / 8 > 0 ? ncu / 8 : 1, bn = NBT * 16;
    int best = 1;
    long long bcost = 1LL << 62;
    for (int a = 1; a <= per_xcd && a <= pl.ntm; a *= 2) {
      const long long c = (long long)a * BM + (long long)((per_xcd + a - 1) / a) * bn;
      if (c < bcost) bcost = c, best = a;
    }
    pl.gm = best;
  }
  pl.T = (KB + KS - 1) / KS;
  const int P = ncu;
  if (!sk) {
    pl.sk_tiles = 0;
    *grid = pl.ntiles < P ? pl.ntiles : P;
  } else if (pl.ntiles >= P) {
    const int rem = pl.ntiles % P;
    pl.sk_tiles = rem ? rem + P : 0;
    if (pl.sk_tiles > pl.ntiles) pl.sk_tiles = pl.ntiles;
    *grid = P;
  } else {
    pl.sk_tiles = pl.ntiles;
    const long long it = (long long)pl.ntiles * pl.T;
    long long g = it / (min_share > 0 ? min_share : 1);
    if (g > P) g = P;
    if (g < pl.ntiles) g = pl.ntiles;
    *grid = (int)g;
  }
  pl.sk_iters = pl.sk_tiles * pl.T;
  return pl;
}

// Tile configurations (BM, WN) and their cost per output element per K-tile relative to the 256 x 256 tile (the
// narrower tiles stage more operand bytes per MFMA and run shorter phases); a partial-tile seam (a 64-256 KiB f32
// partial written and read back by one CU) is priced in 256 x 256 K-tiles.  Measured: scripts/bench_prefill_gemm.py.
// ks: k-steps of 32 per K-tile.  BK = 128 (ks 4) for the 128-row tiles was built and measured no faster (cold caches,
// profiles/r5/prefill_gemm_bk128_ab_cold_mi355x.jsonl: ties or loses by 1-3 %), so every configuration runs BK = 64.
// nw: waves per workgroup (4: two workgroups per CU, twice the columns per wave; TileCfg).
struct SkCfg {
  int bm, wn, ks, nw;
  float cost;
};
static const SkCfg kSkCfgs[] = {{256, 4, 2, 8, 1.00f}, {256, 3, 2, 8, 1.06f}, {256, 2, 2, 8, 1.18f},
                                {128, 4, 2, 8, 1.18f}, {128, 3, 2, 8, 1.28f}, {128, 2, 2, 8, 1.45f},
                                {128, 6, 2, 4, 1.20f}, {128, 4, 2, 4, 1.36f}};
#define LSA_SK_SEAM_KTILES 8.0f

// predicted time (256 x 256 K-tiles) of config c on the shape; *use_sk: whether the stream-K remainder beats whole
// rounds
static float sk_cfg_time(const SkCfg& c, int M, int KB, int NBtot, int ncu, bool* use_sk) {
  const int nbt = (c.nw / 2) * c.wn;
  ncu *= c.nw == 4 ? 2 : 1;  // workgroup slots; a slot of a shared CU runs at about half the rate (cost below)
  const long long tiles = (long long)((M + c.bm - 1) / c.bm) * ((NBtot + nbt - 1) / nbt);
  const float T = (float)((KB + c.ks - 1) / c.ks) * (float)c.ks / 2.0f;  // in 64-deep K-tiles
  const float per_tile = T * c.cost * (float)(c.bm * nbt) / 4096.0f * (c.nw == 4 ? 2.0f : 1.0f);
  const float dp = (float)((tiles + ncu - 1) / ncu) * per_tile;
  const float skt = (float)tiles / ncu * per_tile + LSA_SK_SEAM_KTILES * (c.bm * nbt) / 4096.0f;
  *use_sk = tiles % ncu != 0 && skt < dp;
  return *use_sk ? skt : dp;
}

// epilogue mode of the next launches (lsa_gemm_sk_epilogue): 0 direct, 1 through LDS
static int g_sk_epl = 1;
extern "C" void lsa_gemm_sk_epilogue(int mode) { g_sk_epl = mode ? 1 : 0; }
// K-tile buffers (lsa_gemm_sk_nbuf): 3 wherever three fit the LDS (default), 2 = the two-buffer schedule everywhere
static int g_sk_nbuf = 3;
extern "C" void lsa_gemm_sk_nbuf(int n) { g_sk_nbuf = n == 2 ? 2 : 3; }
// one-phase schedule (four K-tile buffers, one MFMA cluster per K-tile) for the tiles whose four buffers fit (the
// 128-row tiles but 128 x 256); lsa_gemm_sk_one_phase(0) restores the four-phase one.  Default on: interleaved A/B at
// the engine's table configurations (scripts/ab_sk_sched.py, profiles/r6/prefill_gemm_one_phase_ab_mi355x.jsonl):
// 3B o 2048 rows 50.9 -> 48.7 us warm / 65.0 -> 62.6 cold, 3B down 134.2 -> 130.6 cold, 7B qkv 300 rows 74.7 -> 70.8
// cold; the 128 x 128 configurations tie
static int g_sk_one = 1;
extern "C" void lsa_gemm_sk_one_phase(int on) { g_sk_one = on ? 1 : 0; }

template <int BM, int WN, int KS = 2, int NW = 8>
static int sk_launch(int epi, const uint16_t* x, int ldx, int M, int KB, const uint4* w, int NBtot, void* out, int ldo,
                     float* ws, int* tickets, int ncu, int min_share, bool sk, int epl, int xf, int* grid_out,
                     const RopeEpi& re, hipStream_t stream) {
  using C = TileCfg<BM, WN, KS, NW>;
  const int P = ncu * (NW == 4 ? 2 : 1);  // persistent workgroups: one per CU, or two of the 4-wave kind
  int grid = 0;
  SkPlan pl = sk_plan(M, KB, NBtot, BM, C::NBT, KS, P, min_share, sk, &grid);
  pl.epl = epl;
  pl.xf = xf;
  if (pl.sk_tiles > 2 * P || grid > P || (long long)pl.sk_tiles * pl.T * (grid + 1) >= (1LL << 31)) return -3;
  if (grid_out) *grid_out = grid;
  switch (epi) {
#define LSA_SKL(E)                                                                                                \
  do {                                                                                                            \
    if constexpr (C::CAN4) {                                                                                      \
      if (g_sk_one) {                                                                                             \
        hipLaunchKernelGGL((gemm_sk_kernel<BM, WN, E, 4, KS, NW>), dim3(grid), dim3(64 * NW), 0, stream, x, ldx, \
                           M, KB, w, NBtot, out, ldo, pl, ws, tickets, re);                                   \
        break;                                                                                                    \
      }                                                                                                           \
    }                                                                                                             \
    if constexpr (C::CAN3) {                                                                                      \
      if (g_sk_nbuf == 3) {                                                                                       \
        hipLaunchKernelGGL((gemm_sk_kernel<BM, WN, E, 3, KS, NW>), dim3(grid), dim3(64 * NW), 0, stream, x, ldx, \
                           M, KB, w, NBtot, out, ldo, pl, ws, tickets, re);                                   \
        break;                                                                                                    \
      }                                                                                                           \
    }                                                                                                             \
    hipLaunchKernelGGL((gemm_sk_kernel<BM, WN, E, 2, KS, NW>), dim3(grid), dim3(64 * NW), 0, stream, x, ldx, M, \
                       KB, w, NBtot, out, ldo, pl, ws, tickets, re);                                          \
  } while (0)
    case EPI_BF16: LSA_SKL(EPI_BF16); break;
    case EPI_F32: LSA_SKL(EPI_F32); break;
    case EPI_RES: LSA_SKL(EPI_RES); break;
    case EPI_SILU:
      if constexpr (WN % 2 == 0) {
        LSA_SKL(EPI_SILU);
        break;
      } else {
        return -2;
      }
    case EPI_ROPE:
      if constexpr (C::NBT % 8 == 0) {
        LSA_SKL(EPI_ROPE);
        break;
      } else {
        return -2;
      }
#undef LSA_SKL
    default: return -4;
  }
  return (int)hipGetLastError();
}

// M > 64 linear layer (K % 32 == 0, N % 16 == 0; EPI_SILU needs N % 32 == 0).  ws: lsa_gemm_sk_ws_bytes(ncu)
// bytes; tickets: lsa_gemm_sk_tickets(ncu) int32, zero before the first call (every call leaves them zero).
// out: bf16 [M][N] (EPI_BF16), f32 [M][N] (EPI_F32), bf16 [M][N / 2] (EPI_SILU), f32 h [M][N] accumulated (EPI_RES).
// cfg: -1 = the cost model's pick, else an index into kSkCfgs (+ 8: whole tiles only, no stream-K remainder), + 16:
// the epilogue mode given in bit 5 (+ 32 = through LDS) instead of lsa_gemm_sk_epilogue's; *cfg_out = the
// configuration used (bits 0-3).  xf: +1 X in the fragment-major layout of ceil(M / 16) row tiles (common.h xf_off;
// ldx unused), +2 the EPI_SILU output in it -- the prefill activations the next GEMM stages as whole 1 KiB pieces.
static int gemm_sk_impl(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, float* ws,
                        int* tickets, int ncu, int min_share, int cfg, int xf, int* grid_out, int* cfg_out,
                        const RopeEpi& re, hipStream_t stream) {
  if (K % 32 != 0 || N % 16 != 0 || M <= 0 || ncu < 8 || ncu > 1024 || !ws || !tickets) return -1;
  // fragment-major operands: X (+1; its whole buffer, K / 32 x ceil(M / 16) KiB, under the 2 GiB buffer range),
  // the SiLU output (+2; whole 32-column k-steps: N / 2 % 32 == 0)
  if (xf < 0 || xf > 3 || ((xf & 2) && (epi != EPI_SILU || N % 64)) || ((xf & 1) && (long long)(K / 32) * ((M + 15) / 16) >= (1 << 21)))
    return -7;
  if (epi == EPI_SILU && N % 32 != 0) return -2;
  const bool even_wn = epi == EPI_SILU || epi == EPI_ROPE;  // tile configurations with an even n-block count/wave
  const int KB = K / 32, NBtot = N / 16;
  const int ncfg = (int)(sizeof(kSkCfgs) / sizeof(kSkCfgs[0]));
  bool sk = true;
  int epl = g_sk_epl;
  if (cfg >= 0 && (cfg & 16)) {
    epl = (cfg >> 5) & 1;
    cfg &= 15;
  }
  if (cfg < 0) {
    float best = 3.0e38f;
    for (int i = 0; i < ncfg; ++i) {
      if (even_wn && kSkCfgs[i].wn % 2) continue;
      // RoPE: a tile must hold whole 128-column heads (8 n-blocks), or the rotate-half partner of a column lies
      // outside the tile's LDS image (the 4-wave 128 x 192 tile has 12 n-blocks)
      if (epi == EPI_ROPE && ((kSkCfgs[i].nw / 2) * kSkCfgs[i].wn) % 8) continue;
      bool u = false;
      const float t = sk_cfg_time(kSkCfgs[i], M, KB, NBtot, ncu, &u);
      if (t < best) best = t, cfg = i, sk = u;
    }
  } else {
    if (cfg > 15) return -5;
    sk = cfg < 8;
    cfg &= 7;
    if (cfg >= ncfg) return -5;
    // BN 192 -> the 256-column tile (RoPE needs whole 128-column heads; the 4-wave 192-column tile pairs fine for SiLU)
    if (even_wn && (kSkCfgs[cfg].wn % 2 || (epi == EPI_ROPE && ((kSkCfgs[cfg].nw / 2) * kSkCfgs[cfg].wn) % 8)))
      cfg = kSkCfgs[cfg].bm == 256 ? 0 : 3;
  }
  if (cfg_out) *cfg_out = cfg + (sk ? 0 : 8);
  const uint16_t* x = reinterpret_cast<const uint16_t*>(X);
  const uint4* w = reinterpret_cast<const uint4*>(Wf);
  const int ldo = epi == EPI_SILU ? N / 2 : N;
  switch (cfg) {
#define LSA_SKC(I, BMV, WNV) \
  case I: return sk_launch<BMV, WNV>(epi, x, ldx, M, KB, w, NBtot, out, ldo, ws, tickets, ncu, min_share, sk, epl, xf, grid_out, re, stream);
    LSA_SKC(0, 256, 4)
    LSA_SKC(1, 256, 3)
    LSA_SKC(2, 256, 2)
    LSA_SKC(3, 128, 4)
    LSA_SKC(4, 128, 3)
    LSA_SKC(5, 128, 2)
    case 6: return sk_launch<128, 6, 2, 4>(epi, x, ldx, M, KB, w, NBtot, out, ldo, ws, tickets, ncu, min_share, sk, epl, xf, grid_out, re, stream);
    case 7: return sk_launch<128, 4, 2, 4>(epi, x, ldx, M, KB, w, NBtot, out, ldo, ws, tickets, ncu, min_share, sk, epl, xf, grid_out, re, stream);
#undef LSA_SKC
    default: return -5;
  }
}

extern "C" int lsa_gemm_sk(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, float* ws,
                           int* tickets, int ncu, int min_share, int cfg, int xf, int* grid_out, int* cfg_out,
                           hipStream_t stream) {
  if (epi < 0 || epi > 3) return -4;
  return gemm_sk_impl(X, ldx, M, K, Wf, N, out, epi, ws, tickets, ncu, min_share, cfg, xf, grid_out, cfg_out,
                      RopeEpi{}, stream);
}

// the prefill qkv projection with RoPE + the paged bf16 KV-cache append fused into its epilogue (EPI_ROPE above);
// N = (H + 2 Hkv) * 128
extern "C" int lsa_gemm_sk_rope(const void* X, int ldx, int M, int K, const void* Wf, int N, float* ws, int* tickets,
                                int ncu, int min_share, int cfg, const int* pos, const int* tok_seq,
                                const int* block_tables, int max_blocks, const float* cos_t, const float* sin_t,
                                void* q_out, void* kc, void* vc, int H, int Hkv, int xf, int* grid_out, int* cfg_out,
                                hipStream_t stream) {
  if (H <= 0 || Hkv <= 0 || N != (H + 2 * Hkv) * 128 || !pos || !block_tables || !cos_t || !sin_t || !q_out || !kc ||
      !vc)
    return -6;
  const RopeEpi re{pos, tok_seq, block_tables, max_blocks, cos_t, sin_t, reinterpret_cast<uint16_t*>(q_out),
                   reinterpret_cast<uint16_t*>(kc), reinterpret_cast<uint16_t*>(vc), H, Hkv};
  return gemm_sk_impl(X, ldx, M, K, Wf, N, nullptr, EPI_ROPE, ws, tickets, ncu, min_share, cfg, xf & 1, grid_out,
                      cfg_out, re, stream);
}
