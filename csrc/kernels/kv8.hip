// fp8 KV cache (ops.KV_FP8) support kernels.
//
// The cache stores every (token, kv-head) row of 128 values as e4m3 bytes (token-pair order, common.h kv8_off)
// with one f32 scale (written by
// rope_append_kernel<.., KV8> / attn_decode_kernel<.., KV8>).  Decode attention reads the bytes directly
// (attention.hip).  Prefill attention is compute-bound MFMA work on bf16 LDS tiles, so the blocks a prefill batch
// attends to are widened once per layer into a compact bf16 scratch (lsa_kv8_dequant) and the unchanged prefill
// kernels run on that with the table scratch block = seq * mb + j.  Cost: 1 B read + 2 B written per cached
// value, ~3 % of a 2k-token prefill layer's attention time.
#include "common.h"

// grid (mb, nseq * Hkv, 2): block j of sequence seq, kv head hk, K (z = 0) or V (z = 1); 256 threads, each two
// 16-byte units of the tile (token pair p, 8-dim chunk ch: common.h kv8_off) -> 8 bf16 of tokens 2p and 2p + 1.
// Blocks at or past the sequence's context are skipped.
__global__ __launch_bounds__(256) void kv8_dequant_kernel(const uint8_t* __restrict__ kc, const uint8_t* __restrict__ vc,
                                                          const float* __restrict__ ks, const float* __restrict__ vs,
                                                          const int* __restrict__ block_tables, int max_blocks,
                                                          const int* __restrict__ ctx_lens, int Hkv, int mb,
                                                          uint16_t* __restrict__ ko, uint16_t* __restrict__ vo) {
  const int j = blockIdx.x, seq = blockIdx.y / Hkv, hk = blockIdx.y % Hkv;
  if (j * 64 >= ctx_lens[seq]) return;
  const bool isv = blockIdx.z != 0;
  const size_t src = ((size_t)block_tables[(size_t)seq * max_blocks + j] * Hkv + hk) * 64;
  const size_t dst = ((size_t)(seq * mb + j) * Hkv + hk) * 64;
  const uint8_t* tile = (isv ? vc : kc) + src * 128;
  const float* sc = (isv ? vs : ks) + src;
  uint16_t* o = (isv ? vo : ko) + dst * 128;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int unit = threadIdx.x + 256 * i, p = unit >> 4, ch = unit & 15;
    const uint4 q = *reinterpret_cast<const uint4*>(tile + unit * 16);  // == kv8_off(2 p, 8 ch)
    const float2 s2 = *reinterpret_cast<const float2*>(sc + 2 * p);
    float f[8];
    fp8x8_to_f32(make_uint2(q.x, q.y), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= s2.x;
    *reinterpret_cast<uint4*>(o + (2 * p) * 128 + 8 * ch) = pack8(f);
    fp8x8_to_f32(make_uint2(q.z, q.w), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= s2.y;
    *reinterpret_cast<uint4*>(o + (2 * p + 1) * 128 + 8 * ch) = pack8(f);
  }
}

extern "C" int lsa_kv8_dequant(const void* kc, const void* vc, const float* ks, const float* vs, const int* block_tables,
                               int max_blocks, const int* ctx_lens, int nseq, int Hkv, int mb, void* ko, void* vo,
                               hipStream_t s) {
  if (nseq <= 0 || mb <= 0) return 0;
  if (mb > max_blocks) return -1;
  hipLaunchKernelGGL(kv8_dequant_kernel, dim3(mb, nseq * Hkv, 2), dim3(256), 0, s, reinterpret_cast<const uint8_t*>(kc),
                     reinterpret_cast<const uint8_t*>(vc), ks, vs, block_tables, max_blocks, ctx_lens, Hkv, mb,
                     reinterpret_cast<uint16_t*>(ko), reinterpret_cast<uint16_t*>(vo));
  return (int)hipGetLastError();
}
