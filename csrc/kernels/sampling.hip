// Token selection + device-side decode-state update (graph-capturable: no host round trip).
//
//   lsa_argmax_partial   [B, V] f32 logits -> per-chunk packed (orderable key << 32 | ~index) maxima
//   lsa_sample_commit    per row: greedy (temperature <= 0) = reduce the argmax partials; otherwise
//                        repetition penalty (last `window` tokens, llama.cpp semantics), top-k (<= 64)
//                        by a per-chunk bitonic sort in LDS, temperature softmax, top-p nucleus and a
//                        counter-based RNG draw.  Then the decode state is advanced in place:
//                        out_tokens[b, gen_len[b]] = tok, gen_len++, input_ids = tok, positions++,
//                        finished on EOS / length.  A finished row keeps its position (its KV slot is
//                        re-written, never a new block), so a replayed graph can never walk past the
//                        blocks reserved for it.
#include "common.h"

#define LSA_TOPK 64
#define LSA_CHUNK 2048

__device__ __forceinline__ unsigned long long pack_key(float v, int idx) {
  return ((unsigned long long)float_key(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)idx);
}

__global__ __launch_bounds__(256) void argmax_partial_kernel(const float* __restrict__ logits, int V, int chunk,
                                                             unsigned long long* __restrict__ part, int nch) {
  const int c = blockIdx.x, b = blockIdx.y;
  const float* row = logits + (size_t)b * V;
  const int lo = c * chunk, hi = min(V, lo + chunk);
  unsigned long long best = 0ull;
  for (int i = lo + threadIdx.x; i < hi; i += 256) {
    const unsigned long long k = pack_key(row[i], i);
    best = k > best ? k : best;
  }
  best = wave_max_u64(best);
  __shared__ unsigned long long red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b2 = red[0];
    for (int i = 1; i < 4; ++i) b2 = red[i] > b2 ? red[i] : b2;
    part[(size_t)b * nch + c] = b2;
  }
}

struct DecodeState {
  int* out_tokens;  // [B, max_new]
  int max_new;
  int* gen_len;     // [B]
  int* input_ids;   // [B]
  int* positions;   // [B]
  int* finished;    // [B]
  const int* eos;   // [neos]
  int neos;
  const int* limit;   // [B] per-row max new tokens (<= max_new)
  const int* eos_on;  // [B] 0 = ignore EOS for this row
  int* hist;          // [B, window] ring of the context's last tokens (slot = position % window), or null
  int window;
};

__device__ void commit_token(const DecodeState& st, int b, int tok) {
  if (st.finished[b]) return;
  const int n = st.gen_len[b];
  if (n < st.max_new) st.out_tokens[(size_t)b * st.max_new + n] = tok;
  st.gen_len[b] = n + 1;
  bool done = (n + 1) >= min(st.max_new, st.limit[b]);
  if (st.eos_on[b])
    for (int e = 0; e < st.neos; ++e) done |= (tok == st.eos[e]);
  st.input_ids[b] = tok;
  if (st.hist) st.hist[(size_t)b * st.window + (st.positions[b] + 1) % st.window] = tok;  // its position
  if (done) {
    st.finished[b] = 1;
  } else {
    st.positions[b] += 1;
  }
}

__global__ __launch_bounds__(64) void argmax_commit_kernel(const unsigned long long* __restrict__ part, int nch,
                                                           DecodeState st) {
  const int b = blockIdx.x;
  unsigned long long best = 0ull;
  for (int i = threadIdx.x; i < nch; i += 64) {
    const unsigned long long k = part[(size_t)b * nch + i];
    best = k > best ? k : best;
  }
  best = wave_max_u64(best);
  if (threadIdx.x == 0) commit_token(st, b, (int)(0xffffffffu - (uint32_t)(best & 0xffffffffull)));
}

// ---------------------------------------------------------------- sampling path
// bitonic sort (descending by key) of n (power of two) packed keys in LDS with the whole block
__device__ void bitonic_desc(unsigned long long* a, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int ix = i ^ j;
        if (ix > i) {
          const unsigned long long x = a[i], y = a[ix];
          const bool desc = (i & k) == 0;
          if (desc ? (x < y) : (x > y)) {
            a[i] = y;
            a[ix] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// repetition penalty applied in place (llama.cpp / Ollama semantics: logit / pen if > 0, else * pen) to
// each distinct token among the row's last `last_n` context tokens (prompt + generated), read from the
// position-indexed ring `hist` ending at the current input position
__global__ __launch_bounds__(64) void repeat_penalty_kernel(float* __restrict__ logits, int V,
                                                            const int* __restrict__ hist, int window,
                                                            const float* __restrict__ penalty,
                                                            const int* __restrict__ last_n,
                                                            const int* __restrict__ positions) {
  const int b = blockIdx.x;
  const float pen = penalty[b];
  if (pen == 1.0f) return;
  const int* hrow = hist + (size_t)b * window;
  const int p = positions[b];
  const int n = min(min(last_n ? last_n[b] : window, window), p + 1);
  for (int i = threadIdx.x; i < n; i += 64) {
    const int t = hrow[(p - i) % window];
    if (t < 0 || t >= V) continue;
    bool first = true;  // the most recent occurrence applies the penalty, once per distinct token
    for (int k = 0; k < i; ++k) first &= (hrow[(p - k) % window] != t);
    if (!first) continue;
    float* q = logits + (size_t)b * V + t;
    const float v = *q;
    *q = v > 0.f ? v / pen : v * pen;
  }
}

// stage 1: per (chunk, row) top-LSA_TOPK keys of temperature-free logits
__global__ __launch_bounds__(256) void topk_partial_kernel(const float* __restrict__ logits, int V,
                                                           unsigned long long* __restrict__ cand, int nch) {
  __shared__ unsigned long long a[LSA_CHUNK];
  const int c = blockIdx.x, b = blockIdx.y;
  const int lo = c * LSA_CHUNK;
  for (int i = threadIdx.x; i < LSA_CHUNK; i += 256) {
    const int gi = lo + i;
    a[i] = gi < V ? pack_key(logits[(size_t)b * V + gi], gi) : 0ull;
  }
  __syncthreads();
  bitonic_desc(a, LSA_CHUNK);
  for (int i = threadIdx.x; i < LSA_TOPK; i += 256) cand[((size_t)b * nch + c) * LSA_TOPK + i] = a[i];
}

// splitmix64 finalizer of a stream key
__device__ __forceinline__ unsigned long long lsa_key_mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float uniform01(unsigned long long seed, unsigned long long ctr) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// stage 2: one block per row — merge candidates, softmax(T), top-k/top-p, draw, commit
__global__ __launch_bounds__(1024) void sample_commit_kernel(const unsigned long long* __restrict__ cand, int ncand_pow2,
                                                             int ncand, const unsigned long long* __restrict__ amax_part,
                                                             int nch_amax, const float* __restrict__ temperature,
                                                             const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                             const unsigned long long* __restrict__ seeds,
                                                             DecodeState st) {
  extern __shared__ unsigned long long a[];
  const int b = blockIdx.x;
  const float T = temperature[b];
  if (T <= 0.f) {  // greedy row inside a sampled batch
    if (threadIdx.x < 64) {
      unsigned long long best = 0ull;
      for (int i = threadIdx.x; i < nch_amax; i += 64) {
        const unsigned long long k = amax_part[(size_t)b * nch_amax + i];
        best = k > best ? k : best;
      }
      best = wave_max_u64(best);
      if (threadIdx.x == 0) commit_token(st, b, (int)(0xffffffffu - (uint32_t)(best & 0xffffffffull)));
    }
    return;
  }
  for (int i = threadIdx.x; i < ncand_pow2; i += blockDim.x) a[i] = i < ncand ? cand[(size_t)b * ncand + i] : 0ull;
  __syncthreads();
  bitonic_desc(a, ncand_pow2);
  if (threadIdx.x < 64) {
    int k = top_k[b];
    if (k <= 0 || k > LSA_TOPK) k = LSA_TOPK;
    const int i = threadIdx.x;
    const uint32_t* a32 = reinterpret_cast<const uint32_t*>(a);
    const float lmax = key_float(a32[1]);
    const float li = key_float(a32[2 * i + 1]);
    float e = (i < k && a[i] != 0ull) ? __expf((li - lmax) / T) : 0.f;
    const float tot = wave_sum(e);
    float p = e / tot;
    // inclusive prefix sum over the (sorted) probabilities
    float cum = p;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float x = __shfl_up(cum, o, 64);
      if (i >= o) cum += x;
    }
    const float tp = top_p[b];
    // keep token i if the mass before it is < top_p (always keeps the first)
    const bool keep = (i < k) && (i == 0 || (cum - p) < tp) && e > 0.f;
    const float pk = keep ? p : 0.f;
    const float ktot = wave_sum(pk);
    const float pn = pk / ktot;
    float cumk = pn;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float x = __shfl_up(cumk, o, 64);
      if (i >= o) cumk += x;
    }
    // draw g of a request: the request's seed is the stream KEY (scrambled, so seeds 0, 1, 2, ... give unrelated
    // streams) and the draw index the counter; seeds[b] packs the key (low 40 bits) with a counter offset (high 24
    // bits: the tokens a preempted request already generated, so its re-admission continues the same stream
    // whatever slot it lands in).  ops/reference.py draw_seed is the host twin.
    const unsigned long long sv = seeds[b];
    const float u = uniform01(lsa_key_mix(sv & 0xFFFFFFFFFFull), (sv >> 40) + (unsigned long long)st.gen_len[b]);
    // first kept index whose cumulative mass exceeds u (fallback: last kept index)
    int first_hit = (keep && u < cumk) ? i : 64;
    int last_kept = keep ? i : -1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      first_hit = min(first_hit, __shfl_xor(first_hit, o, 64));
      last_kept = max(last_kept, __shfl_xor(last_kept, o, 64));
    }
    const int pick = first_hit < 64 ? first_hit : (last_kept >= 0 ? last_kept : 0);
    if (i == 0) {
      const int tok = (int)(0xffffffffu - (uint32_t)(a[pick] & 0xffffffffull));
      commit_token(st, b, tok);
    }
  }
}

extern "C" int lsa_argmax_commit(const float* logits, int B, int V, unsigned long long* part, int* out_tokens,
                                 int max_new, int* gen_len, int* input_ids, int* positions, int* finished,
                                 const int* eos, int neos, const int* limit, const int* eos_on, hipStream_t s) {
  const int chunk = 4096;
  const int nch = (V + chunk - 1) / chunk;
  hipLaunchKernelGGL(argmax_partial_kernel, dim3(nch, B), dim3(256), 0, s, logits, V, chunk, part, nch);
  DecodeState st{out_tokens, max_new, gen_len, input_ids, positions, finished, eos, neos, limit, eos_on, nullptr, 0};
  hipLaunchKernelGGL(argmax_commit_kernel, dim3(B), dim3(64), 0, s, part, nch, st);
  return (int)hipGetLastError();
}

// workspace: part (B * ceil(V/4096) u64) + cand (B * ceil(V/2048) * 64 u64)
extern "C" int lsa_sample_commit(float* logits, int B, int V, unsigned long long* part, unsigned long long* cand,
                                 int* hist, int window, const float* penalty, const int* last_n,
                                 const float* temperature,
                                 const int* top_k, const float* top_p, const unsigned long long* seeds,
                                 int* out_tokens, int max_new, int* gen_len, int* input_ids, int* positions,
                                 int* finished, const int* eos, int neos, const int* limit, const int* eos_on,
                                 hipStream_t s) {
  if (hist && window > 0 && penalty)
    hipLaunchKernelGGL(repeat_penalty_kernel, dim3(B), dim3(64), 0, s, logits, V, hist, window, penalty, last_n,
                       positions);
  const int chunk = 4096;
  const int nch = (V + chunk - 1) / chunk;
  hipLaunchKernelGGL(argmax_partial_kernel, dim3(nch, B), dim3(256), 0, s, logits, V, chunk, part, nch);
  const int nch2 = (V + LSA_CHUNK - 1) / LSA_CHUNK;
  hipLaunchKernelGGL(topk_partial_kernel, dim3(nch2, B), dim3(256), 0, s, logits, V, cand, nch2);
  const int ncand = nch2 * LSA_TOPK;
  int p2 = 64;
  while (p2 < ncand) p2 <<= 1;
  if (p2 > 8192) return -1;  // V > 262144 unsupported
  DecodeState st{out_tokens, max_new, gen_len, input_ids, positions, finished, eos, neos, limit, eos_on,
                 window > 0 ? hist : nullptr, window};
  hipLaunchKernelGGL(sample_commit_kernel, dim3(B), dim3(1024), p2 * sizeof(unsigned long long), s, cand, p2, ncand,
                     part, nch, temperature, top_k, top_p, seeds, st);
  return (int)hipGetLastError();
}
