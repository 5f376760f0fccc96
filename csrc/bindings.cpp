// pybind11 / torch bindings of the gfx950 kernels (csrc/kernels/*.hip).
// Every op launches on the current HIP stream so it can be captured into a hipGraph
// (torch.cuda.CUDAGraph) and ordered with RCCL collectives issued by torch.distributed.
#ifdef LSA_BINDINGS_SELFTEST
// host-only build of the argument validation (csrc/tests/bindings_selftest.cpp, under ASan / UBSan on the CPU):
// CPU tensors stand in for device tensors, the launchers are stubs, no Python module
#include <ATen/ATen.h>
#include <hip/hip_runtime_api.h>
#else
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#endif

#include "kernels/gemm_sk.h"
#include "kernels/lsa_epi.h"

extern "C" {
int lsa_gemm(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb, int splitk,
             hipStream_t stream);
int lsa_add_rmsnorm(float* h, const float* parts, int nparts, long part_stride, const int* ids, const void* emb,
                    const int* row_idx, int write_h, const void* w, float eps, void* xn, int rows, int D,
                    int xf_mt, long long* ss_out, int ss_ld, int ss_nzero, void* x8, float* sx8, hipStream_t s);
int lsa_prefetch(const void* const* ptrs, const long* bytes, int nr, int wgs, hipStream_t s);
int lsa_res_add_ss(float* h, const float* parts, int nparts, long part_stride, void* xn, int rows, int D, int xf_mt,
                   long long* ss_out, hipStream_t s);
int lsa_a8_gemm(const void* X8, const void* s8, const float* sx, int M, int K, const void* Wq, const float* wscale,
                const void* Sw, int wk, int N, void* out, void* out_s8, int epi, int nb, int splitk, int waves, int depth,
                int xfo, const LsaEpi* ep, hipStream_t stream);
int lsa_quant_xf8(const void* x, int ldx, int M, int K, int MT, void* x8, float* sx, hipStream_t s);
int lsa_quant_xf8_blocks(const void* x, int ldx, int M, int K, int MT, int blk, void* x8, void* s8, hipStream_t s);
int lsa_gemm_ex(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb, int splitk,
                int waves, int div, int xlds, const LsaEpi* ep, hipStream_t stream);
int lsa_fp8_gemm_ex(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N, void* out,
                    int epi, int nb, int splitk, int xfrag, const LsaEpi* ep, hipStream_t stream);
int lsa_rope_append(const void* qkv, const float* qkv_parts, int nparts, long part_stride, const int* pos, const int* tok_seq, const int* block_tables, int max_blocks,
                    const float* cos_t, const float* sin_t, void* q_out, void* kc, void* vc, float* ks, float* vs, int T,
                    int H, int Hkv, hipStream_t s);
int lsa_silu_mul(const void* g, const void* u, void* o, long n, hipStream_t s);
int lsa_attn_decode(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                    const int* pos, int B, int H, int Hkv, float scale, int chunk_blocks, int nsplit, int unsplit_max,
                    void* out, float* opart, float* mlpart, int* counters, int xf_mt, const float* qkv_parts, int nparts,
                    long part_stride,
                    const float* cos_t, const float* sin_t, const float* ks, const float* vs, void* out_s8,
                    const long long* rowss, float inv_k, float eps, hipStream_t s);
int lsa_gemm_rr(int K, const void* Wf, int N, void* out, int epi, int nb, int splitk, int waves, int div,
                const LsaRr* rr, hipStream_t stream);
int lsa_a8_gemm_rr(int K, const void* Wq, const float* wscale, const void* Sw, int wk, int N, void* out, void* out_s8,
                   int epi, int nb, int splitk, int waves, int depth, const LsaRr* rr, hipStream_t stream);
int lsa_kv8_dequant(const void* kc, const void* vc, const float* ks, const float* vs, const int* block_tables,
                    int max_blocks, const int* ctx_lens, int nseq, int Hkv, int mb, void* ko, void* vo, hipStream_t s);
int lsa_attn_prefill(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                     const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv, float scale,
                     void* out, int xf_mt, hipStream_t s);
int lsa_argmax_commit(const float* logits, int B, int V, unsigned long long* part, int* out_tokens, int max_new,
                      int* gen_len, int* input_ids, int* positions, int* finished, const int* eos, int neos,
                      const int* limit, const int* eos_on, hipStream_t s);
int lsa_sample_commit(float* logits, int B, int V, unsigned long long* part, unsigned long long* cand, int* hist,
                      int window, const float* penalty, const int* last_n, const float* temperature, const int* top_k,
                      const float* top_p, const unsigned long long* seeds, int* out_tokens, int max_new, int* gen_len,
                      int* input_ids, int* positions, int* finished, const int* eos, int neos, const int* limit,
                      const int* eos_on, hipStream_t s);
int lsa_fp8_gemm(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N, void* out, int epi,
                 int nb, int splitk, hipStream_t stream);
int lsa_fp8_dequant(const void* Wq, const float* wscale, int N, int K, void* Wf, hipStream_t s);
int lsa_gemm_cfg(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, int nb, int splitk,
                 int waves, int div, int xlds, hipStream_t stream);
int lsa_fp8_gemm_cfg(const void* X, int ldx, int M, int K, const void* Wq, const float* wscale, int N, void* out,
                     int epi, int nb, int splitk, int xfrag, hipStream_t stream);
void lsa_gemm_sk_epilogue(int mode);
void lsa_gemm_sk_nbuf(int n);
void lsa_gemm_sk_one_phase(int on);
void lsa_rmsnorm_xf_tile_min(int rows);
int lsa_gemm_sk_rope(const void* X, int ldx, int M, int K, const void* Wf, int N, float* ws, int* tickets, int ncu,
                     int min_share, int cfg, const int* pos, const int* tok_seq, const int* block_tables,
                     int max_blocks, const float* cos_t, const float* sin_t, void* q_out, void* kc, void* vc, int H,
                     int Hkv, int xf, int* grid_out, int* cfg_out, hipStream_t stream);
int lsa_gemm_sk(const void* X, int ldx, int M, int K, const void* Wf, int N, void* out, int epi, float* ws,
                int* tickets, int ncu, int min_share, int cfg, int xf, int* grid_out, int* cfg_out, hipStream_t stream);
int lsa_silu_parts(const float* parts, int nparts, long part_stride, int M, int F, void* out, hipStream_t s);
int lsa_silu_bf16(const void* y, int M, int F, void* out, hipStream_t s);
void lsa_fp8_gemm_knobs(int waves, int depth);
int lsa_attn_prefill32(const void* q, const void* kc, const void* vc, const int* block_tables, int max_blocks,
                       const int* cu_q, const int* ctx_lens, const int* work, int nwork, int H, int Hkv, float scale,
                       void* out, int ng, int xf_mt, hipStream_t s);
int lsa_quant_rows_fp8(const void* x, int ldx, int M, int K, void* x8, int ld8, float* sx, hipStream_t s);
int lsa_fp8_gemm_t256(const void* X8, int ldx, const float* sx, int M, int K, const void* Wq, const float* sw, int N,
                      void* out, int epi, int splitk, hipStream_t stream);
int lsa_ar_alloc(size_t bytes, void** out);
int lsa_ar_free(void* p);
int lsa_ar_handle(void* p, char* out64);
int lsa_ar_open(const char* in64, void** out);
int lsa_ar_close(void* p);
int lsa_ar_max_world();
int lsa_prefill_qblock();
int lsa_ar_wallclock_khz(int* out);
int lsa_ar_header_bytes();
int lsa_ar_run(float* data, long n, float* out, uint8_t* const* regions, int rank, int world, size_t maxb,
               int nblocks, long long timeout_ticks, int* err, int nslab, long slab_stride, const float* res_h,
               void* res_xn, long long* res_ss, int res_d, int res_xmt, int mode, hipStream_t s);
int lsa_fp4_gemm_ex(const void* X, int ldx, int M, int K, const void* Wq, const void* S, int N, void* out, int epi,
                    int nb, int splitk, int waves, int xfrag, const LsaEpi* ep, hipStream_t stream);
int lsa_fp4_dequant(const void* Wq, const void* S, int N, int K, void* Wf, hipStream_t s);
}

namespace {

#ifdef LSA_BINDINGS_SELFTEST
hipStream_t cur_stream() { return nullptr; }
bool on_dev(const at::Tensor& t) { return t.defined(); }
#else
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
bool on_dev(const at::Tensor& t) { return t.is_cuda(); }
#endif

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, "lsa kernel '", what, "' failed: rc=", rc); }

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(on_dev(t), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

// paged KV cache operands: bf16 [nblk, Hkv, 64, 128], or fp8 (uint8 e4m3 bytes, same shape) with f32
// per-(token, kv-head) scales [nblk, Hkv, 64]
void check_cache(const at::Tensor& kc, const at::Tensor& vc, const c10::optional<at::Tensor>& ks,
                 const c10::optional<at::Tensor>& vs) {
  TORCH_CHECK(ks.has_value() == vs.has_value(), "fp8 cache needs both K and V scales");
  TORCH_CHECK(kc.dim() == 4 && kc.size(2) == 64 && kc.size(3) == 128 && kc.sizes() == vc.sizes() &&
                  kc.is_contiguous() && vc.is_contiguous(), "cache must be contiguous [nblk, Hkv, 64, 128]");
  const at::ScalarType dt = ks.has_value() ? at::kByte : at::kBFloat16;
  need(kc, dt, "kc");
  need(vc, dt, "vc");
  if (ks.has_value()) {
    need(*ks, at::kFloat, "ks");
    need(*vs, at::kFloat, "vs");
    TORCH_CHECK(ks->numel() == kc.numel() / 128 && vs->numel() == kc.numel() / 128 && ks->is_contiguous() &&
                    vs->is_contiguous(), "fp8 cache scales must be contiguous [nblk, Hkv, 64]");
  }
}

template <typename T>
T* ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// Decode epilogue extensions (kernels/lsa_epi.h): rowss = per-row sum of squares of the un-normalised
// input rows (RMS row scale with eps, 1/K); epi 3 (residual) adds into h [M, N] f32, writes bf16(h) to
// xout (fragment-major with xmt row tiles, or row-major when xmt == 0) and accumulates sum h^2 into ss_out.
struct EpiOpts {
  LsaEpi e{};
  bool on = false;
};

EpiOpts epi_opts(int64_t epi, int64_t M, int64_t N, int64_t K, const c10::optional<at::Tensor>& rowss, double eps,
                 const c10::optional<at::Tensor>& h, const c10::optional<at::Tensor>& xout, int64_t xmt,
                 const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& tickets, int64_t ncols) {
  EpiOpts o;
  if (rowss.has_value()) {
    need(*rowss, at::kLong, "rowss");
    TORCH_CHECK(rowss->numel() >= M, "rowss too small");
    o.e.rowss = reinterpret_cast<const long long*>(rowss->data_ptr<int64_t>());
    o.e.inv_k = 1.0f / (float)K;
    o.e.eps = (float)eps;
    o.on = true;
  }
  if (epi == 3) {
    TORCH_CHECK(h.has_value() && xout.has_value() && ss_out.has_value(), "residual epilogue needs h, xout, ss_out");
    need(*h, at::kFloat, "h");
    need(*xout, at::kBFloat16, "xout");
    need(*ss_out, at::kLong, "ss_out");
    TORCH_CHECK(h->is_contiguous() && h->numel() >= M * N, "h must be a contiguous [M, N] f32 tensor");
    TORCH_CHECK(ss_out->numel() >= M, "ss_out too small");
    TORCH_CHECK(xout->numel() >= (xmt ? xmt * 16 * N : M * N), "xout too small");
    o.e.h = h->data_ptr<float>();
    o.e.ldh = (int)N;
    o.e.xout = reinterpret_cast<uint16_t*>(xout->data_ptr());
    o.e.xmt = (int)xmt;
    o.e.ss_out = reinterpret_cast<long long*>(ss_out->data_ptr<int64_t>());
    if (tickets.has_value()) {
      need(*tickets, at::kInt, "tickets");
      TORCH_CHECK(tickets->numel() >= ncols, "tickets: one counter per 16-column block needed");
      o.e.tickets = tickets->data_ptr<int>();
    }
    o.on = true;
  }
  return o;
}

void check_out(int64_t epi, const at::Tensor& out, int64_t splitk, int64_t M, int64_t N, int64_t mt_silu) {
  if (epi == 3 && splitk <= 1) return;  // the residual epilogue writes through h / xout
  if (epi == 1 || epi == 3) {  // f32 slabs (split-K residual: the partials of the splits)
    need(out, at::kFloat, "out");
    TORCH_CHECK(out.numel() >= splitk * M * N, "f32 out too small");
  } else {
    need(out, at::kBFloat16, "out");
    TORCH_CHECK(out.numel() >= (epi == 2 ? (mt_silu ? mt_silu * 16 : M) * (N / 2) : M * N), "bf16 out too small");
  }
}

// out = x @ W^T with W in fragment-major layout (see kernels/gemm.hip)
void gemm(const at::Tensor& x, const at::Tensor& wf, int64_t N, at::Tensor& out, int64_t epi, int64_t nb,
          int64_t splitk, int64_t waves, int64_t div, int64_t xlds, const c10::optional<at::Tensor>& rowss,
          double eps, const c10::optional<at::Tensor>& h, const c10::optional<at::Tensor>& xout, int64_t xmt,
          const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& tickets) {
  need(x, at::kBFloat16, "x");
  need(wf, at::kBFloat16, "wf");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(wf.numel() == N * K, "weight numel mismatch: ", wf.numel(), " vs ", N, "x", K);
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, h, xout, xmt, ss_out, tickets, N / 16);
  if (eo.on) {
    check_out(epi, out, splitk, M, N, 0);
    check(lsa_gemm_ex(x.data_ptr(), x.stride(0), M, K, wf.data_ptr(), N, out.data_ptr(), epi, nb, splitk, waves, div,
                      xlds, &eo.e, cur_stream()),
          "gemm");
    return;
  }
  if (epi == 1) {
    need(out, at::kFloat, "out");
    TORCH_CHECK(out.numel() >= splitk * M * N, "f32 out too small");
  } else {
    need(out, at::kBFloat16, "out");
    TORCH_CHECK(out.numel() >= M * (epi == 2 ? N / 2 : N), "bf16 out too small");
  }
  check(lsa_gemm_cfg(x.data_ptr(), x.stride(0), M, K, wf.data_ptr(), N, out.data_ptr(), epi, nb, splitk, waves, div,
                     xlds, cur_stream()),
        "gemm");
}

// Batch-1 decode GEMM with the residual-reduce prologue (kernels/gemm.hip, lsa_epi.h LsaRr): X = h + sum_s parts[s]
// (h f32 [K]; parts f32 [np, 1, K] split-K slabs), h_out = X.  epi 1: f32 slabs [splitk, 1, N], the column-0
// workgroups add each K slice's sum of X^2 (Q24) into ss_out[0] (the slab consumer applies the row scale);
// epi 2: SiLU(gate) * up bf16 [1, N / 2] with the RMS row scale from the workgroup's own full-row sum (splitk 1).
void gemm_rr(const at::Tensor& h, const at::Tensor& parts, at::Tensor& h_out, const at::Tensor& wf, int64_t N,
             at::Tensor& out, int64_t epi, int64_t nb, int64_t splitk, int64_t waves, int64_t div,
             const c10::optional<at::Tensor>& ss_out, double eps) {
  need(h, at::kFloat, "h");
  need(h_out, at::kFloat, "h_out");
  need(parts, at::kFloat, "parts");
  need(wf, at::kBFloat16, "wf");
  const int64_t K = h.numel();
  TORCH_CHECK(h.is_contiguous() && h_out.is_contiguous() && h_out.numel() >= K, "gemm_rr: h / h_out contiguous [K]");
  TORCH_CHECK(h.data_ptr() != h_out.data_ptr(), "gemm_rr: h_out must not alias h (other workgroups still read h)");
  TORCH_CHECK(parts.dim() == 3 && parts.size(1) == 1 && parts.size(2) == K && parts.stride(2) == 1 &&
                  parts.stride(1) == K, "gemm_rr: parts must be [np, 1, K] slabs");
  TORCH_CHECK(wf.numel() == N * K, "gemm_rr: weight numel mismatch");
  TORCH_CHECK(epi == 1 || epi == 2, "gemm_rr: f32 slabs or silu");
  check_out(epi, out, splitk, 1, N, 0);
  LsaRr rr{};
  rr.h = h.data_ptr<float>();
  rr.parts = parts.data_ptr<float>();
  rr.pstride = parts.stride(0);
  rr.np = (int)parts.size(0);
  rr.h_out = h_out.data_ptr<float>();
  rr.local = epi == 2 ? 1 : 0;
  rr.inv_k = 1.0f / (float)K;
  rr.eps = (float)eps;
  if (epi == 1) {
    TORCH_CHECK(ss_out.has_value(), "gemm_rr: f32 slabs need ss_out");
    need(*ss_out, at::kLong, "ss_out");
    rr.ss_out = reinterpret_cast<long long*>(ss_out->data_ptr<int64_t>());
  }
  check(lsa_gemm_rr((int)K, wf.data_ptr(), (int)N, out.data_ptr(), (int)epi, (int)nb, (int)splitk, (int)waves, (int)div,
                    &rr, cur_stream()),
        "gemm_rr");
}

// same, with X in the fragment-major activation layout (ops.to_xfrag): xf holds ceil(M/16) row tiles
void gemm_xf(const at::Tensor& xf, int64_t M, int64_t K, const at::Tensor& wf, int64_t N, at::Tensor& out,
             int64_t epi, int64_t nb, int64_t splitk, int64_t waves, int64_t div,
             const c10::optional<at::Tensor>& rowss, double eps, const c10::optional<at::Tensor>& h,
             const c10::optional<at::Tensor>& xout, int64_t xmt, const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& tickets) {
  need(xf, at::kBFloat16, "xf");
  need(wf, at::kBFloat16, "wf");
  TORCH_CHECK(M >= 1 && M <= 64 && K % 32 == 0, "gemm_xf: M in 1..64, K % 32 == 0");
  const int64_t mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  TORCH_CHECK(xf.is_contiguous() && xf.numel() >= mt * 16 * K, "xf too small for M=", M, " K=", K);
  TORCH_CHECK(wf.numel() == N * K, "weight numel mismatch");
  check_out(epi, out, splitk, M, N, mt);
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, h, xout, xmt, ss_out, tickets, N / 16);
  check(lsa_gemm_ex(xf.data_ptr(), K, M, K, wf.data_ptr(), N, out.data_ptr(), epi, nb, splitk, waves, div, 2,
                    eo.on ? &eo.e : nullptr, cur_stream()),
        "gemm_xf");
}


// fp8 weights, activations in the fragment-major decode layout (ops.to_xfrag), M <= 64
void fp8_gemm_xf(const at::Tensor& xf, int64_t M, int64_t K, const at::Tensor& wq, const at::Tensor& wscale, int64_t N,
                 at::Tensor& out, int64_t epi, int64_t nb, int64_t splitk, int64_t waves, int64_t depth,
                 const c10::optional<at::Tensor>& rowss,
                 double eps, const c10::optional<at::Tensor>& h, const c10::optional<at::Tensor>& xout, int64_t xmt,
                 const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& tickets) {
  need(xf, at::kBFloat16, "xf");
  need(wscale, at::kFloat, "wscale");
  TORCH_CHECK(on_dev(wq) && wq.element_size() == 1 && wq.numel() == N * K, "wq must be N*K fp8 bytes");
  TORCH_CHECK(M >= 1 && M <= 64 && K % 64 == 0, "fp8_gemm_xf: M in 1..64, K % 64 == 0");
  const int64_t mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  TORCH_CHECK(xf.is_contiguous() && xf.numel() >= mt * 16 * K, "xf too small");
  check_out(epi, out, splitk, M, N, mt);
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, h, xout, xmt, ss_out, tickets, N / 16);
  lsa_fp8_gemm_knobs((int)waves, (int)depth);
  check(lsa_fp8_gemm_ex(xf.data_ptr(), K, M, K, wq.data_ptr(), wscale.data_ptr<float>(), N, out.data_ptr(), epi, nb,
                        splitk, 1, eo.on ? &eo.e : nullptr, cur_stream()),
        "fp8_gemm_xf");
}

// W8A8 / W4A8 decode GEMM (kernels/gemm_fp8a.hip): x8 e4m3 activations in the xf8 layout with per-row f32 scales
// sx and / or per-lane-block E8M0 scales s8; fp8 weights (wscale per channel) or MXFP4 weights (wsc8 = their E8M0
// block-scale words).  xfo 2: the SiLU output as e4m3 + E8M0 blocks into (out, out_s8).
void a8_gemm(const at::Tensor& x8, const c10::optional<at::Tensor>& s8, const c10::optional<at::Tensor>& sx, int64_t M,
             int64_t K, const at::Tensor& wq, const c10::optional<at::Tensor>& wscale,
             const c10::optional<at::Tensor>& wsc8, int64_t N, at::Tensor& out, const c10::optional<at::Tensor>& out_s8,
             int64_t epi, int64_t nb, int64_t splitk, int64_t waves, int64_t depth, int64_t xfo,
             const c10::optional<at::Tensor>& rowss, double eps) {
  const bool fp4 = wsc8.has_value();
  TORCH_CHECK(fp4 != wscale.has_value(), "a8_gemm: exactly one of wscale (fp8) / wsc8 (mxfp4)");
  TORCH_CHECK(M >= 1 && M <= 64 && K % 128 == 0 && N % 16 == 0, "a8_gemm: M in 1..64, K % 128 == 0, N % 16 == 0");
  TORCH_CHECK(epi == 1 || epi == 2, "a8_gemm: f32 slabs or silu");
  TORCH_CHECK(on_dev(wq) && wq.element_size() == 1 && wq.numel() == (fp4 ? N * K / 2 : N * K), "a8_gemm: weight bytes");
  if (fp4) {
    TORCH_CHECK(on_dev(*wsc8) && wsc8->numel() * wsc8->element_size() >= (N / 16) * ((K / 128 + 3) / 4) * 256,
                "a8_gemm: mxfp4 scales too small");
  } else {
    need(*wscale, at::kFloat, "wscale");
    TORCH_CHECK(wscale->numel() >= N, "a8_gemm: wscale too small");
  }
  const int64_t mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  TORCH_CHECK(on_dev(x8) && x8.element_size() == 1 && x8.is_contiguous() && x8.numel() >= mt * 16 * K, "x8 too small");
  TORCH_CHECK(s8.has_value() || sx.has_value(), "a8_gemm: per-row (sx) and / or block (s8) activation scales");
  if (s8.has_value())
    TORCH_CHECK(on_dev(*s8) && s8->element_size() == 1 && s8->numel() >= mt * 64 * (K / 128), "s8 too small");
  if (sx.has_value()) {
    need(*sx, at::kFloat, "sx");
    TORCH_CHECK(sx->numel() >= M, "sx too small");
  }
  if (epi == 2 && xfo == 2) {
    TORCH_CHECK(on_dev(out) && out.element_size() == 1 && out.numel() >= mt * 16 * (N / 2), "e4m3 SiLU out too small");
    TORCH_CHECK(out_s8.has_value() && on_dev(*out_s8) && out_s8->element_size() == 1 &&
                    out_s8->numel() >= mt * 64 * (N / 2 / 128) && (N / 2) % 128 == 0,
                "a8_gemm: e4m3 SiLU output needs out_s8 (and N / 2 % 128 == 0)");
  } else {
    check_out(epi, out, splitk, M, N, xfo ? mt : 0);
  }
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, c10::nullopt, c10::nullopt, 0, c10::nullopt, c10::nullopt, N / 16);
  check(lsa_a8_gemm(x8.data_ptr(), s8.has_value() ? s8->data_ptr() : nullptr,
                    sx.has_value() ? sx->data_ptr<float>() : nullptr, M, K, wq.data_ptr(),
                    fp4 ? nullptr : wscale->data_ptr<float>(), fp4 ? wsc8->data_ptr() : nullptr, fp4 ? 1 : 0, N,
                    out.data_ptr(), out_s8.has_value() ? out_s8->data_ptr() : nullptr, epi, nb, splitk, waves, depth, xfo,
                    eo.on ? &eo.e : nullptr, cur_stream()),
        "a8_gemm");
}

// W8A8 / W4A8 batch-1 decode GEMM with the residual-reduce prologue (kernels/gemm_fp8a.hip RR): X = h + sum_s parts[s]
// quantised in the prologue (e4m3, one E8M0 scale per 32 k); h_out = X.  epi 1: f32 slabs [splitk, 1, N] (ss_out[0] +=
// sum X^2, the slab consumer scales the row); epi 2: the e4m3 SiLU output in the xf8 layout + E8M0 blocks in out_s8
// (splitk 1, the row scale from the workgroup's own full-row sum).
void a8_gemm_rr(const at::Tensor& h, const at::Tensor& parts, at::Tensor& h_out, const at::Tensor& wq,
                const c10::optional<at::Tensor>& wscale, const c10::optional<at::Tensor>& wsc8, int64_t N, at::Tensor& out,
                const c10::optional<at::Tensor>& out_s8, int64_t epi, int64_t nb, int64_t splitk, int64_t waves,
                int64_t depth, const c10::optional<at::Tensor>& ss_out, double eps) {
  const bool fp4 = wsc8.has_value();
  TORCH_CHECK(fp4 != wscale.has_value(), "a8_gemm_rr: exactly one of wscale (fp8) / wsc8 (mxfp4)");
  need(h, at::kFloat, "h");
  need(h_out, at::kFloat, "h_out");
  need(parts, at::kFloat, "parts");
  const int64_t K = h.numel();
  TORCH_CHECK(K % 128 == 0 && N % 16 == 0, "a8_gemm_rr: K % 128 == 0, N % 16 == 0");
  TORCH_CHECK(h.is_contiguous() && h_out.is_contiguous() && h_out.numel() >= K, "a8_gemm_rr: h / h_out contiguous [K]");
  TORCH_CHECK(h.data_ptr() != h_out.data_ptr(), "a8_gemm_rr: h_out must not alias h");
  TORCH_CHECK(parts.dim() == 3 && parts.size(1) == 1 && parts.size(2) == K && parts.stride(2) == 1 &&
                  parts.stride(1) == K, "a8_gemm_rr: parts must be [np, 1, K] slabs");
  TORCH_CHECK(on_dev(wq) && wq.element_size() == 1 && wq.numel() == (fp4 ? N * K / 2 : N * K), "a8_gemm_rr: weight bytes");
  if (fp4) {
    TORCH_CHECK(on_dev(*wsc8) && wsc8->numel() * wsc8->element_size() >= (N / 16) * ((K / 128 + 3) / 4) * 256,
                "a8_gemm_rr: mxfp4 scales too small");
  } else {
    need(*wscale, at::kFloat, "wscale");
    TORCH_CHECK(wscale->numel() >= N, "a8_gemm_rr: wscale too small");
  }
  TORCH_CHECK(epi == 1 || epi == 2, "a8_gemm_rr: f32 slabs or the e4m3 SiLU output");
  if (epi == 2) {
    TORCH_CHECK(on_dev(out) && out.element_size() == 1 && out.numel() >= 16 * (N / 2), "a8_gemm_rr: e4m3 SiLU out too small");
    TORCH_CHECK(out_s8.has_value() && on_dev(*out_s8) && out_s8->element_size() == 1 && out_s8->numel() >= 64 * (N / 2 / 128) &&
                    (N / 2) % 128 == 0, "a8_gemm_rr: the e4m3 SiLU output needs out_s8 (and N / 2 % 128 == 0)");
  } else {
    check_out(epi, out, splitk, 1, N, 0);
  }
  LsaRr rr{};
  rr.h = h.data_ptr<float>();
  rr.parts = parts.data_ptr<float>();
  rr.pstride = parts.stride(0);
  rr.np = (int)parts.size(0);
  rr.h_out = h_out.data_ptr<float>();
  rr.local = epi == 2 ? 1 : 0;
  rr.inv_k = 1.0f / (float)K;
  rr.eps = (float)eps;
  if (epi == 1) {
    TORCH_CHECK(ss_out.has_value(), "a8_gemm_rr: f32 slabs need ss_out");
    need(*ss_out, at::kLong, "ss_out");
    rr.ss_out = reinterpret_cast<long long*>(ss_out->data_ptr<int64_t>());
  }
  check(lsa_a8_gemm_rr((int)K, wq.data_ptr(), fp4 ? nullptr : wscale->data_ptr<float>(),
                       fp4 ? wsc8->data_ptr() : nullptr, fp4 ? 1 : 0, (int)N, out.data_ptr(),
                       out_s8.has_value() ? out_s8->data_ptr() : nullptr, (int)epi, (int)nb, (int)splitk, (int)waves,
                       (int)depth, &rr, cur_stream()),
        "a8_gemm_rr");
}

void quant_xf8_blocks(const at::Tensor& x, int64_t mt, int64_t blk, at::Tensor& x8, at::Tensor& s8) {
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(on_dev(x8) && x8.element_size() == 1 && x8.numel() >= mt * 16 * K, "x8 too small");
  TORCH_CHECK(on_dev(s8) && s8.element_size() == 1 && s8.numel() >= mt * 64 * (K / 128), "s8 too small");
  check(lsa_quant_xf8_blocks(x.data_ptr(), x.stride(0), M, K, (int)mt, (int)blk, x8.data_ptr(), s8.data_ptr(),
                             cur_stream()),
        "quant_xf8_blocks");
}

void quant_xf8(const at::Tensor& x, int64_t mt, at::Tensor& x8, at::Tensor& sx) {
  need(x, at::kBFloat16, "x");
  need(sx, at::kFloat, "sx");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(on_dev(x8) && x8.element_size() == 1 && x8.numel() >= mt * 16 * K && sx.numel() >= M, "x8 / sx too small");
  check(lsa_quant_xf8(x.data_ptr(), x.stride(0), M, K, (int)mt, x8.data_ptr(), sx.data_ptr<float>(), cur_stream()),
        "quant_xf8");
}

// large-M (prefill) linear layer on the stream-K 256x256 tile kernel (kernels/gemm_tile256.hip).  epi: 0 bf16 [M][N],
// 1 f32 [M][N], 2 SiLU(gate) * up bf16 [M][N / 2], 3 h f32 [M][N] += x @ W^T.  ws / tickets: the per-stream
// workspace (ops._sk_workspace).  cfg: -1 = the kernel's cost model, else a tile configuration index (+ 8: whole
// tiles only; + 16 + 32 * mode: that epilogue mode for this call).  xf: + 1 x is a flat buffer in the fragment-major
// layout (ops.to_xfrag) of ``rows`` rows, + 2 the SiLU output is written in it.  Returns grid * 16 + the configuration
// used.
// rows / K of a stream-K GEMM's X: the [M, K] row-major matrix, or (xf & 1) a flat fragment-major buffer of rows rows
static std::pair<int64_t, int64_t> sk_x_shape(const at::Tensor& x, const at::Tensor& wf, int64_t N, int64_t xf,
                                              int64_t rows) {
  need(x, at::kBFloat16, "x");
  need(wf, at::kBFloat16, "wf");
  TORCH_CHECK(N > 0 && wf.numel() % N == 0, "gemm_sk: weight numel not a multiple of N");
  if (xf & 1) {
    const int64_t K = wf.numel() / N;
    TORCH_CHECK(rows > 0 && x.is_contiguous() && x.numel() >= (rows + 15) / 16 * 16 * K,
                "gemm_sk: fragment-major x needs rows and ceil(rows / 16) * 16 * K elements");
    return {rows, K};
  }
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  TORCH_CHECK(wf.numel() == N * x.size(1), "weight numel mismatch");
  return {x.size(0), x.size(1)};
}

int64_t gemm_sk(const at::Tensor& x, const at::Tensor& wf, int64_t N, at::Tensor& out, int64_t epi, at::Tensor& ws,
                at::Tensor& tickets, int64_t ncu, int64_t min_share, int64_t cfg, int64_t xf, int64_t rows) {
  need(ws, at::kFloat, "ws");
  need(tickets, at::kInt, "tickets");
  TORCH_CHECK(xf >= 0 && xf <= 3 && (!(xf & 2) || (epi == 2 && N % 64 == 0)),
              "gemm_sk: xf (+2 only with the SiLU epilogue and N / 2 % 32 == 0)");
  const auto mk = sk_x_shape(x, wf, N, xf, rows);
  const int M = (int)mk.first, K = (int)mk.second;
  TORCH_CHECK(M > 0, "gemm_sk: no rows");
  TORCH_CHECK(ncu >= 8 && ncu <= 1024, "gemm_sk: ncu out of range");
  TORCH_CHECK(ws.numel() * 4 >= lsa_gemm_sk_ws_bytes((int)ncu) && tickets.numel() >= lsa_gemm_sk_tickets((int)ncu),
              "gemm_sk: workspace too small");
  TORCH_CHECK(epi >= 0 && epi <= 3, "gemm_sk: epi");
  if (epi == 1 || epi == 3) {
    need(out, at::kFloat, "out");
    TORCH_CHECK(out.numel() >= (int64_t)M * N, "f32 out too small");
  } else {
    need(out, at::kBFloat16, "out");
    TORCH_CHECK(out.numel() >= (int64_t)((xf & 2) ? (M + 15) / 16 * 16 : M) * (epi == 2 ? N / 2 : N),
                "bf16 out too small");
  }
  TORCH_CHECK(cfg >= -1 && cfg < 64, "gemm_sk: cfg");
  int grid = 0, used = 0;
  check(lsa_gemm_sk(x.data_ptr(), (xf & 1) ? 0 : (int)x.stride(0), M, K, wf.data_ptr(), N, out.data_ptr(), (int)epi,
                    ws.data_ptr<float>(), tickets.data_ptr<int>(), (int)ncu, (int)min_share, (int)cfg, (int)xf, &grid,
                    &used, cur_stream()),
        "gemm_sk");
  return (int64_t)grid * 16 + used;
}

// the prefill qkv projection with RoPE and the paged bf16 KV-cache append in its epilogue (gemm_tile256.hip
// EPI_ROPE): q_out [T, H, 128], kc / vc [blocks, Hkv, 64, 128] bf16, pos / tok_seq [T] int32, block_tables
// [seqs, max_blocks] int32, cos / sin [max_pos, 64] f32.  Returns grid * 16 + the configuration used.
int64_t gemm_sk_rope(const at::Tensor& x, const at::Tensor& wf, at::Tensor& ws, at::Tensor& tickets, int64_t ncu,
                     int64_t min_share, int64_t cfg, const at::Tensor& pos, const c10::optional<at::Tensor>& tok_seq,
                     const at::Tensor& block_tables, const at::Tensor& cos_t, const at::Tensor& sin_t,
                     at::Tensor& q_out, at::Tensor& kc, at::Tensor& vc, int64_t H, int64_t Hkv, int64_t xf,
                     int64_t rows) {
  need(ws, at::kFloat, "ws");
  need(tickets, at::kInt, "tickets");
  need(pos, at::kInt, "pos");
  need(block_tables, at::kInt, "block_tables");
  need(cos_t, at::kFloat, "cos_t");
  need(sin_t, at::kFloat, "sin_t");
  need(q_out, at::kBFloat16, "q_out");
  need(kc, at::kBFloat16, "kc");
  need(vc, at::kBFloat16, "vc");
  TORCH_CHECK(xf == 0 || xf == 1, "gemm_sk_rope: xf 0 | 1");
  const int64_t N = (H + 2 * Hkv) * 128;
  TORCH_CHECK(H > 0 && Hkv > 0, "gemm_sk_rope: heads");
  const auto mk = sk_x_shape(x, wf, N, xf, rows);
  const int64_t M = mk.first, K = mk.second;
  TORCH_CHECK(pos.numel() >= M && q_out.is_contiguous() && q_out.numel() >= M * H * 128, "gemm_sk_rope: q_out / pos");
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(2) == 64 && kc.size(3) == 128 && kc.sizes() == vc.sizes() &&
                  kc.is_contiguous() && vc.is_contiguous(), "gemm_sk_rope: cache [blocks, Hkv, 64, 128]");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.is_contiguous(), "gemm_sk_rope: block_tables [seqs, max_blocks]");
  TORCH_CHECK(cos_t.dim() == 2 && cos_t.size(1) == 64 && cos_t.sizes() == sin_t.sizes(), "gemm_sk_rope: cos / sin");
  if (tok_seq.has_value()) {
    need(*tok_seq, at::kInt, "tok_seq");
    TORCH_CHECK(tok_seq->numel() >= M, "gemm_sk_rope: tok_seq");
  }
  TORCH_CHECK(ncu >= 8 && ncu <= 1024 && ws.numel() * 4 >= lsa_gemm_sk_ws_bytes((int)ncu) &&
                  tickets.numel() >= lsa_gemm_sk_tickets((int)ncu), "gemm_sk_rope: workspace too small");
  int grid = 0, used = 0;
  check(lsa_gemm_sk_rope(x.data_ptr(), xf ? 0 : (int)x.stride(0), (int)M, (int)K, wf.data_ptr(), (int)N, ws.data_ptr<float>(),
                         tickets.data_ptr<int>(), (int)ncu, (int)min_share, (int)cfg, pos.data_ptr<int>(),
                         ptr<int>(tok_seq), block_tables.data_ptr<int>(), (int)block_tables.size(1),
                         cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), q_out.data_ptr(), kc.data_ptr(),
                         vc.data_ptr(), (int)H, (int)Hkv, (int)xf, &grid, &used, cur_stream()),
        "gemm_sk_rope");
  return (int64_t)grid * 16 + used;
}

void fp8_gemm(const at::Tensor& x, const at::Tensor& wq, const at::Tensor& wscale, int64_t N, at::Tensor& out,
              int64_t epi, int64_t nb, int64_t splitk, int64_t waves, int64_t depth,
              const c10::optional<at::Tensor>& rowss, double eps,
              const c10::optional<at::Tensor>& h, const c10::optional<at::Tensor>& xout, int64_t xmt,
              const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& tickets) {
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(on_dev(wq) && wq.element_size() == 1, "wq must be a 1-byte GPU tensor");
  need(wscale, at::kFloat, "wscale");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(wq.numel() == N * K, "fp8 weight numel mismatch");
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, h, xout, xmt, ss_out, tickets, N / 16);
  lsa_fp8_gemm_knobs((int)waves, (int)depth);
  check(lsa_fp8_gemm_ex(x.data_ptr(), x.stride(0), M, K, wq.data_ptr(), wscale.data_ptr<float>(), N, out.data_ptr(),
                        epi, nb, splitk, 0, eo.on ? &eo.e : nullptr, cur_stream()),
        "fp8_gemm");
}

// MXFP4 weights (kernels/gemm_fp4.hip, ops.pack_mxfp4): wq [N/16, K/128, 64, 16] e2m1 nibbles, sw [N/16, KB4, 64, 4]
// E8M0 block scales (KB4 = ceil(K / 512))
void check_fp4(const at::Tensor& wq, const at::Tensor& sw, int64_t N, int64_t K) {
  TORCH_CHECK(N % 16 == 0 && K % 128 == 0, "mxfp4: N % 16 == 0, K % 128 == 0");
  TORCH_CHECK(on_dev(wq) && wq.element_size() == 1 && wq.is_contiguous() && wq.numel() == N * K / 2,
              "wq must be N*K/2 contiguous e2m1 bytes");
  TORCH_CHECK(on_dev(sw) && sw.element_size() == 1 && sw.is_contiguous() && sw.numel() == (N / 16) * ((K / 128 + 3) / 4) * 256,
              "sw must be the [N/16, ceil(K/512), 64, 4] E8M0 scale bytes");
}

void fp4_gemm(const at::Tensor& x, const at::Tensor& wq, const at::Tensor& sw, int64_t N, at::Tensor& out, int64_t epi,
              int64_t nb, int64_t splitk, int64_t waves, const c10::optional<at::Tensor>& rowss, double eps,
              const c10::optional<at::Tensor>& h, const c10::optional<at::Tensor>& xout, int64_t xmt,
              const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& tickets) {
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 64, "fp4_gemm: decode rows 1..64 (prefill dequantises, fp4_dequant)");
  check_fp4(wq, sw, N, K);
  check_out(epi, out, splitk, M, N, 0);
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, h, xout, xmt, ss_out, tickets, N / 16);
  check(lsa_fp4_gemm_ex(x.data_ptr(), x.stride(0), M, K, wq.data_ptr(), sw.data_ptr(), N, out.data_ptr(), epi, nb, splitk,
                        waves, 0, eo.on ? &eo.e : nullptr, cur_stream()),
        "fp4_gemm");
}

void fp4_gemm_xf(const at::Tensor& xf, int64_t M, int64_t K, const at::Tensor& wq, const at::Tensor& sw, int64_t N,
                 at::Tensor& out, int64_t epi, int64_t nb, int64_t splitk, int64_t waves,
                 const c10::optional<at::Tensor>& rowss, double eps, const c10::optional<at::Tensor>& h,
                 const c10::optional<at::Tensor>& xout, int64_t xmt, const c10::optional<at::Tensor>& ss_out,
                 const c10::optional<at::Tensor>& tickets) {
  need(xf, at::kBFloat16, "xf");
  TORCH_CHECK(M >= 1 && M <= 64, "fp4_gemm_xf: M in 1..64");
  check_fp4(wq, sw, N, K);
  const int64_t mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  TORCH_CHECK(xf.is_contiguous() && xf.numel() >= mt * 16 * K, "xf too small");
  check_out(epi, out, splitk, M, N, mt);
  const EpiOpts eo = epi_opts(epi, M, N, K, rowss, eps, h, xout, xmt, ss_out, tickets, N / 16);
  check(lsa_fp4_gemm_ex(xf.data_ptr(), K, M, K, wq.data_ptr(), sw.data_ptr(), N, out.data_ptr(), epi, nb, splitk, waves,
                        1, eo.on ? &eo.e : nullptr, cur_stream()),
        "fp4_gemm_xf");
}

void fp4_dequant(const at::Tensor& wq, const at::Tensor& sw, int64_t N, int64_t K, at::Tensor& wf) {
  check_fp4(wq, sw, N, K);
  need(wf, at::kBFloat16, "wf");
  TORCH_CHECK(wf.is_contiguous() && wf.numel() >= N * K, "fp4_dequant: output too small");
  check(lsa_fp4_dequant(wq.data_ptr(), sw.data_ptr(), N, K, wf.data_ptr(), cur_stream()), "fp4_dequant");
}

void add_rmsnorm(at::Tensor& h, const c10::optional<at::Tensor>& parts, int64_t nparts, int64_t part_stride,
                 const c10::optional<at::Tensor>& ids, const c10::optional<at::Tensor>& emb,
                 const c10::optional<at::Tensor>& row_idx, bool write_h, const at::Tensor& w, double eps,
                 const c10::optional<at::Tensor>& xn, int64_t rows, int64_t xf_mt, const c10::optional<at::Tensor>& ss_out,
                 int64_t ss_ld, int64_t ss_nzero, const c10::optional<at::Tensor>& x8,
                 const c10::optional<at::Tensor>& sx8) {
  need(h, at::kFloat, "h");
  need(w, at::kBFloat16, "w");
  if (xn.has_value()) need(*xn, at::kBFloat16, "xn");
  if (x8.has_value()) {
    TORCH_CHECK(on_dev(*x8) && x8->element_size() == 1 && x8->numel() >= xf_mt * 16 * w.numel(), "x8 too small");
    TORCH_CHECK(sx8.has_value() && sx8->scalar_type() == at::kFloat && sx8->numel() >= rows, "x8 needs sx8 [rows] f32");
  }
  const int D = w.numel();
  if (ss_out.has_value()) {
    need(*ss_out, at::kLong, "ss_out");
    TORCH_CHECK(ss_out->numel() >= (ss_nzero + 1) * ss_ld && ss_ld >= rows, "ss_out too small");
  }
  check(lsa_add_rmsnorm(h.data_ptr<float>(), ptr<const float>(parts), parts.has_value() ? nparts : 0, part_stride,
                        ptr<const int>(ids), ptr<const void>(emb), ptr<const int>(row_idx), write_h ? 1 : 0,
                        w.data_ptr(), (float)eps, xn.has_value() ? xn->data_ptr() : nullptr, rows, D, xf_mt,
                        ss_out.has_value() ? reinterpret_cast<long long*>(ss_out->data_ptr<int64_t>()) : nullptr, (int)ss_ld,
                        (int)ss_nzero, x8.has_value() ? x8->data_ptr() : nullptr,
                        sx8.has_value() ? sx8->data_ptr<float>() : nullptr, cur_stream()),
        "add_rmsnorm");
}

// y: bf16 [M, 2F] (gate/up interleaved per 16 columns, the vendor prefill GEMM's output) -> out bf16 [M, F]
void silu_bf16(const at::Tensor& y, at::Tensor& out) {
  need(y, at::kBFloat16, "y");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(y.dim() == 2 && y.is_contiguous() && y.size(1) % 32 == 0, "silu_bf16: y [M, 2F] contiguous");
  const int M = y.size(0), F = y.size(1) / 2;
  TORCH_CHECK(out.is_contiguous() && out.numel() >= (int64_t)M * F, "silu_bf16: out too small");
  check(lsa_silu_bf16(y.data_ptr(), M, F, out.data_ptr(), cur_stream()), "silu_bf16");
}

// Infinity-Cache warm-up of up to four tensors (the first bytes[k] bytes of each; -1 = all of it)
void prefetch(const std::vector<at::Tensor>& ts, const std::vector<int64_t>& bytes, int64_t wgs) {
  TORCH_CHECK(!ts.empty() && ts.size() <= 4 && bytes.size() == ts.size(), "prefetch: 1-4 tensors, one byte count each");
  const void* ptrs[4];
  long nb[4];
  for (size_t k = 0; k < ts.size(); ++k) {
    TORCH_CHECK(on_dev(ts[k]) && ts[k].is_contiguous(), "prefetch: contiguous GPU tensors");
    const int64_t all = ts[k].numel() * ts[k].element_size();
    ptrs[k] = ts[k].data_ptr();
    nb[k] = (long)(bytes[k] < 0 || bytes[k] > all ? all : bytes[k]);
  }
  check(lsa_prefetch(ptrs, nb, (int)ts.size(), (int)wgs, cur_stream()), "prefetch");
}

// wide raw residual add of the folded-norm decode step: h += sum parts; xn = bf16(h); ss_out[m] += sum h^2 (Q24)
void res_add_ss(at::Tensor& h, const c10::optional<at::Tensor>& parts, int64_t nparts, int64_t part_stride,
                at::Tensor& xn, int64_t rows, int64_t D, int64_t xf_mt, at::Tensor& ss_out) {
  need(h, at::kFloat, "h");
  need(xn, at::kBFloat16, "xn");
  need(ss_out, at::kLong, "ss_out");
  TORCH_CHECK(rows > 0 && D > 0 && D % 8 == 0, "res_add_ss: bad rows / D");
  TORCH_CHECK(h.is_contiguous() && h.numel() >= rows * D, "res_add_ss: h too small");
  TORCH_CHECK(xn.is_contiguous() && xn.numel() >= (xf_mt > 0 ? xf_mt * 16 : rows) * D, "res_add_ss: xn too small");
  TORCH_CHECK(xf_mt <= 0 || (D % 32 == 0 && rows <= 16 * xf_mt), "res_add_ss: xf tiles");
  TORCH_CHECK(ss_out.is_contiguous() && ss_out.numel() >= rows, "res_add_ss: ss_out too small");
  if (parts.has_value() && nparts > 0) {
    need(*parts, at::kFloat, "parts");
    TORCH_CHECK(part_stride >= rows * D && parts->numel() >= (nparts - 1) * part_stride + rows * D,
                "res_add_ss: parts too small");
  }
  check(lsa_res_add_ss(h.data_ptr<float>(), parts.has_value() && nparts > 0 ? parts->data_ptr<float>() : nullptr,
                       parts.has_value() ? (int)nparts : 0, part_stride, xn.data_ptr(), (int)rows, (int)D,
                       (int)(xf_mt > 0 ? xf_mt : 0), reinterpret_cast<long long*>(ss_out.data_ptr<int64_t>()),
                       cur_stream()),
        "res_add_ss");
}

void rope_append(const at::Tensor& qkv, const at::Tensor& pos, const c10::optional<at::Tensor>& tok_seq,
                 const at::Tensor& block_tables, const at::Tensor& cos_t, const at::Tensor& sin_t, at::Tensor& q_out,
                 at::Tensor& kc, at::Tensor& vc, int64_t H, int64_t Hkv, const c10::optional<at::Tensor>& ks,
                 const c10::optional<at::Tensor>& vs) {
  need(pos, at::kInt, "pos");
  check_cache(kc, vc, ks, vs);
  need(block_tables, at::kInt, "block_tables");
  need(cos_t, at::kFloat, "cos");
  need(sin_t, at::kFloat, "sin");
  need(q_out, at::kBFloat16, "q_out");
  // qkv: bf16 [T, n] or f32 split-K slabs [S, T, n]
  const bool parts = qkv.scalar_type() == at::kFloat;
  TORCH_CHECK(parts || qkv.scalar_type() == at::kBFloat16, "qkv must be bf16 or f32 slabs");
  const int T = parts ? qkv.size(1) : qkv.size(0);
  TORCH_CHECK(qkv.size(qkv.dim() - 1) == (H + 2 * Hkv) * 128 && pos.numel() >= T && q_out.numel() >= (int64_t)T * H * 128,
              "rope_append: qkv [.., T, (H + 2 Hkv) * 128], pos [T], q_out [T, H, 128]");
  TORCH_CHECK(cos_t.size(0) >= block_tables.size(1) * 64 && sin_t.size(0) >= block_tables.size(1) * 64,
              "rope tables have fewer rows than the block tables address (", block_tables.size(1) * 64, ")");
  check(lsa_rope_append(parts ? nullptr : qkv.data_ptr(), parts ? qkv.data_ptr<float>() : nullptr,
                        parts ? qkv.size(0) : 0, parts ? qkv.stride(0) : 0, pos.data_ptr<int>(), ptr<const int>(tok_seq), block_tables.data_ptr<int>(),
                        block_tables.size(1), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), q_out.data_ptr(),
                        kc.data_ptr(), vc.data_ptr(), ptr<float>(ks), ptr<float>(vs), T, H, Hkv, cur_stream()),
        "rope_append");
}

void silu_mul(const at::Tensor& g, const at::Tensor& u, at::Tensor& o) {
  need(g, at::kBFloat16, "g");
  need(u, at::kBFloat16, "u");
  need(o, at::kBFloat16, "o");
  TORCH_CHECK(u.numel() == g.numel() && o.numel() >= g.numel() && g.is_contiguous() && u.is_contiguous() &&
                  o.is_contiguous(), "silu_mul: contiguous g, u of equal size and o at least as large");
  check(lsa_silu_mul(g.data_ptr(), u.data_ptr(), o.data_ptr(), g.numel(), cur_stream()), "silu_mul");
}

extern "C" int lsa_attn_set_stamps(void* p);
void attn_set_stamps(const c10::optional<at::Tensor>& st) {
  if (st.has_value()) TORCH_CHECK(on_dev(*st) && st->element_size() == 8, "stamps: int64 GPU tensor");
  check(lsa_attn_set_stamps(st.has_value() ? st->data_ptr() : nullptr), "attn_set_stamps");
}

// diagnostic stamps of the stream-K prefill GEMM (kernels/gemm_tile256.hip g_sk_stamps): [grid][8] int64, sized by the
// caller for the largest grid it launches (<= 2 x CUs)
extern "C" int lsa_sk_set_stamps(unsigned long long* p);
void sk_set_stamps(const c10::optional<at::Tensor>& st) {
  if (st.has_value()) TORCH_CHECK(on_dev(*st) && st->element_size() == 8 && st->numel() >= 2048 * 8,
                                  "stamps: int64 GPU tensor of >= 2048 x 8");
  check(lsa_sk_set_stamps(st.has_value() ? reinterpret_cast<unsigned long long*>(st->data_ptr()) : nullptr),
        "sk_set_stamps");
}

// diagnostic cycle stamps of the 32-row prefill attention (kernels/attention_prefill32.hip g_p32_stamps): the caller
// sizes the buffer for the plan it launches, [nwork * H * NG * 4][8] int64
extern "C" int lsa_p32_set_stamps(void* p);
void attn_prefill_set_stamps(const c10::optional<at::Tensor>& st) {
  if (st.has_value()) TORCH_CHECK(on_dev(*st) && st->element_size() == 8 && st->is_contiguous(), "stamps: int64 GPU tensor");
  check(lsa_p32_set_stamps(st.has_value() ? st->data_ptr() : nullptr), "attn_prefill_set_stamps");
}

void attn_decode(const at::Tensor& q, const at::Tensor& kc, const at::Tensor& vc, const at::Tensor& block_tables,
                 const at::Tensor& pos, int64_t H, int64_t Hkv, double scale, int64_t chunk_blocks, int64_t nsplit,
                 at::Tensor& out, at::Tensor& opart, at::Tensor& mlpart, at::Tensor& counters, int64_t xf_mt,
                 const c10::optional<at::Tensor>& qkv_parts, const c10::optional<at::Tensor>& cos_t,
                 const c10::optional<at::Tensor>& sin_t, int64_t unsplit_max, const c10::optional<at::Tensor>& ks,
                 const c10::optional<at::Tensor>& vs, const c10::optional<at::Tensor>& out_s8 = c10::nullopt,
                 const c10::optional<at::Tensor>& rowss = c10::nullopt, double eps = 1e-5, int64_t hidden = 0) {
  need(q, at::kBFloat16, "q");
  if (rowss.has_value()) {  // residual-reduce decode step: the slabs are the projection of un-normalised rows
    TORCH_CHECK(qkv_parts.has_value() && hidden > 0, "attn_decode rowss: needs qkv_parts and the hidden size");
    need(*rowss, at::kLong, "rowss");
    TORCH_CHECK(rowss->numel() >= pos.size(0), "attn_decode: rowss too small");
  }
  check_cache(kc, vc, ks, vs);
  need(pos, at::kInt, "pos");
  need(block_tables, at::kInt, "block_tables");
  const int B = pos.size(0);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && block_tables.is_contiguous(),
              "block_tables [>= B, max_blocks]");
  TORCH_CHECK(H > 0 && Hkv > 0 && H % Hkv == 0 && kc.size(1) == Hkv, "heads: H % Hkv == 0, cache has Hkv heads");
  if (out_s8.has_value()) {  // e4m3 output (xf8 layout) + E8M0 per (row, head): the W8A8 / W4A8 o projection's input
    TORCH_CHECK(xf_mt > 0 && on_dev(out) && out.element_size() == 1 && out.numel() >= xf_mt * 16 * H * 128,
                "attn_decode: e4m3 out needs xf_mt and xf_mt * 16 * H * 128 bytes");
    TORCH_CHECK(on_dev(*out_s8) && out_s8->element_size() == 1 && out_s8->numel() >= xf_mt * 64 * H,
                "attn_decode: out_s8 too small");
  } else {
    need(out, at::kBFloat16, "out");
    TORCH_CHECK(out.numel() >= (xf_mt ? xf_mt * 16 : B) * H * 128, "attn_decode out too small");
  }
  need(opart, at::kFloat, "opart");
  need(mlpart, at::kFloat, "mlpart");
  need(counters, at::kInt, "counters");
  TORCH_CHECK(opart.numel() >= (int64_t)B * H * nsplit * 128 && mlpart.numel() >= (int64_t)B * H * nsplit * 2 &&
                  counters.numel() >= (int64_t)B * Hkv,
              "attn_decode workspace too small");
  TORCH_CHECK(opart.numel() * 4 < 0x7fffffffLL, "opart must stay below 2 GiB (buffer descriptor range)");
  if (qkv_parts.has_value()) {  // fused RoPE + KV append from the QKV projection's f32 split-K slabs
    need(*qkv_parts, at::kFloat, "qkv_parts");
    TORCH_CHECK(qkv_parts->dim() == 3 && qkv_parts->size(1) >= B && qkv_parts->size(2) == (H + 2 * Hkv) * 128 &&
                    qkv_parts->stride(1) == qkv_parts->size(2) && qkv_parts->stride(2) == 1,
                "qkv_parts must be [S, B, (H + 2 Hkv) * 128] row-major slabs");
    TORCH_CHECK(cos_t.has_value() && sin_t.has_value(), "fused rope needs cos/sin tables");
    need(*cos_t, at::kFloat, "cos");
    need(*sin_t, at::kFloat, "sin");
    // positions come from the device (no host read); every position the block tables address needs a row
    TORCH_CHECK(cos_t->size(0) >= block_tables.size(1) * 64 && sin_t->size(0) >= block_tables.size(1) * 64,
                "rope tables have fewer rows than the block tables address (", block_tables.size(1) * 64, ")");
  }
  check(lsa_attn_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_tables.data_ptr<int>(),
                        block_tables.size(1), pos.data_ptr<int>(), B, H, Hkv, (float)scale, chunk_blocks, nsplit,
                        (int)unsplit_max, out.data_ptr(), opart.data_ptr<float>(), mlpart.data_ptr<float>(), counters.data_ptr<int>(), xf_mt,
                        ptr<const float>(qkv_parts), qkv_parts.has_value() ? qkv_parts->size(0) : 0,
                        qkv_parts.has_value() ? qkv_parts->stride(0) : 0, ptr<const float>(cos_t),
                        ptr<const float>(sin_t), ptr<const float>(ks), ptr<const float>(vs),
                        out_s8.has_value() ? out_s8->data_ptr() : nullptr,
                        rowss.has_value() ? reinterpret_cast<const long long*>(rowss->data_ptr<int64_t>()) : nullptr,
                        rowss.has_value() ? 1.0f / (float)hidden : 0.f, (float)eps, cur_stream()),
        "attn_decode");
}

// fp8 cache blocks of a prefill batch -> compact bf16 scratch [nseq * mb, Hkv, 64, 128] (kernels/kv8.hip)
void kv8_dequant(const at::Tensor& kc, const at::Tensor& vc, const at::Tensor& ks, const at::Tensor& vs,
                 const at::Tensor& block_tables, const at::Tensor& ctx_lens, int64_t mb, at::Tensor& ko, at::Tensor& vo) {
  check_cache(kc, vc, ks, vs);
  need(block_tables, at::kInt, "block_tables");
  need(ctx_lens, at::kInt, "ctx_lens");
  need(ko, at::kBFloat16, "ko");
  need(vo, at::kBFloat16, "vo");
  const int64_t nseq = ctx_lens.numel(), Hkv = kc.size(1);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= nseq && block_tables.is_contiguous(),
              "block_tables must be a contiguous [nseq, max_blocks] table");
  TORCH_CHECK(mb <= block_tables.size(1), "mb exceeds the block table width");
  TORCH_CHECK(ko.numel() >= nseq * mb * Hkv * 64 * 128 && vo.numel() >= nseq * mb * Hkv * 64 * 128, "kv8 scratch too small");
  check(lsa_kv8_dequant(kc.data_ptr(), vc.data_ptr(), ks.data_ptr<float>(), vs.data_ptr<float>(),
                        block_tables.data_ptr<int>(), block_tables.size(1), ctx_lens.data_ptr<int>(), nseq, Hkv, mb,
                        ko.data_ptr(), vo.data_ptr(), cur_stream()),
        "kv8_dequant");
}

void attn_prefill(const at::Tensor& q, const at::Tensor& kc, const at::Tensor& vc, const at::Tensor& block_tables,
                  const at::Tensor& cu_q, const at::Tensor& ctx_lens, const at::Tensor& work, int64_t H, int64_t Hkv,
                  double scale, at::Tensor& out, int64_t rows32, int64_t xf_mt) {
  need(q, at::kBFloat16, "q");
  need(work, at::kInt, "work");
  need(cu_q, at::kInt, "cu_q");
  need(ctx_lens, at::kInt, "ctx_lens");
  need(block_tables, at::kInt, "block_tables");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(q.dim() == 3 && q.size(1) == H && q.size(2) == 128, "q [T, H, 128]");
  // out: [T, H, 128] row-major, or (xf_mt > 0) a flat buffer in the fragment-major layout of xf_mt 16-row tiles (the
  // o projection's stream-K input)
  TORCH_CHECK(xf_mt >= 0 && (xf_mt ? (out.is_contiguous() && xf_mt * 16 >= q.size(0) && out.numel() >= xf_mt * 16 * H * 128)
                                   : out.sizes() == q.sizes()),
              "attn_prefill: out [T, H, 128], or xf_mt >= T / 16 row tiles of fragment-major rows");
  TORCH_CHECK(cu_q.numel() == ctx_lens.numel() + 1 && block_tables.size(0) >= ctx_lens.numel(),
              "cu_q [nseq + 1], ctx_lens [nseq], block_tables [>= nseq, max_blocks]");
  if (rows32) {  // 32 x 32 MFMA kernel, 128 query rows per work item (kernels/attention_prefill32.hip)
    // work [n_workgroups, 4 * NG] of (seq, q_start, t0, t1) (ops.prefill_plan)
    TORCH_CHECK(rows32 == 1, "attn_prefill: rows32 must be 0 or 1");
    TORCH_CHECK(work.dim() == 2 && (work.size(1) == 4 || work.size(1) == 8) && work.is_contiguous(),
                "attn_prefill32 work must be [n, 4 per group] int32");
    check(lsa_attn_prefill32(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_tables.data_ptr<int>(),
                             block_tables.size(1), cu_q.data_ptr<int>(), ctx_lens.data_ptr<int>(), work.data_ptr<int>(),
                             work.size(0), H, Hkv, (float)scale, out.data_ptr(), (int)(work.size(1) / 4), (int)xf_mt,
                             cur_stream()),
          "attn_prefill32");
    return;
  }
  check(lsa_attn_prefill(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_tables.data_ptr<int>(),
                         block_tables.size(1), cu_q.data_ptr<int>(), ctx_lens.data_ptr<int>(), work.data_ptr<int>(),
                         work.size(0), H, Hkv, (float)scale, out.data_ptr(), (int)xf_mt, cur_stream()),
        "attn_prefill");
}

// decode-state operands of the commit kernels: [B] int32 rows, out_tokens [B, max_new]
void check_state(int64_t B, const at::Tensor& out_tokens, const at::Tensor& gen_len, const at::Tensor& input_ids,
                 const at::Tensor& positions, const at::Tensor& finished, const at::Tensor& eos,
                 const at::Tensor& limit, const at::Tensor& eos_on) {
  for (const at::Tensor* t : {&gen_len, &input_ids, &positions, &finished, &limit, &eos_on}) {
    need(*t, at::kInt, "decode state");
    TORCH_CHECK(t->numel() >= B && t->is_contiguous(), "decode state rows: numel < B");
  }
  need(out_tokens, at::kInt, "out_tokens");
  TORCH_CHECK(out_tokens.dim() == 2 && out_tokens.size(0) >= B && out_tokens.is_contiguous(), "out_tokens [B, max_new]");
  need(eos, at::kInt, "eos");
  TORCH_CHECK(eos.numel() >= 1, "eos: at least one id (-1 = none)");
}

void argmax_commit(const at::Tensor& logits, at::Tensor& part, at::Tensor& out_tokens, at::Tensor& gen_len,
                   at::Tensor& input_ids, at::Tensor& positions, at::Tensor& finished, const at::Tensor& eos,
                   const at::Tensor& limit, const at::Tensor& eos_on) {
  need(logits, at::kFloat, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits: contiguous [B, V]");
  const int B = logits.size(0), V = logits.size(1);
  check_state(B, out_tokens, gen_len, input_ids, positions, finished, eos, limit, eos_on);
  need(part, at::kLong, "part");
  TORCH_CHECK(part.numel() >= (int64_t)B * ((V + 4095) / 4096), "argmax partials too small");
  check(lsa_argmax_commit(logits.data_ptr<float>(), B, V, reinterpret_cast<unsigned long long*>(part.data_ptr()),
                          out_tokens.data_ptr<int>(), out_tokens.size(1), gen_len.data_ptr<int>(),
                          input_ids.data_ptr<int>(), positions.data_ptr<int>(), finished.data_ptr<int>(),
                          eos.data_ptr<int>(), eos.numel(), limit.data_ptr<int>(), eos_on.data_ptr<int>(), cur_stream()),
        "argmax_commit");
}

void sample_commit(at::Tensor& logits, at::Tensor& part, at::Tensor& cand, const c10::optional<at::Tensor>& hist,
                   const c10::optional<at::Tensor>& penalty, const c10::optional<at::Tensor>& last_n,
                   const at::Tensor& temperature, const at::Tensor& top_k,
                   const at::Tensor& top_p, const at::Tensor& seeds, at::Tensor& out_tokens, at::Tensor& gen_len,
                   at::Tensor& input_ids, at::Tensor& positions, at::Tensor& finished, const at::Tensor& eos,
                   const at::Tensor& limit, const at::Tensor& eos_on) {
  need(logits, at::kFloat, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits: contiguous [B, V]");
  const int B = logits.size(0), V = logits.size(1);
  check_state(B, out_tokens, gen_len, input_ids, positions, finished, eos, limit, eos_on);
  need(part, at::kLong, "part");
  need(cand, at::kLong, "cand");
  TORCH_CHECK(part.numel() >= (int64_t)B * ((V + 4095) / 4096) && cand.numel() >= (int64_t)B * ((V + 2047) / 2048) * 64,
              "sampling workspace too small");
  need(temperature, at::kFloat, "temperature");
  need(top_p, at::kFloat, "top_p");
  need(top_k, at::kInt, "top_k");
  need(seeds, at::kLong, "seeds");
  TORCH_CHECK(temperature.numel() >= B && top_p.numel() >= B && top_k.numel() >= B && seeds.numel() >= B,
              "sampling parameters: one per row");
  if (hist.has_value()) {
    need(*hist, at::kInt, "hist");
    TORCH_CHECK(hist->dim() == 2 && hist->size(0) >= B && hist->is_contiguous(), "hist [B, W]");
    TORCH_CHECK(penalty.has_value() && penalty->numel() >= B, "repetition penalty: one per row");
  }
  const int window = hist.has_value() ? hist->size(1) : 0;
  check(lsa_sample_commit(logits.data_ptr<float>(), B, V, reinterpret_cast<unsigned long long*>(part.data_ptr()),
                          reinterpret_cast<unsigned long long*>(cand.data_ptr()), ptr<int>(hist), window,
                          ptr<const float>(penalty), ptr<const int>(last_n), temperature.data_ptr<float>(), top_k.data_ptr<int>(),
                          top_p.data_ptr<float>(), reinterpret_cast<const unsigned long long*>(seeds.data_ptr()),
                          out_tokens.data_ptr<int>(), out_tokens.size(1), gen_len.data_ptr<int>(),
                          input_ids.data_ptr<int>(), positions.data_ptr<int>(), finished.data_ptr<int>(),
                          eos.data_ptr<int>(), eos.numel(), limit.data_ptr<int>(), eos_on.data_ptr<int>(), cur_stream()),
        "sample_commit");
}

// per-token fp8 quantisation of bf16 rows: x8 [M, K] uint8 (e4m3fn bits), sx [M] f32 (amax / 448)
void quant_rows_fp8(const at::Tensor& x, at::Tensor& x8, at::Tensor& sx) {
  need(x, at::kBFloat16, "x");
  need(sx, at::kFloat, "sx");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be a row-major matrix");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(on_dev(x8) && x8.element_size() == 1 && x8.dim() == 2 && x8.size(0) >= M && x8.size(1) >= K &&
                  x8.stride(1) == 1, "x8 must be a row-major [M, K] 1-byte tensor");
  TORCH_CHECK(sx.numel() >= M, "sx too small");
  check(lsa_quant_rows_fp8(x.data_ptr(), x.stride(0), M, K, x8.data_ptr(), x8.stride(0), sx.data_ptr<float>(),
                           cur_stream()),
        "quant_rows_fp8");
}

// W8A8 large-M linear layer on the block-scaled fp8 MFMA (kernels/gemm_fp8_tile.hip)
void fp8_gemm_t256(const at::Tensor& x8, const at::Tensor& sx, const at::Tensor& wq, const at::Tensor& sw, int64_t N,
                   at::Tensor& out, int64_t epi, int64_t splitk) {
  need(sx, at::kFloat, "sx");
  need(sw, at::kFloat, "sw");
  TORCH_CHECK(on_dev(x8) && x8.element_size() == 1 && x8.dim() == 2 && x8.stride(1) == 1, "x8: [M, K] bytes");
  const int M = x8.size(0), K = x8.size(1);
  TORCH_CHECK(on_dev(wq) && wq.element_size() == 1 && wq.numel() == N * K, "wq must be N*K fp8 bytes");
  TORCH_CHECK(sx.numel() >= M && sw.numel() >= N, "scale sizes");
  if (epi == 1) {
    need(out, at::kFloat, "out");
    TORCH_CHECK(out.numel() >= splitk * M * N, "f32 out too small");
  } else {
    need(out, at::kBFloat16, "out");
    TORCH_CHECK(out.numel() >= M * (epi == 2 ? N / 2 : N), "bf16 out too small");
  }
  check(lsa_fp8_gemm_t256(x8.data_ptr(), x8.stride(0), sx.data_ptr<float>(), M, K, wq.data_ptr(), sw.data_ptr<float>(),
                          N, out.data_ptr(), epi, splitk, cur_stream()),
        "fp8_gemm_t256");
}

void fp8_dequant(const at::Tensor& wq, const at::Tensor& wscale, int64_t N, int64_t K, at::Tensor& wf) {
  need(wscale, at::kFloat, "wscale");
  need(wf, at::kBFloat16, "wf");
  TORCH_CHECK(wq.numel() == N * K && wf.numel() >= N * K, "fp8_dequant size mismatch");
  check(lsa_fp8_dequant(wq.data_ptr(), wscale.data_ptr<float>(), N, K, wf.data_ptr(), cur_stream()), "fp8_dequant");
}

// ---- one-shot IPC all-reduce (kernels/allreduce.hip); regions are raw device addresses (int64)
int64_t ar_alloc(int64_t bytes) {
  void* p = nullptr;
  check(lsa_ar_alloc((size_t)bytes, &p), "ar_alloc");
  return reinterpret_cast<int64_t>(p);
}

#ifndef LSA_BINDINGS_SELFTEST
py::bytes ar_handle(int64_t p) {
  char h[64];
  check(lsa_ar_handle(reinterpret_cast<void*>(p), h), "ar_handle");
  return py::bytes(h, 64);
}
#endif

int64_t ar_open(const std::string& h) {
  TORCH_CHECK(h.size() == 64, "IPC handle must be 64 bytes");
  void* p = nullptr;
  check(lsa_ar_open(h.data(), &p), "ar_open");
  return reinterpret_cast<int64_t>(p);
}

void ar_run(at::Tensor& data, const c10::optional<at::Tensor>& out, const at::Tensor& regions, int64_t rank,
            int64_t maxb, int64_t nblocks, int64_t timeout_ticks, at::Tensor& err, int64_t nslab = 1,
            const c10::optional<at::Tensor>& res_h = c10::nullopt, const c10::optional<at::Tensor>& res_xn = c10::nullopt,
            const c10::optional<at::Tensor>& res_ss = c10::nullopt, int64_t res_xmt = 0, int64_t mode = 0) {
  // nslab > 1: data is [nslab, n] split-K slabs; the sum lands in slab 0.  mode: bit 0 bf16 payload, bit 1 two-shot
  // (sums only; the caller sized the regions for the two-shot result area)
  need(data, at::kFloat, "data");
  need(regions, at::kLong, "regions");
  need(err, at::kInt, "err");
  TORCH_CHECK(regions.numel() >= 2 && regions.numel() <= 8 && rank >= 0 && rank < regions.numel(),
              "all-reduce: 2..8 regions and 0 <= rank < world");
  TORCH_CHECK(nslab >= 1 && data.numel() % nslab == 0, "all-reduce: numel must split into nslab slabs");
  const int64_t n = data.numel() / nslab;
  TORCH_CHECK(data.is_contiguous() && n % 4 == 0, "all-reduce data: contiguous, slab numel % 4 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(data.data_ptr()) % 16 == 0, "all-reduce data must be 16-B aligned");
  TORCH_CHECK(n * 4 <= maxb, "all-reduce payload exceeds the registered slot size");
  if (out.has_value()) {
    TORCH_CHECK(nslab == 1, "all-gather takes one slab");
    need(*out, at::kFloat, "out");
    TORCH_CHECK(out->is_contiguous() && out->numel() == n * regions.numel(), "all-gather out size");
  }
  TORCH_CHECK(mode >= 0 && mode <= 3 && (mode == 0 || !out.has_value()), "all-reduce mode: 0..3, sums only");
  int64_t D = 0;
  if (res_h.has_value()) {  // residual epilogue: h [rows, D] f32 += the sum; xn = bf16(h); ss[rows] += sum h^2 (Q24)
    TORCH_CHECK(!out.has_value() && res_xn.has_value() && res_ss.has_value(), "all-reduce residual: h, xn, ss");
    need(*res_h, at::kFloat, "res_h");
    need(*res_xn, at::kBFloat16, "res_xn");
    need(*res_ss, at::kLong, "res_ss");
    TORCH_CHECK(res_h->dim() == 2 && res_h->is_contiguous() && res_h->numel() == n, "all-reduce residual: h [rows, D]");
    D = res_h->size(1);
    const int64_t rows = res_h->size(0);
    TORCH_CHECK(D % 256 == 0, "all-reduce residual: D % 256 == 0");
    TORCH_CHECK(res_ss->numel() >= rows && res_xn->is_contiguous() &&
                    res_xn->numel() >= (res_xmt ? res_xmt * 16 : rows) * D && (!res_xmt || rows <= 16 * res_xmt),
                "all-reduce residual: ss / xn too small");
  }
  check(lsa_ar_run(data.data_ptr<float>(), n, ptr<float>(out), reinterpret_cast<uint8_t* const*>(regions.data_ptr()),
                   rank, regions.numel(), maxb, nblocks, timeout_ticks, err.data_ptr<int>(), nslab, n,
                   res_h.has_value() ? res_h->data_ptr<float>() : nullptr, res_xn.has_value() ? res_xn->data_ptr() : nullptr,
                   res_ss.has_value() ? reinterpret_cast<long long*>(res_ss->data_ptr<int64_t>()) : nullptr, (int)D,
                   (int)res_xmt, (int)mode, cur_stream()),
        "ar_run");
}

// ---------------------------------------------------------------------------------------- latency path (B <= 4)
}  // namespace

#ifndef LSA_BINDINGS_SELFTEST
PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for the MI355X NL->SQL / Spark-error inference engine";
  m.def("gemm", &gemm, py::arg("x"), py::arg("wf"), py::arg("N"), py::arg("out"), py::arg("epi"), py::arg("nb"),
        py::arg("splitk"), py::arg("waves") = 4, py::arg("div") = 4, py::arg("xlds") = 0,
        py::arg("rowss") = py::none(), py::arg("eps") = 1e-5, py::arg("h") = py::none(), py::arg("xout") = py::none(), py::arg("xmt") = 0, py::arg("ss_out") = py::none(), py::arg("tickets") = py::none());
  m.def("gemm_xf", &gemm_xf, py::arg("xf"), py::arg("M"), py::arg("K"), py::arg("wf"), py::arg("N"), py::arg("out"),
        py::arg("epi"), py::arg("nb"), py::arg("splitk"), py::arg("waves") = 4, py::arg("div") = 4,
        py::arg("rowss") = py::none(), py::arg("eps") = 1e-5, py::arg("h") = py::none(), py::arg("xout") = py::none(), py::arg("xmt") = 0, py::arg("ss_out") = py::none(), py::arg("tickets") = py::none());
  m.def("gemm_sk", &gemm_sk, py::arg("x"), py::arg("wf"), py::arg("N"), py::arg("out"), py::arg("epi"), py::arg("ws"),
        py::arg("tickets"), py::arg("ncu"), py::arg("min_share") = 0, py::arg("cfg") = -1, py::arg("xf") = 0,
        py::arg("rows") = 0);
  m.def("gemm_sk_rope", &gemm_sk_rope, py::arg("x"), py::arg("wf"), py::arg("ws"), py::arg("tickets"), py::arg("ncu"),
        py::arg("min_share"), py::arg("cfg"), py::arg("pos"), py::arg("tok_seq"), py::arg("block_tables"),
        py::arg("cos_t"), py::arg("sin_t"), py::arg("q_out"), py::arg("kc"), py::arg("vc"), py::arg("H"), py::arg("Hkv"),
        py::arg("xf") = 0, py::arg("rows") = 0);
  m.def("gemm_sk_epilogue", [](int64_t mode) { lsa_gemm_sk_epilogue((int)mode); });
  m.def("gemm_sk_nbuf", [](int64_t n) { lsa_gemm_sk_nbuf((int)n); });
  m.def("gemm_sk_one_phase", [](int64_t on) { lsa_gemm_sk_one_phase((int)on); });
  m.def("rmsnorm_xf_tile_min", [](int64_t rows) { lsa_rmsnorm_xf_tile_min((int)rows); });
  m.def("gemm_sk_ws_bytes", [](int64_t ncu) { return lsa_gemm_sk_ws_bytes((int)ncu); });
  m.def("gemm_sk_tickets", [](int64_t ncu) { return (int64_t)lsa_gemm_sk_tickets((int)ncu); });
  m.def("fp4_gemm", &fp4_gemm, py::arg("x"), py::arg("wq"), py::arg("sw"), py::arg("N"), py::arg("out"), py::arg("epi"),
        py::arg("nb"), py::arg("splitk"), py::arg("waves") = 4, py::arg("rowss") = py::none(), py::arg("eps") = 1e-5,
        py::arg("h") = py::none(), py::arg("xout") = py::none(), py::arg("xmt") = 0, py::arg("ss_out") = py::none(),
        py::arg("tickets") = py::none());
  m.def("fp4_gemm_xf", &fp4_gemm_xf, py::arg("xf"), py::arg("M"), py::arg("K"), py::arg("wq"), py::arg("sw"),
        py::arg("N"), py::arg("out"), py::arg("epi"), py::arg("nb"), py::arg("splitk"), py::arg("waves") = 4,
        py::arg("rowss") = py::none(), py::arg("eps") = 1e-5, py::arg("h") = py::none(), py::arg("xout") = py::none(),
        py::arg("xmt") = 0, py::arg("ss_out") = py::none(), py::arg("tickets") = py::none());
  m.def("fp4_dequant", &fp4_dequant);
  m.def("fp8_gemm", &fp8_gemm, py::arg("x"), py::arg("wq"), py::arg("wscale"), py::arg("N"), py::arg("out"),
        py::arg("epi"), py::arg("nb"), py::arg("splitk"), py::arg("waves") = 4, py::arg("depth") = 1,
        py::arg("rowss") = py::none(), py::arg("eps") = 1e-5, py::arg("h") = py::none(), py::arg("xout") = py::none(), py::arg("xmt") = 0, py::arg("ss_out") = py::none(), py::arg("tickets") = py::none());
  m.def("fp8_gemm_xf", &fp8_gemm_xf, py::arg("xf"), py::arg("M"), py::arg("K"), py::arg("wq"), py::arg("wscale"),
        py::arg("N"), py::arg("out"), py::arg("epi"), py::arg("nb"), py::arg("splitk"), py::arg("waves") = 4,
        py::arg("depth") = 1,
        py::arg("rowss") = py::none(), py::arg("eps") = 1e-5, py::arg("h") = py::none(), py::arg("xout") = py::none(), py::arg("xmt") = 0, py::arg("ss_out") = py::none(), py::arg("tickets") = py::none());
  m.def("prefetch", &prefetch, py::arg("tensors"), py::arg("bytes"), py::arg("wgs") = 512);
  m.def("res_add_ss", &res_add_ss, py::arg("h"), py::arg("parts"), py::arg("nparts"), py::arg("part_stride"),
        py::arg("xn"), py::arg("rows"), py::arg("D"), py::arg("xf_mt"), py::arg("ss_out"));
  m.def("add_rmsnorm", &add_rmsnorm, py::arg("h"), py::arg("parts"), py::arg("nparts"), py::arg("part_stride"),
        py::arg("ids"), py::arg("emb"), py::arg("row_idx"), py::arg("write_h"), py::arg("w"), py::arg("eps"),
        py::arg("xn"), py::arg("rows"), py::arg("xf_mt") = 0, py::arg("ss_out") = py::none(), py::arg("ss_ld") = 0,
        py::arg("ss_nzero") = 0, py::arg("x8") = py::none(), py::arg("sx8") = py::none());
  m.def("a8_gemm", &a8_gemm, py::arg("x8"), py::arg("s8"), py::arg("sx"), py::arg("M"), py::arg("K"), py::arg("wq"),
        py::arg("wscale"), py::arg("wsc8"), py::arg("N"), py::arg("out"), py::arg("out_s8"), py::arg("epi"), py::arg("nb"),
        py::arg("splitk"), py::arg("waves"), py::arg("depth"), py::arg("xfo"), py::arg("rowss") = py::none(),
        py::arg("eps") = 1e-5);
  m.def("quant_xf8_blocks", &quant_xf8_blocks, py::arg("x"), py::arg("mt"), py::arg("blk"), py::arg("x8"), py::arg("s8"));
  m.def("quant_xf8", &quant_xf8, py::arg("x"), py::arg("mt"), py::arg("x8"), py::arg("sx"));
  m.def("attn_set_stamps", &attn_set_stamps, py::arg("stamps") = py::none());
  m.def("sk_set_stamps", &sk_set_stamps, py::arg("stamps") = py::none());
  m.def("attn_prefill_set_stamps", &attn_prefill_set_stamps, py::arg("stamps") = py::none());
  m.def("rope_append", &rope_append, py::arg("qkv"), py::arg("pos"), py::arg("tok_seq"), py::arg("block_tables"),
        py::arg("cos"), py::arg("sin"), py::arg("q_out"), py::arg("kc"), py::arg("vc"), py::arg("H"), py::arg("Hkv"),
        py::arg("ks") = py::none(), py::arg("vs") = py::none());
  m.def("kv8_dequant", &kv8_dequant);
  m.def("silu_mul", &silu_mul);
  m.def("attn_decode", &attn_decode, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("block_tables"),
        py::arg("pos"), py::arg("H"), py::arg("Hkv"), py::arg("scale"), py::arg("chunk_blocks"), py::arg("nsplit"),
        py::arg("out"), py::arg("opart"), py::arg("mlpart"), py::arg("counters"), py::arg("xf_mt") = 0,
        py::arg("qkv_parts") = py::none(),
        py::arg("cos") = py::none(), py::arg("sin") = py::none(), py::arg("unsplit_max") = 4,
        py::arg("ks") = py::none(), py::arg("vs") = py::none(), py::arg("out_s8") = py::none(),
        py::arg("rowss") = py::none(), py::arg("eps") = 1e-5, py::arg("hidden") = 0);
  m.def("a8_gemm_rr", &a8_gemm_rr, py::arg("h"), py::arg("parts"), py::arg("h_out"), py::arg("wq"), py::arg("wscale"),
        py::arg("wsc8"), py::arg("N"), py::arg("out"), py::arg("out_s8"), py::arg("epi"), py::arg("nb"), py::arg("splitk"),
        py::arg("waves"), py::arg("depth"), py::arg("ss_out") = py::none(), py::arg("eps") = 1e-5);
  m.def("gemm_rr", &gemm_rr, py::arg("h"), py::arg("parts"), py::arg("h_out"), py::arg("wf"), py::arg("N"),
        py::arg("out"), py::arg("epi"), py::arg("nb"), py::arg("splitk"), py::arg("waves"), py::arg("div"),
        py::arg("ss_out") = py::none(), py::arg("eps") = 1e-5);
  m.def("attn_prefill", &attn_prefill, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("block_tables"),
        py::arg("cu_q"), py::arg("ctx_lens"), py::arg("work"), py::arg("H"), py::arg("Hkv"), py::arg("scale"),
        py::arg("out"), py::arg("rows32") = 0, py::arg("xf_mt") = 0);
  m.def("argmax_commit", &argmax_commit);
  m.def("sample_commit", &sample_commit);
  m.def("fp8_dequant", &fp8_dequant);
  m.def("quant_rows_fp8", &quant_rows_fp8);
  m.def("fp8_gemm_t256", &fp8_gemm_t256, py::arg("x8"), py::arg("sx"), py::arg("wq"), py::arg("sw"), py::arg("N"),
        py::arg("out"), py::arg("epi"), py::arg("splitk") = 1);
  m.def("silu_parts", [](const at::Tensor& parts, at::Tensor& out) {
    // parts: f32 [S, M, 2F] (gate/up interleaved per 16 rows) -> out bf16 [M, F] = silu(gate) * up
    need(parts, at::kFloat, "parts");
    need(out, at::kBFloat16, "out");
    const int S = parts.size(0), M = parts.size(1), F = parts.size(2) / 2;
    check(lsa_silu_parts(parts.data_ptr<float>(), S, parts.stride(0), M, F, out.data_ptr(), cur_stream()),
          "silu_parts");
  });
  m.def("silu_bf16", &silu_bf16);
  m.def("ar_alloc", &ar_alloc);
  m.def("ar_free", [](int64_t p) { check(lsa_ar_free(reinterpret_cast<void*>(p)), "ar_free"); });
  m.def("ar_handle", &ar_handle);
  m.def("ar_open", &ar_open);
  m.def("ar_close", [](int64_t p) { check(lsa_ar_close(reinterpret_cast<void*>(p)), "ar_close"); });
  m.def("ar_run", &ar_run, py::arg("data"), py::arg("out"), py::arg("regions"), py::arg("rank"), py::arg("maxb"),
        py::arg("nblocks"), py::arg("timeout_ticks"), py::arg("err"), py::arg("nslab") = 1,
        py::arg("res_h") = py::none(), py::arg("res_xn") = py::none(), py::arg("res_ss") = py::none(),
        py::arg("res_xmt") = 0, py::arg("mode") = 0);
  m.def("ar_wallclock_khz", []() {
    int k = 0;
    check(lsa_ar_wallclock_khz(&k), "ar_wallclock_khz");
    return k;
  });
  m.attr("ar_max_world") = lsa_ar_max_world();
  m.attr("ar_header_bytes") = lsa_ar_header_bytes();
  m.attr("prefill_qblock") = lsa_prefill_qblock();
  m.attr("arch") = "gfx950";
}
#endif  // LSA_BINDINGS_SELFTEST
