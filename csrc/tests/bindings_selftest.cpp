// Host-side self-test of the argument validation in csrc/bindings.cpp, built with AddressSanitizer +
// UndefinedBehaviorSanitizer on the CPU (tests/test_native_sanitizers.py).  bindings.cpp is compiled in its
// LSA_BINDINGS_SELFTEST mode: CPU tensors stand in for device tensors, the lsa_* launchers are stubs that only
// count calls (lsa_stub_calls), there is no Python module.  Every case either passes validation and reaches its
// launcher exactly once, or is rejected with a c10::Error before any launcher runs.
#define LSA_BINDINGS_SELFTEST 1
#include "../bindings.cpp"

#include <cstdio>
#include <functional>
#include <string>

extern "C" int lsa_stub_calls;

namespace {

int failures = 0;

at::Tensor T(std::initializer_list<int64_t> shape, at::ScalarType dt) {
  return at::zeros(at::IntArrayRef(shape), at::TensorOptions().dtype(dt));
}
const auto BF = at::kBFloat16;
const auto F32 = at::kFloat;
const auto I32 = at::kInt;
const auto I64 = at::kLong;
const auto U8 = at::kByte;

void expect_ok(const std::string& name, const std::function<void()>& f) {
  const int before = lsa_stub_calls;
  try {
    f();
  } catch (const c10::Error& e) {
    std::printf("FAIL %s: rejected valid arguments: %s\n", name.c_str(), e.what_without_backtrace());
    ++failures;
    return;
  }
  if (lsa_stub_calls != before + 1) {
    std::printf("FAIL %s: launcher called %d times\n", name.c_str(), lsa_stub_calls - before);
    ++failures;
  }
}

void expect_reject(const std::string& name, const std::function<void()>& f) {
  const int before = lsa_stub_calls;
  try {
    f();
  } catch (const c10::Error&) {
    if (lsa_stub_calls != before) {
      std::printf("FAIL %s: launcher ran before the rejection\n", name.c_str());
      ++failures;
    }
    return;
  }
  std::printf("FAIL %s: invalid arguments accepted\n", name.c_str());
  ++failures;
}

const c10::optional<at::Tensor> none = c10::nullopt;

}  // namespace

int main() {
  // ---- decode / prefill GEMMs
  {
    auto x = T({4, 64}, BF), wf = T({128 * 64}, BF), out = T({4, 128}, BF);
    expect_ok("gemm bf16", [&] { gemm(x, wf, 128, out, 0, 1, 1, 4, 4, 0, none, 1e-5, none, none, 0, none, none); });
    auto o32 = T({2, 4, 128}, F32);
    expect_ok("gemm f32 split-K", [&] { gemm(x, wf, 128, o32, 1, 1, 2, 4, 4, 0, none, 1e-5, none, none, 0, none, none); });
    auto bad_w = T({127 * 64}, BF);
    expect_reject("gemm weight numel", [&] { gemm(x, bad_w, 128, out, 0, 1, 1, 4, 4, 0, none, 1e-5, none, none, 0, none, none); });
    auto small = T({4, 64}, BF);
    expect_reject("gemm out too small", [&] { gemm(x, wf, 128, small, 0, 1, 1, 4, 4, 0, none, 1e-5, none, none, 0, none, none); });
    expect_reject("gemm split-K slabs too small", [&] { gemm(x, wf, 128, o32, 1, 1, 4, 4, 4, 0, none, 1e-5, none, none, 0, none, none); });
    expect_reject("gemm residual without h", [&] { gemm(x, wf, 128, out, 3, 1, 1, 4, 4, 0, none, 1e-5, none, none, 0, none, none); });
    auto h = T({4, 128}, F32), xo = T({4, 128}, BF), ss = T({4}, I64), tk = T({8}, I32);
    expect_ok("gemm residual", [&] { gemm(x, wf, 128, out, 3, 1, 1, 4, 4, 0, none, 1e-5, h, xo, 0, ss, tk); });
    auto ss_small = T({2}, I64);
    expect_reject("gemm residual ss too small", [&] { gemm(x, wf, 128, out, 3, 1, 1, 4, 4, 0, none, 1e-5, h, xo, 0, ss_small, tk); });
    auto rowss = T({4}, I64);
    expect_ok("gemm rownorm", [&] { gemm(x, wf, 128, o32, 1, 1, 2, 4, 4, 0, rowss, 1e-5, none, none, 0, none, none); });
    auto rowss_f = T({4}, F32);
    expect_reject("gemm rownorm dtype", [&] { gemm(x, wf, 128, o32, 1, 1, 2, 4, 4, 0, rowss_f, 1e-5, none, none, 0, none, none); });
  }
  {
    auto xf = T({2 * 16 * 64}, BF), wf = T({128 * 64}, BF), o = T({2, 20, 128}, F32);
    expect_ok("gemm_xf", [&] { gemm_xf(xf, 20, 64, wf, 128, o, 1, 2, 2, 4, 4, none, 1e-5, none, none, 0, none, none); });
    auto xs = T({16 * 64}, BF);
    expect_reject("gemm_xf xf too small", [&] { gemm_xf(xs, 20, 64, wf, 128, o, 1, 2, 2, 4, 4, none, 1e-5, none, none, 0, none, none); });
    expect_reject("gemm_xf M > 64", [&] { gemm_xf(xf, 65, 64, wf, 128, o, 1, 2, 2, 4, 4, none, 1e-5, none, none, 0, none, none); });
    expect_reject("gemm_xf K % 32", [&] { gemm_xf(xf, 20, 48, wf, 128, o, 1, 2, 2, 4, 4, none, 1e-5, none, none, 0, none, none); });
  }
  {
    auto xf = T({16 * 128}, BF), wq = T({64 * 128}, U8), sc = T({64}, F32), o = T({1, 4, 64}, F32);
    expect_ok("fp8_gemm_xf", [&] { fp8_gemm_xf(xf, 4, 128, wq, sc, 64, o, 1, 1, 1, 4, 1, none, 1e-5, none, none, 0, none, none); });
    auto wq_bad = T({64 * 127}, U8);
    expect_reject("fp8_gemm_xf wq numel", [&] { fp8_gemm_xf(xf, 4, 128, wq_bad, sc, 64, o, 1, 1, 1, 4, 1, none, 1e-5, none, none, 0, none, none); });
    auto x8 = T({16 * 128}, U8), sx = T({4}, F32), s8 = T({64}, U8);
    expect_ok("a8_gemm", [&] { a8_gemm(x8, none, sx, 4, 128, wq, sc, none, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    expect_ok("a8_gemm block scales", [&] { a8_gemm(x8, s8, none, 4, 128, wq, sc, none, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    expect_reject("a8_gemm K % 128", [&] { a8_gemm(x8, none, sx, 4, 64, wq, sc, none, 128, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    auto sx_small = T({2}, F32);
    expect_reject("a8_gemm sx too small", [&] { a8_gemm(x8, none, sx_small, 4, 128, wq, sc, none, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    expect_reject("a8_gemm no activation scales", [&] { a8_gemm(x8, none, none, 4, 128, wq, sc, none, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    auto s8_small = T({32}, U8);
    expect_reject("a8_gemm s8 too small", [&] { a8_gemm(x8, s8_small, none, 4, 128, wq, sc, none, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    // MXFP4 weights: N * K / 2 bytes + E8M0 words [N/16][ceil(K/512)][64]
    auto w4 = T({64 * 64}, U8), sw4 = T({4 * 64 * 4}, U8);
    expect_ok("a8_gemm mxfp4", [&] { a8_gemm(x8, s8, none, 4, 128, w4, none, sw4, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    expect_reject("a8_gemm both weight scales", [&] { a8_gemm(x8, s8, none, 4, 128, w4, sc, sw4, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    auto sw4_small = T({64}, U8);
    expect_reject("a8_gemm mxfp4 scales", [&] { a8_gemm(x8, s8, none, 4, 128, w4, none, sw4_small, 64, o, none, 1, 1, 1, 4, 1, 1, none, 1e-5); });
    // e4m3 SiLU output: N / 2 % 128 == 0 bytes out + block scales
    auto wq2 = T({256 * 128}, U8), sc2 = T({256}, F32), o8 = T({16 * 128}, U8), os8 = T({64}, U8);
    expect_ok("a8_gemm silu e4m3", [&] { a8_gemm(x8, s8, none, 4, 128, wq2, sc2, none, 256, o8, os8, 2, 4, 1, 4, 1, 2, none, 1e-5); });
    expect_reject("a8_gemm silu e4m3 no scales", [&] { a8_gemm(x8, s8, none, 4, 128, wq2, sc2, none, 256, o8, none, 2, 4, 1, 4, 1, 2, none, 1e-5); });
    auto x = T({300, 128}, BF), xq = T({300, 128}, U8), sxq = T({300}, F32);
    expect_ok("quant_rows_fp8", [&] { quant_rows_fp8(x, xq, sxq); });
    auto xq_small = T({200, 128}, U8);
    expect_reject("quant_rows_fp8 x8 too small", [&] { quant_rows_fp8(x, xq_small, sxq); });
    auto o2 = T({300, 64}, F32), sw = T({64}, F32);
    // stream-K prefill GEMM: workspace of lsa_gemm_sk_ws_bytes(ncu) / tickets(ncu)
    auto wsk = T({2 * 8 * 65536}, F32), tks = T({32}, I32), ob = T({300, 64}, BF), wsb = T({64 * 128}, BF);
    expect_ok("gemm_sk", [&] { gemm_sk(x, wsb, 64, ob, 0, wsk, tks, 8, 0, -1, 0, 0); });
    auto wsk_small = T({65536}, F32);
    expect_reject("gemm_sk workspace", [&] { gemm_sk(x, wsb, 64, ob, 0, wsk_small, tks, 8, 0, -1, 0, 0); });
    expect_reject("gemm_sk residual dtype", [&] { gemm_sk(x, wsb, 64, ob, 3, wsk, tks, 8, 0, -1, 0, 0); });
    auto hs = T({300, 64}, F32), hs_small = T({299, 64}, F32);
    expect_ok("gemm_sk residual", [&] { gemm_sk(x, wsb, 64, hs, 3, wsk, tks, 8, 0, -1, 0, 0); });
    expect_reject("gemm_sk residual too small", [&] { gemm_sk(x, wsb, 64, hs_small, 3, wsk, tks, 8, 0, -1, 0, 0); });
    // fragment-major X (a flat buffer of ceil(300 / 16) * 16 rows) and SiLU output
    auto xfr = T({304 * 128}, BF), xf_small = T({300 * 128}, BF), of = T({304 * 32}, BF);
    expect_ok("gemm_sk fragment-major x", [&] { gemm_sk(xfr, wsb, 64, ob, 0, wsk, tks, 8, 0, -1, 1, 300); });
    expect_reject("gemm_sk fragment-major x too small", [&] { gemm_sk(xf_small, wsb, 64, ob, 0, wsk, tks, 8, 0, -1, 1, 300); });
    expect_reject("gemm_sk fragment-major x without rows", [&] { gemm_sk(xfr, wsb, 64, ob, 0, wsk, tks, 8, 0, -1, 1, 0); });
    expect_ok("gemm_sk fragment-major silu", [&] { gemm_sk(xfr, wsb, 64, of, 2, wsk, tks, 8, 0, -1, 3, 300); });
    expect_reject("gemm_sk fragment-major bf16 out", [&] { gemm_sk(x, wsb, 64, ob, 0, wsk, tks, 8, 0, -1, 2, 0); });
    expect_ok("fp8_gemm_t256", [&] { fp8_gemm_t256(xq, sxq, wq, sw, 64, o2, 1, 1); });
    auto sw_small = T({32}, F32);
    expect_reject("fp8_gemm_t256 weight scales", [&] { fp8_gemm_t256(xq, sxq, wq, sw_small, 64, o2, 1, 1); });
  }
  // ---- normalisation, elementwise
  {
    auto h = T({4, 256}, F32), w = T({256}, BF), xn = T({4, 256}, BF), ss = T({3 * 4}, I64);
    expect_ok("add_rmsnorm", [&] { add_rmsnorm(h, none, 0, 0, none, none, none, true, w, 1e-5, xn, 4, 0, ss, 4, 2, none, none); });
    expect_reject("add_rmsnorm ss too small", [&] { add_rmsnorm(h, none, 0, 0, none, none, none, true, w, 1e-5, xn, 4, 0, ss, 4, 3, none, none); });
    auto x8 = T({8}, U8), sx8 = T({4}, F32);
    expect_reject("add_rmsnorm x8 too small", [&] { add_rmsnorm(h, none, 0, 0, none, none, none, true, w, 1e-5, xn, 4, 1, none, 0, 0, x8, sx8); });
    auto hr = T({4, 1024}, F32), pr = T({2, 4, 1024}, F32), xr = T({4, 1024}, BF), ss1 = T({4}, I64);
    auto ss_small = T({3}, I64), xr_small = T({3, 1024}, BF);
    expect_ok("res_add_ss", [&] { res_add_ss(hr, pr, 2, 4 * 1024, xr, 4, 1024, 0, ss1); });
    expect_reject("res_add_ss ss too small", [&] { res_add_ss(hr, pr, 2, 4 * 1024, xr, 4, 1024, 0, ss_small); });
    expect_reject("res_add_ss xn too small", [&] { res_add_ss(hr, pr, 2, 4 * 1024, xr_small, 4, 1024, 0, ss1); });
    expect_reject("res_add_ss parts too small", [&] { res_add_ss(hr, pr, 3, 4 * 1024, xr, 4, 1024, 0, ss1); });
    auto g = T({1000}, BF), u = T({1000}, BF), o = T({1000}, BF), us = T({999}, BF);
    expect_ok("silu_mul", [&] { silu_mul(g, u, o); });
    {
      auto y = T({4, 64}, BF), so = T({4, 32}, BF), small = T({4, 31}, BF), bad = T({4, 48}, BF);
      expect_ok("silu_bf16", [&] { silu_bf16(y, so); });
      expect_reject("silu_bf16 out too small", [&] { silu_bf16(y, small); });
      expect_reject("silu_bf16 width not a multiple of 32", [&] { silu_bf16(bad, so); });
      auto a = T({1024}, F32), b = T({64}, BF);
      expect_ok("prefetch", [&] { prefetch({a, b}, {-1, 64}, 256); });
      expect_reject("prefetch 5 tensors", [&] { prefetch({a, a, a, a, a}, {-1, -1, -1, -1, -1}, 256); });
      expect_reject("prefetch byte counts", [&] { prefetch({a, b}, {-1}, 256); });
    }
    expect_reject("silu_mul size mismatch", [&] { silu_mul(g, us, o); });
  }
  // ---- attention
  {
    const int64_t B = 2, H = 8, Hkv = 2, nblk = 6, mb = 3;
    auto kc = T({nblk, Hkv, 64, 128}, BF), vc = T({nblk, Hkv, 64, 128}, BF);
    auto bt = T({B, mb}, I32), pos = T({B}, I32), q = T({B, H, 128}, BF), out = T({B, H, 128}, BF);
    auto op = T({B * H * 4 * 128}, F32), ml = T({B * H * 4 * 2}, F32), ctr = T({B * Hkv}, I32);
    expect_ok("attn_decode", [&] { attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml, ctr, 0, none, none, none, 4, none, none); });
    auto ml_small = T({B * H * 4}, F32);
    expect_reject("attn_decode workspace", [&] { attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml_small, ctr, 0, none, none, none, 4, none, none); });
    expect_reject("attn_decode heads", [&] { attn_decode(q, kc, vc, bt, pos, H, 3, 0.08, 2, 4, out, op, ml, ctr, 0, none, none, none, 4, none, none); });
    auto parts = T({2, B, (H + 2 * Hkv) * 128}, F32), cs = T({mb * 64, 64}, F32), cs_short = T({mb * 64 - 1, 64}, F32);
    expect_ok("attn_decode fused rope", [&] { attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml, ctr, 0, parts, cs, cs, 4, none, none); });
    expect_reject("attn_decode rope table", [&] { attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml, ctr, 0, parts, cs_short, cs, 4, none, none); });
    auto parts_bad = T({2, B, (H + Hkv) * 128}, F32);
    expect_reject("attn_decode qkv slabs", [&] { attn_decode(q, kc, vc, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml, ctr, 0, parts_bad, cs, cs, 4, none, none); });
    auto k8 = T({nblk, Hkv, 64, 128}, U8), v8 = T({nblk, Hkv, 64, 128}, U8), ks = T({nblk, Hkv, 64}, F32);
    expect_ok("attn_decode fp8 cache", [&] { attn_decode(q, k8, v8, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml, ctr, 0, none, none, none, 4, ks, ks); });
    expect_reject("attn_decode fp8 cache without V scales", [&] { attn_decode(q, k8, v8, bt, pos, H, Hkv, 0.08, 2, 4, out, op, ml, ctr, 0, none, none, none, 4, ks, none); });
    auto ctx = T({B}, I32), ko = T({B * mb, Hkv, 64, 128}, BF);
    expect_ok("kv8_dequant", [&] { kv8_dequant(k8, v8, ks, ks, bt, ctx, mb, ko, ko); });
    expect_reject("kv8_dequant mb", [&] { kv8_dequant(k8, v8, ks, ks, bt, ctx, mb + 1, ko, ko); });
    // prefill: 2 sequences of 70 and 30 tokens
    auto qp = T({100, H, 128}, BF), outp = T({100, H, 128}, BF), cu = T({B + 1}, I32), work = T({2, 4}, I32);
    expect_ok("attn_prefill32", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work, H, Hkv, 0.08, outp, 1, 0); });
    auto work_bad = T({2, 5}, I32), work8 = T({2, 8}, I32);
    expect_ok("attn_prefill32 paired", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work8, H, Hkv, 0.08, outp, 1, 0); });
    expect_reject("attn_prefill removed split mode", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work8, H, Hkv, 0.08, outp, 3, 0); });
    expect_reject("attn_prefill32 work", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work_bad, H, Hkv, 0.08, outp, 1, 0); });
    auto cu_bad = T({B}, I32);
    expect_reject("attn_prefill offsets", [&] { attn_prefill(qp, kc, vc, bt, cu_bad, ctx, work, H, Hkv, 0.08, outp, 1, 0); });
    expect_reject("attn_prefill rows32 mode", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work, H, Hkv, 0.08, outp, 2, 0); });
    auto outf = T({112 * H * 128}, BF);  // fragment-major output: ceil(100 / 16) = 7 row tiles
    expect_ok("attn_prefill32 fragment-major out", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work, H, Hkv, 0.08, outf, 1, 7); });
    expect_reject("attn_prefill fragment-major tiles", [&] { attn_prefill(qp, kc, vc, bt, cu, ctx, work, H, Hkv, 0.08, outf, 1, 6); });
    auto qkv = T({100, (H + 2 * Hkv) * 128}, BF), tpos = T({100}, I32), tseq = T({100}, I32), qo = T({100, H, 128}, BF);
    expect_ok("rope_append", [&] { rope_append(qkv, tpos, tseq, bt, cs, cs, qo, kc, vc, H, Hkv, none, none); });
    auto qo_small = T({99, H, 128}, BF);
    expect_reject("rope_append q_out", [&] { rope_append(qkv, tpos, tseq, bt, cs, cs, qo_small, kc, vc, H, Hkv, none, none); });
  }
  // ---- sampling / decode state
  {
    const int64_t B = 3, V = 5000;
    auto lg = T({B, V}, F32), part = T({B * 2}, I64), cand = T({B * 3 * 64}, I64);
    auto ot = T({B, 16}, I32), gl = T({B}, I32), ii = T({B}, I32), ps = T({B}, I32), fin = T({B}, I32);
    auto eos = T({1}, I32), lim = T({B}, I32), eon = T({B}, I32);
    expect_ok("argmax_commit", [&] { argmax_commit(lg, part, ot, gl, ii, ps, fin, eos, lim, eon); });
    auto fin_small = T({B - 1}, I32);
    expect_reject("argmax_commit state rows", [&] { argmax_commit(lg, part, ot, gl, ii, ps, fin_small, eos, lim, eon); });
    auto part_small = T({B}, I64);
    expect_reject("argmax_commit partials", [&] { argmax_commit(lg, part_small, ot, gl, ii, ps, fin, eos, lim, eon); });
    auto temp = T({B}, F32), topk = T({B}, I32), topp = T({B}, F32), seeds = T({B}, I64), hist = T({B, 64}, I32);
    auto pen = T({B}, F32), lastn = T({B}, I32);
    expect_ok("sample_commit", [&] { sample_commit(lg, part, cand, hist, pen, lastn, temp, topk, topp, seeds, ot, gl, ii, ps, fin, eos, lim, eon); });
    auto seeds32 = T({B}, I32);
    expect_reject("sample_commit seeds dtype", [&] { sample_commit(lg, part, cand, hist, pen, lastn, temp, topk, topp, seeds32, ot, gl, ii, ps, fin, eos, lim, eon); });
    expect_reject("sample_commit penalty missing", [&] { sample_commit(lg, part, cand, hist, none, lastn, temp, topk, topp, seeds, ot, gl, ii, ps, fin, eos, lim, eon); });
  }
  // ---- one-shot all-reduce
  {
    auto data = T({4096}, F32), regions = T({2}, I64), err = T({1}, I32);
    expect_ok("ar_run", [&] { ar_run(data, none, regions, 0, 1 << 20, 64, 1000, err, 1); });
    expect_reject("ar_run payload > slot", [&] { ar_run(data, none, regions, 0, 1024, 64, 1000, err, 1); });
    expect_reject("ar_run rank", [&] { ar_run(data, none, regions, 2, 1 << 20, 64, 1000, err, 1); });
    auto unaligned = T({4097}, F32).narrow(0, 1, 4096);
    expect_reject("ar_run unaligned", [&] { ar_run(unaligned, none, regions, 0, 1 << 20, 64, 1000, err, 1); });
    auto gout = T({8191}, F32);
    expect_reject("ar_run gather out", [&] { ar_run(data, gout, regions, 0, 1 << 20, 64, 1000, err, 1); });
    auto slabs = T({3, 4096}, F32);
    expect_ok("ar_run slabs", [&] { ar_run(slabs, none, regions, 1, 1 << 20, 64, 1000, err, 3); });
    expect_ok("ar_run bf16 two-shot", [&] { ar_run(slabs, none, regions, 1, 1 << 20, 64, 1000, err, 3, none, none, none, 0, 3); });
    auto gout2 = T({8192}, F32);
    expect_reject("ar_run gather mode", [&] { ar_run(data, gout2, regions, 0, 1 << 20, 64, 1000, err, 1, none, none, none, 0, 1); });
    expect_reject("ar_run mode range", [&] { ar_run(data, none, regions, 0, 1 << 20, 64, 1000, err, 1, none, none, none, 0, 4); });
  }
  if (failures) {
    std::printf("bindings selftest: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("bindings selftest ok (%d launches)\n", lsa_stub_calls);
  return 0;
}
