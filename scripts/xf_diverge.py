"""Diagnostic: record every prefill op's output (fragment-major outputs converted back to rows) with
ops.PREFILL_XF off and on, and print the first op whose outputs differ, plus run-to-run determinism of each mode."""
import sys

import torch

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import ModelRunner  # noqa: E402
from llm_based_apache_spark_optimization_amd.models import get_spec  # noqa: E402
from llm_based_apache_spark_optimization_amd.models.llama import init_random  # noqa: E402

rec = []


def wrap(name, outsel):
    f = getattr(ops, name)

    def g(*a, **k):
        r = f(*a, **k)
        torch.cuda.synchronize()
        rec.append((name, outsel(a, k, r)))
        return r
    setattr(ops, name, g)


def rows_of(t, k, ncol):
    T = k.get("rows")
    if T is not None:
        return ops.from_xfrag(t, T, ncol).float().cpu().clone()
    return t.float().cpu().clone()


wrap("add_rmsnorm", lambda a, k, r: ("h", a[0].float().cpu().clone()))
wrap("linear_res", lambda a, k, r: ("h", a[2].float().cpu().clone()))
wrap("linear_sk", lambda a, k, r: ("out", rows_of(a[3], {"rows": k.get("rows")} if k.get("xf_out") else {}, a[1].N // 2)
                                    if a[2] == "silu" else a[3].float().cpu().clone()))
wrap("rope_append", lambda a, k, r: ("q", a[6].float().cpu().clone()))
wrap("linear", lambda a, k, r: ("y", r.float().cpu().clone()))


def _attn_rec(a, k, r):
    q, kc, vc, bt, cu, ctx, H, Hkv, scale, out = a[:10]
    T = q.shape[0]
    got = ops.from_xfrag(out, T, H * 128) if k.get("xf") else out.reshape(T, -1)
    want = torch.empty_like(q)
    ops.ref.attn_prefill(q, kc, vc, bt, cu, ctx, H, Hkv, scale, want, k.get("kv_scales"))
    want = want.reshape(T, -1).float()
    g = got.float()
    err = ((g - want).norm(dim=1) / want.norm(dim=1).clamp_min(1e-6))
    bad = (err > 1e-2).nonzero().flatten().tolist()
    print("  attn T", T, "cu", cu.tolist(), "ctx", ctx.tolist(), "bt", tuple(bt.shape), "rel err max", float(err.max()),
          "bad rows", len(bad), bad[:8], bad[-8:], flush=True)
    return ("o", g.cpu().clone())


wrap("attn_prefill", _attn_rec)

name = sys.argv[1] if len(sys.argv) > 1 else "tiny-llama3"
spec = get_spec(name)
dev = torch.device("cuda:0")
torch.manual_seed(0)
w = init_random(spec, dev, seed=0, std=0.08)
runs = {}
for tag, xf in (("rm1", False), ("rm2", False), ("xf1", True), ("xf2", True)):
    ops.PREFILL_XF = xf
    rec.clear()
    r = ModelRunner(w, max_slots=2, max_model_len=512)
    if tag.endswith("2"):  # a poisoned cache: a read of a never-written slot shows up as NaN
        r.kv.fill_(float("nan"))
    r.set_slot(0, [1, 2, 3, 4], 4)
    r.set_slot(1, [5, 6], 4)
    r.prefill([(0, [1] + list(range(7, 200)), 0), (1, [1] + list(range(300, 399)), 0)])
    runs[tag] = (list(rec), r.logits_l[:2].float().cpu())
for a, b in (("rm1", "rm2"), ("xf1", "xf2"), ("rm1", "xf1")):
    ra, rb = runs[a][0], runs[b][0]
    print(a, b, "ops", len(ra), len(rb), "logits equal", torch.equal(runs[a][1], runs[b][1]),
          float((runs[a][1] - runs[b][1]).abs().max()))
    for i, ((na, (ka, ta)), (nb, (kb, tb))) in enumerate(zip(ra, rb)):
        if na != nb or ta.shape != tb.shape or not torch.equal(ta, tb):
            d = float((ta - tb).abs().max()) if ta.shape == tb.shape else None
            print("  first divergence at op", i, na, nb, ka, tuple(ta.shape), tuple(tb.shape), "maxdiff", d)
            break
