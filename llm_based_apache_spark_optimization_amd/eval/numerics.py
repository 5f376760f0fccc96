"""Teacher-forced numerics check of the engine's DECODE path against the plain fp32 PyTorch forward.

The engine decodes a batch greedily with its captured graphs; the logits of every step (the decode kernels'
own lm_head output, rows of the batch bucket the benchmark times) are recorded.  The oracle
(``models.llama.reference_forward``) is then fed each sequence's prompt plus the engine's own tokens
(teacher forcing), so position j of both predicts the same token j.  Per position:

* KL(oracle || engine) of the two next-token distributions (nats),
* top-1 agreement (argmax of the engine's logits vs the oracle's),
* top-5 overlap (|top5(engine) n top5(oracle)| / 5).

Statistics are taken over >= 64 positions per checked sequence.  fp8 models are compared with an oracle that
emulates the engine's quantisation (its dequantised weights, the same per-token e4m3 activation rounding for
W8A8 GEMMs, the e4m3 KV rows of an fp8 cache), so the thresholds measure kernels and layouts, not the
quantiser -- and a wrong scale or a scrambled cache layout moves the distributions far past them
(tests/test_numerics_gpu.py injects both and requires the check to fail).
"""
from __future__ import annotations

import contextlib
from typing import Optional, Sequence

import torch

# (mean KL nats PER LAYER, top-5 overlap, top-1 agreement) a healthy engine stays within, per numerics class;
# the KL bound is n_layers x the first entry.  Calibrated on MI355X (profiles/numerics_calibration_mi355x.jsonl,
# scripts/numerics_calibrate.py: duckdb-nsql-7B shape, random init, 4 and 32 layers, batch 4 and 32):
#
#   class   healthy KL / layer      one layer's scale x1.25: KL / layer   swapped cached keys: KL / layer
#   bf16    1.6e-5 .. 2.6e-5         4.8e-3 .. 5.3e-3                      1.9e-2 .. 5.9e-2
#   w8a16   2.8e-4 .. 7.2e-4         5.3e-3 .. 5.6e-3                      2.6e-2 .. 5.7e-2
#   w8a8    4.6e-4 .. 2.1e-3         5.6e-3 .. 6.7e-3                      1.9e-2 .. 7.8e-2
#
# Both the healthy noise and a fault's KL grow ~linearly with depth, so the bound scales with n_layers.  The fp8
# classes' healthy noise is dominated by per-token e4m3 activation rounding that the oracle emulates but cannot
# reproduce bit-exactly (a bf16-level difference flips a rounding: one e4m3 ulp, ~6 %), compounded over a
# random-init network; the fp8 bounds sit 1.6-2.8x above the worst healthy row and 1.6-2.7x below the scale
# fault (bf16: ~10x above, ~19x below).
# Top-5 / top-1 floors are gross-failure guards (at 32 random layers healthy fp8 top-1 is only ~0.4-0.7).
#   w4a8    1.6e-3 .. 3.3e-3         1.2e-2 .. 1.8e-2 (E8M0 fault)         1.7e-2 .. 4.9e-2
# w4a8 = MXFP4 weights with e4m3 activations on the W4A8 projections (ModelRunner.a8_plan): the oracle multiplies
# the dequantised e2m1 weights, so the healthy noise is the activation rounding of every W4A8 input (qkv / gate_up
# per row, o / down per 32-block up to 16 rows); its scale fault is every 8th E8M0 block scale of one layer's down
# projection one binade up (e8m0_fault).  Calibrated in round 4 (profiles/r4/numerics_calibration_w4a8_mi355x.jsonl):
# the bound sits 1.8x above the worst healthy row and 2x below the weakest fault.  w4a8 gates on the mean KL and
# the top-5 overlap only (top-1 is reported): its healthy top-1 sits at 0.3-0.4 on a 32-layer random-init network
# and moves by +-0.05 with the summation order of an equally exact kernel (round 6: the batch-1 residual-reduce
# step's 0.344 vs 0.391, at KL 0.126 vs 0.105 under a 0.192 bound), while the E8M0 fault's KL alone is 2x the bound.
THRESHOLDS = {
    "bf16": (2.5e-4, 0.85, 0.8),
    "w8a16": (2.0e-3, 0.5, 0.4),
    "w8a8": (3.5e-3, 0.4, 0.3),
    "w4a8": (6.0e-3, 0.35, None),
}

# Tied-embedding models (Llama-3.2-3B: lm_head = the embedding table).  With random-init weights the final hidden
# state is dominated by the current token's own embedding row (std 1.0 vs 0.02 for the layers), so the TIED head's
# logits put the input token ~400 logits above every other: KL ~ 0 and top-1 = 1 whatever the layers compute (round
# 3 reported KL 0.0 for every 3B check).  For these models the statistic is taken over what a fault actually moves:
# the final normalised hidden state x (what the lm_head reads), through an UNTIED seeded random probe head
# P [PROBE_V, d] ~ N(0, PROBE_SCALE^2 / d) -- probe logits ~ N(0, PROBE_SCALE^2), a spread distribution whose
# KL(oracle||engine) ~ PROBE_SCALE^2 / 2 x the relative error of x squared -- plus the per-position relative L2
# error of x itself.  Bounds per class: (mean probe KL PER LAYER, mean relative error / sqrt(n_layers)) -- healthy
# probe KL grows ~linearly with depth, the relative error ~ as its square root.  Calibrated on MI355X at the
# Llama-3.2-3B shape (GQA 3:1, tied), 4 and 28 layers, batch 1 and 4 (profiles/r4/numerics_calibration_tied_mi355x.jsonl,
# scripts/numerics_calibrate.py --tied):
#
#   class   healthy KL / layer, rel / sqrt(L)    scale x1.25: KL / layer, rel / sqrt(L)   swapped keys
#   bf16    8.5e-5 .. 9.6e-5, 0.0035 .. 0.0038   2.5e-2 .. 4.2e-2, 0.064 .. 0.075         6.9e-2 .., 0.10 ..
#   w8a16   9.9e-4 .. 2.2e-3, 0.011 .. 0.018     2.8e-2 .. 4.5e-2, 0.066 .. 0.076         7.0e-2 .., 0.10 ..
#   w8a8    1.2e-3 .. 2.8e-3, 0.014 .. 0.020     2.8e-2 .. 5.0e-2, 0.066 .. 0.076         1.1e-1 .., 0.12 ..
#   w4a8    1.1e-2 .. 1.7e-2, 0.043 .. 0.046     6.2e-2 .. 0.11, 0.100 .. 0.133 (E8M0)    7.3e-2 .., 0.10 ..
TIED_THRESHOLDS = {
    "bf16": (4e-4, 0.012),
    "w8a16": (6e-3, 0.035),
    "w8a8": (7e-3, 0.038),
    "w4a8": (3e-2, 0.07),
}
PROBE_V, PROBE_SCALE, PROBE_SEED = 8192, 4.0, 1234


def _probe(d: int, device) -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(PROBE_SEED)
    return (torch.randn(PROBE_V, d, generator=g) * (PROBE_SCALE / d ** 0.5)).to(device)


def tied(weights) -> bool:
    return bool(getattr(weights.spec, "tie_embeddings", False))


def record_decode_logits(eng, prompts: Sequence[Sequence[int]], n_steps: int, hidden: Optional[bool] = None):
    """Greedy-decode ``prompts`` as ONE batch (bucket of len(prompts)), one decode step per engine iteration,
    recording the decode step's logits.  Returns (tokens [P][n_steps + 1], logits [P, n_steps, V] f32) where
    logits[i, j - 1] are the engine's logits that chose token j (j = 1 .. n_steps; token 0 comes from prefill).
    ``hidden`` (default: tied-embedding models): the logits entry is then a pair (logits, final hidden states
    [P, n_steps, d] f32) -- the lm_head input of the same steps."""
    from ..engine import SamplingParams

    r = eng.runner
    hidden = tied(r.w) if hidden is None else hidden
    old = eng.run_ahead
    eng.run_ahead = 1
    try:
        params = SamplingParams(max_tokens=n_steps + 1, temperature=0.0, ignore_eos=True)
        reqs = [eng.add_request(list(p), params) for p in prompts]
        out = torch.zeros(len(prompts), n_steps, r.V, dtype=torch.float32, device=r.device)
        hid = torch.zeros(len(prompts), n_steps, r.d, dtype=torch.float32, device=r.device) if hidden else None
        B = r.bucket(len(prompts))
        while not all(q.done.is_set() for q in reqs):
            eng.step()
            xh = r.final_hidden(B) if hidden else None
            for i, q in enumerate(reqs):
                j = (len(q.output_ids) if q.done.is_set() else q.gen_host) - 1  # token the last step chose
                if 1 <= j <= n_steps and q.slot >= 0:
                    out[i, j - 1].copy_(r.logits[q.slot].float())
                    if hidden:
                        hid[i, j - 1].copy_(xh[q.slot].float())
        return [q.output_ids for q in reqs], ((out, hid) if hidden else out)
    finally:
        eng.run_ahead = old


def compare(engine_logits: torch.Tensor, oracle_logits: torch.Tensor) -> dict:
    """Per-position KL(oracle || engine), top-1 agreement and top-5 overlap over [n, V] logits."""
    e = engine_logits.float()
    o = oracle_logits.float().to(e.device)
    lo, le = torch.log_softmax(o, -1), torch.log_softmax(e, -1)
    kl = (lo.exp() * (lo - le)).sum(-1)
    top1 = (e.argmax(-1) == o.argmax(-1)).float()
    t5e, t5o = e.topk(5, -1).indices, o.topk(5, -1).indices
    top5 = (t5e.unsqueeze(-1) == t5o.unsqueeze(-2)).any(-1).float().mean(-1)
    return {"kl": kl, "top1": top1, "top5": top5}


def compare_hidden(engine_x: torch.Tensor, oracle_x: torch.Tensor) -> dict:
    """Per-position probe-head KL(oracle || engine) and relative L2 error of the final hidden states [n, d]."""
    e, o = engine_x.float(), oracle_x.float().to(engine_x.device)
    P = _probe(e.shape[-1], e.device)
    lo, le = torch.log_softmax(o @ P.t(), -1), torch.log_softmax(e @ P.t(), -1)
    kl = (lo.exp() * (lo - le)).sum(-1)
    rel = (e - o).norm(dim=-1) / o.norm(dim=-1).clamp(min=1e-12)
    return {"probe_kl": kl, "rel": rel}


def numerics_class(runner, decode_batch: int) -> str:
    """Which threshold row applies to the decode path at ``decode_batch`` (see engine/runner.py)."""
    a8 = any(runner.a8_plan(decode_batch))
    if runner.w.layers[0].wqkv.kind != "fp8":
        return "w4a8" if a8 else "bf16"  # MXFP4: the oracle multiplies its dequantised weights; W4A8 rounds activations
    return "w8a8" if a8 or runner.kv_fp8 else "w8a16"


def teacher_forced_check(eng, prompts: Sequence[Sequence[int]], n_steps: int = 64, check_rows: Sequence[int] = (0,),
                         weights=None, prefill_rows: Optional[int] = None) -> dict:
    """Decode ``prompts`` as one batch for ``n_steps`` steps, compare rows ``check_rows`` against the oracle."""
    toks, elog = record_decode_logits(eng, prompts, n_steps)
    return check_recorded(eng, prompts, toks, elog, n_steps, check_rows, weights, prefill_rows)


def check_recorded(eng, prompts, toks, elog, n_steps: int, check_rows: Sequence[int] = (0,), weights=None,
                   prefill_rows: Optional[int] = None) -> dict:
    """Compare recorded decode logits (``record_decode_logits``) of rows ``check_rows`` with the oracle.

    ``weights``: the unsharded weights for the oracle (TP engines hold one shard; default the engine's own).
    ``prefill_rows``: rows of the packed prefill (fp8: > 64 -> W8A8 prefill, emulated by the oracle)."""
    from .. import ops
    from ..models.llama import reference_forward

    r = eng.runner
    B = r.bucket(len(prompts))
    w = weights if weights is not None else r.w
    fp8 = w.layers[0].wqkv.kind == "fp8"
    rows = prefill_rows if prefill_rows is not None else sum(len(p) for p in prompts)
    plan = r.oracle_plan(B)
    ehid = None
    if isinstance(elog, tuple):
        elog, ehid = elog
    kls, t1s, t5s, pks, rels = [], [], [], [], []
    for i in sorted(set(check_rows)):
        p = list(prompts[i])
        aq = len(p) if (fp8 and rows > 64 and ops.FP8_W8A8) else 0
        lg, xo = reference_forward(w, p + list(toks[i][:n_steps]), act_quant_rows=aq, decode_a8=plan,
                                   kv_fp8=r.kv_fp8, return_hidden=True)
        c = compare(elog[i], lg[len(p):len(p) + n_steps])
        kls.append(c["kl"])
        t1s.append(c["top1"])
        t5s.append(c["top5"])
        if ehid is not None:
            ch = compare_hidden(ehid[i], xo[len(p):len(p) + n_steps])
            pks.append(ch["probe_kl"])
            rels.append(ch["rel"])
        del lg, xo
    kl, t1, t5 = torch.cat(kls), torch.cat(t1s), torch.cat(t5s)
    cls = numerics_class(r, B)
    kl_layer, t5_min, t1_min = THRESHOLDS[cls]
    nl = len(r.w.layers)
    kl_max = round(kl_layer * nl, 6)
    res = {"tokens_checked": int(kl.numel()), "decode_batch": len(prompts), "class": cls,
           "mean_kl": round(float(kl.mean()), 6), "max_kl": round(float(kl.max()), 6),
           "top1_agree": round(float(t1.mean()), 4), "top5_overlap": round(float(t5.mean()), 4)}
    if ehid is None:
        res["ok"] = bool(res["mean_kl"] < kl_max and res["top5_overlap"] >= t5_min
                         and (t1_min is None or res["top1_agree"] >= t1_min))
        res["criterion"] = (f"{cls}: teacher-forced over {n_steps} decode steps: mean KL(oracle||engine) < {kl_max} "
                            f"({kl_layer} x {nl} layers), top-5 overlap >= {t5_min}"
                            + (f", top-1 agreement >= {t1_min}" if t1_min is not None else " (top-1 reported only)"))
        return res
    pk, rel = torch.cat(pks), torch.cat(rels)
    pk_layer, rel_c = TIED_THRESHOLDS[cls]
    pk_max = round(pk_layer * nl, 6)
    rel_max = round(rel_c * nl ** 0.5, 5)
    res.update(tied_head=True, probe_kl=round(float(pk.mean()), 6), probe_kl_max=round(float(pk.max()), 6),
               hidden_rel_err=round(float(rel.mean()), 5), hidden_rel_err_max=round(float(rel.max()), 5))
    res["ok"] = bool(res["probe_kl"] < pk_max and res["hidden_rel_err"] < rel_max
                     and (t1_min is None or res["top1_agree"] >= t1_min))
    res["criterion"] = (f"{cls}, tied lm_head: teacher-forced over {n_steps} decode steps: mean KL(oracle||engine) of an "
                        f"untied random probe head over the final hidden state < {pk_max} ({pk_layer} x {nl} layers), "
                        f"mean relative L2 error of the final hidden state < {rel_max} ({rel_c} x sqrt({nl})), top-1 agreement of the tied "
                        f"head >= {t1_min or 0} (its KL is reported, but a random-init tied head is near one-hot)")
    return res


# ---- fault injection (tests/test_numerics_gpu.py, scripts/numerics_calibrate.py): the check must catch these
@contextlib.contextmanager
def scale_fault(eng, layer: int = 1, factor: float = 1.25):
    """One layer's down-projection dequantisation scale (fp8) / weights (bf16) x ``factor`` in the ENGINE; MXFP4: a
    wrong E8M0 block scale instead (``e8m0_fault``: every 8th block of that layer's down projection one binade up)."""
    lw = eng.runner.w.layers[layer].w_down
    if lw.kind == "mxfp4":
        with e8m0_fault(eng, layer):
            yield
        return
    saved = lw.scale.clone() if lw.scale is not None else lw.data.clone()
    if lw.scale is not None:
        lw.scale.mul_(factor)
    else:
        lw.data.copy_((lw.data.float() * factor).to(lw.data.dtype))
    try:
        yield
    finally:
        (lw.scale if lw.scale is not None else lw.data).copy_(saved)


@contextlib.contextmanager
def e8m0_fault(eng, layer: int = 1, every: int = 8, delta: int = 1):
    """MXFP4: every ``every``-th E8M0 block-scale byte of one layer's down projection + ``delta`` in the ENGINE (those
    32-weight blocks scaled by 2^delta) -- the wrong-block-scale bug class of the W4A8 / W4A16 kernels."""
    lw = eng.runner.w.layers[layer].w_down
    assert lw.kind == "mxfp4", lw.kind
    saved = lw.scale.clone()
    v = lw.scale.view(-1)
    v[::every] = (v[::every].int() + delta).clamp(0, 254).to(v.dtype)
    try:
        yield
    finally:
        lw.scale.copy_(saved)


@contextlib.contextmanager
def kv_swap_fault(eng):
    """Keys of positions 2k and 2k + 1 exchanged in the first cache block of every sequence and layer after
    prefill (values left in place): a KV layout bug."""
    r = eng.runner
    orig = r.prefill

    def prefill_swapping(seqs, *a, **k):
        orig(seqs, *a, **k)
        for slot, _, _ in seqs:
            blk = int(r.block_tables[slot, 0])
            for l in range(r.L):
                kc = r.kv[l, 0, blk]  # [Hkv, 64, D] (bytes for the fp8 cache)
                ev, od = kc[:, 0:32:2].clone(), kc[:, 1:32:2].clone()
                kc[:, 0:32:2], kc[:, 1:32:2] = od, ev
                if r.kv_fp8:  # the per-token scales move with their rows
                    ks = r.kv_scale[l, 0, blk]
                    e2, o2 = ks[:, 0:32:2].clone(), ks[:, 1:32:2].clone()
                    ks[:, 0:32:2], ks[:, 1:32:2] = o2, e2

    r.prefill = prefill_swapping
    try:
        yield
    finally:
        del r.prefill
