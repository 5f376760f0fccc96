"""Per-launch check of the block decode step inside a real engine (eager): every ops.decode_block call of the
first decode steps is re-run on CPU copies of its inputs (the fp32 reference path) and compared."""
import dataclasses
import json
import os
import sys

import torch

sys.path.insert(0, ".")
os.environ["LSA_DECODE_BLOCK"] = "1"
from llm_based_apache_spark_optimization_amd import ops  # noqa: E402
from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner, SamplingParams  # noqa: E402
from llm_based_apache_spark_optimization_amd.models import get_spec  # noqa: E402
from llm_based_apache_spark_optimization_amd.models.llama import init_random  # noqa: E402

real = ops.decode_block
calls = [0]
cpu_w = {}


def cpuw(w):
    if w is None:
        return None
    k = id(w)
    if k not in cpu_w:
        cpu_w[k] = ops.PackedWeight.from_dense(w.dense().cpu())
    return cpu_w[k]


def checked(attn, wo, h, x, ss1, ss2, wgu, act, wd, wq, qout, B, eps, cnt, err, cfg=None, **kw):
    calls[0] += 1
    if calls[0] > 12:
        return real(attn, wo, h, x, ss1, ss2, wgu, act, wd, wq, qout, B, eps, cnt, err, cfg=cfg, **kw)
    torch.cuda.synchronize()
    c = {k: v.detach().cpu().clone() for k, v in dict(attn=attn, h=h, x=x, ss1=ss1, ss2=ss2, act=act, qout=qout,
                                                       cnt=cnt, err=err).items()}
    cfg = cfg or ops.decode_block_cfg(B)
    real(attn, wo, h, x, ss1, ss2, wgu, act, wd, wq, qout, B, eps, cnt, err, cfg=cfg, **kw)
    torch.cuda.synchronize()
    real(c["attn"], cpuw(wo), c["h"], c["x"], c["ss1"], c["ss2"], cpuw(wgu), c["act"], cpuw(wd), cpuw(wq), c["qout"],
         B, eps, c["cnt"], c["err"], cfg=cfg)
    rel = lambda a, b: float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))
    nq = wq.N if wq is not None else 0
    out = {"call": calls[0], "B": B, "err": int(err[0]), "ss1_in": ops.ss_float(c["ss1"][:B]).tolist()[:4],
           "h_row": [rel(h[m].cpu(), c["h"][m]) for m in range(B)],
           "ss2": [rel(ops.ss_float(ss2[m:m + 1].cpu()), ops.ss_float(c["ss2"][m:m + 1])) for m in range(B)],
           "act_row": [rel(a, b) for a, b in zip(ops.from_xfrag(act, B, wd.K).cpu(), ops.from_xfrag(c["act"], B, wd.K))]}
    if wq is not None:
        qg = qout[: B * nq].view(B, nq).cpu()
        out["q_row"] = [rel(qg[m], c["qout"][: B * nq].view(B, nq)[m]) for m in range(B)]
    print(json.dumps(out), flush=True)


ops.decode_block = checked
spec = dataclasses.replace(get_spec("duckdb-nsql"), n_layers=3, name="duckdb-nsql-3l")
dev = torch.device("cuda:0")
w = init_random(spec, dev, seed=5, kind="bf16")
r = ModelRunner(w, max_slots=32, max_model_len=512, use_graphs=False, num_kv_blocks=32 * 8 + 1)
assert r.block_decode
eng = LLMEngine(r, name=spec.name)
g = torch.Generator().manual_seed(1)
prompts = [[1] + torch.randint(3, 30000, (20 + 5 * i,), generator=g).tolist() for i in range(3)]
res = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
print(json.dumps({"tokens": [q.token_ids for q in res]}))
