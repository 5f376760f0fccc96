"""Run the same model on CPU (reference ops) and GPU (HIP ops) and report the first op whose
output diverges — a bisecting debug tool for engine-level mismatches."""
import sys, torch
sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd import ops
from llm_based_apache_spark_optimization_amd.engine import ModelRunner
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import from_hf_state_dict
from transformers import LlamaConfig, LlamaForCausalLM

name = sys.argv[1] if len(sys.argv) > 1 else "tiny-llama3"
spec = get_spec(name)
torch.manual_seed(0)
m = LlamaForCausalLM(LlamaConfig(**spec.to_hf_config(), initializer_range=0.08)).to(torch.bfloat16).float().eval()
sd = m.state_dict()
trace = {}
def wrap(fname, out_arg):
    f = getattr(ops, fname)
    def g(*a, **k):
        r = f(*a, **k)
        o = k.get("out") if out_arg == "out" else (a[out_arg] if isinstance(out_arg, int) and len(a) > out_arg else k.get("xn"))
        if o is None: o = r
        trace.setdefault(cur[0], []).append((fname, o.detach().float().cpu().clone()))
        return r
    setattr(ops, fname, g)
cur = ["cpu"]
for fn, oa in [("linear", "out"), ("add_rmsnorm", 3), ("attn_prefill", 9), ("attn_decode", 8)]:
    wrap(fn, oa)
prompts = [[1] + list(range(5, 60)), [1] + list(range(100, 300, 3))]
for dev in ["cpu", "cuda"]:
    cur[0] = dev
    w = from_hf_state_dict(spec, sd, dev)
    r = ModelRunner(w, max_slots=4, max_model_len=512, use_graphs=False)
    seqs = []
    for i, p in enumerate(prompts):
        r.set_slot(i, [1 + 4 * i + j for j in range(4)], 4)
        seqs.append((i, p, 0))
    r.prefill(seqs)
    if dev == "cuda": torch.cuda.synchronize()
a, b = trace["cpu"], trace["cuda"]
print(len(a), len(b))
for i, ((fa, ta), (fb, tb)) in enumerate(zip(a, b)):
    if ta.shape != tb.shape:
        print(i, fa, fb, "shape", ta.shape, tb.shape); continue
    rel = ((ta - tb).norm() / (ta.norm() + 1e-9)).item()
    flag = "  <-- DIFF" if rel > 2e-2 else ""
    print(i, fa, tuple(ta.shape), f"{rel:.2e}{flag}")
    if flag: 
        print(ta.flatten()[:8], tb.flatten()[:8]); break
