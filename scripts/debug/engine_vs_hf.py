import sys, torch
sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner, SamplingParams
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import from_hf_state_dict
from transformers import LlamaConfig, LlamaForCausalLM
name = sys.argv[1]
spec = get_spec(name)
torch.manual_seed(0)
m = LlamaForCausalLM(LlamaConfig(**spec.to_hf_config(), initializer_range=0.08)).to(torch.bfloat16).float().eval()
prompts = [[1] + list(range(5, 60)), [1] + list(range(100, 300, 3))]
for p in prompts:
    with torch.no_grad():
        out = m.generate(torch.tensor([p]), max_new_tokens=12, do_sample=False, eos_token_id=None, pad_token_id=0)
        lg = m(torch.tensor([p])).logits[0, -1]
    print("HF ", out[0, len(p):].tolist(), "argmax", int(lg.argmax()), lg.topk(3))
for dev, graphs in [("cpu", False), ("cuda", False), ("cuda", True)]:
    w = from_hf_state_dict(spec, m.state_dict(), dev)
    eng = LLMEngine(ModelRunner(w, max_slots=4, max_model_len=512, use_graphs=graphs))
    res = eng.generate(prompts, SamplingParams(max_tokens=12, ignore_eos=True))
    print(dev, graphs, [r.token_ids for r in res])
    print("   logits top", eng.runner.logits_l[:2].float().cpu().topk(3))
