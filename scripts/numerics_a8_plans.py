import dataclasses, json, sys
sys.path.insert(0, ".")
import torch
from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner
from llm_based_apache_spark_optimization_amd.eval import numerics as nm
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import init_random
gpu = torch.device("cuda:0")
for name in ("llama3.2", "duckdb-nsql"):
    spec = dataclasses.replace(get_spec(name), n_layers=4, name=name + "-4l")
    w = init_random(spec, gpu, seed=5, kind="mxfp4")
    for B in (1, 4):
        for cfg in ({}, {"a8_od_max_batch": 0}, {"a8_od_max_batch": 0, "a8_min_batch": 64, "a8_mlp_min_batch": 64}):
            r = ModelRunner(w, max_slots=32, max_model_len=512, use_graphs=True, num_kv_blocks=32 * 8 + 1)
            for k, v in cfg.items():
                setattr(r, k, v)
            eng = LLMEngine(r, name=spec.name)
            g = torch.Generator().manual_seed(3)
            prompts = [[1] + torch.randint(3, 30000, (100 + 7 * i,), generator=g).tolist() for i in range(B)]
            res = nm.teacher_forced_check(eng, prompts, 64, check_rows=(0, B - 1) if B > 1 else (0,))
            print(json.dumps({"model": name, "B": B, "cfg": cfg, "plan": r.a8_plan(B), **{k: res.get(k) for k in ("ok", "mean_kl", "probe_kl", "hidden_rel_err", "top1_agree")}}), flush=True)
            del eng, r
            torch.cuda.empty_cache()
