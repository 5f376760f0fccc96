"""BASELINE config 1 (CPU plumbing): the engine's model path vs HuggingFace transformers on CPU.

A tiny random-init Llama of each served architecture (MHA duckdb-nsql shape; GQA + llama3-scaled
RoPE + tied embeddings Llama-3.2 shape) is built in transformers, its state dict loaded into the
engine (CPU reference ops, bf16 weights / bf16 activations) and compared: prefill logits and
teacher-forced greedy decoding through the paged KV cache and the native scheduler.
"""
import json

import pytest
import torch

from llm_based_apache_spark_optimization_amd.engine import LLMEngine, ModelRunner, SamplingParams
from llm_based_apache_spark_optimization_amd.models import get_spec
from llm_based_apache_spark_optimization_amd.models.llama import from_hf_state_dict
from llm_based_apache_spark_optimization_amd.ops import reference as ref


def hf_model(name, init=0.08, seed=0):
    from transformers import LlamaConfig, LlamaForCausalLM

    spec = get_spec(name)
    torch.manual_seed(seed)
    m = LlamaForCausalLM(LlamaConfig(**spec.to_hf_config(), initializer_range=init))
    inv = m.model.rotary_emb.inv_freq.clone()
    m = m.to(torch.bfloat16).float().eval()
    m.model.rotary_emb.inv_freq.copy_(inv)
    return spec, m


@pytest.mark.parametrize("name", ["tiny-nsql", "tiny-llama3"])
def test_greedy_matches_transformers(name):
    spec, m = hf_model(name)
    eng = LLMEngine(ModelRunner(from_hf_state_dict(spec, m.state_dict(), "cpu"), max_slots=4, max_model_len=512))
    prompts = [[1] + list(range(5, 60)), [1] + list(range(100, 300, 3))]
    res = eng.generate(prompts, SamplingParams(max_tokens=10, ignore_eos=True))
    for p, r in zip(prompts, res):
        with torch.no_grad():
            lg = m(torch.tensor([p + r.token_ids])).logits[0, len(p) - 1:-1]
        chosen = lg.gather(1, torch.tensor(r.token_ids).view(-1, 1)).squeeze(1)
        gap = lg.max(1).values - chosen
        assert (gap <= 0.05 * lg.max(1).values.abs() + 0.05).all(), gap


@pytest.mark.parametrize("name", ["tiny-nsql", "tiny-llama3"])
def test_prefill_logits(name):
    """Prefill logits (300 rows: the residual-epilogue path, ops.linear_res) vs transformers."""
    spec, m = hf_model(name)
    r = ModelRunner(from_hf_state_dict(spec, m.state_dict(), "cpu"), max_slots=2, max_model_len=512)
    p = [1] + list(range(7, 300))
    r.set_slot(0, list(range(1, 6)), 4)
    r.prefill([(0, p, 0)])
    with torch.no_grad():
        want = m(torch.tensor([p])).logits[0, -1:]
    rel = (r.logits_l[:1] - want).norm() / want.norm()
    assert rel < 3e-2


def test_rope_tables_match_transformers():
    spec, m = hf_model("tiny-llama3")
    c, s = ref.rope_tables(128, 300, spec.rope_theta, spec.rope_scaling)
    hc, hs = m.model.rotary_emb(torch.zeros(1, 300, 128), torch.arange(300)[None])
    assert torch.allclose(c, hc[0, :, :64], atol=1e-4) and torch.allclose(s, hs[0, :, :64], atol=1e-4)


def test_llama3_scaling_changes_low_frequencies():
    sc = get_spec("llama3.2").rope_scaling
    c, _ = ref.rope_tables(128, 20000, 500000.0, sc)
    c0, _ = ref.rope_tables(128, 20000, 500000.0, None)
    assert torch.allclose(c[:, :8], c0[:, :8], atol=1e-6)
    assert not torch.allclose(c[-1, -4:], c0[-1, -4:])


@pytest.mark.parametrize("name", ["tiny-nsql", "tiny-llama3"])
def test_repeat_penalty_matches_transformers(name):
    """Ollama's repeat_penalty through the engine (greedy, context < the 64-token window) vs HF's
    RepetitionPenaltyLogitsProcessor semantics applied to teacher-forced transformers logits."""
    spec, m = hf_model(name)
    eng = LLMEngine(ModelRunner(from_hf_state_dict(spec, m.state_dict(), "cpu"), max_slots=2, max_model_len=256))
    p = [1] + [7, 9, 7, 11, 13, 9, 7, 21, 9, 7]
    pen = 1.8
    r = eng.generate([p], SamplingParams(max_tokens=14, ignore_eos=True, repeat_penalty=pen))[0]
    with torch.no_grad():
        lg = m(torch.tensor([p + r.token_ids])).logits[0, len(p) - 1:-1]
    for i, t in enumerate(r.token_ids):
        row = lg[i].clone()
        seen = torch.tensor(sorted(set(p + r.token_ids[:i])))
        s = row[seen]
        row[seen] = torch.where(s < 0, s * pen, s / pen)
        assert row.max() - row[t] <= 0.05 * row.max().abs() + 0.05, (i, t, int(row.argmax()))


def test_repeat_penalty_ollama_options():
    sp = SamplingParams.from_ollama_options({"repeat_penalty": 1.1, "repeat_last_n": 32, "temperature": 0})
    assert sp.repeat_penalty == 1.1 and sp.repeat_last_n == 32 and sp.needs_sampler
    assert not SamplingParams.from_ollama_options({}).needs_sampler


@pytest.mark.parametrize("name", ["tiny-nsql", "tiny-llama3"])
def test_safetensors_checkpoint_dir_loads(name, tmp_path):
    """An HF checkpoint directory (config.json + *.safetensors, written by transformers' save_pretrained)
    loads through the safe loader into the same weights as the in-memory state dict: identical spec
    fields and identical prefill logits; the TP=2 shards split the projections in halves."""
    from llm_based_apache_spark_optimization_amd.models.llama import load_safetensors_dir

    spec, m = hf_model(name)
    m.to(torch.bfloat16).save_pretrained(str(tmp_path), safe_serialization=True)
    w = load_safetensors_dir(str(tmp_path), "cpu", name=name)
    for f in ("n_layers", "hidden", "n_heads", "n_kv_heads", "ffn", "vocab_size", "rope_theta", "rms_eps", "tie_embeddings"):
        assert getattr(w.spec, f) == getattr(spec, f), f
    assert (w.spec.rope_scaling is None) == (spec.rope_scaling is None)
    assert w.spec.template == spec.template  # the served name selects the Ollama template
    p = [1] + list(range(7, 120))
    outs = []
    for weights in (w, from_hf_state_dict(spec, m.state_dict(), "cpu")):
        r = ModelRunner(weights, max_slots=1, max_model_len=256)
        r.set_slot(0, list(range(1, 3)), 4)
        r.prefill([(0, p, 0)])
        outs.append(r.logits_l[:1].clone())
    assert torch.equal(outs[0], outs[1])
    # the serving factory path (weights-only directory: byte tokenizer fallback)
    from llm_based_apache_spark_optimization_amd.engine import build_engine

    eng = build_engine(name, device="cpu", checkpoint=str(tmp_path), max_slots=2, max_model_len=256)
    r = eng.generate(["Select all records"], SamplingParams(max_tokens=4, ignore_eos=True))[0]
    assert r.eval_count == 4
    if spec.n_kv_heads % 2:
        return  # tiny-llama3 has one kv head: not TP-shardable
    w0 = load_safetensors_dir(str(tmp_path), "cpu", name=name, tp_rank=0, tp_size=2)
    w1 = load_safetensors_dir(str(tmp_path), "cpu", name=name, tp_rank=1, tp_size=2)
    assert w0.layers[0].wo.K == w.layers[0].wo.K // 2 and w1.layers[0].wqkv.N == w.layers[0].wqkv.N // 2
    assert w0.lm_head.N + w1.lm_head.N == w.lm_head.N


def test_hf_tokenizer_checkpoint_llama3_specials(tmp_path):
    """A checkpoint directory's tokenizer.json (a byte-level BPE trained here with the Llama-3 special
    tokens; no hub download is possible) is used by the serving factory: the rendered llama3 chat
    template maps each header/end-of-turn marker to ONE special id, text round-trips, and <|eot_id|>
    terminates generation."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    from llm_based_apache_spark_optimization_amd.engine import build_engine
    from llm_based_apache_spark_optimization_amd.models.templates import render
    from llm_based_apache_spark_optimization_amd.models.tokenizer import LLAMA3_SPECIALS, HFTokenizer
    from llm_based_apache_spark_optimization_amd.prompts import EXPLAIN_SYSTEM

    spec, m = hf_model("tiny-llama3")
    m.to(torch.bfloat16).save_pretrained(str(tmp_path), safe_serialization=True)
    bpe = Tokenizer(models.BPE())
    bpe.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    bpe.decoder = decoders.ByteLevel()
    corpus = ["The following Spark error occurred: AnalysisException UNRESOLVED_COLUMN", "SELECT * FROM temp_view;",
              "Please analyze this error and suggest possible solutions.", EXPLAIN_SYSTEM] * 20
    bpe.train_from_iterator(corpus, trainers.BpeTrainer(vocab_size=420, special_tokens=list(LLAMA3_SPECIALS),
                                                        initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    bpe.save(str(tmp_path / "tokenizer.json"))
    ids = {s: bpe.token_to_id(s) for s in LLAMA3_SPECIALS}
    cfg = json.loads((tmp_path / "config.json").read_text())
    cfg.update(bos_token_id=ids["<|begin_of_text|>"], eos_token_id=[ids["<|end_of_text|>"], ids["<|eot_id|>"]])
    (tmp_path / "config.json").write_text(json.dumps(cfg))

    eng = build_engine("llama3.2", device="cpu", checkpoint=str(tmp_path), max_slots=2, max_model_len=512)
    assert isinstance(eng.tok, HFTokenizer) and eng.spec.template == "llama3"
    text = render("llama3", "The following Spark error occurred: x", EXPLAIN_SYSTEM)
    enc = eng.tok.encode(text, add_bos=False)
    for s in ("<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"):
        assert enc.count(ids[s]) == text.count(s) > 0, s
    assert eng.tok.decode(eng.tok.encode("SELECT * FROM temp_view;", add_bos=False)) == "SELECT * FROM temp_view;"
    assert ids["<|eot_id|>"] in eng.runner.eos_list
    r = eng.generate(["SELECT"], SamplingParams(max_tokens=3, ignore_eos=True), system=EXPLAIN_SYSTEM)[0]
    assert r.eval_count == 3 and isinstance(r.text, str)


def test_full_width_duckdb_nsql_layers_match_transformers():
    """BASELINE config 1 at the served model's full width: duckdb-nsql-7B's exact shapes (d 4096, 32 MHA heads,
    ffn 11008, vocab 32000, untied head) with 2 of its 32 layers, random-init in transformers, through the engine on
    CPU: prefill logits and greedy decoding vs HF (the tiny configs above check the same path at test sizes)."""
    import dataclasses

    from transformers import LlamaConfig, LlamaForCausalLM

    spec = dataclasses.replace(get_spec("duckdb-nsql"), n_layers=2)
    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig(**spec.to_hf_config(), initializer_range=0.02))
    inv = m.model.rotary_emb.inv_freq.clone()
    m = m.to(torch.bfloat16).float().eval()
    m.model.rotary_emb.inv_freq.copy_(inv)
    assert (m.config.hidden_size, m.config.intermediate_size, m.config.vocab_size) == (4096, 11008, 32000)
    eng = LLMEngine(ModelRunner(from_hf_state_dict(spec, m.state_dict(), "cpu"), max_slots=2, max_model_len=256))
    p = [1] + list(range(300, 340))
    r = eng.generate([p], SamplingParams(max_tokens=6, ignore_eos=True))[0]
    with torch.no_grad():
        lg = m(torch.tensor([p + r.token_ids])).logits[0, len(p) - 1:-1]
    chosen = lg.gather(1, torch.tensor(r.token_ids).view(-1, 1)).squeeze(1)
    gap = lg.max(1).values - chosen
    assert (gap <= 0.05 * lg.max(1).values.abs() + 0.05).all(), gap
