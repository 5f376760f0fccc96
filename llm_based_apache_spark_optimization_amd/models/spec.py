"""Model specifications served by the engine.

The reference never names architectures: it addresses Ollama tags (`duckdb-nsql`, `llama3.2`,
`mistral` — FastAPI/app.py:86,106, Flask/app.py:103,161, Model_Evaluation_&_Comparision.py:69,83).
These are the published configs behind those tags (SURVEY.md §2.5 "Model specs"), plus tiny
configurations of the same architecture for CPU tests.
"""
from __future__ import annotations

import dataclasses
from typing import Optional


@dataclasses.dataclass(frozen=True)
class ModelSpec:
    name: str
    vocab_size: int
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn: int
    rope_theta: float
    rms_eps: float = 1e-5
    head_dim: int = 128
    tie_embeddings: bool = False
    max_position: int = 4096
    rope_scaling: Optional[dict] = None
    bos_id: int = 1
    eos_ids: tuple = (2,)
    template: str = "raw"  # prompt template id (models/templates.py)
    hf_id: str = ""

    @property
    def qkv_dim(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    @property
    def params(self) -> int:
        d, L = self.hidden, self.n_layers
        per = d * self.qkv_dim + self.n_heads * self.head_dim * d + 3 * d * self.ffn + 2 * d
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return L * per + emb + d

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * self.n_kv_heads * self.head_dim * dtype_bytes

    def to_hf_config(self) -> dict:
        cfg = dict(
            architectures=["LlamaForCausalLM"], model_type="llama", vocab_size=self.vocab_size,
            hidden_size=self.hidden, intermediate_size=self.ffn, num_hidden_layers=self.n_layers,
            num_attention_heads=self.n_heads, num_key_value_heads=self.n_kv_heads, head_dim=self.head_dim,
            rms_norm_eps=self.rms_eps, rope_theta=self.rope_theta, max_position_embeddings=self.max_position,
            tie_word_embeddings=self.tie_embeddings, bos_token_id=self.bos_id, eos_token_id=list(self.eos_ids),
            hidden_act="silu", attention_bias=False, mlp_bias=False,
        )
        if self.rope_scaling:
            cfg["rope_scaling"] = dict(self.rope_scaling)
        return cfg


LLAMA3_SCALING = {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                  "original_max_position_embeddings": 8192}

SPECS: dict[str, ModelSpec] = {
    # motherduckdb/DuckDB-NSQL-7B-v0.1 (Llama-2-7B architecture)
    "duckdb-nsql": ModelSpec(
        name="duckdb-nsql", vocab_size=32000, hidden=4096, n_layers=32, n_heads=32, n_kv_heads=32, ffn=11008,
        rope_theta=10000.0, rms_eps=1e-5, max_position=16384, bos_id=1, eos_ids=(2,), template="duckdb-nsql",
        hf_id="motherduckdb/DuckDB-NSQL-7B-v0.1"),
    # meta-llama/Llama-3.2-3B-Instruct
    "llama3.2": ModelSpec(
        name="llama3.2", vocab_size=128256, hidden=3072, n_layers=28, n_heads=24, n_kv_heads=8, ffn=8192,
        rope_theta=500000.0, rms_eps=1e-5, tie_embeddings=True, max_position=131072, rope_scaling=LLAMA3_SCALING,
        bos_id=128000, eos_ids=(128001, 128008, 128009), template="llama3", hf_id="meta-llama/Llama-3.2-3B-Instruct"),
    # mistralai/Mistral-7B-Instruct-v0.3 (eval harness third model)
    "mistral": ModelSpec(
        name="mistral", vocab_size=32768, hidden=4096, n_layers=32, n_heads=32, n_kv_heads=8, ffn=14336,
        rope_theta=1000000.0, rms_eps=1e-5, max_position=32768, bos_id=1, eos_ids=(2,), template="mistral",
        hf_id="mistralai/Mistral-7B-Instruct-v0.3"),
    # tiny configs of the same architectures (tests / CPU plumbing)
    "tiny-nsql": ModelSpec(
        name="tiny-nsql", vocab_size=512, hidden=256, n_layers=2, n_heads=2, n_kv_heads=2, ffn=512,
        rope_theta=10000.0, max_position=2048, bos_id=1, eos_ids=(2,), template="duckdb-nsql"),
    "tiny-llama3": ModelSpec(
        name="tiny-llama3", vocab_size=640, hidden=384, n_layers=2, n_heads=3, n_kv_heads=1, ffn=768,
        rope_theta=500000.0, tie_embeddings=True, max_position=4096, rope_scaling=LLAMA3_SCALING, bos_id=1,
        eos_ids=(2,), template="llama3"),
}

ALIASES = {
    "duckdb-nsql:latest": "duckdb-nsql", "duckdb-nsql:7b": "duckdb-nsql", "duckdb-nsql-7b": "duckdb-nsql",
    "llama3.2:latest": "llama3.2", "llama3.2:3b": "llama3.2", "llama-3.2-3b": "llama3.2",
    "mistral:latest": "mistral", "mistral:7b": "mistral",
}


def get_spec(name: str) -> ModelSpec:
    key = ALIASES.get(name, name)
    if key not in SPECS:
        raise KeyError(f"unknown model {name!r}; known: {sorted(SPECS)}")
    return SPECS[key]


def spec_from_hf_config(cfg: dict, name: str = "custom", template: str = "raw") -> ModelSpec:
    eos = cfg.get("eos_token_id", 2)
    eos = tuple(eos) if isinstance(eos, (list, tuple)) else (eos,)
    # checkpoints written by transformers >= 5 carry RoPE as one "rope_parameters" dict (rope_theta +
    # rope_type + the scaling fields); older ones (the hub's Llama-2 / Llama-3.2 / Mistral configs) use
    # top-level "rope_theta" and an optional "rope_scaling" dict
    rp = cfg.get("rope_parameters") or {}
    theta = cfg.get("rope_theta", rp.get("rope_theta", 10000.0))
    scaling = cfg.get("rope_scaling")
    if scaling is None and rp.get("rope_type", "default") not in ("default", None):
        scaling = {k: v for k, v in rp.items() if k != "rope_theta"}
    if scaling is not None and scaling.get("rope_type", scaling.get("type", "default")) == "default":
        scaling = None
    return ModelSpec(
        name=name, vocab_size=cfg["vocab_size"], hidden=cfg["hidden_size"], n_layers=cfg["num_hidden_layers"],
        n_heads=cfg["num_attention_heads"], n_kv_heads=cfg.get("num_key_value_heads", cfg["num_attention_heads"]),
        ffn=cfg["intermediate_size"], rope_theta=float(theta), rms_eps=cfg.get("rms_norm_eps", 1e-5),
        head_dim=cfg.get("head_dim") or cfg["hidden_size"] // cfg["num_attention_heads"],
        tie_embeddings=cfg.get("tie_word_embeddings", False), max_position=cfg.get("max_position_embeddings", 4096),
        rope_scaling=scaling, bos_id=cfg.get("bos_token_id", 1) or 1, eos_ids=eos, template=template)
