"""Model family: Llama-architecture decoders (duckdb-nsql-7B, Llama-3.2-3B, Mistral-7B)."""
from .spec import ModelSpec, SPECS, get_spec, spec_from_hf_config  # noqa: F401
from .templates import render, apply_stops  # noqa: F401
from .tokenizer import ByteTokenizer, HFTokenizer, tokenizer_for  # noqa: F401
