"""Inference engine: ModelRunner (device execution + hipGraph decode) and LLMEngine (batching)."""
from .engine import GenerationResult, LLMEngine, Request, SamplingParams  # noqa: F401
from .runner import ModelRunner  # noqa: F401
from .factory import build_engine  # noqa: F401
