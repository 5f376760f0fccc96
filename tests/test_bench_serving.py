"""The co-serving load generator end to end on CPU (fake engine behind the real FastAPI app + uvicorn)."""
from llm_based_apache_spark_optimization_amd import bench_serving


def test_bench_serving_fake_engine():
    out = bench_serving.run(bench_serving_args(qps=40, duration=0.5))
    assert out["failed"] == 0 and out["requests"] > 5
    assert out["nl2sql"]["n"] + out["explain_error"]["n"] == out["requests"]
    assert out["nl2sql"]["p50_s"] is not None and out["output_tokens_per_sec"] > 0


def test_bench_serving_streaming_fake_engine():
    out = bench_serving.run(bench_serving_args(qps=40, duration=0.5, stream=True))
    assert out["failed"] == 0 and out["requests"] > 5
    assert out["nl2sql"]["ttft_p50_s"] is not None and out["nl2sql"]["ttft_p50_s"] <= out["nl2sql"]["p99_s"]


def test_bench_serving_option_less_fake_engine():
    out = bench_serving.run(bench_serving_args(qps=40, duration=0.5, option_less=True))
    assert out["failed"] == 0 and out["requests"] > 5 and out["option_less"] is True


def test_synthetic_prompts_sizes():
    import random

    rng = random.Random(0)
    e = bench_serving.synthetic_spark_error(rng, 1024)
    assert "UNRESOLVED_COLUMN" in e and 3500 < len(e) < 5000
    s = bench_serving.synthetic_schema(rng)
    assert all(line.endswith(")") and " (" in line for line in s.splitlines())


def bench_serving_args(**kw):
    import argparse

    a = argparse.Namespace(qps=8.0, duration=1.0, explain_frac=0.3, explain_tokens=256, new_tokens=16,
                           nl2sql_dtype="bf16", explain_dtype="bf16", max_batch=8, max_model_len=1024,
                           concurrency=32, timeout=30.0, engine="fake", seed=0, option_less=False)
    for k, v in kw.items():
        setattr(a, k, v)
    return a
