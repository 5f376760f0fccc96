"""NL->SQL accuracy / latency comparison across models.

Reproduces Model_Evaluation_&_Comparision.py: the single-query evaluation (taxi schema, one question,
an 8-line expected SQL; C21) and the 4-query evaluation (C22) over ``mistral``, ``llama3.2`` and
``duckdb-nsql``, with the same metrics — exact match after ``strip()``, Levenshtein distance
(native C++ ``_lsa_runtime.levenshtein`` in place of the python-Levenshtein extension) and end-to-end
client wall-clock latency around each ``generate`` call — and the same printed summary.  Additions:
p50 latency, output tokens and tokens/s per model (from the engine's ``eval_count`` /
``eval_duration``, which the reference discarded), a JSON report, and the Markdown model-comparison report of
``eval.report`` (the reference's hand-written ``Model_Comparision_Report.docx``).

    python -m llm_based_apache_spark_optimization_amd.eval.harness --engine hip --max-tokens 128
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from typing import Callable, Optional, Sequence

from .. import prompts
from ..runtime.native import levenshtein

GenerateFn = Callable[..., object]


def _gen(generate: GenerateFn, model: str, system: str, prompt: str, options: Optional[dict]):
    t0 = time.time()
    res = generate(model=model, system=system, prompt=prompt, options=options)
    return res, time.time() - t0


def evaluate_single(generate: GenerateFn, model_name: str, options: Optional[dict] = None, verbose: bool = True):
    res, latency = _gen(generate, model_name, prompts.EVAL_SINGLE_SYSTEM, prompts.EVAL_SINGLE_PROMPT, options)
    generated_sql = res.response.strip()
    exact_match = 1 if generated_sql == prompts.EVAL_EXPECTED_SQL else 0
    edit_distance = levenshtein(generated_sql, prompts.EVAL_EXPECTED_SQL)
    if verbose:
        print(f"Model: {model_name}")
        print(f"Generated SQL:\n{generated_sql}")
        print(f"Exact Match: {exact_match}")
        print(f"Edit Distance: {edit_distance}")
        print(f"Latency: {latency:.4f} sec")
        print("=" * 80)
    return {"model": model_name, "generated_sql": generated_sql, "exact_match": exact_match,
            "edit_distance": edit_distance, "latency": latency,
            "eval_count": getattr(res, "eval_count", 0), "eval_duration": getattr(res, "eval_duration", 0)}


def evaluate_multi(generate: GenerateFn, models: Sequence[str], queries=prompts.EVAL_QUERIES,
                   options: Optional[dict] = None, verbose: bool = True) -> dict:
    results = {m: {"exact_match": 0, "total_edit_distance": 0, "total_latency": 0, "queries": []} for m in models}
    for model in models:
        if verbose:
            print(f"Evaluating model: {model}\n" + "=" * 80)
        for query in queries:
            res, latency = _gen(generate, model, prompts.EVAL_MULTI_SYSTEM, query["nl"], options)
            generated_sql = res.response.strip()
            expected_sql = query["expected_sql"].strip()
            exact_match = int(generated_sql == expected_sql)
            edit_distance = levenshtein(generated_sql, expected_sql)
            r = results[model]
            r["exact_match"] += exact_match
            r["total_edit_distance"] += edit_distance
            r["total_latency"] += latency
            r["queries"].append({"query": query["nl"], "generated_sql": generated_sql, "expected_sql": expected_sql,
                                 "exact_match": exact_match, "edit_distance": edit_distance, "latency": latency,
                                 "eval_count": getattr(res, "eval_count", 0),
                                 "eval_duration": getattr(res, "eval_duration", 0)})
            if verbose:
                print(f"Query: {query['nl']}")
                print(f"Generated SQL: {generated_sql}")
                print(f"Expected SQL: {expected_sql}")
                print(f"Exact Match: {exact_match}, Edit Distance: {edit_distance}, Latency: {latency:.4f} sec")
                print("-" * 80)
    return results


def summarize(results: dict, n_queries: int, verbose: bool = True) -> dict:
    out = {}
    if verbose:
        print("\n\nFinal Evaluation Summary:\n" + "=" * 100)
    for model, data in results.items():
        lats = [q["latency"] for q in data["queries"]]
        toks = sum(q["eval_count"] for q in data["queries"])
        dur = sum(q["eval_duration"] for q in data["queries"]) / 1e9
        s = {"exact_match_rate": data["exact_match"] / n_queries * 100,
             "avg_edit_distance": data["total_edit_distance"] / n_queries,
             "avg_latency": data["total_latency"] / n_queries,
             "p50_latency": statistics.median(lats) if lats else 0.0,
             "output_tokens": toks, "decode_tokens_per_s": (toks / dur) if dur else 0.0}
        out[model] = s
        if verbose:
            print(f"Model: {model}")
            print(f"Exact Match Rate: {s['exact_match_rate']:.2f}%")
            print(f"Average Edit Distance: {s['avg_edit_distance']:.2f}")
            print(f"Average Latency: {s['avg_latency']:.4f} sec")
            print(f"p50 Latency: {s['p50_latency']:.4f} sec   output tokens: {toks}   "
                  f"decode tok/s: {s['decode_tokens_per_s']:.1f}")
            print("=" * 100)
    return out


def main(argv=None) -> int:
    from .. import client
    from ..config import Settings

    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--engine", default="hip", choices=["hip", "fake", "remote"])
    ap.add_argument("--remote-url", default="http://127.0.0.1:8000")
    ap.add_argument("--models", default=",".join(prompts.EVAL_MODELS))
    ap.add_argument("--max-tokens", type=int, default=128, help="num_predict per request")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--json", default="", help="write the report here")
    ap.add_argument("--report", default="", help="write the Markdown model-comparison report here (eval.report)")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    s = Settings(engine=a.engine, remote_url=a.remote_url)
    from ..serving.service import backend_from_settings

    client.set_backend(backend_from_settings(s))
    opts = {"num_predict": a.max_tokens, "temperature": a.temperature}
    models = [m for m in a.models.split(",") if m]
    single = [evaluate_single(client.generate, m, opts, verbose=not a.quiet) for m in models]
    multi = evaluate_multi(client.generate, models, options=opts, verbose=not a.quiet)
    summary = summarize(multi, len(prompts.EVAL_QUERIES), verbose=not a.quiet)
    report = {"single": single, "multi": multi, "summary": summary, "options": opts}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(report, f, indent=1)
    if a.report:
        from .report import render

        with open(a.report, "w") as f:
            f.write(render(report, random_weights=a.engine != "remote"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
