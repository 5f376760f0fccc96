"""The model-comparison report (the reference's ``Model_Comparision_Report.docx``, C23) generated from a harness run.

The reference published a hand-written Word report of one evaluation: a metrics table (exact match, edit distance,
latency, "issues" per model), an accuracy / latency analysis, the structural errors seen in the generated SQL (prose
around the query, invalid identifiers), and recommendations (best model for accuracy, for speed, trade-offs).  This
module renders the same sections as Markdown from ``eval.harness``'s JSON report, with the structural checks made
mechanical instead of by eye:

* ``extra_text`` -- text outside the SQL statement (after stripping a code fence): an explanation before the first SQL
  keyword or after the final ``;`` (the reference's "Mistral: unnecessary explanation included");
* ``valid`` -- the extracted statement compiles against the evaluation's taxi schema in an in-memory SQLite database
  (``EXPLAIN``); the error names the offending token or identifier (the reference's "V VendortID" syntax error).

Published numbers of the reference's run (its report, section 4.1) are printed next to the measured ones.  With
random-init weights (the benchmark path: no checkpoints can be downloaded) exact match and edit distance are
meaningless and the report says so; latency and decode rate are real.

    python -m llm_based_apache_spark_optimization_amd.eval.report --json harness.json --out report.md
"""
from __future__ import annotations

import argparse
import json
import re
import sqlite3
import sys
from typing import Optional

from .. import prompts

# The reference report's section 4.1 (single-query evaluation of its Ollama deployment): edit distance and latency
PUBLISHED = {
    "mistral": {"exact_match": 0, "edit_distance": 456, "latency": 53.73, "issues": "extra text, unnecessary explanation"},
    "llama3.2": {"exact_match": 0, "edit_distance": 589, "latency": 31.09, "issues": "syntax errors (V VendortID)"},
    "duckdb-nsql": {"exact_match": 0, "edit_distance": 57, "latency": 33.65, "issues": "closest to expected output"},
}

_SQL_START = re.compile(r"\b(SELECT|WITH|INSERT|UPDATE|DELETE|CREATE)\b", re.IGNORECASE)
_FENCE = re.compile(r"```(?:sql)?\s*(.*?)```", re.IGNORECASE | re.DOTALL)


def _schema_ddl() -> str:
    m = re.search(r"CREATE TABLE.*?\);", prompts.EVAL_SINGLE_SYSTEM, re.DOTALL)
    return m.group(0) if m else ""


def structural_checks(text: str) -> dict:
    """{sql, extra_text, valid, error} for one generated answer (see the module docstring)."""
    body = text.strip()
    fenced = _FENCE.search(body)
    outside = ""
    if fenced:
        outside = (body[:fenced.start()] + body[fenced.end():]).strip()
        body = fenced.group(1).strip()
    m = _SQL_START.search(body)
    if m is None:
        return {"sql": "", "extra_text": bool(body), "valid": False, "error": "no SQL statement"}
    prefix, sql = body[:m.start()].strip(), body[m.start():]
    semi = sql.find(";")
    suffix = sql[semi + 1:].strip() if semi >= 0 else ""
    sql = sql[:semi + 1] if semi >= 0 else sql.strip()
    res = {"sql": sql, "extra_text": bool(prefix or suffix or outside), "valid": True, "error": ""}
    con = sqlite3.connect(":memory:")
    try:
        con.execute(_schema_ddl())
        con.execute("EXPLAIN " + sql.rstrip(";"))
    except sqlite3.Error as e:
        res.update(valid=False, error=str(e))
    finally:
        con.close()
    return res


def _issues(chk: dict) -> str:
    out = []
    if chk["extra_text"]:
        out.append("extra text around the query")
    if not chk["valid"]:
        out.append(f"invalid SQL ({chk['error']})")
    return ", ".join(out) or "valid SQL, no extra text"


def render(rep: dict, title: str = "Model comparison report (MI355X engine)", random_weights: bool = True) -> str:
    """Markdown report of one harness JSON (``eval.harness --json``)."""
    single = {r["model"]: r for r in rep.get("single", [])}
    multi, summ = rep.get("multi", {}), rep.get("summary", {})
    models = list(single) or list(multi)
    L = [f"# {title}", ""]
    opts = rep.get("options", {})
    L += ["## 1. Setup", "",
          f"Models: {', '.join(models)}, served by this repository's engine (greedy, num_predict "
          f"{opts.get('num_predict', '?')}).  Schema: the reference's taxi table; prompts: its single query and its "
          f"four-query set (`prompts.EVAL_*`).", ""]
    if random_weights:
        L += ["Weights are random-init (no checkpoint download is possible here): exact match and edit distance are "
              "computed exactly as the reference does but say nothing about the models; latency and decode rate are "
              "the engine's real numbers.", ""]
    L += ["## 2. Metrics", "",
          "Exact match (generated SQL == expected after strip), edit distance (Levenshtein, lower is better), latency "
          "(client wall clock around each generate call, lower is better), decode tokens/s; structural checks: text "
          "outside the statement, and whether the statement compiles against the taxi schema (SQLite `EXPLAIN`).", ""]
    L += ["## 3. Results", "", "### 3.1 Single query (the reference report's table)", "",
          "| model | exact match | edit distance | latency | issues | reference: edit distance / latency |",
          "|---|---|---|---|---|---|"]
    checks = {}
    for m in models:
        r = single.get(m, {})
        chk = structural_checks(r.get("generated_sql", "")) if "generated_sql" in r else None
        checks[m] = chk
        pub = PUBLISHED.get(m)
        ref = f"{pub['edit_distance']} / {pub['latency']:.2f} s" if pub else "—"
        L.append(f"| {m} | {r.get('exact_match', '—')} | {r.get('edit_distance', '—')} | "
                 f"{r.get('latency', float('nan')):.3f} s | {_issues(chk) if chk else '—'} | {ref} |")
    L += ["", "### 3.2 Four-query set", "",
          "| model | exact match rate | avg edit distance | avg latency | p50 latency | decode tok/s | valid SQL |",
          "|---|---|---|---|---|---|---|"]
    for m in models:
        s = summ.get(m, {})
        qs = multi.get(m, {}).get("queries", [])
        valid = sum(structural_checks(q.get("generated_sql", ""))["valid"] for q in qs)
        L.append(f"| {m} | {s.get('exact_match_rate', 0):.2f}% | {s.get('avg_edit_distance', 0):.2f} | "
                 f"{s.get('avg_latency', 0):.3f} s | {s.get('p50_latency', 0):.3f} s | "
                 f"{s.get('decode_tokens_per_s', 0):.1f} | {valid} / {len(qs)} |")
    # analysis (the reference's 4.2 - 4.4 and 5)
    L += ["", "## 4. Analysis", ""]
    if single:
        best_acc = min(models, key=lambda m: single[m].get("edit_distance", 1 << 30))
        fastest = min(models, key=lambda m: single[m].get("latency", float("inf")))
        slowest = max(models, key=lambda m: single[m].get("latency", 0.0))
        L.append(f"- Accuracy: {sum(single[m].get('exact_match', 0) for m in models)} exact matches; lowest edit "
                 f"distance {best_acc} ({single[best_acc]['edit_distance']}).")
        L.append(f"- Latency: fastest {fastest} ({single[fastest]['latency']:.3f} s), slowest {slowest} "
                 f"({single[slowest]['latency']:.3f} s).")
        sp = [f"{m} {PUBLISHED[m]['latency'] / single[m]['latency']:.0f}x" for m in models
              if m in PUBLISHED and single[m].get("latency")]
        if sp:
            L.append(f"- Against the reference's published single-query latencies: {', '.join(sp)} faster.")
    for m in models:
        chk = checks.get(m)
        if chk:
            L.append(f"- Structure, {m}: {_issues(chk)}.")
    if single:
        L += ["", "## 5. Recommendations", "",
              f"- Best for accuracy (lowest edit distance): {best_acc}.",
              f"- Best for speed (lowest latency): {fastest}."]
        if best_acc != fastest:
            L.append(f"- Trade-off: {best_acc} is the more accurate, {fastest} the faster; "
                     f"their latencies differ by {abs(single[best_acc]['latency'] - single[fastest]['latency']):.3f} s.")
    return "\n".join(L) + "\n"


def main(argv: Optional[list] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--json", required=True, help="eval.harness --json output")
    ap.add_argument("--out", default="", help="write the Markdown here (default: stdout)")
    ap.add_argument("--trained-weights", action="store_true", help="the run served real checkpoints")
    a = ap.parse_args(argv)
    with open(a.json) as f:
        rep = json.load(f)
    md = render(rep, random_weights=not a.trained_weights)
    if a.out:
        with open(a.out, "w") as f:
            f.write(md)
    else:
        sys.stdout.write(md)
    return 0


if __name__ == "__main__":
    sys.exit(main())
