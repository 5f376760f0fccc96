"""Byte-level prompt contracts, executor semantics and the eval harness metrics (CPU)."""
import os

import pytest

from llm_based_apache_spark_optimization_amd import prompts
from llm_based_apache_spark_optimization_amd.client import FakeBackend, GenerateResponse
from llm_based_apache_spark_optimization_amd.eval import evaluate_multi, evaluate_single, summarize
from llm_based_apache_spark_optimization_amd.runtime import native
from llm_based_apache_spark_optimization_amd.serving.executor import (SQLExecutionError, SqliteExecutor,
                                                                      clean_sql, infer_spark_type, read_csv)

REF = "/root/reference/Model_Evaluation_&_Comparision.py"


def test_nl2sql_prompt_contract():
    schema = prompts.table_schema_text([("Incubation_Center", "string"), ("Age", "int")])
    assert schema == "Incubation_Center (string)\nAge (int)"
    assert prompts.nl2sql_system(schema) == ("Table name is temp_view. The structure of the table is:\n"
                                             "Incubation_Center (string)\nAge (int)")


def test_explain_prompt_contract():
    assert prompts.explain_prompt("boom") == (
        "The following Spark error occurred:\n\nboom\n\nPlease analyze this error and suggest possible solutions.")
    assert prompts.EXPLAIN_SYSTEM == ("You are an AI that helps troubleshoot Apache Spark errors. "
                                      "Provide clear, concise solutions.")


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree not mounted")
def test_eval_strings_byte_identical_to_reference():
    src = open(REF).read()
    exp = src[src.index('EXPECTED_SQL = """') + 18:src.index('""".strip()')].strip()
    assert exp == prompts.EVAL_EXPECTED_SQL
    i = src.index('system="""') + 10
    assert src[i:src.index('""",', i)] == prompts.EVAL_SINGLE_SYSTEM
    i = src.index('system="Here') + 8
    assert src[i:src.index('",', i)] == prompts.EVAL_MULTI_SYSTEM
    for q in prompts.EVAL_QUERIES:
        assert f'"{q["nl"]}"' in src and f'"{q["expected_sql"]}"' in src


def test_levenshtein_native():
    assert native.NATIVE
    assert native.levenshtein("kitten", "sitting") == 3
    assert native.levenshtein("", "abc") == 3
    assert native.levenshtein("héllo", "hello") == 1  # code points, not bytes
    assert native.levenshtein_batch(["a", "ab"], ["b", "ab"]) == [1, 0]


@pytest.mark.parametrize("vals,t", [(["1", "2", ""], "int"), (["1", "3000000000"], "bigint"), (["1.5", "2"], "double"),
                                    (["true", "False"], "boolean"), (["2024-01-02"], "date"),
                                    (["2024-01-02 10:00:00", "2024-01-03"], "timestamp"), (["x", "1"], "string"),
                                    ([""], "string")])
def test_spark_type_inference(vals, t):
    assert infer_spark_type(vals) == t


def test_executor_roundtrip_and_errors(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text("name,age,score\nann,30,1.5\nbob,40,2.5\n")
    ex = SqliteExecutor()
    t = ex.load_csv(str(p))
    assert t.dtypes == [("name", "string"), ("age", "int"), ("score", "double")]
    s = ex.session(t)
    r = s.sql("```sql\nSELECT name, age FROM temp_view WHERE age > 35;\n```")
    assert r.columns == ["name", "age"] and r.rows == [("bob", 40)]
    with pytest.raises(SQLExecutionError) as e:
        s.sql("SELECT nme FROM temp_view")
    assert str(e.value).startswith("[UNRESOLVED_COLUMN.WITH_SUGGESTION] A column or function parameter with name `nme`")
    assert "`temp_view`.`name`" in str(e.value)
    with pytest.raises(SQLExecutionError) as e:
        s.sql("SELECT * FROM taxi")
    assert "[TABLE_OR_VIEW_NOT_FOUND] The table or view `taxi` cannot be found." in str(e.value)
    with pytest.raises(SQLExecutionError) as e:
        s.sql("SELEC * FROM temp_view")
    assert "[PARSE_SYNTAX_ERROR]" in str(e.value)
    assert clean_sql("SELECT 1;;") == "SELECT 1"
    with pytest.raises(SQLExecutionError):
        read_csv(str(tmp_path / "missing.csv"))


def test_eval_harness_metrics_and_summary(capsys):
    answers = {q["nl"]: q["expected_sql"] for q in prompts.EVAL_QUERIES}
    fb = FakeBackend(sql=lambda p, s: answers.get(p, prompts.EVAL_EXPECTED_SQL if "total fare amount" in p else "x"))
    one = evaluate_single(fb.generate, "duckdb-nsql")
    assert one["exact_match"] == 1 and one["edit_distance"] == 0
    res = evaluate_multi(lambda **kw: fb.generate(kw["model"], kw["prompt"], kw["system"], kw["options"]),
                         ["duckdb-nsql"])
    summ = summarize(res, 4)
    assert summ["duckdb-nsql"]["exact_match_rate"] == 100.0 and summ["duckdb-nsql"]["avg_edit_distance"] == 0
    out = capsys.readouterr().out
    assert "Final Evaluation Summary:" in out and "Exact Match Rate: 100.00%" in out
    # the multi-query system prompt (with the reference's trailing comma) was sent verbatim
    assert fb.calls[-1]["system"] == prompts.EVAL_MULTI_SYSTEM


def test_generate_response_is_ollama_shaped():
    r = GenerateResponse(model="m", response="SELECT 1", eval_count=10, eval_duration=2_000_000_000)
    assert r.response == r["response"] == "SELECT 1" and r.tokens_per_second == 5.0


def test_eval_report_structural_checks_and_render():
    """eval.report: the reference's hand-written comparison report (Model_Comparision_Report.docx) generated from a
    harness run -- structural checks made mechanical (text around the statement; the statement compiled against the
    taxi schema) and the report's sections with the published reference numbers beside the measured ones."""
    from llm_based_apache_spark_optimization_amd.eval.report import render, structural_checks

    ok = structural_checks(prompts.EVAL_EXPECTED_SQL)
    assert ok["valid"] and not ok["extra_text"], ok
    chatty = structural_checks("To achieve this, you can use the following query:\n```sql\nSELECT * FROM taxi;\n```")
    assert chatty["valid"] and chatty["extra_text"] and chatty["sql"] == "SELECT * FROM taxi;"
    bad = structural_checks("SELECT V VendortID, SUM(total_amount) FROM taxi GROUP BY VendorID;")
    assert not bad["valid"] and "no such column" in bad["error"], bad  # the reference's llama3.2 error
    assert structural_checks("")["error"] == "no SQL statement"

    answers = {q["nl"]: q["expected_sql"] for q in prompts.EVAL_QUERIES}
    fb = FakeBackend(sql=lambda p, s: answers.get(p, "Sure! SELECT VendorID FROM taxi;"))
    gen = lambda **kw: fb.generate(kw["model"], kw["prompt"], kw["system"], kw["options"])  # noqa: E731
    models = ["mistral", "duckdb-nsql"]
    single = [evaluate_single(gen, m, verbose=False) for m in models]
    assert single[0]["generated_sql"].startswith("Sure!")
    multi = evaluate_multi(gen, models, verbose=False)
    md = render({"single": single, "multi": multi, "summary": summarize(multi, 4, verbose=False),
                 "options": {"num_predict": 8}})
    for section in ("## 1. Setup", "## 3. Results", "### 3.2 Four-query set", "## 4. Analysis", "## 5. Recommendations"):
        assert section in md, section
    assert "extra text around the query" in md and "456 / 53.73 s" in md and "4 / 4" in md
