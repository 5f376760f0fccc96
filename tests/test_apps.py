"""Contract tests of the FastAPI and Flask apps with the deterministic fake model backend, the SQLite
executor and a SQLite history store."""
import io
import json
import os
import threading

import pytest

from llm_based_apache_spark_optimization_amd import prompts
from llm_based_apache_spark_optimization_amd.client import FakeBackend
from llm_based_apache_spark_optimization_amd.config import Settings
from llm_based_apache_spark_optimization_amd.serving.history import HistoryStore
from llm_based_apache_spark_optimization_amd.serving.service import make_context

CSV = "Incubation_Center,Name_of_startup,Location of company,Sector,Funding\nA,Alpha,Pune,AI,100\nB,Beta,Delhi,EdTech,250\nC,Gamma,Pune,AI,75\n"


@pytest.fixture
def ctx(tmp_path):
    s = Settings(input_dir=str(tmp_path / "in"), output_dir=str(tmp_path / "out"),
                 history_dsn="sqlite:///" + str(tmp_path / "h.db"), engine="fake", secret_key="test")
    s.ensure_dirs()
    with open(os.path.join(s.input_dir, "Listofstartups.csv"), "w") as f:
        f.write(CSV)
    return make_context(s, backend=FakeBackend())


# ----------------------------------------------------------------------------------- FastAPI
@pytest.fixture
def api(ctx):
    from fastapi.testclient import TestClient

    from llm_based_apache_spark_optimization_amd.serving.fastapi_app import create_app

    return TestClient(create_app(ctx))


def test_fastapi_success(api, ctx):
    r = api.post("/process-data/", json={"input_text": "Select 10 records", "file_name": "Listofstartups.csv"})
    assert r.status_code == 200
    d = r.json()
    assert d["message"] == "Query executed successfully!"
    assert d["sql_query"] == "SELECT * FROM temp_view LIMIT 10;"
    assert d["input_file_name"] == "Listofstartups.csv" and d["input_data"] == "Select 10 records"
    assert d["output_file"].endswith("_Listofstartups.csv.csv") and os.path.exists(d["output_file"])
    with open(d["output_file"]) as f:
        assert f.readline().startswith("Incubation_Center,Name_of_startup")
    # the NL->SQL call used the reference's exact system prompt
    call = ctx.backend.calls[0]
    assert call["model"] == "duckdb-nsql"
    assert call["system"] == ("Table name is temp_view. The structure of the table is:\nIncubation_Center (string)\n"
                              "Name_of_startup (string)\nLocation of company (string)\nSector (string)\nFunding (int)")
    recs, has_next = ctx.history.page(1)
    assert recs[0]["sql_query"] == d["sql_query"] and not has_next


def test_fastapi_missing_file(api, ctx):
    r = api.post("/process-data/", json={"input_text": "x", "file_name": "nope.csv"})
    assert r.status_code == 200
    assert r.json() == {"error": "CSV file not found at " + os.path.join(ctx.settings.input_dir, "nope.csv")}


def test_fastapi_sql_error_explained(api, ctx):
    ctx.backend.sql = lambda p, s: "SELECT * FROM temp_view WHERE name = 'abc';"
    r = api.post("/process-data/", json={"input_text": "find abc", "file_name": "Listofstartups.csv"})
    d = r.json()
    assert d["error"] == "SQL execution failed"
    assert d["sql_query"] == "SELECT * FROM temp_view WHERE name = 'abc';"
    assert d["error_details"] == ctx.backend.explanation
    explain_call = ctx.backend.calls[-1]
    assert explain_call["model"] == "llama3.2" and explain_call["system"] == prompts.EXPLAIN_SYSTEM
    assert explain_call["prompt"].startswith("The following Spark error occurred:\n\n[UNRESOLVED_COLUMN.WITH_SUGGESTION]")
    assert explain_call["prompt"].endswith("\n\nPlease analyze this error and suggest possible solutions.")


def test_fastapi_nl2sql_and_explain(api):
    r = api.post("/nl2sql", json={"table_schema": "a (int)", "question": "all rows"})
    assert r.json()["sql_query"] == "SELECT * FROM temp_view LIMIT 10;"
    r = api.post("/nl2sql", json={"file_name": "Listofstartups.csv", "question": "all rows"})
    assert "Funding (int)" in r.json()["table_schema"]
    r = api.post("/explain_error", json={"error_message": "[TABLE_OR_VIEW_NOT_FOUND] x"})
    assert "column" in r.json()["explanation"]
    assert api.post("/nl2sql", json={"question": "q"}).status_code == 422


def test_fastapi_ollama_api_and_ops(api):
    r = api.post("/api/generate", json={"model": "duckdb-nsql", "prompt": "q", "system": "s"})
    d = r.json()
    assert d["response"] and d["done"] is True and "eval_count" in d
    r = api.post("/api/generate", json={"model": "duckdb-nsql", "prompt": "q", "stream": True})
    lines = [json.loads(x) for x in r.text.splitlines() if x.strip()]
    assert r.headers["content-type"].startswith("application/x-ndjson") and lines[-1]["done"] is True
    assert all(x["done"] is False for x in lines[:-1]) and lines[-1]["response"] == ""
    assert "".join(x["response"] for x in lines) == d["response"] and "eval_count" in lines[-1]
    assert any(m["name"] == "llama3.2" for m in api.get("/api/tags").json()["models"])
    assert api.get("/health").json()["ok"] is True
    api.post("/nl2sql", json={"table_schema": "a (int)", "question": "all rows"})
    m = api.get("/metrics").text
    assert "lsa_requests_total" in m and "lsa_stage_seconds_bucket" in m


def test_fastapi_concurrent_requests_do_not_clobber(api, ctx):
    outs = []

    def go(i):
        r = api.post("/process-data/", json={"input_text": f"q{i}", "file_name": "Listofstartups.csv"})
        outs.append(r.json()["output_file"])

    ts = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert len(set(outs)) == 6 and all(os.path.exists(o) for o in outs)


def test_engine_failure_is_explained_not_500(api, ctx):
    ctx.backend.fail_next = RuntimeError("engine replica died")
    r = api.post("/process-data/", json={"input_text": "q", "file_name": "Listofstartups.csv"})
    d = r.json()
    assert r.status_code == 200 and d["error"] == "SQL execution failed"
    assert d["error_details"] == ctx.backend.explanation


# ----------------------------------------------------------------------------------- Flask
@pytest.fixture
def web(ctx):
    from llm_based_apache_spark_optimization_amd.serving.flask_app import create_app

    app = create_app(ctx)
    app.testing = True
    return app.test_client()


def _upload(web, text, job=None, name="Listofstartups.csv"):
    data = {"file_name": (io.BytesIO(CSV.encode()), name), "input_text": text}
    if job:
        data["job"] = job
    return web.post("/process-data/", data=data, content_type="multipart/form-data")


def test_flask_home_and_success_flow(web, ctx):
    assert b"AI powered SparkSQL Studio" in web.get("/").data
    r = _upload(web, "Select 10 records", job="abc123")
    assert r.json == {"redirect": "/show"}
    st = web.get("/status?job=abc123").json
    assert st["status"] == "done" and st["redirect"] == "/show"
    page = web.get("/show").data.decode()
    assert "SELECT * FROM temp_view LIMIT 10;" in page and "Listofstartups.csv" in page
    recs, _ = ctx.history.page(1)
    assert recs[0]["output_file"].endswith("_Listofstartups.csv")  # basename persisted (Flask/app.py:133)


def test_flask_status_sequence(web, ctx):
    seen = []
    orig = ctx.status.update

    def spy(job, message, status="running", **kw):
        seen.append(message)
        return orig(job, message, status, **kw)

    ctx.status.update = spy
    _upload(web, "Select 10 records", job="j1")
    assert seen[:7] == ["Uploading file...", "CSV file loading into Spark.", "Generating SQL query...",
                        "SQL query generated successfully.", "Executing query in Spark...",
                        "Saving results to CSV...", "Saving results to MySQL..."]


def test_flask_error_flow(web, ctx):
    ctx.backend.sql = lambda p, s: "SELECT nosuchcol FROM temp_view"
    r = _upload(web, "bad", job="e1")
    target = r.json["redirect"]
    assert target.startswith("/err_sol?")
    page = web.get(target).data.decode()
    assert "UNRESOLVED_COLUMN" in page and "Suggested Solution" in page and "nosuchcol" in page
    assert web.get("/status?job=e1").json["message"] == "Error resolved"


def test_flask_history_pagination(web, ctx):
    for i in range(11):
        ctx.history.insert(f"f{i}.csv", f"q{i}", f"SELECT {i}", f"o{i}.csv")
    p1 = web.get("/history").data.decode()
    assert "q10" in p1 and "q3" in p1 and "q2" not in p1 and "Next" in p1  # 8 per page, newest first
    p2 = web.get("/history?page=2").data.decode()
    assert "q2" in p2 and "q0" in p2 and "Next" not in p2 and "Prev" in p2


def test_history_store_sqlite_contract(tmp_path):
    h = HistoryStore("sqlite:///" + str(tmp_path / "x.db"))
    assert h.page(1) == ([], False)
    h.insert("a.csv", "q", "SELECT 1", "o.csv")
    recs, nxt = h.page(1, 8)
    assert set(recs[0]) == {"id", "input_file_name", "input_data", "sql_query", "output_file"} and not nxt


def test_run_client_against_app(api, ctx):
    """The manual client (reference FastAPI/run.ipynb, C20) drives every JSON endpoint."""
    from llm_based_apache_spark_optimization_amd.tools.run_client import ApiClient

    c = ApiClient(base_url="", session=api)
    d = c.process_data("Listofstartups.csv", "Select 10 records")
    assert d["message"] == "Query executed successfully!"
    assert c.nl2sql("Name (string)\nAge (int)", "Select 10 records")["sql_query"].startswith("SELECT")
    assert c.explain_error("[UNRESOLVED_COLUMN.WITH_SUGGESTION] x")["explanation"]
    assert c.generate("duckdb-nsql", "Select 10 records", "T (int)")["response"].startswith("SELECT")
    with pytest.raises(ValueError):
        c.process_data("", "")  # the notebook's empty payload is rejected client-side


def test_explain_error_without_num_predict_is_not_truncated(tmp_path):
    """The reference's option-less ollama.generate call (FastAPI/app.py:105-109) generates until EOS or the
    context window; a served /explain_error without num_predict must not stop at a fixed cap (it used to
    be cut at 256 tokens).  Tiny Llama-3 engine on CPU with EOS disabled: the answer runs to the window."""
    from fastapi.testclient import TestClient

    from llm_based_apache_spark_optimization_amd.client import EngineService
    from llm_based_apache_spark_optimization_amd.engine import build_engine
    from llm_based_apache_spark_optimization_amd.serving.fastapi_app import create_app

    s = Settings(input_dir=str(tmp_path / "in"), output_dir=str(tmp_path / "out"),
                 history_dsn="sqlite:///" + str(tmp_path / "h.db"), engine="hip", secret_key="test",
                 explain_model="tiny-llama3", nl2sql_model="tiny-nsql")
    assert s.max_new_tokens < 0  # the service default is Ollama's: no num_predict

    def factory(model):
        eng = build_engine(model, device="cpu", max_slots=2, max_model_len=1024)
        eng.runner.set_eos([-1])  # random weights: never stop early, so the length is the window's
        return eng

    svc = EngineService(factory, defaults={"temperature": 0.0, "num_predict": s.max_new_tokens})
    try:
        api = TestClient(create_app(make_context(s, backend=svc)))
        r = api.post("/explain_error", json={"error_message": "[UNRESOLVED_COLUMN.WITH_SUGGESTION] A column "
                                                               "with name `Locaton` cannot be resolved."})
        assert r.status_code == 200, r.text
        body = r.json()
        assert body["eval_count"] > 256
        assert body["eval_count"] + body["prompt_eval_count"] == 1024  # stopped by the context window only
    finally:
        svc.loop("tiny-llama3").close()
