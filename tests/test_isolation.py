"""Request isolation and input hardening (SURVEY.md §5 race detection / security):

* FastAPI ``file_name`` cannot leave the configured input directory (absolute paths, ``..``, symlinks);
* the Spark backend registers each request's ``temp_view`` in a private ``newSession()`` so concurrent
  requests never see each other's CSV (the reference shared one global view: FastAPI/app.py:19,94).
pyspark is not importable here, so the Spark path runs against a fake session object with the same
surface (``newSession``, ``read.csv``, ``createOrReplaceTempView``, ``sql``, ``catalog.dropTempView``).
"""
import os
import threading

import pytest

from llm_based_apache_spark_optimization_amd.client import FakeBackend
from llm_based_apache_spark_optimization_amd.config import Settings
from llm_based_apache_spark_optimization_amd.serving.executor import SparkExecutor
from llm_based_apache_spark_optimization_amd.serving.pipeline import resolve_input
from llm_based_apache_spark_optimization_amd.serving.service import make_context

CSV = "Name,Age\nAda,36\nBob,41\n"


@pytest.fixture
def ctx(tmp_path):
    s = Settings(input_dir=str(tmp_path / "in"), output_dir=str(tmp_path / "out"),
                 history_dsn="sqlite:///" + str(tmp_path / "h.db"), engine="fake", secret_key="test")
    s.ensure_dirs()
    with open(os.path.join(s.input_dir, "people.csv"), "w") as f:
        f.write(CSV)
    with open(tmp_path / "secret.csv", "w") as f:
        f.write("token\nhunter2\n")
    return make_context(s, backend=FakeBackend())


@pytest.fixture
def api(ctx):
    from fastapi.testclient import TestClient

    from llm_based_apache_spark_optimization_amd.serving.fastapi_app import create_app

    return TestClient(create_app(ctx))


def test_resolve_input(tmp_path):
    root = tmp_path / "in"
    (root / "sub").mkdir(parents=True)
    (root / "sub" / "a.csv").write_text("x\n1\n")
    os.symlink(tmp_path, root / "escape")
    assert resolve_input(str(root), "sub/a.csv") == os.path.realpath(root / "sub" / "a.csv")
    for bad in ("/etc/passwd", "../secret.csv", "sub/../../secret.csv", "escape/secret.csv", "", ".", "a\x00b"):
        assert resolve_input(str(root), bad) is None, bad


@pytest.mark.parametrize("name", ["/etc/passwd", "../secret.csv", "../../../../etc/passwd"])
def test_process_data_rejects_traversal(api, ctx, name):
    r = api.post("/process-data/", json={"input_text": "Select 10 records", "file_name": name})
    assert r.status_code == 200 and r.json()["error"].startswith("Invalid file name")
    assert ctx.backend.calls == []  # nothing outside input_dir was read, no LLM call made


@pytest.mark.parametrize("name", ["/etc/passwd", "../secret.csv"])
def test_nl2sql_rejects_traversal(api, ctx, name):
    r = api.post("/nl2sql", json={"question": "everything", "file_name": name})
    assert r.status_code == 400
    assert "hunter2" not in r.text and "root:" not in r.text
    assert ctx.backend.calls == []


def test_process_data_inside_input_dir_still_works(api):
    r = api.post("/process-data/", json={"input_text": "Select 10 records", "file_name": "people.csv"})
    d = r.json()
    assert d["message"] == "Query executed successfully!" and d["output_file"].endswith("_people.csv.csv")


# ----------------------------------------------------------------------------------- fake Spark
class _FakeDF:
    def __init__(self, session, rows, columns):
        self.session, self.rows, self.columns = session, rows, columns
        self.dtypes = [(c, "string") for c in columns]

    def createOrReplaceTempView(self, name):
        self.session.views[name] = self

    def collect(self):
        return self.rows


class _FakeCatalog:
    def __init__(self, session):
        self.session = session

    def dropTempView(self, name):
        self.session.views.pop(name, None)


class _FakeReader:
    def __init__(self, session):
        self.session = session

    def csv(self, path, header=True, inferSchema=True):
        with open(path) as f:
            lines = [ln.strip().split(",") for ln in f if ln.strip()]
        return _FakeDF(self.session, [tuple(r) for r in lines[1:]], lines[0])


class FakeSparkSession:
    """Per-session temp-view catalog, like SparkSession: views registered in one session are
    invisible to its siblings from newSession()."""

    def __init__(self, barrier=None):
        self.views = {}
        self.read = _FakeReader(self)
        self.catalog = _FakeCatalog(self)
        self.children = []
        self.barrier = barrier

    def newSession(self):
        s = FakeSparkSession(self.barrier)
        self.children.append(s)
        return s

    def sql(self, q):
        if self.barrier is not None:
            self.barrier.wait(timeout=10)  # both requests have registered their view before either queries
        name = q.split("FROM")[1].split()[0].strip(";")
        if name not in self.views:
            raise RuntimeError(f"[TABLE_OR_VIEW_NOT_FOUND] The table or view `{name}` cannot be found.")
        return self.views[name]


def test_spark_sessions_isolate_concurrent_requests(tmp_path):
    root = FakeSparkSession(threading.Barrier(2))
    ex = SparkExecutor(spark=root)
    paths = []
    for i, body in enumerate(("Name\nAda\n", "Name\nBob\n")):
        p = tmp_path / f"u{i}.csv"
        p.write_text(body)
        paths.append(str(p))
    out = [None, None]

    def job(i):
        sess = ex.session(ex.load_csv(paths[i]))
        out[i] = sess.sql("SELECT * FROM temp_view")
        sess.close()

    ts = [threading.Thread(target=job, args=(i,)) for i in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert out[0].rows == [("Ada",)] and out[1].rows == [("Bob",)]
    assert root.views == {}  # nothing registered on the shared session
    assert all(c.views == {} for c in root.children)  # dropped on close


def test_spark_errors_are_sql_errors(tmp_path):
    from llm_based_apache_spark_optimization_amd.serving.executor import SQLExecutionError

    ex = SparkExecutor(spark=FakeSparkSession())
    p = tmp_path / "x.csv"
    p.write_text("a\n1\n")
    sess = ex.session(ex.load_csv(str(p)))
    with pytest.raises(SQLExecutionError, match="TABLE_OR_VIEW_NOT_FOUND"):
        sess.sql("SELECT * FROM other_view")
