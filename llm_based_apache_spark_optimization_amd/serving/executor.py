"""SQL execution backends behind the NL->SQL pipeline.

The reference runs the generated SQL on a local PySpark session: ``spark.read.csv(path, header=True,
inferSchema=True)`` (FastAPI/app.py:76, Flask/app.py:95), ``df.dtypes`` for the schema text,
``createOrReplaceTempView("temp_view")`` and ``spark.sql(query)`` (FastAPI/app.py:94-97), and on
success ``coalesce(1).write...csv`` (FastAPI/app.py:122).  Spark errors (``AnalysisException`` etc.)
are stringified and sent to the explain model.

* ``SqliteExecutor`` (default; no JVM needed): Spark-style CSV schema inference (int / bigint /
  double / boolean / date / timestamp / string), a ``temp_view`` table in an in-memory SQLite
  database, and Spark-formatted error messages (``[UNRESOLVED_COLUMN.WITH_SUGGESTION] ...``,
  ``[TABLE_OR_VIEW_NOT_FOUND] ...``, ``[PARSE_SYNTAX_ERROR] ...``) so the explain path sees the same
  kind of text it would get from Spark.
* ``SparkExecutor``: the real thing when ``pyspark`` is installed.
"""
from __future__ import annotations

import csv
import dataclasses
import datetime as _dt
import difflib
import os
import re
import sqlite3
import threading
from typing import Any, List, Optional, Sequence, Tuple


class SQLExecutionError(Exception):
    """An error raised while analysing/executing the SQL (message formatted like Spark's)."""


@dataclasses.dataclass
class Table:
    name: str
    columns: List[str]
    dtypes: List[Tuple[str, str]]
    rows: List[tuple]


@dataclasses.dataclass
class Result:
    columns: List[str]
    rows: List[tuple]


INT_MIN, INT_MAX = -(2 ** 31), 2 ** 31 - 1
_TS_FORMATS = ("%Y-%m-%d %H:%M:%S", "%Y-%m-%dT%H:%M:%S", "%Y-%m-%d %H:%M:%S.%f", "%Y-%m-%dT%H:%M:%S.%f",
               "%Y-%m-%d %H:%M")
_DATE_FORMATS = ("%Y-%m-%d",)


def _is_int(v: str) -> Optional[int]:
    if re.fullmatch(r"[+-]?\d+", v):
        return int(v)
    return None


def _is_double(v: str) -> bool:
    if re.fullmatch(r"[+-]?(inf|infinity|nan)", v.lower()):
        return False
    try:
        float(v)
        return True
    except ValueError:
        return False


def _parse_ts(v: str, fmts) -> Optional[_dt.datetime]:
    for f in fmts:
        try:
            return _dt.datetime.strptime(v, f)
        except ValueError:
            continue
    return None


def infer_spark_type(values: Sequence[str]) -> str:
    """Spark CSV ``inferSchema`` type of a column from its non-empty string values."""
    vals = [v for v in values if v != ""]
    if not vals:
        return "string"
    ints = [_is_int(v) for v in vals]
    if all(i is not None for i in ints):
        return "int" if all(INT_MIN <= i <= INT_MAX for i in ints) else "bigint"
    if all(_is_double(v) for v in vals):
        return "double"
    if all(v.lower() in ("true", "false") for v in vals):
        return "boolean"
    if all(_parse_ts(v, _DATE_FORMATS) for v in vals):
        return "date"
    if all(_parse_ts(v, _TS_FORMATS + _DATE_FORMATS) for v in vals):
        return "timestamp"
    return "string"


def _convert(v: str, t: str) -> Any:
    if v == "":
        return None
    if t in ("int", "bigint"):
        return int(v)
    if t == "double":
        return float(v)
    if t == "boolean":
        return 1 if v.lower() == "true" else 0
    if t == "timestamp":
        ts = _parse_ts(v, _TS_FORMATS + _DATE_FORMATS)
        return ts.strftime("%Y-%m-%d %H:%M:%S") if ts else v
    return v


_SQLITE_TYPE = {"int": "INTEGER", "bigint": "INTEGER", "double": "REAL", "boolean": "INTEGER", "date": "TEXT",
                "timestamp": "TEXT", "string": "TEXT"}


def _q(name: str) -> str:
    return '"' + name.replace('"', '""') + '"'


def read_csv(path: str, name: str = "temp_view") -> Table:
    """CSV with a header row -> Table with Spark-inferred dtypes (a directory reads every *.csv in it,
    like ``spark.read.csv(dir)``)."""
    files = [path]
    if os.path.isdir(path):
        files = sorted(os.path.join(path, f) for f in os.listdir(path) if f.lower().endswith(".csv"))
        if not files:
            raise SQLExecutionError(f"[PATH_NOT_FOUND] Path does not exist: file:{path}.")
    if not os.path.exists(files[0]):
        raise SQLExecutionError(f"[PATH_NOT_FOUND] Path does not exist: file:{path}.")
    header, raw = None, []
    for fn in files:
        with open(fn, newline="", encoding="utf-8-sig") as f:
            rd = csv.reader(f)
            h = next(rd, None)
            if h is None:
                continue
            header = header or h
            raw.extend(r + [""] * (len(header) - len(r)) if len(r) < len(header) else r[: len(header)] for r in rd)
    if header is None:
        return Table(name, [], [], [])
    cols = [c if c else f"_c{i}" for i, c in enumerate(header)]
    types = [infer_spark_type([r[i] for r in raw]) for i in range(len(cols))]
    rows = [tuple(_convert(r[i], types[i]) for i in range(len(cols))) for r in raw]
    return Table(name, cols, list(zip(cols, types)), rows)


class SqliteExecutor:
    """Spark-SQL-flavoured execution on SQLite (thread-safe; one connection per request)."""

    name = "sqlite"

    def __init__(self):
        self._lock = threading.Lock()

    def load_csv(self, path: str) -> Table:
        return read_csv(path)

    def session(self, table: Table, view: str = "temp_view") -> "SqliteSession":
        return SqliteSession(table, view)

    @staticmethod
    def table_of(loaded) -> Table:
        return loaded


class SqliteSession:
    def __init__(self, table: Table, view: str = "temp_view"):
        self.table, self.view = table, view
        self.conn = sqlite3.connect(":memory:", check_same_thread=False)
        cols = ", ".join(f"{_q(c)} {_SQLITE_TYPE[t]}" for c, t in table.dtypes)
        self.conn.execute(f"CREATE TABLE {_q(view)} ({cols})")
        if table.rows:
            ph = ", ".join("?" for _ in table.columns)
            self.conn.executemany(f"INSERT INTO {_q(view)} VALUES ({ph})", table.rows)

    def sql(self, query: str) -> Result:
        q = clean_sql(query)
        try:
            cur = self.conn.execute(q)
            cols = [d[0] for d in (cur.description or [])]
            return Result(cols, cur.fetchall())
        except sqlite3.Error as e:
            raise SQLExecutionError(spark_style_error(str(e), q, self.table, self.view)) from None

    def close(self) -> None:
        self.conn.close()


def clean_sql(text: str) -> str:
    """Strip markdown fences and trailing semicolons the way Spark's parser tolerates them."""
    t = text.strip()
    m = re.search(r"```(?:sql)?\s*(.*?)```", t, re.S | re.I)
    if m:
        t = m.group(1).strip()
    while t.endswith(";"):
        t = t[:-1].rstrip()
    return t


def _pos_of(token: str, q: str) -> int:
    i = q.find(token)
    return max(0, i)


def spark_style_error(msg: str, query: str, table: Table, view: str) -> str:
    """Translate a SQLite error into Spark's error-class message format."""
    m = re.search(r"no such column: (\S+)", msg)
    if m:
        col = m.group(1).split(".")[-1].strip('"`')
        cands = [f"`{view}`.`{c}`" for c in table.columns]
        close = difflib.get_close_matches(col, table.columns, n=5, cutoff=0.0)
        sugg = ", ".join(f"`{view}`.`{c}`" for c in close) or ", ".join(cands[:5])
        return (f"[UNRESOLVED_COLUMN.WITH_SUGGESTION] A column or function parameter with name `{col}` cannot be "
                f"resolved. Did you mean one of the following? [{sugg}].; line 1 pos {_pos_of(col, query)};\n"
                f"'Project [*]\n+- SubqueryAlias {view}\n   +- View (`{view}`, [{', '.join(table.columns)}])")
    m = re.search(r"no such table: (\S+)", msg)
    if m:
        t = m.group(1).strip('"`')
        return (f"[TABLE_OR_VIEW_NOT_FOUND] The table or view `{t}` cannot be found. Verify the spelling and "
                f"correctness of the schema and catalog.\nIf you did not qualify the name with a schema, verify the "
                f"current_schema() output, or qualify the name with the correct schema and catalog.; line 1 pos "
                f"{_pos_of(t, query)};")
    m = re.search(r'near "([^"]*)": syntax error', msg)
    if m or "syntax error" in msg or "incomplete input" in msg:
        tok = m.group(1) if m else "end of input"
        return f"\n[PARSE_SYNTAX_ERROR] Syntax error at or near '{tok}'.(line 1, pos {_pos_of(tok, query)})\n\n== SQL ==\n{query}\n"
    m = re.search(r"no such function: (\S+)", msg)
    if m:
        fn = m.group(1)
        return (f"[UNRESOLVED_ROUTINE] Cannot resolve function `{fn}` on search path [`system`.`builtin`, "
                f"`system`.`session`, `spark_catalog`.`default`].; line 1 pos {_pos_of(fn, query)}")
    return f"[INTERNAL_ERROR] {msg}"


def write_csv(result: Result, path: str) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(result.columns)
        w.writerows(result.rows)
    return path


class SparkExecutor:
    """The reference's backend: a process-wide SparkSession in local mode (FastAPI/app.py:19,
    Flask/app.py:16).

    The reference registered every upload as the global view ``temp_view`` on that one session
    (FastAPI/app.py:94, Flask/app.py:111), so two concurrent requests replaced each other's view and a
    query could run against another user's CSV.  Here each request gets its own
    ``spark.newSession()``: sessions share the SparkContext (and its executors) but not the temp-view
    catalog, so every request sees exactly its own ``temp_view``.  The view is dropped on ``close()``.
    ``spark`` may be injected (tests use a fake session object; pyspark is optional)."""

    name = "spark"

    def __init__(self, app_name: str = "LSA-Spark", spark=None):
        if spark is None:  # pragma: no cover - needs pyspark + a JVM
            from pyspark.sql import SparkSession

            spark = SparkSession.builder.appName(app_name).getOrCreate()
        self.spark = spark

    def load_csv(self, path: str):
        sess = self.spark.newSession()  # request-private temp-view catalog (shared SparkContext)
        df = sess.read.csv(path, header=True, inferSchema=True)
        return Table("temp_view", list(df.columns), list(df.dtypes), []), df, sess

    @staticmethod
    def table_of(loaded) -> Table:
        return loaded[0]

    def session(self, loaded, view: str = "temp_view"):
        table, df, spark = loaded
        df.createOrReplaceTempView(view)  # registers in the request's own session only

        class _S:
            def __init__(self):
                self.table = table
                self.spark = spark

            def sql(self, q):
                try:
                    out = spark.sql(q)
                    return Result(list(out.columns), [tuple(r) for r in out.collect()])
                except Exception as e:  # noqa: BLE001
                    raise SQLExecutionError(str(e)) from None

            def close(self):
                try:
                    spark.catalog.dropTempView(view)
                except Exception:  # noqa: BLE001 - best effort
                    pass

        return _S()


def make_executor(kind: str = "sqlite"):
    if kind == "spark":
        return SparkExecutor()
    return SqliteExecutor()
