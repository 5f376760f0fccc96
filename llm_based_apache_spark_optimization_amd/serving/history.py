"""Query-history store (the reference's MySQL ``query_results`` table).

Schema (inferred from FastAPI/app.py:40-43, Flask/app.py:218, hist.html:24-27):
``query_results(id auto-increment PK, input_file_name, input_data, sql_query, output_file)``.
Backends: SQLite (default, ``sqlite:///path``) and MySQL (``mysql://user:pw@host[:port]/db`` when
``mysql.connector`` is importable).  Unlike the reference, a failing store never raises into the
request (FastAPI/app.py:50-51 only printed) and cursors are always bound before ``finally``
(the Flask UnboundLocalError of Flask/app.py:46-50,229-233 is fixed).
"""
from __future__ import annotations

import logging
import re
import sqlite3
import threading
from typing import Optional

log = logging.getLogger(__name__)

_DDL_SQLITE = """CREATE TABLE IF NOT EXISTS query_results (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    input_file_name TEXT, input_data TEXT, sql_query TEXT, output_file TEXT)"""
_DDL_MYSQL = """CREATE TABLE IF NOT EXISTS query_results (
    id INT AUTO_INCREMENT PRIMARY KEY,
    input_file_name TEXT, input_data TEXT, sql_query TEXT, output_file TEXT)"""


class HistoryStore:
    def __init__(self, dsn: str = "sqlite:///:memory:"):
        self.dsn = dsn
        self._lock = threading.Lock()
        if dsn.startswith("sqlite:///"):
            self.kind = "sqlite"
            path = dsn[len("sqlite:///"):] or ":memory:"
            self._conn = sqlite3.connect(path, check_same_thread=False)
            self._conn.execute(_DDL_SQLITE)
            self._conn.commit()
            self._ph = "?"
        elif dsn.startswith("mysql://"):
            self.kind = "mysql"
            m = re.match(r"mysql://([^:@/]+)(?::([^@/]*))?@([^:/]+)(?::(\d+))?/(\w+)", dsn)
            if not m:
                raise ValueError(f"bad mysql dsn {dsn!r}")
            self._mysql = dict(user=m.group(1), password=m.group(2) or "", host=m.group(3),
                               port=int(m.group(4) or 3306), database=m.group(5))
            self._ph = "%s"
            with self._cursor() as (conn, cur):
                cur.execute(_DDL_MYSQL)
                conn.commit()
        else:
            raise ValueError(f"unsupported history dsn {dsn!r}")

    # -------------------------------------------------------------------------------- plumbing
    class _Ctx:
        def __init__(self, store):
            self.s = store
            self.conn = self.cur = None

        def __enter__(self):
            import mysql.connector  # noqa: F401 - optional dependency

            self.conn = mysql.connector.connect(**self.s._mysql)
            self.cur = self.conn.cursor(dictionary=True)
            return self.conn, self.cur

        def __exit__(self, *exc):
            if self.cur is not None:
                self.cur.close()
            if self.conn is not None:
                self.conn.close()
            return False

    def _cursor(self):
        return HistoryStore._Ctx(self)

    # -------------------------------------------------------------------------------- API
    def insert(self, input_file_name: str, input_data: str, sql_query: str, output_file: str) -> Optional[int]:
        q = (f"INSERT INTO query_results (input_file_name, input_data, sql_query, output_file) "
             f"VALUES ({self._ph}, {self._ph}, {self._ph}, {self._ph})")
        vals = (input_file_name, input_data, sql_query, output_file)
        try:
            if self.kind == "sqlite":
                with self._lock:
                    cur = self._conn.execute(q, vals)
                    self._conn.commit()
                    return cur.lastrowid
            with self._cursor() as (conn, cur):
                cur.execute(q, vals)
                conn.commit()
                return cur.lastrowid
        except Exception as e:  # noqa: BLE001 - history must never fail the request
            log.error("history insert failed: %s", e)
            return None

    def count(self) -> int:
        try:
            if self.kind == "sqlite":
                with self._lock:
                    return int(self._conn.execute("SELECT COUNT(*) FROM query_results").fetchone()[0])
            with self._cursor() as (_, cur):
                cur.execute("SELECT COUNT(*) as total FROM query_results")
                return int(cur.fetchone()["total"])
        except Exception as e:  # noqa: BLE001
            log.error("history count failed: %s", e)
            return 0

    def page(self, page: int = 1, limit: int = 8) -> tuple[list, bool]:
        """Records ``ORDER BY id DESC LIMIT limit OFFSET (page-1)*limit`` and whether a next page exists."""
        page = max(1, int(page))
        off = (page - 1) * limit
        q = f"SELECT * FROM query_results ORDER BY id DESC LIMIT {self._ph} OFFSET {self._ph}"
        try:
            if self.kind == "sqlite":
                with self._lock:
                    cur = self._conn.execute(q, (limit, off))
                    cols = [d[0] for d in cur.description]
                    recs = [dict(zip(cols, r)) for r in cur.fetchall()]
            else:
                with self._cursor() as (_, cur):
                    cur.execute(q, (limit, off))
                    recs = list(cur.fetchall())
        except Exception as e:  # noqa: BLE001
            log.error("history page failed: %s", e)
            return [], False
        return recs, (page * limit) < self.count()
