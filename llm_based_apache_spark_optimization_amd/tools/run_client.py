"""Manual client of the FastAPI service (the counterpart of the reference's ``FastAPI/run.ipynb``,
SURVEY.md C20: one ``requests.post`` of ``{"file_name", "input_text"}`` to ``/process-data/``).

The reference notebook posts empty strings, so Spark ends up reading the whole input *directory*; this
client requires both fields and can also drive the north-star endpoints (``/nl2sql``,
``/explain_error``) and the Ollama-compatible ``/api/generate``.

    python -m llm_based_apache_spark_optimization_amd.tools.run_client process-data Listofstartups.csv "Select 10 records"
    python -m llm_based_apache_spark_optimization_amd.tools.run_client nl2sql "Name (string)\\nAge (int)" "How many rows?"
    python -m llm_based_apache_spark_optimization_amd.tools.run_client explain-error "[UNRESOLVED_COLUMN.WITH_SUGGESTION] ..."
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Any, Optional

DEFAULT_URL = "http://127.0.0.1:8000"


class ApiClient:
    """Thin JSON client.  ``session`` is anything with ``.post(url, json=...)`` returning a response with
    ``.status_code`` and ``.json()`` — an ``httpx.Client`` (default) or a FastAPI ``TestClient``."""

    def __init__(self, base_url: str = DEFAULT_URL, session: Any = None, timeout_s: float = 600.0):
        self.base = base_url.rstrip("/")
        if session is None:
            import httpx

            session = httpx.Client(timeout=timeout_s)
        self.session = session

    def _post(self, path: str, body: dict) -> dict:
        url = path if not self.base else self.base + path
        r = self.session.post(url, json=body)
        if r.status_code != 200:
            raise RuntimeError(f"POST {path} -> HTTP {r.status_code}: {r.text[:500]}")
        return r.json()

    def process_data(self, file_name: str, input_text: str) -> dict:
        if not file_name or not input_text:
            raise ValueError("file_name and input_text are both required")
        return self._post("/process-data/", {"file_name": file_name, "input_text": input_text})

    def nl2sql(self, table_schema: str, question: str) -> dict:
        return self._post("/nl2sql", {"table_schema": table_schema, "question": question})

    def explain_error(self, error_message: str) -> dict:
        return self._post("/explain_error", {"error_message": error_message})

    def generate(self, model: str, prompt: str, system: str = "", options: Optional[dict] = None) -> dict:
        body = {"model": model, "prompt": prompt, "system": system, "stream": False}
        if options:
            body["options"] = options
        return self._post("/api/generate", body)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--url", default=DEFAULT_URL)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("process-data")
    p.add_argument("file_name")
    p.add_argument("input_text")
    p = sub.add_parser("nl2sql")
    p.add_argument("table_schema")
    p.add_argument("question")
    p = sub.add_parser("explain-error")
    p.add_argument("error_message")
    p = sub.add_parser("generate")
    p.add_argument("model")
    p.add_argument("prompt")
    p.add_argument("--system", default="")
    a = ap.parse_args(argv)
    c = ApiClient(a.url)
    if a.cmd == "process-data":
        out = c.process_data(a.file_name, a.input_text)
    elif a.cmd == "nl2sql":
        out = c.nl2sql(a.table_schema.replace("\\n", "\n"), a.question)
    elif a.cmd == "explain-error":
        out = c.explain_error(a.error_message)
    else:
        out = c.generate(a.model, a.prompt, a.system)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
