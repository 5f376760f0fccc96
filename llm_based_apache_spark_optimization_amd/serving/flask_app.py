"""Flask web UI (the reference's Flask/app.py surface).

Routes and contracts kept from the reference:

* ``GET /``                upload form (fields ``file_name`` = CSV file, ``input_text`` = question)
* ``POST /process-data/``  multipart upload -> pipeline -> ``{"redirect": "/show"}`` or
                           ``{"redirect": "/err_sol?file_name=..&table_schema=..&sql_query=..&error_message=..&err=.."}``
* ``GET /status``          ``{"status": idle|running|done, "message": ...}`` — per request when the page
                           sends ``?job=<id>`` (its own id, posted as the ``job`` form field), else the
                           most recent request; once done it also carries ``redirect`` (the reference's
                           page expected it but the server never sent it, Flask/templates/index.html:78-83)
* ``GET /err_sol``         error + suggested-solution page from the query string
* ``GET /show``            result page from ``session["result"]``
* ``GET /history?page=N``  8 rows per page, ``ORDER BY id DESC`` (Flask/app.py:214-224)

Additions: ``POST /nl2sql``, ``POST /explain_error`` (JSON), ``GET /metrics``, ``GET /health``.
Fixed reference bugs: per-request status/ids, unique upload + output names per request (no
clobbering), no Windows-path rewrite of the output path (Flask/app.py:135-136), secret from settings.
"""
from __future__ import annotations

import os
import time
from typing import Optional
from urllib.parse import urlencode

from flask import Flask, jsonify, render_template, request, session, url_for
from werkzeug.utils import secure_filename

from .. import prompts
from ..client import EngineUnavailable
from ..utils.metrics import REGISTRY
from ..utils.tracing import new_request_id
from .pipeline import ST_UPLOAD, unique_path
from .service import AppContext, make_context

HERE = os.path.dirname(os.path.abspath(__file__))


def create_app(ctx: Optional[AppContext] = None) -> Flask:
    ctx = ctx or make_context()
    s = ctx.settings
    app = Flask(__name__, template_folder=os.path.join(HERE, "templates"), static_folder=os.path.join(HERE, "static"))
    app.secret_key = s.secret_key
    app.config["LSA_CTX"] = ctx

    @app.errorhandler(EngineUnavailable)
    def engine_down(exc):  # a dead engine answers at once instead of after the request timeout
        return jsonify({"error": "engine unavailable", "detail": str(exc)}), 503

    @app.after_request
    def cors(resp):  # the reference enabled CORS for every origin (Flask/app.py:13)
        resp.headers.setdefault("Access-Control-Allow-Origin", "*")
        return resp

    @app.route("/")
    def home():
        return render_template("studio.html")

    @app.route("/status")
    def get_status():
        return jsonify(ctx.status.get(request.args.get("job")))

    @app.route("/process-data/", methods=["POST"])
    def process_data():
        t0 = time.perf_counter()
        job = request.form.get("job") or new_request_id()
        ctx.status.update(job, ST_UPLOAD)
        upload = request.files.get("file_name")
        input_text = request.form.get("input_text", "")
        fname = secure_filename(upload.filename) if upload is not None and upload.filename else ""
        if not fname:
            err = "No CSV file was uploaded (form field 'file_name')."
            try:  # like the reference, every failure is routed to the explain model
                expl = ctx.pipeline.explain(err).response
            except Exception as e:  # noqa: BLE001
                expl = f"(explanation unavailable: {e})"
            target = url_for("err_sol", file_name="", table_schema="", sql_query="", error_message=err, err=expl)
            ctx.status.update(job, "Error resolved", status="done", redirect=target)
            return jsonify({"redirect": target})
        # unique per request: concurrent uploads of the same name never overwrite each other
        path = unique_path(os.path.join(s.input_dir, fname))
        upload.save(path)
        res = ctx.pipeline.run(path, fname, input_text, output_name=lambda ts: f"{ts}_{fname}", job=job,
                               history_name=os.path.basename)
        REGISTRY.observe("lsa_request_seconds", time.perf_counter() - t0, "e2e latency", route="flask-process")
        if res.ok:
            session["result"] = {"input_file_name": fname, "input_text": input_text, "sql_query": res.sql_query,
                                 "output_file": res.output_file}
            target = url_for("show_result")
        else:
            target = url_for("err_sol", file_name=fname, table_schema=res.table_schema, sql_query=res.sql_query,
                             error_message=res.error_message, err=res.explanation)
        ctx.status.update(job, ctx.status.get(job).get("message", ""), status="done", redirect=target)
        return jsonify({"redirect": target})

    @app.route("/err_sol")
    def err_sol():
        a = request.args
        return render_template("error_solution.html", error_message=a.get("error_message", "Unknown error"),
                               err=a.get("err", "No solution available"), file_name=a.get("file_name", "Unknown"),
                               table_schema=a.get("table_schema", "Unknown"), sql_query=a.get("sql_query", "Unknown"))

    @app.route("/show")
    def show_result():
        return render_template("result.html", result=session.get("result", {}))

    @app.route("/history")
    def history():
        try:
            page = max(1, int(request.args.get("page", 1)))
        except ValueError:
            page = 1
        records, has_next = ctx.history.page(page, s.history_page_size)
        return render_template("history.html", records=records, page=page, has_next=has_next)

    @app.route("/nl2sql", methods=["POST"])
    def nl2sql():
        d = request.get_json(force=True, silent=True) or {}
        q = d.get("question") or d.get("input_text")
        schema = d.get("table_schema") or d.get("schema_text")
        if not q or schema is None:
            return jsonify({"error": "question and table_schema are required"}), 422
        r = ctx.pipeline.nl2sql(schema, q, d.get("options"))
        return jsonify({"sql_query": r.response, "model": r.model, "eval_count": r.eval_count,
                        "eval_duration": r.eval_duration})

    @app.route("/explain_error", methods=["POST"])
    def explain_error():
        d = request.get_json(force=True, silent=True) or {}
        if not d.get("error_message"):
            return jsonify({"error": "error_message is required"}), 422
        r = ctx.pipeline.explain(d["error_message"], d.get("options"))
        return jsonify({"explanation": r.response, "model": r.model, "eval_count": r.eval_count,
                        "eval_duration": r.eval_duration})

    @app.route("/metrics")
    def metrics():
        from .fastapi_app import export_backend_gauges

        export_backend_gauges(ctx.backend)
        return REGISTRY.render(), 200, {"Content-Type": "text/plain; version=0.0.4"}

    @app.route("/health")
    def health():
        return jsonify(ctx.backend.health())

    # keep the helper importable for templates/tests
    app.jinja_env.globals["schema_prompt"] = prompts.nl2sql_system
    app.jinja_env.globals["urlencode"] = urlencode
    return app


def main(argv=None) -> None:  # pragma: no cover - server entry point
    import argparse

    from ..config import Settings
    from ..utils import setup_logging

    ap = argparse.ArgumentParser(description="Flask web UI for the MI355X NL->SQL service")
    Settings.add_cli(ap)
    settings = Settings.from_cli(ap.parse_args(argv))
    setup_logging(settings.log_level)
    create_app(make_context(settings)).run(host=settings.host, port=settings.flask_port, threaded=True)


if __name__ == "__main__":  # pragma: no cover
    main()
