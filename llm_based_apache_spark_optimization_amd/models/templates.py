"""Prompt templates applied to (system, prompt) before tokenisation.

The reference passes ``system=`` and ``prompt=`` to ``ollama.generate`` and Ollama wraps them in each
model's Modelfile TEMPLATE before tokenising.  These reproduce those wrappers:

* ``duckdb-nsql`` — the Alpaca-style instruction format of the DuckDB-NSQL model card, with the
  request's system text (the table schema) as the ``### Input`` block and the user's question as
  ``### Question``.
* ``llama3`` — the Llama-3 chat format used by Ollama's ``llama3.2`` tag (system header with the
  knowledge-cutoff line, user turn, open assistant turn).
* ``mistral`` — ``[INST] system\\n\\nprompt [/INST]``.
* ``raw`` — system and prompt concatenated.

Parity note: the exact Modelfile bytes are not in the reference tree and cannot be fetched here, so
byte-for-byte equality with Ollama is unpinned; the structure matches the public model cards.
"""
from __future__ import annotations

DUCKDB_NSQL = (
    "### Instruction:\n"
    "Your task is to generate valid duckdb SQL to answer the following question, given a duckdb database schema.\n\n"
    "### Input:\n"
    "{system}\n\n"
    "### Question:\n"
    "{prompt}\n\n"
    "### Response (use duckdb shorthand if possible):\n"
)

LLAMA3_SYSTEM_HEAD = "Cutting Knowledge Date: December 2023\n\n"
LLAMA3 = (
    "<|start_header_id|>system<|end_header_id|>\n\n"
    "{head}{system}<|eot_id|>"
    "<|start_header_id|>user<|end_header_id|>\n\n"
    "{prompt}<|eot_id|>"
    "<|start_header_id|>assistant<|end_header_id|>\n\n"
)

MISTRAL = "[INST] {body} [/INST]"


def render(template: str, prompt: str, system: str = "") -> str:
    if template == "duckdb-nsql":
        return DUCKDB_NSQL.format(system=system.strip(), prompt=prompt.strip())
    if template == "llama3":
        return LLAMA3.format(head=LLAMA3_SYSTEM_HEAD, system=system, prompt=prompt)
    if template == "mistral":
        body = f"{system}\n\n{prompt}" if system else prompt
        return MISTRAL.format(body=body)
    if template == "raw":
        return f"{system}\n\n{prompt}" if system else prompt
    raise KeyError(f"unknown template {template!r}")


STOP_STRINGS = {
    "duckdb-nsql": ("### Instruction:", "### Input:", "### Question:"),
    "llama3": ("<|eot_id|>", "<|start_header_id|>"),
    "mistral": ("[INST]",),
    "raw": (),
}


def apply_stops(text: str, template: str, extra: tuple = ()) -> str:
    """Cut generated text at the first stop string (Ollama's Modelfile ``stop`` parameters)."""
    cut = len(text)
    for s in tuple(STOP_STRINGS.get(template, ())) + tuple(extra):
        i = text.find(s)
        if i >= 0:
            cut = min(cut, i)
    return text[:cut]
