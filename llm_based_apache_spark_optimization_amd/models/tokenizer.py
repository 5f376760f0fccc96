"""Tokenizers.

* ``HFTokenizer`` wraps a HuggingFace ``tokenizer.json`` (the fast ``tokenizers`` library) or a
  SentencePiece ``tokenizer.model`` when a checkpoint directory provides one — the real vocabularies
  of duckdb-nsql (Llama-2 SentencePiece, 32k), Llama-3.2 (tiktoken-BPE, 128,256) and Mistral v0.3.
* ``ByteTokenizer`` is the self-contained fallback used with random-init weights (no checkpoint can
  be downloaded here): UTF-8 bytes mapped onto ids [n_special, n_special + 256) of the model's
  vocabulary, with the model's BOS/EOS ids and chat-template special tokens mapped to reserved ids
  so templated prompts round-trip.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

from .spec import ModelSpec


class ByteTokenizer:
    def __init__(self, vocab_size: int, bos_id: int = 1, eos_ids: Sequence[int] = (2,), offset: int = 3,
                 specials: Sequence[str] = ()):
        self.vocab_size = vocab_size
        self.bos_id = bos_id
        self.eos_ids = tuple(eos_ids)
        self.offset = offset
        assert offset + 256 <= vocab_size or vocab_size >= 259, "vocab too small for byte fallback"
        # special strings (e.g. "<|eot_id|>") get reserved ids after the byte range
        self.special_to_id = {}
        nxt = offset + 256
        for s in specials:
            if nxt < vocab_size:
                self.special_to_id[s] = nxt
                nxt += 1
        self.id_to_special = {v: k for k, v in self.special_to_id.items()}

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        ids = [self.bos_id] if add_bos else []
        i = 0
        specials = sorted(self.special_to_id, key=len, reverse=True)
        while i < len(text):
            for s in specials:
                if text.startswith(s, i):
                    ids.append(self.special_to_id[s])
                    i += len(s)
                    break
            else:
                ids.extend(b + self.offset for b in text[i].encode("utf-8"))
                i += 1
        return ids

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        out = bytearray()
        text = []
        for t in ids:
            t = int(t)
            if self.offset <= t < self.offset + 256:
                out.append(t - self.offset)
            elif t in self.id_to_special and not skip_special:
                text.append(out.decode("utf-8", errors="replace"))
                out = bytearray()
                text.append(self.id_to_special[t])
        text.append(out.decode("utf-8", errors="replace"))
        return "".join(text)


class HFTokenizer:
    def __init__(self, path: str, bos_id: Optional[int] = None, eos_ids: Sequence[int] = ()):
        tj = os.path.join(path, "tokenizer.json")
        sp = os.path.join(path, "tokenizer.model")
        self._sp = None
        self._tk = None
        if os.path.exists(tj):
            from tokenizers import Tokenizer

            self._tk = Tokenizer.from_file(tj)
        elif os.path.exists(sp):
            import sentencepiece as spm

            self._sp = spm.SentencePieceProcessor(model_file=sp)
        else:
            raise FileNotFoundError(f"no tokenizer.json / tokenizer.model in {path}")
        self.bos_id = bos_id if bos_id is not None else (self._sp.bos_id() if self._sp else 1)
        self.eos_ids = tuple(eos_ids) or ((self._sp.eos_id(),) if self._sp else (2,))

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        if self._tk is not None:
            ids = self._tk.encode(text, add_special_tokens=False).ids
        else:
            ids = self._sp.encode(text)
        return ([self.bos_id] if add_bos else []) + list(ids)

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        ids = [int(i) for i in ids]
        if self._tk is not None:
            return self._tk.decode(ids, skip_special_tokens=skip_special)
        return self._sp.decode(ids)


LLAMA3_SPECIALS = ("<|begin_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>",
                   "<|end_of_text|>")
MISTRAL_SPECIALS = ("[INST]", "[/INST]")


def tokenizer_for(spec: ModelSpec, path: Optional[str] = None):
    # a checkpoint directory with its tokenizer files: the real tokenizer; weights-only directories
    # fall back to the byte tokenizer below
    if path and any(os.path.exists(os.path.join(path, f)) for f in ("tokenizer.json", "tokenizer.model")):
        return HFTokenizer(path, spec.bos_id, spec.eos_ids)
    specials = LLAMA3_SPECIALS if spec.template == "llama3" else MISTRAL_SPECIALS if spec.template == "mistral" else ()
    tok = ByteTokenizer(spec.vocab_size, bos_id=spec.bos_id if spec.bos_id < spec.vocab_size else 1,
                        eos_ids=[e for e in spec.eos_ids if e < spec.vocab_size] or [2], specials=specials)
    if spec.template == "llama3":  # the end-of-turn marker terminates generation
        eot = tok.special_to_id.get("<|eot_id|>")
        if eot is not None:
            tok.eos_ids = tuple(sorted(set(tok.eos_ids) | {eot}))
    return tok
