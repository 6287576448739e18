"""Tokenizers.

* ``HFTokenizer`` -- a real tokenizer loaded from a local model directory (the model
  PVC), via `tokenizers`/`transformers` (no network).
* ``ByteTokenizer`` -- offline fallback used with random-init weights: UTF-8 bytes are
  token ids [3, 259); 0/1/2 are pad/bos/eos.  Ids outside the byte range (which random
  weights emit) decode to a printable placeholder character, so text round-trips and
  the HTTP API stays well-formed.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


class ByteTokenizer:
    OFFSET = 3

    def __init__(self, vocab_size: int = 512, bos_id: int = 1, eos_id: int = 2):
        self.vocab_size = vocab_size
        self.bos_token_id = bos_id
        self.eos_token_id = eos_id
        self.name = "byte"

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = [b + self.OFFSET for b in text.encode("utf-8")]
        return ([self.bos_token_id] + ids) if add_bos else ids

    def decode(self, ids, skip_special: bool = True) -> str:
        # vectorised: a finishing decode batch detokenises 256 x 256 ids at once (a per-id
        # Python loop took ~40 ms of host time per such step)
        a = np.asarray(ids, dtype=np.int64).reshape(-1)
        if skip_special:
            a = a[(a != self.bos_token_id) & (a != self.eos_token_id) & (a != 0)]
        b = a - self.OFFSET
        # ids outside the byte range -> printable ASCII placeholder 33 + (id % 94)
        out = np.where((b >= 0) & (b < 256), b, 33 + (a % 94)).astype(np.uint8)
        return out.tobytes().decode("utf-8", errors="replace")

    def decode_token(self, i: int) -> str:
        return self.decode([i])


class HFTokenizer:
    def __init__(self, path: str):
        from transformers import AutoTokenizer  # local files only

        self.tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.vocab_size = len(self.tok)
        self.bos_token_id = self.tok.bos_token_id
        self.eos_token_id = self.tok.eos_token_id
        self.name = path
        self.chat_template = getattr(self.tok, "chat_template", None)

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        return self.tok.encode(text, add_special_tokens=add_bos)

    def decode(self, ids, skip_special: bool = True) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=skip_special)

    def decode_token(self, i: int) -> str:
        return self.tok.decode([i])


def get_tokenizer(model_path: Optional[str], vocab_size: int, bos_id: int, eos_id: int):
    if model_path and os.path.isdir(model_path) and any(
            os.path.exists(os.path.join(model_path, f))
            for f in ("tokenizer.json", "tokenizer.model", "tokenizer_config.json")):
        try:
            return HFTokenizer(model_path)
        except Exception:  # pragma: no cover - depends on local files
            pass
    return ByteTokenizer(vocab_size, bos_id, eos_id)
