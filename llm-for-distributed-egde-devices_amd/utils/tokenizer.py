"""Tokenizer loading.

With a Hugging Face checkpoint directory (the reference's ``save_pretrained`` layout,
download.py:20-24) the checkpoint's own tokenizer is used (``transformers.AutoTokenizer``,
local files only).  Sets ``pad = eos`` when missing, like every reference loader
(e.g. Llama_bf16_updated.py:27-28).  Without checkpoint files (offline, random-init
benchmarks) a deterministic byte-level tokenizer stands in: ids 3..258 are the UTF-8 bytes.
"""
from __future__ import annotations

import os
from typing import List, Optional


class ByteTokenizer:
    pad_token_id = 0
    bos_token_id = 1
    eos_token_id = 2
    OFFSET = 3

    def __init__(self, vocab_size: int = 259):
        assert vocab_size >= 259, "byte tokenizer needs >= 259 ids"
        self.vocab_size = vocab_size

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = [b + self.OFFSET for b in text.encode("utf-8")]
        return ([self.bos_token_id] if add_bos else []) + ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        bs = bytes(i - self.OFFSET for i in ids if self.OFFSET <= i < self.OFFSET + 256)
        return bs.decode("utf-8", errors="replace")

    def __call__(self, text: str):
        return {"input_ids": self.encode(text)}


class HFTokenizer:
    def __init__(self, path: str):
        from transformers import AutoTokenizer
        self.tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        if self.tok.pad_token is None:
            self.tok.pad_token = self.tok.eos_token
        self.eos_token_id = self.tok.eos_token_id
        self.pad_token_id = self.tok.pad_token_id
        self.bos_token_id = self.tok.bos_token_id

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        return self.tok(text, truncation=True)["input_ids"]

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        return self.tok.decode(ids, skip_special_tokens=skip_special_tokens)


def load_tokenizer(path: Optional[str], vocab_size: int = 32000):
    if path and os.path.isdir(path) and any(os.path.exists(os.path.join(path, f)) for f in
                                            ("tokenizer.json", "tokenizer.model", "vocab.json", "vocab.txt")):
        return HFTokenizer(path)
    return ByteTokenizer(max(259, vocab_size))
