"""Reversible byte-level tokenizer (stand-in for the reference's TF-Text
subword converters `ted_hrlr_translate_pt_en_converter`, loaded at
english_portugese_dataset.py:9-18, which need TensorFlow and a download).

ids: 0 PAD, 1 UNK, 2 [START], 3 [END], 4 + byte. Any object with the same
`tokenize` / `detokenize` / `lookup` / `start_end` methods can be used by the
Tester instead (e.g. a `tokenizers` wrapper around a trained vocabulary).
"""
from __future__ import annotations

from typing import List, Sequence, Union

import torch

PAD, UNK, START, END = 0, 1, 2, 3
OFFSET = 4


class ByteTokenizer:
    def __init__(self, vocab_size: int = 260):
        if vocab_size < OFFSET + 256:
            raise ValueError("ByteTokenizer needs a vocabulary of at least 260 ids")
        self.vocab_size = vocab_size

    def start_end(self):
        return START, END

    def encode(self, text: str, add_start_end: bool = True) -> List[int]:
        ids = [OFFSET + b for b in text.encode("utf-8")]
        return [START] + ids + [END] if add_start_end else ids

    def tokenize(self, texts: Union[str, Sequence[str]]) -> torch.Tensor:
        """Right-padded int64 [B, L] with [START] ... [END]."""
        if isinstance(texts, str):
            texts = [texts]
        rows = [self.encode(t) for t in texts]
        L = max(len(r) for r in rows)
        out = torch.zeros(len(rows), L, dtype=torch.int64)
        for i, r in enumerate(rows):
            out[i, : len(r)] = torch.tensor(r, dtype=torch.int64)
        return out

    def lookup(self, ids: Sequence[int]) -> List[str]:
        names = {PAD: "[PAD]", UNK: "[UNK]", START: "[START]", END: "[END]"}
        out = []
        for i in ids:
            i = int(i)
            if i in names:
                out.append(names[i])
            elif OFFSET <= i < OFFSET + 256:
                out.append(bytes([i - OFFSET]).decode("latin-1"))
            else:
                out.append(f"<{i}>")
        return out

    def detokenize(self, ids: Sequence[int]) -> str:
        bs = bytes(int(i) - OFFSET for i in ids if OFFSET <= int(i) < OFFSET + 256)
        return bs.decode("utf-8", errors="replace")
