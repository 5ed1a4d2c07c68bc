"""WordPiece tokenizer handle (C++ in libhcrag_hip.so)."""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_char_p, c_int32, c_int64, c_void_p
from typing import List, Sequence

import numpy as np

from ._lib import check, lib


class WordPieceTokenizer:
    """BERT uncased WordPiece: ``encode(texts, max_len) -> (ids, mask, lengths)``."""

    def __init__(self, vocab_path: str = None, vocab_tokens: Sequence[str] = None,
                 lowercase: bool = True, strip_accents: int = -1):
        self._h = c_void_p()
        if vocab_path is not None:
            check(lib().hcr_wordpiece_create(vocab_path.encode(), int(lowercase),
                                             int(strip_accents), ctypes.byref(self._h)))
        else:
            data = ("\n".join(vocab_tokens) + "\n").encode("utf-8")
            check(lib().hcr_wordpiece_create_from_buffer(data, len(data), int(lowercase),
                                                         int(strip_accents), ctypes.byref(self._h)))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().hcr_wordpiece_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def vocab_size(self) -> int:
        return int(lib().hcr_wordpiece_vocab_size(self._h))

    def encode(self, texts: List[str], max_len: int = 256, pad_to_longest: bool = True):
        n = len(texts)
        enc = [t.encode("utf-8", "replace") for t in texts]
        arr = (c_char_p * max(n, 1))(*enc)
        tl = np.array([len(b) for b in enc] or [0], dtype=np.int64)
        ids = np.zeros((n, max_len), dtype=np.int32)
        mask = np.zeros((n, max_len), dtype=np.int32)
        lens = np.zeros(n, dtype=np.int32)
        check(lib().hcr_tokenize(self._h, arr, tl.ctypes.data_as(POINTER(c_int64)), n, int(max_len),
                                 ids.ctypes.data_as(POINTER(c_int32)),
                                 mask.ctypes.data_as(POINTER(c_int32)),
                                 lens.ctypes.data_as(POINTER(c_int32))))
        if pad_to_longest and n:
            L = int(lens.max())
            ids, mask = ids[:, :L].copy(), mask[:, :L].copy()
        return ids, mask, lens
