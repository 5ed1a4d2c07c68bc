"""Drop-ins for the reference's similarity functions, backed by the HIP index.

* ``batch_semantic_similarity`` — experiments/isRelevant.py:197-210 (every node's
  ``(cos+1)/2`` score, node order; ``[]`` for no nodes).
* ``EmbeddingSearch.find_similar_content`` — experiments/main.py:831-857 (top-k by cosine,
  then ``>= similarity_threshold``; result dicts ``content/metadata/similarity_score``).
* ``EmbeddingSearch.search_by_category`` — experiments/main.py:859-905 (rows whose
  ``metadata['type'] == category``; ``rank/similarity_score/content/metadata``; no threshold).

Differences from the reference, on purpose: exact score ties are ordered by row id
ascending (the reference's ``np.argsort`` is unstable, its tie order unspecified).
"""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ._lib import HCR_SCORE_COSINE, HCR_SCORE_UNIT
from .index import VectorIndex

_scratch: Dict[tuple, VectorIndex] = {}
_scratch_lock = threading.Lock()


def _embedding_of(x) -> np.ndarray:
    """Accept a QueryInput/NodeInput-like object (``.embeddings``) or a raw vector."""
    e = getattr(x, "embeddings", x)
    return np.asarray(e, dtype=np.float64).reshape(-1)


def _scratch_index(dim: int, device: int) -> VectorIndex:
    key = (dim, device)
    ix = _scratch.get(key)
    if ix is None:
        ix = VectorIndex(dim, dtype="f32", device=device)
        _scratch[key] = ix
    return ix


def batch_semantic_similarity(query, nodes: Sequence[Any], device: int = 0) -> List[float]:
    """GPU ``batch_semantic_similarity`` (experiments/isRelevant.py:197-210).

    ``query`` / ``nodes`` are QueryInput / NodeInput-like objects (``.embeddings``) or raw
    vectors.  Rows are stored as float32 and scored exactly in fp64 on the GPU.
    """
    if not nodes:
        return []
    q = _embedding_of(query)
    E = np.stack([_embedding_of(n) for n in nodes])
    if E.shape[1] != q.shape[0]:
        raise ValueError(
            f"Incompatible dimension for X and Y matrices: X.shape[1] == {q.shape[0]} "
            f"while Y.shape[1] == {E.shape[1]}")
    with _scratch_lock:
        ix = _scratch_index(q.shape[0], device)
        ix.reset()
        ix.add(E.astype(np.float32), normalize=False)
        s = ix.score_all(q.astype(np.float32).reshape(1, -1), score_mode=HCR_SCORE_UNIT)[0]
    return [float(v) for v in s]


class EmbeddingSearch:
    """Search half of ``EmbeddingRAGSystem`` (experiments/main.py:738-905) on the GPU index.

    ``embeddings``: (N, D) matrix (the reference's ``embeddings_matrix``, :762);
    ``texts`` / ``metadata``: per-row lists (:763-764).  ``embedder``: optional object with
    ``encode(List[str]) -> ndarray`` used when a query is given as text (:807, :869).
    """

    def __init__(self, embeddings, texts: Optional[List[str]] = None,
                 metadata: Optional[List[dict]] = None, dtype: str = "f32", device: int = 0,
                 embedder=None):
        E = np.asarray(embeddings)
        if E.ndim != 2:
            raise ValueError("embeddings must be a 2-D matrix")
        self.index = VectorIndex(E.shape[1], dtype=dtype, device=device, capacity=E.shape[0])
        self.index.add(E, normalize=(dtype != "f32"))
        n = E.shape[0]
        self.texts_list = list(texts) if texts is not None else [None] * n
        self.metadata_list = list(metadata) if metadata is not None else [{} for _ in range(n)]
        self.embedder = embedder

    def _query_vec(self, query) -> np.ndarray:
        if isinstance(query, str):
            if self.embedder is None:
                raise ValueError("text query given but no embedder attached")
            return np.asarray(self.embedder.encode([query]), dtype=np.float32)[0]
        return np.asarray(query, dtype=np.float32).reshape(-1)

    def find_similar_content(self, query_embedding, top_k: int = 5,
                             similarity_threshold: float = 0.3) -> List[dict]:
        q = self._query_vec(query_embedding)
        k = max(1, min(int(top_k), len(self.index)))
        s, ids = self.index.search(q.reshape(1, -1), k, HCR_SCORE_COSINE,
                                   float(similarity_threshold))
        out = []
        for sc, i in zip(s[0], ids[0]):
            if i < 0:
                continue
            out.append({"content": self.texts_list[i], "metadata": self.metadata_list[i],
                        "similarity_score": float(sc)})
        return out[:top_k]

    def search_by_category(self, query, category_filter: Optional[str] = None,
                           top_k: int = 5) -> dict:
        q = self._query_vec(query)
        if category_filter:
            mask = np.array([(m or {}).get("type") == category_filter
                             for m in self.metadata_list], dtype=bool)
        else:
            mask = np.ones(len(self.metadata_list), dtype=bool)
        if not mask.any():
            return {"results": [], "summary": "No items match the filter criteria"}
        k = max(1, min(int(top_k), int(mask.sum())))
        self.index.set_rowmask(mask if category_filter else None)
        try:
            s, ids = self.index.search(q.reshape(1, -1), k, HCR_SCORE_COSINE)
        finally:
            self.index.set_rowmask(None)
        results = []
        for rank, (sc, i) in enumerate(zip(s[0], ids[0])):
            if i < 0:
                continue
            results.append({"rank": rank + 1, "similarity_score": float(sc),
                            "content": self.texts_list[i], "metadata": self.metadata_list[i]})
        return {"results": results,
                "summary": f"Found {len(results)} results in {category_filter or 'all categories'}"}
