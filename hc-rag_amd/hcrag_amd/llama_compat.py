"""LlamaIndex plugin surface backed by the HIP index.

Drop-in points in the reference: ``Settings.embed_model = HuggingFaceEmbedding(...)``
(graph_builder.py:146-149, query_interface.py:136-139), ``SimplePropertyGraphStore()``
(graph_builder.py:161) and ``VectorContextRetriever(graph_store, embed_model=...,
similarity_top_k=10)`` (query_interface.py:200-204).

llama-index-core (pinned 0.12.46, uv.lock:1467-1468) is not installed in this image, so the
query / result containers below are duck-typed with the pinned field names; when llama_index
IS importable the real classes are used instead and ``MI355XVectorStore`` can be passed where
a ``BasePydanticVectorStore`` is expected.

Semantics kept from the reference path (``SimpleVectorStore.query`` ->
``get_top_k_embeddings``): cosine similarity, best ``similarity_top_k`` first, ids are the
node ids, ``filters`` (ExactMatch / EQ on metadata keys) restrict the candidate rows.
Difference on purpose: exact ties are ordered by insertion order (llama-index's heap order
keeps the later node on a tie); zero-norm rows score 0 (llama-index yields NaN).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ._lib import HCR_SCORE_COSINE
from .index import VectorIndex

try:  # pragma: no cover - llama_index is absent in this image
    from llama_index.core.vector_stores.types import (VectorStoreQuery,  # type: ignore
                                                      VectorStoreQueryResult)
    HAVE_LLAMA = True
except Exception:
    HAVE_LLAMA = False

    @dataclass
    class VectorStoreQuery:  # type: ignore[no-redef]
        """Field names of llama_index.core.vector_stores.types.VectorStoreQuery (0.12.x)."""
        query_embedding: Optional[List[float]] = None
        similarity_top_k: int = 1
        doc_ids: Optional[List[str]] = None
        node_ids: Optional[List[str]] = None
        query_str: Optional[str] = None
        output_fields: Optional[List[str]] = None
        embedding_field: Optional[str] = None
        mode: str = "default"
        alpha: Optional[float] = None
        filters: Any = None
        mmr_threshold: Optional[float] = None
        sparse_top_k: Optional[int] = None
        hybrid_top_k: Optional[int] = None

    @dataclass
    class VectorStoreQueryResult:  # type: ignore[no-redef]
        nodes: Optional[Sequence[Any]] = None
        similarities: Optional[List[float]] = None
        ids: Optional[List[str]] = None


@dataclass
class TextNodeLite:
    """Minimal node record (id, text, metadata, embedding) used when llama_index is absent."""
    id_: str
    text: str = ""
    metadata: Dict[str, Any] = field(default_factory=dict)
    embedding: Optional[List[float]] = None

    @property
    def node_id(self) -> str:
        return self.id_

    def get_embedding(self):
        return self.embedding


def _node_id(n) -> str:
    return getattr(n, "node_id", None) or getattr(n, "id_", None) or getattr(n, "id")


def _node_embedding(n):
    e = getattr(n, "embedding", None)
    if e is None and hasattr(n, "get_embedding"):
        e = n.get_embedding()
    if e is None:
        raise ValueError(f"node {_node_id(n)} has no embedding")
    return e


def _filter_pairs(filters) -> List[tuple]:
    """(key, value) equality pairs of a MetadataFilters-like object (AND semantics)."""
    if filters is None:
        return []
    out = []
    for f in getattr(filters, "filters", filters):
        op = str(getattr(f, "operator", "==")).lower()
        if op not in ("==", "filteroperator.eq", "eq"):
            raise NotImplementedError(f"metadata filter operator {op!r} not supported")
        out.append((f.key, f.value))
    return out


class MI355XVectorStore:
    """``SimpleVectorStore``-compatible store whose ``query`` runs on the MI355X index.

    stores_text = False / is_embedding_query = True, like SimpleVectorStore.
    """

    stores_text: bool = False
    is_embedding_query: bool = True
    flat_metadata: bool = True

    def __init__(self, dim: int, dtype: str = "f16", device: int = 0):
        self.dim = int(dim)
        self._index = VectorIndex(dim, dtype=dtype, device=device)
        self._ids: List[str] = []
        self._row_of: Dict[str, int] = {}
        self._metadata: List[dict] = []
        self._deleted = np.zeros(0, dtype=bool)
        self._nodes: List[Any] = []

    @property
    def client(self):
        return self._index

    def add(self, nodes: Sequence[Any], **kwargs) -> List[str]:
        if not nodes:
            return []
        E = np.asarray([_node_embedding(n) for n in nodes], dtype=np.float32)
        self._index.add(E, normalize=True)
        ids = []
        for n in nodes:
            nid = _node_id(n)
            self._row_of[nid] = len(self._ids)
            self._ids.append(nid)
            self._metadata.append(dict(getattr(n, "metadata", {}) or {}))
            self._nodes.append(n)
            ids.append(nid)
        self._deleted = np.concatenate([self._deleted, np.zeros(len(nodes), dtype=bool)])
        return ids

    def delete(self, ref_doc_id: str, **delete_kwargs) -> None:
        """Tombstone the rows of ``ref_doc_id`` (node id or metadata 'ref_doc_id')."""
        for r, (nid, md) in enumerate(zip(self._ids, self._metadata)):
            if nid == ref_doc_id or md.get("ref_doc_id") == ref_doc_id:
                self._deleted[r] = True

    def _mask(self, query) -> Optional[np.ndarray]:
        pairs = _filter_pairs(getattr(query, "filters", None))
        want_ids = getattr(query, "node_ids", None) or getattr(query, "doc_ids", None)
        if not pairs and not want_ids and not self._deleted.any():
            return None
        m = ~self._deleted.copy()
        for key, val in pairs:
            m &= np.array([md.get(key) == val for md in self._metadata], dtype=bool)
        if want_ids:
            s = set(want_ids)
            m &= np.array([nid in s or md.get("ref_doc_id") in s
                           for nid, md in zip(self._ids, self._metadata)], dtype=bool)
        return m

    def query(self, query, **kwargs):
        if query.query_embedding is None:
            raise ValueError("query_embedding is required")
        k = int(query.similarity_top_k or 1)
        n = len(self._ids)
        if n == 0:
            return VectorStoreQueryResult(nodes=[], similarities=[], ids=[])
        mask = self._mask(query)
        if mask is not None and not mask.any():
            return VectorStoreQueryResult(nodes=[], similarities=[], ids=[])
        self._index.set_rowmask(mask)
        try:
            kk = max(1, min(k, n, 256))
            s, i = self._index.search(np.asarray(query.query_embedding, dtype=np.float32)[None],
                                      kk, HCR_SCORE_COSINE)
        finally:
            if mask is not None:
                self._index.set_rowmask(None)
        rows = [int(r) for r in i[0] if r >= 0]
        return VectorStoreQueryResult(nodes=[self._nodes[r] for r in rows],
                                      similarities=[float(x) for x in s[0][:len(rows)]],
                                      ids=[self._ids[r] for r in rows])


class MI355XVectorRetriever:
    """``VectorContextRetriever``-style retriever (query_interface.py:200-204): embeds the
    query with ``embed_model`` and returns ``[(node, score)]`` of the ``similarity_top_k``
    best nodes of ``vector_store``.  (The graph-expansion part of VectorContextRetriever —
    ``get_rel_map`` over the property graph — is Python dict walking, out of scope.)"""

    def __init__(self, vector_store: MI355XVectorStore, embed_model=None,
                 similarity_top_k: int = 4, filters=None):
        self.vector_store = vector_store
        self.embed_model = embed_model
        self.similarity_top_k = similarity_top_k
        self.filters = filters

    def retrieve(self, query) -> List[tuple]:
        if isinstance(query, str):
            if self.embed_model is None:
                raise ValueError("text query needs an embed_model")
            emb = self.embed_model.get_query_embedding(query)
        else:
            emb = getattr(query, "embedding", None) or query
        res = self.vector_store.query(VectorStoreQuery(query_embedding=list(emb),
                                                       similarity_top_k=self.similarity_top_k,
                                                       filters=self.filters))
        return list(zip(res.nodes, res.similarities))


class MI355XPropertyGraphStore:
    """Vector half of a ``PropertyGraphStore`` (second form):
    ``supports_vector_queries = True`` and ``vector_query(VectorStoreQuery) -> (nodes,
    scores)``, the call ``VectorContextRetriever`` makes instead of a separate vector store
    when the graph store holds the node embeddings (``SimplePropertyGraphStore`` at
    graph_builder.py:161 keeps them on ``LabelledNode.embedding``).  Triplets / relations stay
    with the caller's graph store; ``get(ids=...)`` returns the stored node objects."""

    supports_structured_queries: bool = False
    supports_vector_queries: bool = True

    def __init__(self, dim: int, dtype: str = "f16", device: int = 0):
        self._vs = MI355XVectorStore(dim, dtype=dtype, device=device)
        self._by_id: Dict[str, Any] = {}

    def upsert_nodes(self, nodes: Sequence[Any]) -> None:
        fresh = []
        for n in nodes:
            nid = _node_id(n)
            if nid in self._by_id:
                self._vs.delete(nid)
            self._by_id[nid] = n
            if getattr(n, "embedding", None) is not None:
                fresh.append(n)
        if fresh:
            self._vs.add(fresh)

    def get(self, properties: Optional[dict] = None, ids: Optional[List[str]] = None) -> List[Any]:
        out = [self._by_id[i] for i in (ids or list(self._by_id)) if i in self._by_id]
        if properties:
            out = [n for n in out if all((getattr(n, "properties", None) or
                                          getattr(n, "metadata", {}) or {}).get(k) == v
                                         for k, v in properties.items())]
        return out

    def vector_query(self, query, **kwargs):
        res = self._vs.query(query)
        return list(res.nodes), list(res.similarities)


__all__ = ["MI355XVectorStore", "MI355XVectorRetriever", "MI355XPropertyGraphStore", "VectorStoreQuery",
           "VectorStoreQueryResult", "TextNodeLite", "HAVE_LLAMA"]
