"""LlamaIndex plugin surface backed by the HIP library.

Drop-in points in the reference:
  * ``Settings.embed_model = HuggingFaceEmbedding(model_name=config.EMBEDDING_MODEL)``
    (graph_builder.py:146-149, query_interface.py:136-139)          -> ``MI355XEmbedding``
  * ``property_graph_store=SimplePropertyGraphStore()`` (graph_builder.py:161, 493-498)
                                                                     -> ``MI355XPropertyGraphStore``
  * ``VectorContextRetriever(index.property_graph_store, embed_model=Settings.embed_model,
    similarity_top_k=10)`` (query_interface.py:200-204)             -> unchanged: it calls the
    store's ``vector_query`` (``supports_vector_queries = True``) and ``get_rel_map``; or
    ``MI355XVectorContextRetriever`` where llama_index is absent.
  * ``SimpleVectorStore`` (the index's vector store)                 -> ``MI355XVectorStore``

When llama-index-core (pinned 0.12.46, uv.lock:1467-1468) is importable the classes subclass
the real ones: ``BaseEmbedding``, ``BasePydanticVectorStore``, ``SimplePropertyGraphStore``
(graph half inherited; only the vector half is replaced) and ``BaseRetriever`` -- so the
reference's callers accept them unchanged.  It is NOT installed in this image (nor on the GPU
box), so the classes below fall back to self-contained implementations with the pinned field
and method names, and those are what the tests exercise.  The llama-index semantics restated
here (get_top_k_embeddings, LabelledPropertyGraph.get_rel_map, VectorContextRetriever's triplet
scoring) are from the pinned version's published source -- parity unpinned by any reference test.

Semantics kept from the reference path (``SimpleVectorStore.query`` -> ``get_top_k_embeddings``):
cosine similarity in fp64, best ``similarity_top_k`` first, ids are the node ids, ``filters``
(ExactMatch / EQ on metadata keys) restrict the candidate rows.  Differences on purpose: exact
ties are ordered by insertion order (llama-index's heap order keeps the later node on a tie);
zero-norm rows score 0 (llama-index yields NaN).  Any similarity_top_k >= 1 is served (above
2048 by the library's sorted full scan, hcrag_index.hip deep_topk).
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ._lib import HCR_SCORE_COSINE
from .index import VectorIndex

_log = logging.getLogger(__name__)

MAX_TOP_K = None          # hcr_search takes any k >= 1 (r05: k > 2048 by the sorted full scan)

try:  # pragma: no cover - llama_index is absent in this image
    from llama_index.core.vector_stores.types import (BasePydanticVectorStore,  # type: ignore
                                                      VectorStoreQuery, VectorStoreQueryResult)
    from llama_index.core.base.embeddings.base import BaseEmbedding  # type: ignore
    from llama_index.core.graph_stores import SimplePropertyGraphStore  # type: ignore
    from llama_index.core.base.base_retriever import BaseRetriever  # type: ignore
    from llama_index.core.schema import NodeWithScore, QueryBundle, TextNode  # type: ignore
    from pydantic import PrivateAttr
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
    class NodeWithScore:  # type: ignore[no-redef]
        node: Any
        score: Optional[float] = None

    @dataclass
    class QueryBundle:  # type: ignore[no-redef]
        query_str: str
        embedding: Optional[List[float]] = None

        @property
        def embedding_strs(self) -> List[str]:
            return [self.query_str]


# ---------------------------------------------------------------------------------------------
# node / relation records (llama_index.core.graph_stores.types field names)
# ---------------------------------------------------------------------------------------------
@dataclass
class TextNodeLite:
    """Minimal text node (id, text, metadata, embedding) used when llama_index is absent."""
    id_: str
    text: str = ""
    metadata: Dict[str, Any] = field(default_factory=dict)
    embedding: Optional[List[float]] = None

    @property
    def node_id(self) -> str:
        return self.id_

    def get_embedding(self):
        return self.embedding


@dataclass
class EntityNodeLite:
    """``EntityNode``: id = name, label, properties, optional embedding."""
    name: str
    label: str = "entity"
    properties: Dict[str, Any] = field(default_factory=dict)
    embedding: Optional[List[float]] = None

    @property
    def id(self) -> str:
        return self.name

    def __str__(self) -> str:
        return self.name


@dataclass
class ChunkNodeLite:
    """``ChunkNode``: a source text chunk (label "text_chunk")."""
    text: str
    id_: str
    label: str = "text_chunk"
    properties: Dict[str, Any] = field(default_factory=dict)
    embedding: Optional[List[float]] = None

    @property
    def id(self) -> str:
        return self.id_

    def __str__(self) -> str:
        return self.text


@dataclass
class RelationLite:
    """``Relation``: label, source_id, target_id, properties."""
    label: str
    source_id: str
    target_id: str
    properties: Dict[str, Any] = field(default_factory=dict)

    @property
    def id(self) -> str:
        return self.label


KG_SOURCE_REL = "SOURCE"     # llama_index.core.graph_stores.types.KG_SOURCE_REL


def _node_id(n) -> str:
    for attr in ("node_id", "id_", "id"):
        v = getattr(n, attr, None)
        if v is not None and not callable(v):
            return str(v)
    raise ValueError(f"node without an id: {n!r}")


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


def _check_top_k(k: int) -> int:
    k = int(k or 1)
    if k < 1:
        raise ValueError(f"similarity_top_k must be >= 1, got {k}")
    return k


# ---------------------------------------------------------------------------------------------
# the GPU vector half: an id-keyed set of rows on one hcr_index
# ---------------------------------------------------------------------------------------------
class _GpuRows:
    """Node embeddings on the MI355X index, keyed by node id (metadata kept host-side for the
    equality filters).  Deletes and replacements tombstone a row (masked out of every search);
    once tombstones reach COMPACT_MIN rows and COMPACT_FRAC of the index, the live rows are
    re-ingested into a fresh index and the old one's HBM is freed (``compact``)."""

    COMPACT_MIN = 1024
    COMPACT_FRAC = 0.25

    def __init__(self, dim: int, dtype: str, device: int):
        self.dim = int(dim)
        self.dtype, self.device = dtype, device
        self.index = VectorIndex(dim, dtype=dtype, device=device)
        # fp32 rows are stored as given (exact sklearn / llama-index cosine of the node
        # embeddings); 16-bit rows are L2-normalised in fp64 before rounding
        self.normalize = dtype not in ("f32", "float32")
        self.ids: List[str] = []
        self.meta: List[dict] = []
        self.nodes: List[Any] = []
        self.row_of: Dict[str, int] = {}
        self.deleted = np.zeros(0, dtype=bool)

    def add(self, nodes: Sequence[Any]) -> List[str]:
        if not nodes:
            return []
        E = np.asarray([_node_embedding(n) for n in nodes], dtype=np.float32)
        if E.ndim != 2 or E.shape[1] != self.dim:
            raise ValueError(f"embeddings must be {self.dim}-wide, got {E.shape}")
        for n in nodes:                                  # re-added ids replace the old row
            nid = _node_id(n)
            if nid in self.row_of:
                self.deleted[self.row_of[nid]] = True
        self.index.add(E, normalize=self.normalize)
        out = []
        for n in nodes:
            nid = _node_id(n)
            self.row_of[nid] = len(self.ids)
            self.ids.append(nid)
            self.meta.append(dict(getattr(n, "metadata", None) or getattr(n, "properties", None) or {}))
            self.nodes.append(n)
            out.append(nid)
        self.deleted = np.concatenate([self.deleted, np.zeros(len(nodes), dtype=bool)])
        self._maybe_compact()
        return out

    def delete(self, pred) -> None:
        for r, (nid, md) in enumerate(zip(self.ids, self.meta)):
            if not self.deleted[r] and pred(nid, md):
                self.deleted[r] = True
                if self.row_of.get(nid) == r:
                    del self.row_of[nid]
        self._maybe_compact()

    def _maybe_compact(self) -> None:
        """Compaction after an add / delete that already took effect: a failure to rebuild (the
        fresh index needs HBM for the live rows while the old one is still held) leaves the
        tombstoned index in place -- every search stays exact, the rows stay masked -- and is
        logged, so the caller's add / delete still succeeds."""
        nd = int(self.deleted.sum())
        if nd >= self.COMPACT_MIN and nd >= self.COMPACT_FRAC * len(self.ids):
            try:
                self.compact()
            except Exception as exc:                    # noqa: BLE001 -- kept tombstoned
                _log.warning("vector store compaction failed (%s); rows stay tombstoned", exc)

    def compact(self) -> None:
        """Re-ingest the live rows (their nodes' embeddings, in insertion order, so ties still
        break by insertion order) into a fresh index; the tombstoned rows' HBM is released.  On
        failure the half-built index is closed and this object is unchanged."""
        live = np.flatnonzero(~self.deleted)
        fresh = VectorIndex(self.dim, dtype=self.dtype, device=self.device)
        try:
            if live.size:
                E = np.asarray([_node_embedding(self.nodes[r]) for r in live], dtype=np.float32)
                fresh.add(E, normalize=self.normalize)
        except BaseException:
            fresh.close()
            raise
        old, self.index = self.index, fresh
        old.close()
        self.ids = [self.ids[r] for r in live]
        self.meta = [self.meta[r] for r in live]
        self.nodes = [self.nodes[r] for r in live]
        self.row_of = {nid: j for j, nid in enumerate(self.ids)}
        self.deleted = np.zeros(len(self.ids), dtype=bool)

    def mask(self, query) -> Optional[np.ndarray]:
        pairs = _filter_pairs(getattr(query, "filters", None))
        want = getattr(query, "node_ids", None) or getattr(query, "doc_ids", None)
        if not pairs and not want and not self.deleted.any():
            return None
        m = ~self.deleted.copy()
        for key, val in pairs:
            m &= np.array([md.get(key) == val for md in self.meta], dtype=bool)
        if want:
            s = set(want)
            m &= np.array([nid in s or md.get("ref_doc_id") in s
                           for nid, md in zip(self.ids, self.meta)], dtype=bool)
        return m

    def query(self, query) -> Tuple[List[Any], List[float], List[str]]:
        if query.query_embedding is None:
            raise ValueError("query_embedding is required")
        k = _check_top_k(query.similarity_top_k)
        n = len(self.ids)
        if n == 0:
            return [], [], []
        m = self.mask(query)
        if m is not None and not m.any():
            return [], [], []
        self.index.set_rowmask(m)
        try:
            s, i = self.index.search(np.asarray(query.query_embedding, dtype=np.float32)[None],
                                     min(k, n), HCR_SCORE_COSINE)
        finally:
            if m is not None:
                self.index.set_rowmask(None)
        rows = [int(r) for r in i[0] if r >= 0]
        return ([self.nodes[r] for r in rows], [float(x) for x in s[0][:len(rows)]],
                [self.ids[r] for r in rows])


# ---------------------------------------------------------------------------------------------
# SimpleVectorStore replacement
# ---------------------------------------------------------------------------------------------
class _VectorStoreImpl:
    stores_text: bool = False
    is_embedding_query: bool = True
    flat_metadata: bool = True

    def _init_rows(self, dim, dtype, device):
        self._rows = _GpuRows(dim, dtype, device)

    @property
    def client(self):
        return self._rows.index

    def add(self, nodes: Sequence[Any], **kwargs) -> List[str]:
        return self._rows.add(nodes)

    def delete(self, ref_doc_id: str, **delete_kwargs) -> None:
        """Drop the rows of ``ref_doc_id`` (node id or metadata 'ref_doc_id')."""
        self._rows.delete(lambda nid, md: nid == ref_doc_id or md.get("ref_doc_id") == ref_doc_id)

    def query(self, query, **kwargs):
        nodes, sims, ids = self._rows.query(query)
        return VectorStoreQueryResult(nodes=nodes, similarities=sims, ids=ids)


if HAVE_LLAMA:  # pragma: no cover
    class MI355XVectorStore(_VectorStoreImpl, BasePydanticVectorStore):
        """``BasePydanticVectorStore`` whose ``query`` runs on the MI355X index."""
        _rows: Any = PrivateAttr()

        def __init__(self, dim: int, dtype: str = "f16", device: int = 0, **kw):
            super().__init__(stores_text=False, **kw)
            self._init_rows(dim, dtype, device)

        @classmethod
        def class_name(cls) -> str:
            return "MI355XVectorStore"
else:
    class MI355XVectorStore(_VectorStoreImpl):
        """``SimpleVectorStore``-compatible store whose ``query`` runs on the MI355X index."""

        def __init__(self, dim: int, dtype: str = "f16", device: int = 0):
            self.dim = int(dim)
            self._init_rows(dim, dtype, device)


# ---------------------------------------------------------------------------------------------
# SimplePropertyGraphStore replacement
# ---------------------------------------------------------------------------------------------
class _GraphImpl:
    """Graph half (nodes, relations, get_rel_map, persist) of a ``SimplePropertyGraphStore``
    (``LabelledPropertyGraph``), used when llama_index is absent.  No pickle: persist writes
    JSON."""

    def _init_graph(self):
        self._nodes: Dict[str, Any] = {}
        self._rels: Dict[Tuple[str, str, str], Any] = {}

    # -- nodes / relations --------------------------------------------------------------------
    def _put_nodes(self, nodes):
        for n in nodes:
            self._nodes[_node_id(n)] = n

    def upsert_relations(self, relations: Sequence[Any]) -> None:
        for r in relations:
            self._rels[(r.source_id, r.label, r.target_id)] = r

    def get(self, properties: Optional[dict] = None, ids: Optional[List[str]] = None) -> List[Any]:
        out = [self._nodes[i] for i in (ids if ids is not None else list(self._nodes)) if i in self._nodes]
        if properties:
            out = [n for n in out if all((getattr(n, "properties", None) or
                                          getattr(n, "metadata", None) or {}).get(k) == v
                                         for k, v in properties.items())]
        return out

    def get_triplets(self, entity_names=None, relation_names=None, properties=None, ids=None):
        out = []
        for (s, lbl, t), r in self._rels.items():
            if s not in self._nodes or t not in self._nodes:
                continue
            src, dst = self._nodes[s], self._nodes[t]
            if entity_names and s not in entity_names and t not in entity_names:
                continue
            if relation_names and lbl not in relation_names:
                continue
            if ids and s not in ids and t not in ids:
                continue
            if properties and not all((r.properties or {}).get(k) == v for k, v in properties.items()):
                continue
            out.append((src, r, dst))
        return out

    def get_rel_map(self, graph_nodes: Sequence[Any], depth: int = 2, limit: int = 30,
                    ignore_rels: Optional[List[str]] = None) -> List[Tuple[Any, Any, Any]]:
        """Triplets within ``depth`` hops of ``graph_nodes`` (breadth first, each triplet once,
        relations in ``ignore_rels`` skipped), at most ``limit``."""
        ignore = set(ignore_rels or [])
        frontier = {_node_id(n) for n in graph_nodes}
        seen_nodes = set(frontier)
        seen, out = set(), []
        for _ in range(max(depth, 0)):
            nxt = set()
            for (s, lbl, t), r in self._rels.items():
                if lbl in ignore or (s, lbl, t) in seen:
                    continue
                if s in frontier or t in frontier:
                    if s not in self._nodes or t not in self._nodes:
                        continue
                    seen.add((s, lbl, t))
                    out.append((self._nodes[s], r, self._nodes[t]))
                    nxt.update({s, t} - seen_nodes)
            seen_nodes |= nxt
            frontier = nxt
            if not frontier:
                break
        return out[:limit]

    def delete(self, entity_names=None, relation_names=None, properties=None, ids=None) -> None:
        gone = set(ids or []) | set(entity_names or [])
        if properties:
            gone |= {_node_id(n) for n in self.get(properties=properties)}
        for nid in gone:
            self._nodes.pop(nid, None)
        self._rels = {k: r for k, r in self._rels.items()
                      if k[0] not in gone and k[2] not in gone and
                      not (relation_names and k[1] in relation_names)}
        if gone:
            self._vec.delete(lambda nid, md: nid in gone)

    def structured_query(self, query: str, param_map: Optional[dict] = None):
        raise NotImplementedError("structured queries are not supported (as SimplePropertyGraphStore)")

    def get_schema(self, refresh: bool = False):
        return {"node_labels": sorted({getattr(n, "label", "") for n in self._nodes.values()}),
                "relation_labels": sorted({k[1] for k in self._rels})}

    # -- persistence (JSON, no pickle) ---------------------------------------------------------
    def persist(self, persist_path: str, fs=None) -> None:
        def node_rec(n):
            rec = {"id": _node_id(n), "label": getattr(n, "label", "text_chunk"),
                   "properties": dict(getattr(n, "properties", None) or getattr(n, "metadata", None) or {}),
                   "embedding": list(map(float, n.embedding)) if getattr(n, "embedding", None) is not None else None}
            if hasattr(n, "text"):
                rec["text"] = n.text
            return rec
        doc = {"dim": self._vec.dim, "nodes": [node_rec(n) for n in self._nodes.values()],
               "relations": [{"label": r.label, "source_id": r.source_id, "target_id": r.target_id,
                              "properties": dict(r.properties or {})} for r in self._rels.values()]}
        os.makedirs(os.path.dirname(os.path.abspath(persist_path)), exist_ok=True)
        with open(persist_path, "w", encoding="utf-8") as fh:
            json.dump(doc, fh, default=str)


if HAVE_LLAMA:  # pragma: no cover
    class MI355XPropertyGraphStore(SimplePropertyGraphStore):
        """``SimplePropertyGraphStore`` with the vector half on the MI355X: the graph (nodes,
        relations, get_rel_map, persist) is the inherited llama-index implementation; node
        embeddings are also indexed on the GPU and ``vector_query`` runs there."""
        supports_vector_queries: bool = True
        _vec: Any = None

        def __init__(self, dim: int, dtype: str = "f16", device: int = 0, **kw):
            super().__init__(**kw)
            self._vec = _GpuRows(dim, dtype, device)

        def upsert_nodes(self, nodes):
            super().upsert_nodes(nodes)
            emb = [n for n in nodes if getattr(n, "embedding", None) is not None]
            self._vec.add(emb)

        def delete(self, entity_names=None, relation_names=None, properties=None, ids=None):
            gone = set(ids or []) | set(entity_names or [])
            super().delete(entity_names=entity_names, relation_names=relation_names,
                           properties=properties, ids=ids)
            if gone:
                self._vec.delete(lambda nid, md: nid in gone)

        def vector_query(self, query, **kwargs):
            nodes, sims, _ = self._vec.query(query)
            return list(nodes), list(sims)
else:
    class MI355XPropertyGraphStore(_GraphImpl):
        """``SimplePropertyGraphStore`` drop-in (graph_builder.py:161): nodes, relations,
        ``get`` / ``get_triplets`` / ``get_rel_map`` / ``delete`` / ``persist``, and the vector
        half -- ``supports_vector_queries = True``, ``vector_query`` on the MI355X index -- which
        ``VectorContextRetriever`` (query_interface.py:200-204) calls."""
        supports_structured_queries: bool = False
        supports_vector_queries: bool = True

        def __init__(self, dim: int, dtype: str = "f16", device: int = 0):
            self._init_graph()
            self._vec = _GpuRows(dim, dtype, device)

        def upsert_nodes(self, nodes: Sequence[Any]) -> None:
            self._put_nodes(nodes)
            emb = [n for n in nodes if getattr(n, "embedding", None) is not None]
            self._vec.add(emb)

        def vector_query(self, query, **kwargs):
            nodes, sims, _ = self._vec.query(query)
            return list(nodes), list(sims)

        @classmethod
        def from_persist_path(cls, persist_path: str, dtype: str = "f16", device: int = 0, fs=None):
            with open(persist_path, encoding="utf-8") as fh:
                doc = json.load(fh)
            st = cls(doc["dim"], dtype=dtype, device=device)
            nodes = []
            for rec in doc["nodes"]:
                if rec.get("label") == "text_chunk" and "text" in rec:
                    nodes.append(ChunkNodeLite(text=rec["text"], id_=rec["id"],
                                               properties=rec["properties"], embedding=rec["embedding"]))
                else:
                    nodes.append(EntityNodeLite(name=rec["id"], label=rec["label"],
                                                properties=rec["properties"], embedding=rec["embedding"]))
            st.upsert_nodes(nodes)
            st.upsert_relations([RelationLite(**r) for r in doc["relations"]])
            return st


# ---------------------------------------------------------------------------------------------
# VectorContextRetriever (vector half + the graph expansion's scoring)
# ---------------------------------------------------------------------------------------------
class _VectorContextImpl:
    """``VectorContextRetriever.retrieve_from_graph`` semantics (llama-index-core 0.12.46,
    recalled): query embedding -> ``VectorStoreQuery(similarity_top_k, filters)`` -> the graph
    store's ``vector_query`` (or a separate vector store + ``graph_store.get``) ->
    ``get_rel_map(kg_nodes, depth=path_depth, ignore_rels=[SOURCE], limit)`` -> each triplet
    scored max(score(source), score(target)) (0 for an endpoint outside the top-k), sorted by
    score descending, optional ``similarity_score`` cutoff.  Returns NodeWithScore of the
    triplets rendered as text ("src -> rel -> dst")."""

    def _setup(self, graph_store, embed_model, vector_store, similarity_top_k, path_depth,
               limit, similarity_score, filters, include_text):
        self._graph_store = graph_store
        self._embed_model = embed_model
        self._vector_store = vector_store
        self._similarity_top_k = _check_top_k(similarity_top_k)
        self._path_depth = path_depth
        self._limit = limit
        self._similarity_score = similarity_score
        self._filters = filters
        self._include_text = include_text

    def _query_embedding(self, query_bundle) -> List[float]:
        if getattr(query_bundle, "embedding", None) is not None:
            return list(query_bundle.embedding)
        if self._embed_model is None:
            raise ValueError("text query needs an embed_model")
        strs = getattr(query_bundle, "embedding_strs", None) or [query_bundle.query_str]
        return list(self._embed_model.get_agg_embedding_from_queries(strs))

    def retrieve_from_graph(self, query_bundle) -> List[Any]:
        q = VectorStoreQuery(query_embedding=self._query_embedding(query_bundle),
                             similarity_top_k=self._similarity_top_k, filters=self._filters)
        gs = self._graph_store
        if getattr(gs, "supports_vector_queries", False):
            kg_nodes, scores = gs.vector_query(q)
            kg_ids = [_node_id(n) for n in kg_nodes]
        elif self._vector_store is not None:
            res = self._vector_store.query(q)
            kg_ids, scores = list(res.ids or []), list(res.similarities or [])
            kg_nodes = gs.get(ids=kg_ids)
        else:
            raise ValueError("graph store has no vector queries and no vector_store was given")
        triplets = gs.get_rel_map(kg_nodes, depth=self._path_depth, limit=self._limit,
                                  ignore_rels=[KG_SOURCE_REL])
        pos = {nid: i for i, nid in enumerate(kg_ids)}
        scored = []
        for t in triplets:
            s1 = scores[pos[_node_id(t[0])]] if _node_id(t[0]) in pos else 0.0
            s2 = scores[pos[_node_id(t[2])]] if _node_id(t[2]) in pos else 0.0
            scored.append((t, max(s1, s2)))
        scored.sort(key=lambda x: x[1], reverse=True)
        if self._similarity_score is not None:
            scored = [x for x in scored if x[1] >= self._similarity_score]
        return [NodeWithScore(node=_triplet_node(t), score=s) for t, s in scored]

    def retrieve(self, query) -> List[Any]:
        qb = QueryBundle(query_str=query) if isinstance(query, str) else query
        return self.retrieve_from_graph(qb)


def _triplet_node(t):
    text = f"{t[0]} -> {t[1].label} -> {t[2]}"
    if HAVE_LLAMA:  # pragma: no cover
        return TextNode(text=text)
    return TextNodeLite(id_=f"{_node_id(t[0])}|{t[1].label}|{_node_id(t[2])}", text=text)


if HAVE_LLAMA:  # pragma: no cover
    class MI355XVectorContextRetriever(_VectorContextImpl, BaseRetriever):
        def __init__(self, graph_store, embed_model=None, vector_store=None, similarity_top_k=4,
                     path_depth=1, limit=30, similarity_score=None, filters=None,
                     include_text=True, **kw):
            BaseRetriever.__init__(self, **kw)
            self._setup(graph_store, embed_model, vector_store, similarity_top_k, path_depth,
                        limit, similarity_score, filters, include_text)

        def _retrieve(self, query_bundle):
            return self.retrieve_from_graph(query_bundle)
else:
    class MI355XVectorContextRetriever(_VectorContextImpl):
        def __init__(self, graph_store, embed_model=None, vector_store=None, similarity_top_k=4,
                     path_depth=1, limit=30, similarity_score=None, filters=None,
                     include_text=True):
            self._setup(graph_store, embed_model, vector_store, similarity_top_k, path_depth,
                        limit, similarity_score, filters, include_text)


class MI355XVectorRetriever:
    """Plain vector retriever: ``retrieve(str | embedding) -> [(node, score)]`` of the
    ``similarity_top_k`` best nodes of a vector store (the vector half of the above)."""

    def __init__(self, vector_store, embed_model=None, similarity_top_k: int = 4, filters=None):
        self.vector_store = vector_store
        self.embed_model = embed_model
        self.similarity_top_k = _check_top_k(similarity_top_k)
        self.filters = filters

    def retrieve(self, query) -> List[tuple]:
        if isinstance(query, str):
            if self.embed_model is None:
                raise ValueError("text query needs an embed_model")
            emb = self.embed_model.get_query_embedding(query)
        else:
            emb = getattr(query, "embedding", None)
            emb = query if emb is None else emb
        res = self.vector_store.query(VectorStoreQuery(query_embedding=list(emb),
                                                       similarity_top_k=self.similarity_top_k,
                                                       filters=self.filters))
        return list(zip(res.nodes, res.similarities))


# ---------------------------------------------------------------------------------------------
# BaseEmbedding (HuggingFaceEmbedding replacement)
# ---------------------------------------------------------------------------------------------
if HAVE_LLAMA:  # pragma: no cover
    from .encoder import MI355XEmbedding as _DuckEmbedding

    class MI355XEmbedding(BaseEmbedding):
        """``BaseEmbedding`` subclass (graph_builder.py:146-149, query_interface.py:136-139):
        the sentence-embedding forward on the MI355X (reference precision by default)."""
        _impl: Any = PrivateAttr()

        def __init__(self, model_name: str, embed_batch_size: int = 10, dtype: str = "f32",
                     device: int = 0, max_length: Optional[int] = None,
                     query_instruction: Optional[str] = None,
                     text_instruction: Optional[str] = None, **kw):
            super().__init__(model_name=model_name, embed_batch_size=embed_batch_size, **kw)
            self._impl = _DuckEmbedding(model_name, embed_batch_size=embed_batch_size, dtype=dtype,
                                        device=device, max_length=max_length,
                                        query_instruction=query_instruction,
                                        text_instruction=text_instruction)

        @classmethod
        def class_name(cls) -> str:
            return "MI355XEmbedding"

        def _get_query_embedding(self, query: str) -> List[float]:
            return self._impl._get_query_embedding(query)

        async def _aget_query_embedding(self, query: str) -> List[float]:
            return self._impl._get_query_embedding(query)

        def _get_text_embedding(self, text: str) -> List[float]:
            return self._impl._get_text_embedding(text)

        def _get_text_embeddings(self, texts: List[str]) -> List[List[float]]:
            return self._impl._get_text_embeddings(texts)
else:
    from .encoder import MI355XEmbedding  # noqa: F401  (duck-typed BaseEmbedding surface)


__all__ = ["MI355XVectorStore", "MI355XVectorRetriever", "MI355XVectorContextRetriever",
           "MI355XPropertyGraphStore", "MI355XEmbedding", "VectorStoreQuery",
           "VectorStoreQueryResult", "NodeWithScore", "QueryBundle", "TextNodeLite",
           "EntityNodeLite", "ChunkNodeLite", "RelationLite", "KG_SOURCE_REL", "HAVE_LLAMA",
           "MAX_TOP_K"]
