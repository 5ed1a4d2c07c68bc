"""Drop-in for the reference's isRelevant scoring (experiments/isRelevant.py), the non-LLM
metrics and every combiner on the GPU (hcr_relevance_combine, csrc/relevance.hip).

Same names and behaviour as the reference module:
  * ``QueryIntent``, ``ScorerType``, ``CompositeWeights`` (:12-116; weights must sum to 1 and
    be non-negative, ValueError otherwise), ``priority_matrix`` (:128-169)
  * ``batch_semantic_similarity`` (:197-210) -> the exact fp64 GPU cosine, ``(cos+1)/2``
  * ``batch_entity_match`` (:300-324), ``batch_node_type_priority`` (:327-346)
  * ``batch_isRelevant`` (:425-501), ``isRelevant`` (:406-422)
The LLM judge (:213-297) is an external service call and out of scope: scorers that need it
take ``llm_scores`` (one float per node) or an ``llm_judge(query, nodes) -> List[float]``
callable, and raise ValueError without either.  ``score_retrieved`` is the batched form for
many queries x their retrieved top-k nodes.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import Enum
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np

from ._lib import check, lib

_c = __import__("ctypes")


class QueryIntent(Enum):
    PRODUCT_SEARCH = "product_search"
    DOCUMENT_REQUEST = "document_request"
    TECHNICAL_SUPPORT = "technical_support"
    COMPARISON_REQUEST = "comparison_request"
    SPECIFICATION_INQUIRY = "specification_inquiry"


class ScorerType(Enum):
    COMPOSITE = "composite"
    PARALLEL = "parallel"
    ROUTER = "router"
    ROUTER_ALL = "router_all"
    ROUTER_TWO_SEM_LLM = "router_two_sem_llm"
    ROUTER_TWO_ENT_TYPE = "router_two_ent_type"
    ROUTER_SINGLE_SEM = "router_single_sem"
    ROUTER_SINGLE_LLM = "router_single_llm"
    ROUTER_SINGLE_ENT = "router_single_ent"
    ROUTER_SINGLE_TYPE = "router_single_type"


@dataclass
class QueryInput:
    """isRelevant.py:20-25."""
    text: str
    embeddings: np.ndarray
    entities: List[str]
    intent: QueryIntent


@dataclass
class NodeInput:
    """isRelevant.py:28-34."""
    text: str
    embeddings: np.ndarray
    graph_relations: Dict[str, Any]
    node_type: str
    entities: List[str]


# hcr_rel_scorer codes (include/hcrag.h)
_SCORER_CODE = {ScorerType.COMPOSITE: 0, ScorerType.PARALLEL: 1, ScorerType.ROUTER: 2,
                ScorerType.ROUTER_ALL: 3, ScorerType.ROUTER_TWO_SEM_LLM: 4,
                ScorerType.ROUTER_TWO_ENT_TYPE: 5, ScorerType.ROUTER_SINGLE_SEM: 6,
                ScorerType.ROUTER_SINGLE_LLM: 7, ScorerType.ROUTER_SINGLE_ENT: 8,
                ScorerType.ROUTER_SINGLE_TYPE: 9}
# scorers whose combination reads the LLM score (isRelevant.py:504-514)
_NEEDS_LLM = {ScorerType.COMPOSITE, ScorerType.PARALLEL, ScorerType.ROUTER, ScorerType.ROUTER_ALL,
              ScorerType.ROUTER_TWO_SEM_LLM, ScorerType.ROUTER_SINGLE_LLM}


@dataclass
class CompositeWeights:
    """isRelevant.py:37-98."""
    semantic_similarity: float = 0.3
    llm_judge: float = 0.45
    entity_match: float = 0.15
    node_type_priority: float = 0.10

    def __post_init__(self):
        total = self.semantic_similarity + self.llm_judge + self.entity_match + self.node_type_priority
        if abs(total - 1.0) > 0.001:
            raise ValueError(f"Weights must sum to 1.0, got {total}")
        for f in ("semantic_similarity", "llm_judge", "entity_match", "node_type_priority"):
            if getattr(self, f) < 0:
                raise ValueError(f"Weight {f} must be non-negative, got {getattr(self, f)}")

    @classmethod
    def create_balanced(cls):
        return cls(0.25, 0.25, 0.25, 0.25)

    @classmethod
    def create_semantic_focused(cls):
        return cls(0.6, 0.2, 0.1, 0.1)

    @classmethod
    def create_llm_focused(cls):
        return cls(0.2, 0.6, 0.1, 0.1)

    @classmethod
    def create_entity_focused(cls):
        return cls(0.2, 0.2, 0.4, 0.2)

    @classmethod
    def from_dict(cls, w: Dict[str, float]):
        return cls(semantic_similarity=w.get("semantic_similarity", 0.3),
                   llm_judge=w.get("llm_judge", 0.45), entity_match=w.get("entity_match", 0.15),
                   node_type_priority=w.get("node_type_priority", 0.10))

    def to_dict(self) -> Dict[str, float]:
        return {"semantic_similarity": self.semantic_similarity, "llm_judge": self.llm_judge,
                "entity_match": self.entity_match, "node_type_priority": self.node_type_priority}

    def as_array(self) -> np.ndarray:
        return np.array([self.semantic_similarity, self.llm_judge, self.entity_match,
                         self.node_type_priority], dtype=np.float64)


DEFAULT_COMPOSITE_WEIGHTS = CompositeWeights()

priority_matrix = {
    QueryIntent.PRODUCT_SEARCH: {"product": 1.0, "category": 0.8, "specification": 0.6,
                                 "document": 0.3, "annotation": 0.2, "unknown": 0.1},
    QueryIntent.DOCUMENT_REQUEST: {"document": 1.0, "specification": 0.7, "annotation": 0.6,
                                   "product": 0.4, "category": 0.2, "unknown": 0.1},
    QueryIntent.TECHNICAL_SUPPORT: {"document": 1.0, "specification": 0.9, "annotation": 0.7,
                                    "product": 0.6, "category": 0.3, "unknown": 0.1},
    QueryIntent.COMPARISON_REQUEST: {"product": 1.0, "specification": 0.8, "category": 0.6,
                                     "document": 0.4, "annotation": 0.3, "unknown": 0.1},
    QueryIntent.SPECIFICATION_INQUIRY: {"specification": 1.0, "product": 0.7, "annotation": 0.6,
                                        "document": 0.5, "category": 0.3, "unknown": 0.1},
}


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(_c.c_void_p)


class _Tables:
    """Entity vocabulary -> bitsets, node types / intents -> table indices."""

    def __init__(self, query_entities: Sequence[Sequence[str]], node_entities: Sequence[Sequence[str]],
                 node_types: Sequence[str], intents: Sequence[QueryIntent]):
        vocab: Dict[str, int] = {}
        for ents in list(query_entities) + list(node_entities):
            for e in ents:
                vocab.setdefault(e, len(vocab))
        self.words = max(1, (len(vocab) + 31) // 32)

        def bits(ents):
            b = np.zeros(self.words, dtype=np.uint32)
            for e in set(ents):
                i = vocab[e]
                b[i >> 5] |= np.uint32(1 << (i & 31))
            return b
        self.qbits = np.stack([bits(e) for e in query_entities]) if len(query_entities) else \
            np.zeros((0, self.words), np.uint32)
        self.nbits = np.stack([bits(e) for e in node_entities]) if len(node_entities) else \
            np.zeros((0, self.words), np.uint32)
        self.ncount = np.array([len(set(e)) for e in node_entities], dtype=np.int32)
        # type columns: the matrix's own types, then any other type -> "unknown" column
        intents_all = list(QueryIntent)
        types = sorted({t for row in priority_matrix.values() for t in row})
        col = {t: i for i, t in enumerate(types)}
        self.prio = np.array([[priority_matrix[it].get(t, priority_matrix[it]["unknown"])
                               for t in types] for it in intents_all], dtype=np.float64)
        unk = col["unknown"]
        self.ntype = np.array([col.get(t, unk) for t in node_types], dtype=np.int32)
        self.intent = np.array([intents_all.index(QueryIntent(getattr(i, "value", i)))
                                for i in intents], dtype=np.int32)
        self.n_types = len(types)
        self.n_intents = len(intents_all)


def _combine(cos: np.ndarray, ids: Optional[np.ndarray], t: _Tables, scorer: ScorerType,
             weights: CompositeWeights, llm: Optional[np.ndarray], device: int) -> np.ndarray:
    cos = np.ascontiguousarray(cos, dtype=np.float64)
    nq, nn = cos.shape
    out = np.empty((nq, nn), dtype=np.float64)
    ids_a = None if ids is None else np.ascontiguousarray(ids, dtype=np.int64)
    llm_a = None if llm is None else np.ascontiguousarray(llm, dtype=np.float64).reshape(nq, nn)
    w = weights.as_array()
    check(lib().hcr_relevance_combine(
        int(device), _ptr(cos), _ptr(ids_a), nq, nn, int(t.nbits.shape[0]), _ptr(t.nbits),
        _ptr(t.ncount), t.words, _ptr(t.qbits), _ptr(t.ntype), _ptr(t.intent), _ptr(t.prio),
        t.n_intents, t.n_types, _ptr(llm_a), _SCORER_CODE[scorer], _ptr(w), _ptr(out)))
    return out


def batch_semantic_similarity(query, nodes, device: int = 0) -> List[float]:
    from .retrieval import batch_semantic_similarity as _bss
    return _bss(query, nodes, device=device)


def _cosines(query, nodes, device: int) -> np.ndarray:
    """Exact fp64 cosines of the query against every node (retrieval's scratch index, cosine
    mode; the kernel applies (cos + 1) / 2 like isRelevant.py:208)."""
    from . import retrieval as R
    from ._lib import HCR_SCORE_COSINE
    q = R._embedding_of(query)
    E = np.stack([R._embedding_of(n) for n in nodes])
    if E.shape[1] != q.shape[0]:
        raise ValueError(f"Incompatible dimension for X and Y matrices: X.shape[1] == "
                         f"{q.shape[0]} while Y.shape[1] == {E.shape[1]}")
    with R._scratch_lock:
        ix = R._scratch_index(q.shape[0], device)
        ix.reset()
        ix.add(E.astype(np.float32), normalize=False)
        return ix.score_all(q.astype(np.float32).reshape(1, -1), score_mode=HCR_SCORE_COSINE)[0]


def _single(query, nodes, scorer: ScorerType, llm=None, device: int = 0,
            weights: CompositeWeights = DEFAULT_COMPOSITE_WEIGHTS, cos=None) -> List[float]:
    if not nodes:
        return []
    t = _Tables([getattr(query, "entities", [])], [getattr(n, "entities", []) for n in nodes],
                [getattr(n, "node_type", "unknown") for n in nodes],
                [getattr(query, "intent", QueryIntent.PRODUCT_SEARCH)])
    if cos is None:
        cos = _cosines(query, nodes, device) if scorer not in (
            ScorerType.ROUTER_SINGLE_ENT, ScorerType.ROUTER_SINGLE_TYPE,
            ScorerType.ROUTER_TWO_ENT_TYPE, ScorerType.ROUTER_SINGLE_LLM) else np.zeros(len(nodes))
    out = _combine(np.asarray(cos, np.float64).reshape(1, -1), None, t, scorer, weights,
                   None if llm is None else np.asarray(llm, np.float64), device)
    return [float(v) for v in out[0]]


def batch_entity_match(query, nodes, device: int = 0) -> List[float]:
    """isRelevant.py:300-324 on the GPU."""
    return _single(query, nodes, ScorerType.ROUTER_SINGLE_ENT, device=device)


def batch_node_type_priority(query, nodes, device: int = 0) -> List[float]:
    """isRelevant.py:327-346 on the GPU."""
    return _single(query, nodes, ScorerType.ROUTER_SINGLE_TYPE, device=device)


def _llm_scores(query, nodes, scorer, llm_scores, llm_judge, batch_size):
    if scorer not in _NEEDS_LLM:
        return None
    if llm_scores is not None:
        s = list(llm_scores)
    elif llm_judge is not None:
        s = []
        for i in range(0, len(nodes), max(1, int(batch_size))):   # isRelevant.py:517-527
            s.extend(llm_judge(query, nodes[i:i + batch_size]))
    else:
        raise ValueError(f"scorer {scorer.value} needs LLM judge scores: pass llm_scores= or "
                         "llm_judge= (the reference's LLM call is out of scope here)")
    if len(s) != len(nodes):
        raise ValueError("one LLM score per node expected")
    return np.asarray(s, dtype=np.float64)


def batch_isRelevant(query, nodes: Sequence[Any], scorer_type: ScorerType, batch_size: int = 10,
                     weights: CompositeWeights = DEFAULT_COMPOSITE_WEIGHTS,
                     llm_scores: Optional[Sequence[float]] = None,
                     llm_judge: Optional[Callable] = None, device: int = 0) -> List[float]:
    """isRelevant.py:425-501 with the non-LLM metrics and the combination on the GPU."""
    if not nodes:
        return []
    nodes = list(nodes)
    llm = _llm_scores(query, nodes, scorer_type, llm_scores, llm_judge, batch_size)
    return _single(query, nodes, scorer_type, llm=llm, device=device, weights=weights)


def isRelevant(query, node, scorer_type: ScorerType,
               weights: CompositeWeights = DEFAULT_COMPOSITE_WEIGHTS, **kw) -> float:
    """isRelevant.py:406-422."""
    return batch_isRelevant(query, [node], scorer_type, batch_size=1, weights=weights, **kw)[0]


def score_retrieved(cos: np.ndarray, ids: np.ndarray, query_entities: Sequence[Sequence[str]],
                    query_intents: Sequence[QueryIntent], node_entities: Sequence[Sequence[str]],
                    node_types: Sequence[str], scorer_type: ScorerType = ScorerType.ROUTER_ALL,
                    weights: CompositeWeights = DEFAULT_COMPOSITE_WEIGHTS,
                    llm_scores: Optional[np.ndarray] = None, device: int = 0) -> np.ndarray:
    """Relevance of every (query, retrieved node): ``cos`` / ``ids`` are a search's [nq][k]
    exact cosines and global row ids (-1 = padding -> -inf); node arrays are per corpus row."""
    t = _Tables(query_entities, node_entities, node_types, query_intents)
    if scorer_type in _NEEDS_LLM and llm_scores is None:
        raise ValueError(f"scorer {scorer_type.value} needs llm_scores")
    return _combine(cos, ids, t, scorer_type, weights, llm_scores, device)


__all__ = ["QueryIntent", "ScorerType", "QueryInput", "NodeInput", "CompositeWeights", "DEFAULT_COMPOSITE_WEIGHTS",
           "priority_matrix", "batch_semantic_similarity", "batch_entity_match",
           "batch_node_type_priority", "batch_isRelevant", "isRelevant", "score_retrieved"]
