"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's non-LLM isRelevant metrics
and combiners, the checker for hcr_relevance_combine (hc-rag_amd/csrc/relevance.hip).

Follows /root/reference/experiments/isRelevant.py:
  * batch_semantic_similarity  :197-210  ((cos + 1) / 2; cos given here)
  * batch_entity_match         :300-324  (set intersection ratio; 0.5 / 0.1 with no query entities)
  * batch_node_type_priority   :327-346  (priority_matrix :128-169, "unknown" fallback)
  * batch_isRelevant combiners :445-501  (composite / parallel / router variants)
The reference module itself is not importable here (it imports ``openai``);
parity of this restatement is pinned by the known answers in tests/test_relevance.py, which
are worked by hand from those lines.  Pure Python on purpose (small cases only).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

# experiments/isRelevant.py:128-169 (intent -> node type -> priority)
PRIORITY_MATRIX: Dict[str, Dict[str, float]] = {
    "product_search": {"product": 1.0, "category": 0.8, "specification": 0.6, "document": 0.3,
                       "annotation": 0.2, "unknown": 0.1},
    "document_request": {"document": 1.0, "specification": 0.7, "annotation": 0.6,
                         "product": 0.4, "category": 0.2, "unknown": 0.1},
    "technical_support": {"document": 1.0, "specification": 0.9, "annotation": 0.7,
                          "product": 0.6, "category": 0.3, "unknown": 0.1},
    "comparison_request": {"product": 1.0, "specification": 0.8, "category": 0.6,
                           "document": 0.4, "annotation": 0.3, "unknown": 0.1},
    "specification_inquiry": {"specification": 1.0, "product": 0.7, "annotation": 0.6,
                              "document": 0.5, "category": 0.3, "unknown": 0.1},
}


def entity_match(query_entities: Sequence[str], node_entities: Sequence[str]) -> float:
    """isRelevant.py:305-322."""
    q, n = set(query_entities), set(node_entities)
    if len(q) == 0:
        return 0.5 if len(n) == 0 else 0.1
    return len(q.intersection(n)) / len(q)


def node_type_priority(intent: str, node_type: str) -> float:
    """isRelevant.py:332-344."""
    row = PRIORITY_MATRIX[intent]
    return row[node_type] if node_type in row else row["unknown"]


def combine(scorer: str, sem: float, llm: float, ent: float, typ: float,
            w: Sequence[float] = (0.3, 0.45, 0.15, 0.10)) -> float:
    """isRelevant.py:448-499 (single-metric routers :449-457, combiners :479-497)."""
    if scorer == "router_single_sem":
        return sem
    if scorer == "router_single_ent":
        return ent
    if scorer == "router_single_type":
        return typ
    if scorer == "router_single_llm":
        return llm
    if scorer == "parallel":
        return max(sem, llm, ent, typ)
    if scorer == "router":
        return (sem + llm + typ) / 3
    if scorer == "router_all":
        return (sem + llm + ent + typ) / 4
    if scorer == "router_two_sem_llm":
        return (sem + llm) / 2
    if scorer == "router_two_ent_type":
        return (ent + typ) / 2
    return sem * w[0] + llm * w[1] + ent * w[2] + typ * w[3]     # composite / fallback


def batch_relevance(cos: Sequence[float], query_entities: Sequence[str], intent: str,
                    node_entities: Sequence[Sequence[str]], node_types: Sequence[str],
                    scorer: str, llm: Optional[Sequence[float]] = None,
                    w: Sequence[float] = (0.3, 0.45, 0.15, 0.10)) -> List[float]:
    """batch_isRelevant (:425-501) for one query with the semantic cosines given."""
    out = []
    for j, c in enumerate(cos):
        sem = (c + 1) / 2
        ent = entity_match(query_entities, node_entities[j])
        typ = node_type_priority(intent, node_types[j])
        l = float(llm[j]) if llm is not None else 0.0
        out.append(combine(scorer, sem, l, ent, typ, w))
    return out
