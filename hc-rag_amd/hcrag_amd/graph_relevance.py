"""Retrieve -> NodeInput -> isRelevant with the per-node re-encode batched away (SURVEY.md
§8(f) rank 4).

The reference turns every retrieved row back into a ``NodeInput`` by re-encoding its text one
row at a time (``model.encode([content])[0]``):
  * experiments/graph_relevance_integration.py:38-85 (``convert_rag_result_to_node_input``),
    driven by ``get_graph_nodes_for_query`` (:149-212) and ``score_query_against_graph``
    (:214-305), which then calls ``isRelevant`` once per (node, scorer);
  * experiments/enhanced_rag_system.py:110-200 (``retrieve_and_rank`` /
    ``_create_node_input_from_result``), one ``isRelevant`` per node again.
Here the node embeddings of a whole result list come from one place:
  * ``node_embeddings="index"`` (default): the rows the search just ranked, read back from the
    resident index (``hcr_index_get_rows``) -- the vectors the corpus was built from, so the
    same values the re-encode produces (the encoder is deterministic); used when the index
    stores fp32 rows, since fp16/bf16 storage has rounded them;
  * otherwise, and for nodes that carry no row id (subgraph-expansion nodes), ONE batched
    ``embedder.encode(texts)`` call for all of them.
Scoring is ``relevance.batch_isRelevant`` -- one GPU launch per scorer for every node.

Graph expansion itself (the Neo4j subgraph, :185-208) and the LLM query parser of
``process_query`` are out of scope: expansion nodes are passed in as ``connected_results``
(dicts with ``content`` / ``metadata``), the LLM judge as ``llm_scores`` / ``llm_judge``.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .relevance import NodeInput, QueryInput, QueryIntent, ScorerType, batch_isRelevant

# graph_relevance_integration.py:90-97
_KEYWORDS = ["mountain bike", "road bike", "bike", "bicycle", "frame", "handlebar", "wheel",
             "tire", "brake", "gear", "pedal", "chain", "saddle", "helmet", "red", "black",
             "blue", "white", "green", "small", "medium", "large", "xl", "xs"]


def extract_entities_from_content(content: str) -> List[str]:
    """graph_relevance_integration.py:87-110: listed keywords found in the text (list order),
    else the first three words longer than 2 characters, lower-cased and stripped; at most 5."""
    low = content.lower()
    found = [k for k in _KEYWORDS if k in low]
    if not found:
        found = [w.lower().strip('.,!?') for w in content.split()[:3] if len(w) > 2]
    return found[:5]


def extract_entities_simple(text: str) -> List[str]:
    """enhanced_rag_system.py:102-108."""
    stop = ['find', 'show', 'what', 'where', 'when', 'how']
    return [w.lower().strip('.,!?') for w in text.split()
            if len(w) > 3 and w.lower() not in stop][:5]


def infer_query_intent(query: str) -> QueryIntent:
    """graph_relevance_integration.py:112-127 (first matching keyword group wins)."""
    q = query.lower()
    for words, intent in ((["find", "search", "show", "get", "buy"], QueryIntent.PRODUCT_SEARCH),
                          (["manual", "document", "guide", "instructions"], QueryIntent.DOCUMENT_REQUEST),
                          (["help", "support", "problem", "issue", "fix"], QueryIntent.TECHNICAL_SUPPORT),
                          (["compare", "vs", "versus", "difference"], QueryIntent.COMPARISON_REQUEST),
                          (["spec", "specification", "details", "features"],
                           QueryIntent.SPECIFICATION_INQUIRY)):
        if any(w in q for w in words):
            return intent
    return QueryIntent.PRODUCT_SEARCH


def infer_query_intent_enhanced(query: str) -> QueryIntent:
    """enhanced_rag_system.py:87-100 (its own keyword groups and order)."""
    q = query.lower()
    for words, intent in ((['manual', 'documentation', 'guide', 'instruction'], QueryIntent.DOCUMENT_REQUEST),
                          (['compare', 'vs', 'versus', 'difference'], QueryIntent.COMPARISON_REQUEST),
                          (['spec', 'specification', 'technical', 'details'],
                           QueryIntent.SPECIFICATION_INQUIRY),
                          (['help', 'support', 'troubleshoot', 'fix', 'problem'],
                           QueryIntent.TECHNICAL_SUPPORT)):
        if any(w in q for w in words):
            return intent
    return QueryIntent.PRODUCT_SEARCH


def node_type_from_metadata(metadata: Dict[str, Any]) -> str:
    """graph_relevance_integration.py:48-63."""
    t = metadata.get("type")
    if t == "database_table":
        name = metadata.get("table_name", "unknown").lower()
        if name in ["product"]:
            return "product"
        if name in ["productcategory", "category"]:
            return "category"
        return "specification"
    if t == "pdf_document":
        return "document"
    if t == "json_table":
        return "specification"
    return "unknown"


def node_type_from_metadata_enhanced(metadata: Dict[str, Any]) -> str:
    """enhanced_rag_system.py:174-184."""
    t = metadata.get("type")
    if t == "database_table":
        name = metadata.get("table_name", "").lower()
        if "product" in name:
            return "product"
        if "category" in name:
            return "category"
        return "specification"
    if t == "pdf_document":
        return "document"
    return "specification"


class GraphRelevanceScorer:
    """``GraphRelevanceScorer`` (graph_relevance_integration.py:23-305) over an
    ``EmbeddingSearch`` (the search half of ``EmbeddingRAGSystem``) and an embedder with
    ``encode(List[str]) -> ndarray`` (``SentenceEmbedder``)."""

    def __init__(self, search, embedder=None, node_embeddings: str = "index", device: int = 0):
        if node_embeddings not in ("index", "encode"):
            raise ValueError("node_embeddings must be 'index' or 'encode'")
        self.search = search
        self.embedder = embedder if embedder is not None else getattr(search, "embedder", None)
        self.node_embeddings = node_embeddings
        self.device = device
        self.encode_calls = 0           # batched encode calls made for nodes (tests / stats)

    def close(self):
        pass

    # -- query side ---------------------------------------------------------------------
    def _encode(self, texts: List[str]) -> np.ndarray:
        if self.embedder is None:
            raise ValueError("no embedder attached (needed to encode text)")
        return np.asarray(self.embedder.encode(list(texts)), dtype=np.float32)

    _extract_entities_from_content = staticmethod(extract_entities_from_content)
    _infer_query_intent = staticmethod(infer_query_intent)

    def create_query_input(self, query: str) -> QueryInput:
        """:129-147."""
        return QueryInput(text=query, embeddings=self._encode([query])[0],
                          entities=extract_entities_from_content(query),
                          intent=infer_query_intent(query))

    # -- results -> NodeInputs ----------------------------------------------------------
    def _node(self, result: Dict[str, Any], emb: np.ndarray, is_connected: bool) -> NodeInput:
        content = result.get("content", "") or ""
        metadata = result.get("metadata", {}) or {}
        return NodeInput(text=content, embeddings=emb,
                         graph_relations={"similarity_score": result.get("similarity_score", 0.0),
                                          "is_connected": is_connected, "metadata": metadata},
                         node_type=node_type_from_metadata(metadata),
                         entities=extract_entities_from_content(content))

    def convert_rag_results_to_node_inputs(self, results: Sequence[Dict[str, Any]],
                                           is_connected: bool = False,
                                           row_ids: Optional[Sequence[int]] = None) -> List[NodeInput]:
        """:38-85 for a whole result list: embeddings from the index rows (``row_ids``) when
        they are stored exactly, else one batched encode of every content."""
        results = list(results)
        if not results:
            return []
        embs: List[Optional[np.ndarray]] = [None] * len(results)
        ix = self.search.index
        if row_ids is not None and self.node_embeddings == "index" and ix.dtype == "f32":
            for j, r in enumerate(row_ids):
                if r is not None and 0 <= int(r) < len(ix):
                    embs[j] = ix.get_rows(int(r), 1)[0]
        todo = [j for j, e in enumerate(embs) if e is None]
        if todo:
            enc = self._encode([results[j].get("content", "") or "" for j in todo])
            self.encode_calls += 1
            for j, e in zip(todo, enc):
                embs[j] = e
        return [self._node(r, e, is_connected) for r, e in zip(results, embs)]

    def convert_rag_result_to_node_input(self, result: Dict[str, Any],
                                         is_connected: bool = False) -> NodeInput:
        """:38-85 (one result; one encode)."""
        return self.convert_rag_results_to_node_inputs([result], is_connected)[0]

    def _search(self, query_vec: np.ndarray, top_k: int, threshold: float):
        from ._lib import HCR_SCORE_COSINE
        ix = self.search.index
        k = max(1, min(int(top_k), len(ix)))
        s, ids = ix.search(query_vec.reshape(1, -1).astype(np.float32), k, HCR_SCORE_COSINE,
                           float(threshold))
        results, rows = [], []
        for sc, i in zip(s[0], ids[0]):
            if i < 0:
                continue
            results.append({"content": self.search.texts_list[i],
                            "metadata": self.search.metadata_list[i],
                            "similarity_score": float(sc)})
            rows.append(int(i))
        return results[:top_k], rows[:top_k]

    def get_graph_nodes_for_query(self, query: str, top_k: int = 10,
                                  similarity_threshold: float = 0.25,
                                  expand_subgraph: bool = True,
                                  connected_results: Optional[Sequence[Dict[str, Any]]] = None,
                                  query_embedding: Optional[np.ndarray] = None
                                  ) -> Tuple[List[NodeInput], Dict[str, Any]]:
        """:149-212: the top-k direct matches, then (``expand_subgraph``) the caller's
        ``connected_results`` (similarity 0, ``is_connected`` True)."""
        qv = self._encode([query])[0] if query_embedding is None else np.asarray(query_embedding, np.float32)
        results, rows = self._search(qv, top_k, similarity_threshold)
        nodes = self.convert_rag_results_to_node_inputs(results, False, rows)
        if expand_subgraph and results and connected_results:
            conn = [{"content": c.get("content", ""), "metadata": c.get("metadata", {}),
                     "similarity_score": 0.0} for c in connected_results]
            nodes.extend(self.convert_rag_results_to_node_inputs(conn, True))
        meta = {"search_text": query, "results": results, "query_embedding": qv,
                "summary": f"Found {len(results)} results with average similarity: "
                           f"{(np.mean([r['similarity_score'] for r in results]) if results else 0):.3f}"}
        return nodes, meta

    def score_query_against_graph(self, query: str, top_k: int = 10,
                                  similarity_threshold: float = 0.25,
                                  expand_subgraph: bool = True,
                                  scorer_types: Optional[List[ScorerType]] = None,
                                  connected_results: Optional[Sequence[Dict[str, Any]]] = None,
                                  llm_scores: Optional[Sequence[float]] = None,
                                  llm_judge: Optional[Callable] = None) -> Dict[str, Any]:
        """:214-305: every node scored by every scorer (one GPU launch per scorer), sorted by
        relevance (stable, descending).  A scorer that cannot run (LLM scores needed but not
        given) yields an empty list, as the reference's per-node ``except`` does."""
        if scorer_types is None:
            scorer_types = [ScorerType.COMPOSITE, ScorerType.PARALLEL, ScorerType.ROUTER]
        query_input = self.create_query_input(query)
        nodes, meta = self.get_graph_nodes_for_query(query, top_k, similarity_threshold,
                                                     expand_subgraph, connected_results,
                                                     query_embedding=query_input.embeddings)
        if not nodes:
            return {"query": query, "query_input": query_input, "nodes_found": 0,
                    "results": {}, "error": "No nodes found for scoring"}
        results: Dict[str, List[Dict[str, Any]]] = {}
        errors: Dict[str, str] = {}
        for sc in scorer_types:
            try:
                scores = batch_isRelevant(query_input, nodes, sc, llm_scores=llm_scores,
                                          llm_judge=llm_judge, device=self.device)
            except ValueError as e:
                errors[sc.value] = str(e)
                results[sc.value] = []
                continue
            scored = [{"node_index": i, "relevance_score": s, "node_type": n.node_type,
                       "is_connected": n.graph_relations.get("is_connected", False),
                       "similarity_score": n.graph_relations.get("similarity_score", 0.0),
                       "content_preview": n.text[:100] + "..." if len(n.text) > 100 else n.text,
                       "entities": n.entities, "node_data": n}
                      for i, (n, s) in enumerate(zip(nodes, scores))]
            scored.sort(key=lambda x: x["relevance_score"], reverse=True)
            results[sc.value] = scored
        out = {"query": query, "query_input": query_input, "nodes_found": len(nodes),
               "query_metadata": meta, "results": results}
        if errors:
            out["errors"] = errors
        return out


def retrieve_and_rank(scorer: GraphRelevanceScorer, query: str, top_k: int = 20,
                      similarity_threshold: float = 0.25,
                      scorer_type: ScorerType = ScorerType.COMPOSITE,
                      llm_scores: Optional[Sequence[float]] = None,
                      llm_judge: Optional[Callable] = None):
    """enhanced_rag_system.py:110-170: 2*top_k candidates above 0.7*threshold, relevance of
    all of them in one launch, ``combined = 0.7 * relevance + 0.3 * similarity``, the top_k by
    combined score.  Returns (scored_nodes, query_input); ([], None) without candidates."""
    qv = scorer._encode([query])[0]
    results, rows = scorer._search(qv, top_k * 2, similarity_threshold * 0.7)
    if not results:
        return [], None
    query_input = QueryInput(text=query, embeddings=qv, entities=extract_entities_simple(query),
                             intent=infer_query_intent_enhanced(query))
    nodes = scorer.convert_rag_results_to_node_inputs(results, False, rows)
    for n in nodes:          # enhanced_rag_system.py:171-200: its own type / entity rules
        md = n.graph_relations["metadata"]
        n.node_type = node_type_from_metadata_enhanced(md)
        n.entities = extract_entities_simple(n.text)
        n.graph_relations = {"metadata": md}
    rel = batch_isRelevant(query_input, nodes, scorer_type, llm_scores=llm_scores,
                           llm_judge=llm_judge, device=scorer.device)
    scored = [{"content": r["content"], "metadata": r["metadata"],
               "similarity_score": r["similarity_score"], "relevance_score": s,
               "combined_score": s * 0.7 + r["similarity_score"] * 0.3, "node_input": n}
              for r, n, s in zip(results, nodes, rel)]
    scored.sort(key=lambda x: x["combined_score"], reverse=True)
    return scored[:top_k], query_input


__all__ = ["GraphRelevanceScorer", "retrieve_and_rank", "extract_entities_from_content",
           "extract_entities_simple", "infer_query_intent", "infer_query_intent_enhanced",
           "node_type_from_metadata", "node_type_from_metadata_enhanced"]
