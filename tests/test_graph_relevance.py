"""Retrieve -> NodeInput -> isRelevant with batched node embeddings (SURVEY.md §8(f) rank 4;
experiments/graph_relevance_integration.py:38-305, experiments/enhanced_rag_system.py:
87-200).  CPU: the keyword / intent / node-type rules against hand-worked answers from those
lines.  GPU: the whole pipeline against the reference's per-node loop restated over the oracle
(sklearn cosine + one encode per node + oracle.relevance), same ids, same node embeddings,
scores within 1e-9 (fp32 vs fp64 vector storage), and the encode-call count it saves."""
import zlib

import numpy as np
import pytest

from oracle import relevance as R


def test_entity_intent_type_rules():
    from hcrag_amd import graph_relevance as G
    from hcrag_amd.relevance import QueryIntent as QI
    # keywords in list order, substring matches (:87-110)
    assert G.extract_entities_from_content("Red Mountain Bike with brakes") == \
        ["mountain bike", "bike", "brake", "red"]
    assert G.extract_entities_from_content("Quarterly sales summary, 2021") == \
        ["quarterly", "sales", "summary"]
    assert G.extract_entities_from_content("An ox is") == []
    assert len(G.extract_entities_from_content("bike frame wheel tire gear chain")) == 5
    assert G.extract_entities_simple("Find the best touring bicycles, please!") == \
        ["best", "touring", "bicycles", "please"]
    # first matching group wins (:112-127); "show" precedes "help"
    assert G.infer_query_intent("show me the manual") == QI.PRODUCT_SEARCH
    assert G.infer_query_intent("user manual for the frame") == QI.DOCUMENT_REQUEST
    assert G.infer_query_intent("fix a flat") == QI.TECHNICAL_SUPPORT
    assert G.infer_query_intent("road vs mountain") == QI.COMPARISON_REQUEST
    assert G.infer_query_intent("frame details") == QI.SPECIFICATION_INQUIRY
    assert G.infer_query_intent("bikes") == QI.PRODUCT_SEARCH
    assert G.infer_query_intent_enhanced("technical guide") == QI.DOCUMENT_REQUEST
    assert G.infer_query_intent_enhanced("technical help") == QI.SPECIFICATION_INQUIRY
    # node types (:48-63 and enhanced :171-182)
    assert G.node_type_from_metadata({"type": "database_table", "table_name": "Product"}) == "product"
    assert G.node_type_from_metadata({"type": "database_table", "table_name": "ProductModel"}) == "specification"
    assert G.node_type_from_metadata({"type": "database_table", "table_name": "Category"}) == "category"
    assert G.node_type_from_metadata({"type": "json_table"}) == "specification"
    assert G.node_type_from_metadata({}) == "unknown"
    assert G.node_type_from_metadata_enhanced({"type": "database_table", "table_name": "ProductModel"}) == "product"
    assert G.node_type_from_metadata_enhanced({}) == "specification"


class _Embedder:
    """Deterministic text -> unit fp32 vector; counts encode calls and texts."""

    def __init__(self, dim):
        self.dim, self.calls, self.texts = dim, 0, 0

    def vec(self, t):
        v = np.random.default_rng(zlib.crc32(t.encode())).standard_normal(self.dim)
        return (v / np.linalg.norm(v)).astype(np.float32)

    def encode(self, texts):
        self.calls += 1
        self.texts += len(texts)
        return np.stack([self.vec(t) for t in texts])


def _corpus(emb, n):
    rng = np.random.default_rng(7)
    words = ["bike", "red", "frame", "manual", "wheel", "gear", "helmet", "road bike", "chain",
             "saddle", "blue", "summary", "sales"]
    tables = [{"type": "database_table", "table_name": t} for t in ("Product", "ProductCategory", "SalesOrder")]
    tables += [{"type": "pdf_document"}, {"type": "json_table"}, {"type": "other"}]
    texts = [" ".join(rng.choice(words, 4)) + f" item {i}" for i in range(n)]
    meta = [dict(tables[i % len(tables)], row=i) for i in range(n)]
    return texts, meta, emb.encode(texts)


@pytest.mark.gpu
def test_graph_relevance_pipeline_matches_reference_loop():
    from sklearn.metrics.pairwise import cosine_similarity
    from hcrag_amd import EmbeddingSearch
    from hcrag_amd import graph_relevance as G
    from hcrag_amd.relevance import ScorerType
    emb = _Embedder(64)
    texts, meta, E = _corpus(emb, 500)
    search = EmbeddingSearch(E, texts, meta, dtype="f32", embedder=emb)
    sc = G.GraphRelevanceScorer(search, emb)
    query = "show me a red mountain bike frame"
    q = emb.vec(query)
    connected = [{"content": "helmet and saddle accessories"}, {"content": "blue chain", "metadata": {"type": "json_table"}}]
    llm = np.linspace(0.2, 0.9, 8 + len(connected))
    emb.calls = emb.texts = 0
    out = sc.score_query_against_graph(query, top_k=8, similarity_threshold=-1.0,
                                       scorer_types=[ScorerType.COMPOSITE, ScorerType.ROUTER_TWO_ENT_TYPE,
                                                     ScorerType.ROUTER_SINGLE_SEM, ScorerType.PARALLEL],
                                       connected_results=connected, llm_scores=llm)
    # one query encode + one batched encode for the connected nodes; direct matches reuse rows
    assert emb.calls == 2 and emb.texts == 1 + len(connected)
    # the reference's loop: sklearn fp64 cosine + argsort top-k, one encode per node
    cs = cosine_similarity([q.astype(np.float64)], E.astype(np.float64))[0]
    top = np.argsort(cs)[::-1][:8]
    nodes = out["results"]["composite"]
    assert out["nodes_found"] == 10
    by_index = sorted(nodes, key=lambda x: x["node_index"])
    for j, i in enumerate(top):
        n = by_index[j]["node_data"]
        assert n.text == texts[i] and not by_index[j]["is_connected"]
        np.testing.assert_array_equal(n.embeddings, emb.vec(texts[i]))     # == the re-encode
        assert n.node_type == G.node_type_from_metadata(meta[i])
        assert abs(n.graph_relations["similarity_score"] - cs[i]) < 1e-6
    ents = [by_index[j]["node_data"].entities for j in range(10)]
    types = [by_index[j]["node_data"].node_type for j in range(10)]
    node_vecs = [emb.vec(by_index[j]["node_data"].text) for j in range(10)]
    cos_ref = cosine_similarity([q.astype(np.float64)], np.stack(node_vecs).astype(np.float64))[0]
    q_ents = G.extract_entities_from_content(query)
    for name, res in out["results"].items():
        exp = R.batch_relevance(cos_ref, q_ents, "product_search", ents, types, name, list(llm))
        got = sorted(res, key=lambda x: x["node_index"])
        np.testing.assert_allclose([g["relevance_score"] for g in got], exp, rtol=0, atol=1e-9)
        rel = [x["relevance_score"] for x in res]
        assert rel == sorted(rel, reverse=True)
    # an LLM scorer without scores -> empty list + recorded error, like the reference's except
    out2 = sc.score_query_against_graph(query, top_k=4, similarity_threshold=-1.0,
                                        scorer_types=[ScorerType.ROUTER, ScorerType.ROUTER_SINGLE_ENT])
    assert out2["results"]["router"] == [] and "router" in out2["errors"]
    assert len(out2["results"]["router_single_ent"]) == 4
    # f16 storage rounds the rows: the scorer falls back to one batched encode
    s16 = G.GraphRelevanceScorer(EmbeddingSearch(E, texts, meta, dtype="f16", embedder=emb), emb)
    emb.calls = emb.texts = 0
    nodes16, _ = s16.get_graph_nodes_for_query(query, top_k=5, similarity_threshold=-1.0)
    assert emb.calls == 2 and emb.texts == 6
    for n in nodes16:
        np.testing.assert_array_equal(n.embeddings, emb.vec(n.text))


@pytest.mark.gpu
def test_retrieve_and_rank_matches_reference_loop():
    from sklearn.metrics.pairwise import cosine_similarity
    from hcrag_amd import EmbeddingSearch
    from hcrag_amd import graph_relevance as G
    from hcrag_amd.relevance import ScorerType
    emb = _Embedder(48)
    texts, meta, E = _corpus(emb, 300)
    sc = G.GraphRelevanceScorer(EmbeddingSearch(E, texts, meta, dtype="f32", embedder=emb), emb)
    query = "technical details of the road bike gear"
    ranked, qi = G.retrieve_and_rank(sc, query, top_k=6, similarity_threshold=-1.0,
                                     scorer_type=ScorerType.ROUTER_TWO_ENT_TYPE)
    q = emb.vec(query).astype(np.float64)
    cs = cosine_similarity([q], E.astype(np.float64))[0]
    cand = np.argsort(cs)[::-1][:12]
    ents = [G.extract_entities_simple(texts[i]) for i in cand]
    types = [G.node_type_from_metadata_enhanced(meta[i]) for i in cand]
    rel = R.batch_relevance(cs[cand], G.extract_entities_simple(query),
                            G.infer_query_intent_enhanced(query).value, ents, types,
                            "router_two_ent_type")
    comb = [r * 0.7 + cs[i] * 0.3 for r, i in zip(rel, cand)]
    order = sorted(range(12), key=lambda j: comb[j], reverse=True)[:6]
    assert [r["content"] for r in ranked] == [texts[cand[j]] for j in order]
    np.testing.assert_allclose([r["combined_score"] for r in ranked], [comb[j] for j in order],
                               rtol=0, atol=1e-6)
    assert qi.intent == G.infer_query_intent_enhanced(query)
    assert G.retrieve_and_rank(sc, query, top_k=3, similarity_threshold=2.0) == ([], None)
