"""CPU: pin the oracle to the reference's known answers and to sklearn goldens."""
import glob
import json
import os

import numpy as np
import pytest

from oracle import cosine_topk as O


def _vec(name, ka):
    d = ka["dim"]
    if name == "ones":
        return np.ones(d)
    if name == "-ones":
        return -np.ones(d)
    if name == "e0":
        v = np.zeros(d); v[0] = 1.0; return v
    if name == "e1":
        v = np.zeros(d); v[1] = 1.0; return v
    if name == "random":
        return np.array(ka["random_node"])
    raise KeyError(name)


def test_known_answers(golden_dir):
    """tests/unit/test_milestone1_core_components.py:108-175 through the oracle."""
    ka = json.load(open(os.path.join(golden_dir, "known_answers.json")))
    np.random.seed(ka["random_node_seed"])
    assert np.array_equal(np.random.rand(ka["dim"]), np.array(ka["random_node"]))
    for case in ka["cases"]:
        got = O.batch_semantic_similarity(_vec(case["query"], ka),
                                          [_vec(n, ka) for n in case["nodes"]])
        assert len(got) == len(case["nodes"])
        if "tol" in case:
            for g, e in zip(got, case["expected"]):
                assert abs(g - e) < case["tol"]
        if "range" in case:
            lo, hi = case["range"]
            assert all(lo <= g <= hi for g in got)
            np.testing.assert_allclose(got, case["expected"], rtol=0, atol=1e-15)


def test_empty_nodes():
    assert O.batch_semantic_similarity(np.ones(4), []) == []


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(
    os.path.dirname(__file__), "golden", "cos_*.npz"))))
def test_oracle_matches_sklearn_goldens(path):
    g = np.load(path)
    E, Q, k = g["E"], g["Q"], int(g["k"])
    s, i = O.cosine_topk(Q, E, k)
    np.testing.assert_array_equal(i, g["ids"])
    np.testing.assert_allclose(s, g["scores"], rtol=0, atol=1e-12)


def test_oracle_vs_installed_sklearn_random():
    from sklearn.metrics.pairwise import cosine_similarity
    rng = np.random.default_rng(0)
    X = rng.standard_normal((5, 33))
    Y = rng.standard_normal((40, 33))
    Y[3] = 0
    np.testing.assert_allclose(O.cosine_similarity64(X, Y), cosine_similarity(X, Y),
                               rtol=0, atol=1e-14)


def test_oracle_chunked_equals_unchunked_with_mask_threshold():
    rng = np.random.default_rng(1)
    E = rng.standard_normal((300, 16))
    Q = rng.standard_normal((4, 16))
    mask = rng.random(300) > 0.3
    a = O.cosine_topk(Q, E, 9, score_mode=1, threshold=0.55, rowmask=mask, chunk_rows=64)
    b = O.cosine_topk(Q, E, 9, score_mode=1, threshold=0.55, rowmask=mask, chunk_rows=1 << 20)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0], b[0])
    assert np.all(mask[a[1][a[1] >= 0]])
    assert np.all(a[0][a[1] >= 0] >= 0.55)


def test_find_similar_content_and_category():
    rng = np.random.default_rng(2)
    M = rng.standard_normal((50, 8))
    q = M[4] + 0.01
    r = O.find_similar_content(q, M, top_k=5, similarity_threshold=0.3)
    assert r[0][0] == 4 and all(s >= 0.3 for _, s in r)
    valid = [i for i in range(50) if i % 2 == 0]
    c = O.search_by_category(q, M, valid, top_k=3)
    assert [x[0] for x in c] == [1, 2, 3] and c[0][2] == 4


def test_llama_semantics_cutoff_strict():
    s, ids = O.llama_get_top_k_embeddings([1.0, 0.0], [[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]],
                                          similarity_top_k=2, similarity_cutoff=0.0)
    assert ids == [0, 2] and abs(s[0] - 1.0) < 1e-15
