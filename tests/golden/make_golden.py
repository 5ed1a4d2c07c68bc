"""Generate the committed golden fixtures for the cosine top-k path.

Expected outputs come from the third-party engine the reference itself calls,
``sklearn.metrics.pairwise.cosine_similarity`` (pinned 1.7.0, uv.lock:2977-2978; installed
1.7.2), on the reference's float64 path (experiments/main.py:762,841), followed by the
reference's top-k (experiments/main.py:844) under the deterministic tie rule (score desc,
row asc).  The known answers restate tests/unit/test_milestone1_core_components.py:108-175.
No reference module is imported (none is importable here).

Run:  python tests/golden/make_golden.py   (writes tests/golden/*.npz, known_answers.json)
"""
import json
import os

import numpy as np
from sklearn.metrics.pairwise import cosine_similarity

HERE = os.path.dirname(os.path.abspath(__file__))


def topk_rows(sim, k):
    order = np.lexsort((np.arange(sim.shape[0]), -sim))
    return order[:k]


def make_case(name, N, D, B, k, seed, planted=True, dup=True, zero=True):
    rng = np.random.default_rng(seed)
    E = rng.standard_normal((N, D)).astype(np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    E = E.astype(np.float16)                      # the index's storage dtype
    if zero:
        E[7] = 0                                  # zero-norm row: sklearn scores it 0
    if dup:
        E[N - 1] = E[3]                           # exact duplicate: tie broken by row id
        E[N - 2] = E[3]
    Q = rng.standard_normal((B, D)).astype(np.float32)
    if planted:                                   # half the queries: a corpus row + noise
        src = rng.integers(0, N, size=B // 2)
        Q[: B // 2] = E[src].astype(np.float32) + 0.05 * rng.standard_normal((B // 2, D)).astype(np.float32) / np.sqrt(D)
    Q[B - 1] = E[3].astype(np.float32)            # hits the duplicate triple exactly
    S = cosine_similarity(Q, E.astype(np.float64))  # reference path: fp64 matrix
    ids = np.stack([topk_rows(S[b], k) for b in range(B)]).astype(np.int64)
    sc = np.take_along_axis(S, ids, axis=1)
    np.savez(os.path.join(HERE, f"{name}.npz"), E=E, Q=Q, k=k, ids=ids, scores=sc)
    return name


def known_answers():
    """tests/unit/test_milestone1_core_components.py:108-175 re-stated as data."""
    np.random.seed(42)
    ones = np.ones(384)
    a = np.zeros(384); a[0] = 1.0
    b = np.zeros(384); b[1] = 1.0
    rnd = np.random.rand(384)                     # first draw after seed(42), as in the test
    def bss(q, nodes):
        s = cosine_similarity(q.reshape(1, -1), np.array(nodes))[0]
        return [float((v + 1) / 2) for v in s]
    return {
        "source": "tests/unit/test_milestone1_core_components.py:108-175",
        "dim": 384,
        "random_node_seed": 42,
        "random_node": rnd.tolist(),
        "cases": [
            {"name": "identical", "query": "ones", "nodes": ["ones"], "expected": [1.0], "tol": 1e-10},
            {"name": "opposite", "query": "ones", "nodes": ["-ones"], "expected": [0.0], "tol": 1e-10},
            {"name": "orthogonal", "query": "e0", "nodes": ["e1"], "expected": [0.5], "tol": 1e-10},
            {"name": "multi", "query": "ones", "nodes": ["ones", "-ones", "random"],
             "expected": bss(ones, [ones, -ones, rnd]), "range": [-1e-10, 1.0 + 1e-10]},
        ],
        "sklearn_version_used": __import__("sklearn").__version__,
    }


if __name__ == "__main__":
    make_case("cos_n1000_d384_b8_k5", 1000, 384, 8, 5, seed=1)
    make_case("cos_n500_d768_b8_k32", 500, 768, 8, 32, seed=2)
    make_case("cos_n300_d1024_b8_k64", 300, 1024, 8, 64, seed=3)
    make_case("cos_n700_d100_b8_k10", 700, 100, 8, 10, seed=4)   # dim not a multiple of 64
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(known_answers(), f, indent=1)
    print("ok")
