"""CPU ORACLE — test infrastructure only, never the product path.

Restates, in float64 numpy, the reference's cosine-similarity + top-k semantics.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.

Pinning (see tests/test_oracle.py):
  * the reference's own known-answer test
    ``tests/unit/test_milestone1_core_components.py:108-175`` (identical -> 1.0,
    opposite -> 0.0, orthogonal -> 0.5, range check), re-stated as fixtures in
    ``tests/golden/known_answers.json``;
  * the installed third-party engine the reference calls,
    ``sklearn.metrics.pairwise.cosine_similarity`` (pinned 1.7.0 at uv.lock:2977-2978,
    installed 1.7.2), via seeded golden vectors in ``tests/golden/*.npz`` produced by
    ``tests/golden/make_golden.py``.

Reference call sites restated here:
  * ``experiments/isRelevant.py:197-210`` ``batch_semantic_similarity``:
    ``cosine_similarity(q[1,D], E[n,D])[0]`` then ``(s + 1) / 2``; ``[]`` for no nodes.
  * ``experiments/main.py:831-857`` ``find_similar_content``: cosine over the whole matrix,
    ``np.argsort(sim)[::-1][:top_k]`` (:844), then keep ``sim >= threshold`` (:848-849).
  * ``experiments/main.py:859-905`` ``search_by_category``: same over the rows whose
    ``metadata['type'] == category`` (:872-885), no threshold.
  * sklearn ``cosine_similarity`` (installed ``sklearn/metrics/pairwise.py:1683-1738``):
    ``normalize(X) @ normalize(Y).T``; both inputs cast to float64 unless both are float32
    (``_return_float_dtype`` :51-72 — the reference's matrix is always float64,
    ``experiments/main.py:762``); row norms below ``10 * eps`` are treated as 1
    (``sklearn/preprocessing/_data.py:118``, ``_handle_zeros_in_scale``), so a zero row
    scores 0.

Tie rule: the reference's ``argsort(...)[::-1]`` uses numpy's unstable default sort, so
its order among exactly equal scores is unspecified.  The oracle (and the HIP path) use
the deterministic rule (score desc, row id asc).
"""
from __future__ import annotations

import numpy as np

_EPS64 = np.finfo(np.float64).eps


def row_norms64(X: np.ndarray) -> np.ndarray:
    """sklearn ``row_norms`` in float64 with ``_handle_zeros_in_scale`` (norm < 10 eps -> 1)."""
    X = np.asarray(X, dtype=np.float64)
    n = np.sqrt(np.einsum("ij,ij->i", X, X))
    n[n < 10 * _EPS64] = 1.0
    return n


def normalize64(X: np.ndarray) -> np.ndarray:
    """sklearn ``normalize(X, norm='l2')`` in float64 (``preprocessing/_data.py:2011-2015``)."""
    X = np.asarray(X, dtype=np.float64)
    return X / row_norms64(X)[:, None]


def cosine_similarity64(X: np.ndarray, Y: np.ndarray) -> np.ndarray:
    """sklearn ``cosine_similarity(X, Y)`` on the reference's float64 path."""
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    Y = np.atleast_2d(np.asarray(Y, dtype=np.float64))
    if X.shape[1] != Y.shape[1]:
        raise ValueError(
            f"Incompatible dimension for X and Y matrices: X.shape[1] == {X.shape[1]} "
            f"while Y.shape[1] == {Y.shape[1]}")
    return normalize64(X) @ normalize64(Y).T


def topk_order(sim: np.ndarray, k: int) -> np.ndarray:
    """Indices of the k best entries of a 1-D score vector, (score desc, index asc)."""
    n = sim.shape[0]
    k = min(k, n)
    if k <= 0:
        return np.zeros(0, dtype=np.int64)
    # argpartition first for large n (pure speed; the final order is the lexsort below)
    if n > 4 * k + 64:
        part = np.argpartition(-sim, k - 1)[:k]
        kth = sim[part].min()
        cand = np.nonzero(sim >= kth)[0]
    else:
        cand = np.arange(n)
    order = np.lexsort((cand, -sim[cand]))[:k]
    return cand[order].astype(np.int64)


def cosine_topk(Q: np.ndarray, E: np.ndarray, k: int, score_mode: int = 0,
                threshold: float = -np.inf, rowmask: np.ndarray | None = None,
                chunk_rows: int = 1 << 20):
    """Batched reference semantics: per query, top-k rows by cosine, then ``>= threshold``.

    Returns (scores float64 [B,k], ids int64 [B,k]); empty slots have id -1, score -inf.
    ``score_mode`` 1 applies the ``(s+1)/2`` map of ``experiments/isRelevant.py:208``
    before the threshold.  ``rowmask`` (bool [N]) restricts the candidate rows
    (``experiments/main.py:872-885``).  Streams E in row chunks (the 10M x 768 fp64
    matrix would not fit host RAM), keeping a running (score desc, id asc) top-k.
    """
    Q = np.atleast_2d(np.asarray(Q, dtype=np.float64))
    B = Q.shape[0]
    N = E.shape[0]
    if Q.shape[1] != E.shape[1]:
        raise ValueError("dimension mismatch")
    Qn = normalize64(Q)
    best_s = np.full((B, 0), -np.inf)
    best_i = np.zeros((B, 0), dtype=np.int64)
    for r0 in range(0, N, chunk_rows):
        r1 = min(N, r0 + chunk_rows)
        Ec = normalize64(E[r0:r1])
        S = Qn @ Ec.T
        ids = np.arange(r0, r1, dtype=np.int64)
        if rowmask is not None:
            keep = np.asarray(rowmask[r0:r1], dtype=bool)
            S = S[:, keep]
            ids = ids[keep]
        if S.shape[1] == 0:
            continue
        cs = np.concatenate([best_s, S], axis=1)
        ci = np.concatenate([best_i, np.broadcast_to(ids, (B, ids.shape[0]))], axis=1)
        kk = min(k, cs.shape[1])
        ns = np.empty((B, kk))
        ni = np.empty((B, kk), dtype=np.int64)
        for b in range(B):
            o = np.lexsort((ci[b], -cs[b]))[:kk]
            ns[b] = cs[b, o]
            ni[b] = ci[b, o]
        best_s, best_i = ns, ni
    out_s = np.full((B, k), -np.inf)
    out_i = np.full((B, k), -1, dtype=np.int64)
    s = best_s if score_mode == 0 else (best_s + 1.0) / 2.0
    ok = s >= threshold
    for b in range(B):
        sel = np.nonzero(ok[b])[0]
        out_s[b, :sel.size] = s[b, sel]
        out_i[b, :sel.size] = best_i[b, sel]
    return out_s, out_i


def batch_semantic_similarity(query_embedding: np.ndarray, node_embeddings) -> list:
    """``experiments/isRelevant.py:197-210``: ``[(s+1)/2 for s in cosine(q, E)[0]]``."""
    if len(node_embeddings) == 0:
        return []
    E = np.array([np.asarray(e) for e in node_embeddings])
    sims = cosine_similarity64(np.asarray(query_embedding).reshape(1, -1), E)[0]
    return [(s + 1) / 2 for s in sims]


def find_similar_content(query_embedding: np.ndarray, matrix: np.ndarray, top_k: int = 5,
                         similarity_threshold: float = 0.3):
    """``experiments/main.py:831-857``: [(row, score)] for top-k rows with score >= threshold."""
    sims = cosine_similarity64([query_embedding], matrix)[0]
    top = topk_order(sims, top_k)
    return [(int(i), float(sims[i])) for i in top if sims[i] >= similarity_threshold]


def search_by_category(query_embedding: np.ndarray, matrix: np.ndarray, valid_indices,
                       top_k: int = 5):
    """``experiments/main.py:859-905``: rank/score/original row over a filtered subset."""
    valid = list(valid_indices)
    if not valid:
        return []
    sims = cosine_similarity64(np.atleast_2d(query_embedding), matrix[valid])[0]
    top = topk_order(sims, top_k)
    return [(r + 1, float(sims[i]), int(valid[i])) for r, i in enumerate(top)]


def llama_get_top_k_embeddings(query_embedding, embeddings, similarity_top_k=None,
                               embedding_ids=None, similarity_cutoff=None):
    """llama-index-core 0.12.46 ``get_top_k_embeddings`` + default cosine ``similarity``
    (third-party, not vendored, not installed; restated from its published source —
    parity unpinned by any reference test).  Per row ``dot/(|q||e|)`` in float64, strict
    ``> cutoff``, keep the best k, sort by similarity desc.  Zero norm gives NaN.
    """
    import heapq
    if embedding_ids is None:
        embedding_ids = list(range(len(embeddings)))
    q = np.asarray(query_embedding, dtype=np.float64)
    heap = []
    with np.errstate(divide="ignore", invalid="ignore"):
        for i, emb in enumerate(np.asarray(embeddings, dtype=np.float64)):
            sim = float(np.dot(q, emb) / (np.linalg.norm(q) * np.linalg.norm(emb)))
            if similarity_cutoff is None or sim > similarity_cutoff:
                heapq.heappush(heap, (sim, embedding_ids[i]))
                if similarity_top_k and len(heap) > similarity_top_k:
                    heapq.heappop(heap)
    res = sorted(heap, key=lambda x: x[0], reverse=True)
    return [s for s, _ in res], [n for _, n in res]
