"""GPU parity of the one-wave-per-SIMD query-stationary kernel (QW1, score_qw1.h) at D = 1024 (its
default from 257 queries: configs[4]'s shape, bge-large) on L2-normalised corpora.  Ids are compared EXACTLY with the fp64
oracle and scores to 1e-12; the stats must show that QW1 ran (score_kernel 7), so a silent
reroute fails.  Reference: experiments/main.py:841-844 (cosine_similarity + argsort[::-1][:k])."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu

QW1 = 7          # hcr_search_stats.score_kernel of QW1


@pytest.fixture(scope="module")
def hc():
    import hcrag_amd
    if hcrag_amd.device_count() == 0:
        pytest.fail("GPU test collected but no HIP device visible")
    return hcrag_amd


def _check(got_s, got_i, exp_s, exp_i, tol=1e-12):
    np.testing.assert_array_equal(got_i, exp_i)
    ok = exp_i >= 0
    np.testing.assert_allclose(got_s[ok], exp_s[ok], rtol=0, atol=tol)


def _planted(rng, E, B, noise=0.2):
    N, D = E.shape
    Q = rng.standard_normal((B, D)).astype(np.float32)
    src = rng.integers(0, N, B // 2)
    Q[: B // 2] = E[src] + noise * rng.standard_normal((B // 2, D)).astype(np.float32)
    return Q, src


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("D,opt", [(1024, -1), (1024, 1)])
@pytest.mark.parametrize("B,k", [(257, 10), (1024, 32), (1100, 64)])
def test_qw1_parity(hc, dtype, D, opt, B, k):
    """N not a multiple of the 32 / 16-row stage (the last tile ends past the corpus), hundreds
    of tiles per workgroup (the seeded pre-pass runs), padded query blocks (257, 1100: the
    192-query blocks of D = 1024 and the 256-padded pre-pass)."""
    rng = np.random.default_rng(D * 10 + B + k + opt)
    N = 90000 + 45
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q, src = _planted(rng, E, B)
    with hc.VectorIndex(D, dtype) as ix:
        ix.set_option(ix.OPT_QW1, opt)
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == QW1, st
        assert st["uncertified_queries"] == 0, st
    sub = np.r_[0:24, B // 2: B // 2 + 24, B - 16:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(s[sub], i[sub], es, ei)
    np.testing.assert_array_equal(i[: B // 2, 0], src)


def test_qw1_off_routes_elsewhere(hc):
    """HCR_OPT_QW1 = 0: D = 1024 on v4 (and QW1's option is ignored at D = 768: QW); the same
    exact results."""
    rng = np.random.default_rng(5)
    for D, want, want1 in ((768, 6, 6), (1024, 4, QW1)):
        N, B, k = 20000 + 7, 300, 16
        E = rng.standard_normal((N, D)).astype(np.float32)
        Q, _ = _planted(rng, E, B)
        with hc.VectorIndex(D, "f16") as ix:
            ix.add(E, normalize=True)
            R = ix.get_rows()
            ix.set_option(ix.OPT_QW1, 0)
            s0, i0 = ix.search(Q, k)
            assert ix.last_stats()["score_kernel"] == want
            ix.set_option(ix.OPT_QW1, 1)
            s1, i1 = ix.search(Q, k)
            assert ix.last_stats()["score_kernel"] == want1
        np.testing.assert_array_equal(i0, i1)
        np.testing.assert_array_equal(s0, s1)
        es, ei = O.cosine_topk(Q[:32], R, k)
        _check(s1[:32], i1[:32], es, ei)


def test_qw1_small_corpus_and_tail(hc):
    """Corpora of one partial stage up to a few stages: empty partitions, a last tile with a
    single live row, fewer tiles than partitions."""
    rng = np.random.default_rng(78)
    B, k = 300, 7
    for D, opt in ((1024, 1), (1024, -1)):
        for N in (1, 15, 17, 33, 100, 2049):
            E = rng.standard_normal((N, D)).astype(np.float32)
            Q = rng.standard_normal((B, D)).astype(np.float32)
            with hc.VectorIndex(D, "bf16") as ix:
                ix.set_option(ix.OPT_QW1, opt)
                ix.add(E, normalize=True)
                R = ix.get_rows()
                s, i = ix.search(Q, k)
                assert ix.last_stats()["score_kernel"] == QW1
                es, ei = O.cosine_topk(Q, R, k)
                _check(s, i, es, ei)


def test_qw1_duplicate_cluster_compaction(hc):
    """600 identical rows in one partition: all appended for the queries equal to them
    (candidate-buffer compactions inside the QW1 tile loop), then the k-th-score tie settled by
    widening / the exact fallback; ids identical to the oracle."""
    rng = np.random.default_rng(4)
    for D, opt in ((1024, 1),):
        N, B, k = 40000, 512, 32
        E = rng.standard_normal((N, D)).astype(np.float32)
        E /= np.linalg.norm(E, axis=1, keepdims=True)
        E[1000:1600] = E[1000]
        Q, _ = _planted(rng, E, B)
        Q[:8] = E[1000] + 1e-3 * rng.standard_normal((8, D)).astype(np.float32)
        with hc.VectorIndex(D, "f16") as ix:
            ix.set_option(ix.OPT_QW1, opt)
            ix.add(E, normalize=True)
            R = ix.get_rows()
            s, i = ix.search(Q, k)
            st = ix.last_stats()
            assert st["score_kernel"] == QW1 and st["uncertified_queries"] == 0, st
        sub = np.r_[0:16, B - 16:B]
        es, ei = O.cosine_topk(Q[sub], R, k)
        _check(s[sub], i[sub], es, ei)


def test_qw1_configs4_batch_grid(hc):
    """configs[4]'s batch (8192 queries, top-64) at D = 1024 on a reduced corpus: 43 query
    blocks of 192 over a multi-round grid (qw1_partitions), k' = 128."""
    rng = np.random.default_rng(41)
    N, D, B, k = 30000 + 3, 1024, 8192, 64
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q, src = _planted(rng, E, B)
    with hc.VectorIndex(D, "bf16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == QW1 and st["uncertified_queries"] == 0, st
        assert st["workgroups"] > 256, st
    sub = np.r_[0:8, 4090:4100, B - 8:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(s[sub], i[sub], es, ei)
    np.testing.assert_array_equal(i[: B // 2, 0], src)


_COLD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import hcrag_amd as hc
from oracle import cosine_topk as O
rng = np.random.default_rng(12)
for D in (1024,):
    N, B, k = 40000 + 13, 600, 32
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == 7 and st["uncertified_queries"] == 0, st
    sub = np.r_[0:16, B - 16:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    assert np.array_equal(i[sub], ei), D
    assert np.max(np.abs(s[sub] - es)) < 1e-12, D
print("cold ok")
"""


@pytest.mark.parametrize("env", [{"HCRAG_NO_PREPASS": "1", "HCRAG_QW1": "1"},
                                 {"HCRAG_PREPASS_MIN_TILES": "1", "HCRAG_SEED_RANK": "1",
                                  "HCRAG_QW1": "-1"}])
def test_qw1_cold_and_aggressive_seeds(env):
    """QW1 with no seed at all (every wave appends and compacts from an empty bound) and with the
    most aggressive seed (short lists, seed-aware certificate, rigorous re-runs), in a subprocess
    (the hooks are read once per process; HCRAG_QW1 sets the option's default)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _COLD, root, os.path.join(root, "hc-rag_amd")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "cold ok" in r.stdout
