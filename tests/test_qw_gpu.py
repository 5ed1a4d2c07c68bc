"""GPU parity of the wide query-stationary score kernel (QW, score_qw.h): batches above 256
queries on L2-normalised corpora at D = 384 and 768 -- the configs[2] regime (10M x 768,
B = 1024, top-32) at reduced N.  Ids are compared EXACTLY with the fp64 oracle and scores to
1e-12, and the stats must show that QW ran (score_kernel 6), so a silent reroute fails."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu

QW = 6          # hcr_search_stats.score_kernel of the QW kernel


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


def _planted(rng, E, B, noise=0.2, with_src=False):
    """B queries, the first B // 2 a corpus row + N(0, noise^2) noise (that row is their
    nearest neighbour), the rest random; optionally the planted rows' indices too."""
    N, D = E.shape
    Q = rng.standard_normal((B, D)).astype(np.float32)
    src = rng.integers(0, N, B // 2)
    Q[: B // 2] = E[src] + noise * rng.standard_normal((B // 2, D)).astype(np.float32)
    return (Q, src) if with_src else Q


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("D", [384, 768])
@pytest.mark.parametrize("B,k", [(130, 10), (256, 10), (257, 10), (512, 32), (1024, 32), (1100, 64)])
def test_qw_parity(hc, dtype, D, B, k):
    """N not a multiple of the 32 / 64-row stage (the last tile ends past the corpus), several
    hundred tiles per workgroup (the seeded pre-pass runs), padded query blocks (257, 1100)."""
    rng = np.random.default_rng(D * 10 + B + k)
    N = 120000 + 45
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q, src = _planted(rng, E, B, with_src=True)
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == QW, st
        assert st["uncertified_queries"] == 0, st
    sub = np.r_[0:24, B // 2: B // 2 + 24, B - 16:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(s[sub], i[sub], es, ei)
    # every planted query (not only the oracle subset) finds its own row first
    np.testing.assert_array_equal(i[: B // 2, 0], src)


def test_qw_small_corpus_and_tail(hc):
    """Corpora of one partial stage up to a few stages: empty partitions, a last tile with a
    single live row, fewer tiles than partitions."""
    rng = np.random.default_rng(77)
    D, B, k = 768, 300, 7
    for N in (1, 31, 33, 100, 2049):
        E = rng.standard_normal((N, D)).astype(np.float32)
        Q = rng.standard_normal((B, D)).astype(np.float32)
        with hc.VectorIndex(D, "f16") as ix:
            ix.add(E, normalize=True)
            R = ix.get_rows()
            s, i = ix.search(Q, k)
            assert ix.last_stats()["score_kernel"] == QW
            es, ei = O.cosine_topk(Q, R, k)
            _check(s, i, es, ei)


def test_qw_duplicate_cluster_compaction(hc):
    """600 identical rows in one partition: every one is appended for the queries that equal
    them (candidate-buffer compactions inside the QW tile loop), then the tie at the k-th score
    is settled by widening / the exact fallback; ids still identical to the oracle."""
    rng = np.random.default_rng(3)
    N, D, B, k = 60000, 384, 512, 32
    E = rng.standard_normal((N, D)).astype(np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    E[1000:1600] = E[1000]
    Q = _planted(rng, E, B)
    Q[:8] = E[1000] + 1e-3 * rng.standard_normal((8, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == QW and st["uncertified_queries"] == 0, st
    sub = np.r_[0:16, B - 16:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(s[sub], i[sub], es, ei)


def test_qw_masked_and_raw_route_to_v4(hc):
    """A row mask or a raw (non-normalised) corpus is not a QW case: v4 runs, results exact."""
    rng = np.random.default_rng(9)
    N, D, B, k = 30000, 384, 400, 10
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = _planted(rng, E, B)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E * rng.uniform(0.5, 2, (N, 1)).astype(np.float32), normalize=False)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        assert ix.last_stats()["score_kernel"] == 4
        es, ei = O.cosine_topk(Q[:32], R, k)
        _check(s[:32], i[:32], es, ei)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        mask = rng.random(N) < 0.6
        ix.set_rowmask(mask)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        assert ix.last_stats()["score_kernel"] == 4
        es, ei = O.cosine_topk(Q[:32], R, k, rowmask=mask)
        _check(s[:32], i[:32], es, ei)


_COLD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import hcrag_amd as hc
from oracle import cosine_topk as O
rng = np.random.default_rng(11)
for D in (384, 768):
    N, B, k = 50000 + 13, 600, 32
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == 6 and st["uncertified_queries"] == 0, st
    sub = np.r_[0:16, B - 16:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    assert np.array_equal(i[sub], ei), D
    assert np.max(np.abs(s[sub] - es)) < 1e-12, D
print("cold ok")
"""


@pytest.mark.parametrize("env", [{"HCRAG_NO_PREPASS": "1"},
                                 {"HCRAG_PREPASS_MIN_TILES": "1", "HCRAG_SEED_RANK": "1"}])
def test_qw_cold_and_aggressive_seeds(env):
    """QW with no seed at all (every wave appends and compacts from an empty bound) and with the
    most aggressive seed (short lists, seed-aware certificate, rigorous re-runs), in a subprocess
    (the hooks are read once per process)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _COLD, root, os.path.join(root, "hc-rag_amd")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "cold ok" in r.stdout


@pytest.mark.parametrize("D,N", [(384, 400000 + 3), (768, 300000 + 11)])
def test_qw_maxonly_prepass_forms_agree(hc, D, N):
    """The sampling pre-pass on QW's MAXONLY form (HCR_OPT_PREPASS 2, the default under QW from
    257 queries) and on v4's (1): N not a multiple of the 256-row sampled tile (the last unit
    ends past the corpus: NaN rows), several partitions of whole 128-row units; the seeds only
    steer which rows are appended, so both give ids identical to the oracle and identical
    scores."""
    rng = np.random.default_rng(D + 7)
    B, k = 512, 16
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = _planted(rng, E, B)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        out = {}
        for form in (2, 1, 0):
            ix.set_option(ix.OPT_PREPASS, form)
            out[form] = ix.search(Q, k)
            st = ix.last_stats()
            assert st["score_kernel"] == QW and st["uncertified_queries"] == 0, st
    for form in (1, 0):
        np.testing.assert_array_equal(out[form][1], out[2][1])
        np.testing.assert_array_equal(out[form][0], out[2][0])
    sub = np.r_[0:12, B - 12:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(out[2][0][sub], out[2][1][sub], es, ei)


@pytest.mark.parametrize("D", [384, 768])
def test_qw_dma_modes_agree(hc, D):
    """Both stage DMA-issue modes of QW (HCR_OPT_QW_DM 0: at the stage barrier, 3: spread over
    the MFMA groups, -1: the default) on one index, one and four query blocks: ids identical to
    the oracle and to each other."""
    rng = np.random.default_rng(D + 3)
    N = 90000 + 13
    E = rng.standard_normal((N, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        for B in (200, 1024):
            Q = _planted(rng, E, B)
            sub = np.r_[0:16, B - 16:B]
            es, ei = O.cosine_topk(Q[sub], R, 16)
            for dm in (0, 3, -1):
                ix.set_option(ix.OPT_QW_DM, dm)
                s, i = ix.search(Q, 16)
                st = ix.last_stats()
                assert st["score_kernel"] == QW and st["uncertified_queries"] == 0, (dm, st)
                _check(s[sub], i[sub], es, ei)


@pytest.mark.parametrize("B", [200, 600])
def test_qw_stagger_agrees(hc, B):
    """HCR_OPT_QW_STAGGER (D = 384: waves 4-7 run each stage's test one stage late, two
    accumulator sets) against the oracle and the plain form, one and three query blocks, an
    odd stage count and a corpus tail, planted queries, a duplicate cluster (appends and
    compactions in the late epilogue)."""
    rng = np.random.default_rng(B + 21)
    D, k = 384, 16
    N = 64 * 777 + 29
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[1000:1400] = E[5] + 1e-3 * rng.standard_normal((400, D)).astype(np.float32)
    Q, src = _planted(rng, E, B, with_src=True)
    Q[:3] = E[5]
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        sub = np.r_[0:24, B - 16:B]
        es, ei = O.cosine_topk(Q[sub], R, k)
        outs = []
        for stg in (0, 1, 2):
            ix.set_option(ix.OPT_QW_STAGGER, stg)
            s, i = ix.search(Q, k)
            st = ix.last_stats()
            assert st["score_kernel"] == QW and st["uncertified_queries"] == 0, (stg, st)
            _check(s[sub], i[sub], es, ei)
            np.testing.assert_array_equal(i[3: B // 2, 0], src[3:])
            outs.append((s, i))
        for o in outs[1:]:
            np.testing.assert_array_equal(outs[0][1], o[1])
        np.testing.assert_array_equal(outs[0][0], outs[1][0])
