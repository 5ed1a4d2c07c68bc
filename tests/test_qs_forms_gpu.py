"""GPU parity of the query-stationary kernel's 256-query forms (score_qs.h, NQ = 2 on 128-row
tiles, 129-256 queries): at D = 384 (KS = 12) with 64-deep (HCR_OPT_QS_FORM 1) and 128-deep
(form 3, the default) ring stages, and at D = 128 / 192 (KS = 4 / 6: 64-deep) -- L2-normalised
(UNIT epilogue) and raw corpora, a row mask, bf16.  Ids are compared EXACTLY with the fp64 oracle
and scores to 1e-12; the stats must show that QS ran (score_kernel 5), so a silent reroute
fails.  Reference: experiments/main.py:841-844 (cosine_similarity + argsort[::-1][:k]) and
:872-885 (the category filter)."""
import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu

QS = 5           # hcr_search_stats.score_kernel of the query-stationary kernel


@pytest.fixture(scope="module")
def hc():
    import hcrag_amd
    if hcrag_amd.device_count() == 0:
        pytest.fail("GPU test collected but no HIP device visible")
    return hcrag_amd


def _planted(rng, E, B, noise=0.2):
    N, D = E.shape
    Q = rng.standard_normal((B, D)).astype(np.float32)
    src = rng.integers(0, N, B // 2)
    Q[: B // 2] = E[src] + noise * rng.standard_normal((B // 2, D)).astype(np.float32)
    return Q, src


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("D,form", [(128, 0), (192, 0), (384, 1), (384, 3)])
@pytest.mark.parametrize("B,k", [(200, 10), (256, 32)])
@pytest.mark.parametrize("normalize", [True, False])
def test_qs_form_parity(hc, dtype, D, form, B, k, normalize):
    """N not a multiple of the 128-row tile, tens of tiles per workgroup (the seeded pre-pass
    runs), a padded second query block (200), the UNIT and the inverse-norm epilogues."""
    rng = np.random.default_rng(D * 7 + B + k + int(normalize) + form)
    N = 120000 + 77
    E = rng.standard_normal((N, D)).astype(np.float32)
    if not normalize:
        E *= rng.uniform(0.5, 2.0, (N, 1)).astype(np.float32)
    Q, src = _planted(rng, E, B)
    with hc.VectorIndex(D, dtype) as ix:
        ix.set_option(ix.OPT_QS_FORM, form)
        ix.set_option(ix.OPT_QW_MIN, 1 << 30)      # (r05: QW takes 129+ queries at D = 384 by default)
        ix.add(E, normalize=normalize)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        st = ix.last_stats()
        assert st["score_kernel"] == QS, st
        assert st["uncertified_queries"] == 0, st
    sub = np.r_[0:16, B // 2: B // 2 + 16, B - 8:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    np.testing.assert_array_equal(i[sub], ei)
    np.testing.assert_allclose(s[sub], es, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(i[: B // 2, 0], src)


def test_qs_rowmask_and_forms_agree(hc):
    """A category mask (the mask words ride the tile-start DMA of wave NW-3), and the 64- vs
    128-deep forms on the same index: identical ids and scores."""
    rng = np.random.default_rng(11)
    N, D, B, k = 70000 + 3, 384, 256, 16
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q, _ = _planted(rng, E, B)
    mask = rng.random(N) < 0.6
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        ix.set_rowmask(mask)
        R = ix.get_rows()
        ix.set_option(ix.OPT_QS_FORM, 3)
        s4, i4 = ix.search(Q, k)
        assert ix.last_stats()["score_kernel"] == QS
        ix.set_option(ix.OPT_QS_FORM, 1)
        s8, i8 = ix.search(Q, k)
        assert ix.last_stats()["score_kernel"] == QS
        with pytest.raises(Exception):
            ix.set_option(ix.OPT_QS_FORM, 2)          # QS4: removed
    np.testing.assert_array_equal(i4, i8)
    np.testing.assert_array_equal(s4, s8)
    es, ei = O.cosine_topk(Q[:24], R, k, rowmask=mask)
    np.testing.assert_array_equal(i4[:24], ei)
    np.testing.assert_allclose(s4[:24], es, rtol=0, atol=1e-12)
