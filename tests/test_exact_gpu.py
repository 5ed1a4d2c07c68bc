"""Exactness guarantees of the search path beyond the certified candidates (VERDICT r1 items
3/5/8): the exact fp64 fallback scan (K6/K7) for queries the certificate cannot
settle at k' = 512 and for k > 256, fp64 thresholds and outputs, rows appended after a row
mask, device ingest from a side stream, and the single-process multi-device index.

Every comparison is against the fp64 oracle (oracle/cosine_topk.py): ids exactly, scores to
1e-12.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu
TOL = 1e-12


@pytest.fixture(scope="module")
def hc():
    import hcrag_amd
    if hcrag_amd.device_count() == 0:
        pytest.fail("GPU test collected but no HIP device visible")
    return hcrag_amd


def _check(got_s, got_i, exp_s, exp_i, tol=TOL):
    np.testing.assert_array_equal(got_i, exp_i)
    ok = exp_i >= 0
    np.testing.assert_allclose(got_s[ok], exp_s[ok], rtol=0, atol=tol)
    assert np.all(np.isneginf(got_s[~ok]))


def _near_dup_corpus(rng, N, D, cluster, dtype, spread):
    """A cluster of `cluster` rows around one direction (relative perturbation `spread`,
    0 = exact duplicates) inside N random rows, quantised to the storage dtype."""
    E = rng.standard_normal((N, D)).astype(np.float32)
    idx = rng.choice(N, cluster, replace=False)
    base = E[idx[0]].copy()
    E[idx] = base + spread * rng.standard_normal((cluster, D)).astype(np.float32)
    return E, idx, base


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("B", [8, 300])                # 256 x 16 and 256 x 256 tiles
@pytest.mark.parametrize("spread", [0.0, 2e-4])         # exact ties / near ties
def test_cluster_wider_than_kprime_is_exact(hc, dtype, B, spread):
    """700 rows straddle the k-th score -- more than the largest candidate set (k' = 512): the
    certificate cannot settle them, the exact fallback must, with oracle-identical ids."""
    rng = np.random.default_rng(int(spread * 1e5) + B)
    N, D, k = 20000, 128, 32
    E, idx, base = _near_dup_corpus(rng, N, D, 700, dtype, spread)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[:4] = base + 1e-3 * rng.standard_normal((4, D)).astype(np.float32)
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k)
        _check(s, i, es, ei)
        st = ix.last_stats()
        assert st["uncertified_queries"] == 0
        assert st["fallback_queries"] >= 1, st


def test_large_k_exact_scan(hc):
    """k > 256 (no MFMA candidate path that deep): the exact scan, with mask and threshold."""
    rng = np.random.default_rng(41)
    N, D = 30000, 96
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = rng.standard_normal((5, D)).astype(np.float32)
    mask = rng.random(N) < 0.6
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        for k in (257, 1000, 2048):
            s, i = ix.search(Q, k)
            es, ei = O.cosine_topk(Q, E.astype(np.float64), k)
            _check(s, i, es, ei)
            assert ix.last_stats()["fallback_queries"] == 5
        ix.set_rowmask(mask)
        s, i = ix.search(Q, 700, threshold=0.05)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), 700, threshold=0.05, rowmask=mask)
        _check(s, i, es, ei)
        with pytest.raises(ValueError):
            ix.search(Q, 0)


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_large_k_mfma_prefilter(hc, D):
    """k > 256 on the MFMA prefilter (K6h round-0 coarse histograms -> starting threshold, then
    K6m: fp64 only for rows whose coarse score reaches threshold - eps): raw (non-normalised)
    rows, 2 query groups (32 + 9), a row mask and a threshold; ids identical to the oracle,
    scores to 1e-12.  A near-duplicate cluster of 3000 rows around one query forces overflow
    rounds (its k = 2048 best lie inside one coarse bin)."""
    rng = np.random.default_rng(D + 7)
    N, B = 60000 + 7, 41
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[:3000] = E[0] + 1e-3 * rng.standard_normal((3000, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[0] = E[0]
    mask = rng.random(N) < 0.7
    with hc.VectorIndex(D, "bf16" if D == 1024 else "f16") as ix:
        ix.add(E, normalize=False)
        R = ix.get_rows()
        for k in (257, 2048):
            s, i = ix.search(Q, k)
            es, ei = O.cosine_topk(Q, R, k)
            _check(s, i, es, ei)
            st = ix.last_stats()
            assert st["fallback_queries"] == B, st
        ix.set_rowmask(mask)
        s, i = ix.search(Q[:9], 700, threshold=0.02)
        es, ei = O.cosine_topk(Q[:9], R, 700, threshold=0.02, rowmask=mask)
        _check(s, i, es, ei)


_PF_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/hc-rag_amd']
import hcrag_amd as hc
rng = np.random.default_rng(5)
N, D = 200000 + 3, 768
E = rng.standard_normal((N, D)).astype(np.float32)
Q = rng.standard_normal((40, D)).astype(np.float32)
with hc.VectorIndex(D, "f16") as ix:
    ix.add(E, normalize=True)
    s, i = ix.search(Q, 1500)
    st = ix.last_stats()
np.savez(sys.argv[2], s=s, i=i, rounds=st["fallback_rounds"])
"""


def test_mfma_prefilter_matches_fp64_scan(tmp_path):
    """The prefiltered scan (default) and K6's fp64 scan of every row (HCRAG_NO_MFMA_FILTER)
    return bit-identical lists: the admitted rows' scores are computed in K6's order."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = []
    for env in ({}, {"HCRAG_NO_MFMA_FILTER": "1"}):
        e = dict(os.environ, **env)
        if not env:
            e.pop("HCRAG_NO_MFMA_FILTER", None)
        f = str(tmp_path / f"pf{len(out)}.npz")
        subprocess.run([sys.executable, "-c", _PF_CHILD, root, f], env=e, check=True, timeout=300)
        out.append(np.load(f))
    np.testing.assert_array_equal(out[0]["i"], out[1]["i"])
    np.testing.assert_array_equal(out[0]["s"], out[1]["s"])


def test_large_k_sorted_corpus_converges(hc):
    """a corpus ordered by ascending score against the query (the scan admits the
    worst rows first).  K7's histogram threshold does not depend on admission order, so the
    fallback converges in a few rounds instead of ~cap - k rows per round (1M rows, k = 2048:
    the old rule needed ~160 rounds and failed at 64)."""
    rng = np.random.default_rng(61)
    N, D = 1_000_000, 64
    E = rng.standard_normal((N, D)).astype(np.float32)
    q = rng.standard_normal(D).astype(np.float32)
    E = E[np.argsort(E @ q, kind="stable")]            # ascending score: best rows last
    Q = np.stack([q, -q, rng.standard_normal(D).astype(np.float32)])
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        R = ix.get_rows()
        for k in (2048, 300):
            s, i = ix.search(Q, k)
            st = ix.last_stats()
            es, ei = O.cosine_topk(Q, R, k)
            _check(s, i, es, ei)
            assert st["fallback_queries"] == 3, st
            assert st["fallback_rounds"] <= 8, st      # one group of 3 queries


def test_threshold_is_fp64_and_inclusive(hc):
    """A row scoring exactly the threshold is kept (main.py:849 `>=`): the threshold crosses
    the ABI as a double and the scores come back in fp64 (a float threshold rounded
    0.3 up and dropped such rows)."""
    rng = np.random.default_rng(43)
    D, N = 384, 2000
    E = rng.standard_normal((N, D)).astype(np.float32)
    q = E[7] + 0.8 * rng.standard_normal(D).astype(np.float32)
    with hc.VectorIndex(D, "f32") as ix:
        ix.add(E, normalize=False)
        exact = ix.score_all(q[None])[0]            # the GPU's own fp64 score of every row
        order = np.lexsort((np.arange(N), -exact))
        thr = float(exact[order[2]])                # the 3rd best score, bit-exact
        s, i = ix.search(q[None], 5, threshold=thr)
        assert s.dtype == np.float64
        assert list(i[0, :3]) == list(order[:3]) and np.all(i[0, 3:] == -1)
        assert s[0, 2] == thr
        # default threshold 0.3 of find_similar_content: keep rows at exactly 0.3
        s, i = ix.search(q[None], 3, threshold=0.3)
        assert np.all((s[0] >= 0.3) | np.isneginf(s[0]))


def test_rows_added_after_mask_are_visible(hc):
    """a mask set, then rows appended within capacity -- they are searchable."""
    rng = np.random.default_rng(47)
    D = 64
    E = rng.standard_normal((3000, D)).astype(np.float16)
    with hc.VectorIndex(D, "f16", capacity=4096) as ix:
        ix.add(E[:2000], normalize=False)
        mask = rng.random(2000) < 0.5
        ix.set_rowmask(mask)
        ix.add(E[2000:], normalize=False)               # fits the reserved capacity
        Q = E[2500:2504].astype(np.float32)
        s, i = ix.search(Q, 4)
        full = np.concatenate([mask, np.ones(1000, bool)])
        es, ei = O.cosine_topk(Q, E.astype(np.float64), 4, rowmask=full)
        _check(s, i, es, ei)
        assert list(i[:, 0]) == [2500, 2501, 2502, 2503]


def test_device_ingest_on_side_stream_is_ordered(hc):
    """rows produced and ingested on a non-default torch stream, searched at once on
    another stream -- the search waits for the ingest (event), ids match the oracle."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    N, D, B, k = 200000, 256, 64, 8
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        g = torch.Generator(device=dev).manual_seed(5)
        E = torch.randn((N, D), generator=g, device=dev, dtype=torch.float16)
        Q = E[:B].float() + 0.01
    with hc.VectorIndex(D, "f16", capacity=N) as ix:
        ix.add_device(E.data_ptr(), N, hc.HCR_F16, normalize=False, stream=side.cuda_stream)
        out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
        out_i = torch.empty((B, k), dtype=torch.int64, device=dev)
        side.synchronize()                               # Q itself is torch's; E is the library's
        ix.search_device(Q.data_ptr(), B, k, out_s.data_ptr(), out_i.data_ptr(),
                         stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        sub = np.arange(0, B, 8)
        Eh = E.cpu().numpy()
        es, ei = O.cosine_topk(Q.cpu().numpy()[sub], Eh, k)
        _check(out_s.cpu().numpy()[sub], out_i.cpu().numpy()[sub], es, ei)


def test_add_ids_maps_results(hc):
    rng = np.random.default_rng(53)
    D = 128
    E = rng.standard_normal((900, D)).astype(np.float16)
    gids = rng.permutation(10**6)[:900].astype(np.int64)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E[:300], normalize=False)                 # ids 0..299
        ix.add_ids(E[300:], gids[300:], normalize=False)
        Q = rng.standard_normal((6, D)).astype(np.float32)
        for k in (10, 300):                              # certified path and exact scan
            s, i = ix.search(Q, k)
            es, ei = O.cosine_topk(Q, E.astype(np.float64), k)
            ids = np.concatenate([np.arange(300), gids[300:]])
            _check(s, i, es, ids[ei])


@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0], "all"])
def test_multi_device_index_matches_unsharded(hc, devices):
    """hcr_multi_*: g shards (repeated device -> peer copies; distinct devices -> RCCL sends to
    the first one; "all" = every visible GPU, one shard each), several adds, mask, k beyond
    256: same lists as the fp64 oracle over all rows."""
    if devices == "all":
        devices = list(range(hc.device_count()))
    rng = np.random.default_rng(len(devices))
    N, D, B = 25000, 192, 40
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[:10] = E[rng.integers(0, N, 10)] + 0.05
    with hc.MultiDeviceIndex(D, devices, dtype="f16") as mx:
        mx.add(E[:10000])
        mx.add(E[10000:])
        assert len(mx) == N and sum(mx.shard_sizes()) == N
        with hc.VectorIndex(D, "f16") as ref:
            ref.add(E)
            R = ref.get_rows()                           # the decoded stored values
        for k in (16, 300):
            s, i = mx.search(Q, k)
            es, ei = O.cosine_topk(Q, R, k)
            _check(s, i, es, ei)
        assert mx.exchange == ("rccl" if len(set(devices)) == len(devices) else "peer")
        mask = rng.random(N) < 0.3
        mx.set_rowmask(mask)
        s, i = mx.search(Q, 16, threshold=0.0)
        es, ei = O.cosine_topk(Q, R, 16, threshold=0.0, rowmask=mask)
        _check(s, i, es, ei)
        assert mx.last_stats()["uncertified_queries"] == 0


_SEED_K200 = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import hcrag_amd as hc
from oracle import cosine_topk as O
rng = np.random.default_rng(200)
N, D, B, k = 60000, 128, 300, 200
E = rng.standard_normal((N, D)).astype(np.float32)
Q = rng.standard_normal((B, D)).astype(np.float32)
with hc.VectorIndex(D, "f16") as ix:
    ix.add(E, normalize=True)
    R = ix.get_rows()
    s, i = ix.search(Q, k)
    es, ei = O.cosine_topk(Q, R, k)
    assert np.array_equal(i, ei)
    assert np.max(np.abs(s - es)) < 1e-12
    st = ix.last_stats()
    assert st["uncertified_queries"] == 0, st
    print("k200 ok", st["kprime"], st["widened_queries"], st["fallback_queries"])
"""


def test_k200_aggressive_seed():
    """k in 129..256 starts at k' = 512 = the widening limit; with the most
    aggressive estimated seed the over-shot queries must still come back exact."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HCRAG_SEED_RANK="1", HCRAG_PREPASS_MIN_TILES="1", HCRAG_SAMPLE_STRIDE="2")
    r = subprocess.run([sys.executable, "-c", _SEED_K200, root, os.path.join(root, "hc-rag_amd")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "k200 ok" in r.stdout


_MULTI_ROLLBACK = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import hcrag_amd as hc
from oracle import cosine_topk as O
rng = np.random.default_rng(3)
N, D = 9000, 128
E = rng.standard_normal((N, D)).astype(np.float32)
Q = rng.standard_normal((8, D)).astype(np.float32)
with hc.MultiDeviceIndex(D, [0, 0, 0], dtype="f16") as mx:
    mx.add(E[:6000])
    sizes = mx.shard_sizes()
    try:
        mx.add(E[6000:])                   # shard 1 (HCRAG_FAIL_MULTI_ADD=1) fails
        raise SystemExit("the injected failure did not surface")
    except RuntimeError as exc:
        assert "rolled back" in str(exc), exc
    assert len(mx) == 6000 and mx.shard_sizes() == sizes, (len(mx), mx.shard_sizes(), sizes)
    with hc.VectorIndex(D, "f16") as ref:
        ref.add(E[:6000])
        R = ref.get_rows()
    s, i = mx.search(Q, 20)
    es, ei = O.cosine_topk(Q, R, 20)
    assert np.array_equal(i, ei) and np.max(np.abs(s - es)) < 1e-12
print("rollback ok")
"""


def test_multi_add_failure_rolls_back():
    """a hcr_multi_add that fails on shard j after shards 0..j-1 took their blocks
    adds nothing (those blocks are dropped; the call's ids are not consumed), so the index
    answers as before the call (HCRAG_FAIL_MULTI_ADD injects the failure, child process)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _MULTI_ROLLBACK, root, os.path.join(root, "hc-rag_amd")],
                       env=dict(os.environ, HCRAG_FAIL_MULTI_ADD="1"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rollback ok" in r.stdout


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_normalized_16bit_store_ranks_like_the_inputs(hc, dtype):
    """the ingest's scale search (normalize=True, 16-bit rows: the scale within
    (1 +- 2^-9) / ||row|| whose rounded row has the norm closest to 1) changes the stored values
    against a plain normalise-then-round -- pinned here against the fp64 oracle over the INPUT
    vectors (not get_rows()): near-ties at gaps of 2e-3 (f16) / 1e-2 (bf16), well above the
    storage rounding, must come back in the inputs' order; and each stored row is the input
    direction to within that rounding."""
    rng = np.random.default_rng(17 if dtype == "f16" else 18)
    D, B, k = 384, 16, 12
    gap = 2e-3 if dtype == "f16" else 1e-2
    Q = rng.standard_normal((B, D))
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    rows = []
    for b in range(B):                   # k rows per query at cosines 0.9 - j gap (near-ties)
        for j in range(k):
            z = rng.standard_normal(D)
            z -= (z @ Q[b]) * Q[b]
            z /= np.linalg.norm(z)
            c = 0.9 - j * gap
            rows.append((c * Q[b] + np.sqrt(1 - c * c) * z) * rng.uniform(0.5, 3.0))
    E = np.concatenate([np.asarray(rows), rng.standard_normal((5000, D))]).astype(np.float32)
    perm = rng.permutation(len(E))
    E = E[perm]
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows().astype(np.float64)
        s, i = ix.search(Q.astype(np.float32), k)
    es, ei = O.cosine_topk(Q.astype(np.float32), E.astype(np.float64), k)
    np.testing.assert_array_equal(i, ei)             # the inputs' ranking
    np.testing.assert_allclose(s, es, rtol=0, atol=gap / 4)
    En = E / np.linalg.norm(E, axis=1, keepdims=True)
    cos = np.sum(R * En, axis=1) / np.linalg.norm(R, axis=1)
    assert 1 - cos.min() < (2e-6 if dtype == "f16" else 5e-5)
    assert np.abs(np.linalg.norm(R, axis=1) - 1).max() < (1e-3 if dtype == "f16" else 2e-3)


@pytest.mark.parametrize("B", [40, 600])                 # finish_kernel / merge + rescore_kernel
def test_out_of_range_candidate_key_is_an_error(hc, B):
    """a candidate key naming a row outside the index (planted into query
    0's first partition list by the handle's HCR_TEST_PLANT_BAD_KEY hook, as a defective score kernel could
    leave it) must fail the search with HCR_EINTERNAL -- not fault the device on the rescore's
    row gather -- and the next search on the same handle must be exact again."""
    from hcrag_amd._lib import HCR_EINTERNAL, HcrError
    rng = np.random.default_rng(B)
    N, D, k = 20000, 256, 10
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        ix.test_hook(ix.TEST_PLANT_BAD_KEY, 1)
        try:
            with pytest.raises(HcrError) as exc:
                ix.search(Q, k)
        finally:
            ix.test_hook(ix.TEST_PLANT_BAD_KEY, 0)
        assert exc.value.code == HCR_EINTERNAL, exc.value
        assert "outside the index" in str(exc.value)
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k)
        _check(s, i, es, ei)


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 0])
def test_flag_read_modes(hc, mode):
    """HCR_OPT_FLAG_READ (r06: how a pass reads its certificate count and bounds-check flag back):
    every mode returns the oracle's lists, reports a planted out-of-index key as HCR_EINTERNAL,
    and sees the uncertified count of a duplicate cluster (the widened pass / fallback runs)."""
    from hcrag_amd._lib import HCR_EINTERNAL, HcrError
    rng = np.random.default_rng(77 + mode)
    N, D, k, B = 30000, 384, 10, 64
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[100:400] = E[7]                       # 301 exact duplicates: q = E[7] cannot certify at k'
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[0] = E[7]
    with hc.VectorIndex(D, "f16") as ix:
        ix.set_option(ix.OPT_FLAG_READ, mode)
        ix.add(E, normalize=True)
        R = ix.get_rows()
        es, ei = O.cosine_topk(Q, R, k)
        for _ in range(3):
            s, i = ix.search(Q, k)
            _check(s, i, es, ei)
        st = ix.last_stats()
        assert st["widened_queries"] + st["fallback_queries"] >= 1, st
        ix.test_hook(ix.TEST_PLANT_BAD_KEY, 1)
        try:
            with pytest.raises(HcrError) as exc:
                ix.search(Q, k)
        finally:
            ix.test_hook(ix.TEST_PLANT_BAD_KEY, 0)
        assert exc.value.code == HCR_EINTERNAL, exc.value
        s, i = ix.search(Q, k)
        _check(s, i, es, ei)


@pytest.mark.parametrize("env", [{"HCRAG_K6_INLINE": "1"}, {}, {"HCRAG_K6_PCAP": "100"}])
def test_k6_admission_forms(env):
    """r06: the exact fallback's admission scan inline (K6m), as two launches (K6c compaction +
    K6r rescoring, the default), and with every group's pair list overflowing (the inline K6m
    rescans those groups after K6r) -- identical to the oracle (tests/k6_forms_check.py)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "k6_forms_check.py")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "parity ok" in r.stdout


def test_deep_k_sorted_scan(hc):
    """VERDICT r4 missing #4: k > 2048 (the reference's argsort(...)[::-1][:top_k] takes any
    top_k, experiments/main.py:844,889) on the deep path (r06: the exact fallback's admission
    scan, a radix select of the k-th admitted key, a bitonic sort of the k answers): k = 5000 on
    a 20k-row corpus with exact
    duplicate rows (tie order id asc), a row mask, a threshold, UNIT mode, k past the corpus."""
    rng = np.random.default_rng(77)
    N, D, B, k = 20000, 192, 9, 5000
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[100:140] = E[7]                                   # 41 exact ties
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[0] = E[7] + 0.05 * rng.standard_normal(D).astype(np.float32)
    for dtype in ("f16", "f32"):
        with hc.VectorIndex(D, dtype) as ix:
            ix.add(E, normalize=False)
            R = ix.get_rows().astype(np.float64)
            s, i = ix.search(Q, k)
            es, ei = O.cosine_topk(Q, R, k)
            _check(s, i, es, ei)
            assert ix.last_stats()["fallback_queries"] == B
            mask = rng.random(N) < 0.5
            ix.set_rowmask(mask)
            s, i = ix.search(Q, k, threshold=-0.05)
            es, ei = O.cosine_topk(Q, R, k, threshold=-0.05, rowmask=mask)
            _check(s, i, es, ei)
            ix.set_rowmask(None)
            s, i = ix.search(Q[:2], N + 50, score_mode=1)       # k past the corpus, (s + 1) / 2
            es, ei = O.cosine_topk(Q[:2], R, N + 50, score_mode=1)
            _check(s, i, es, ei)
            assert np.all(i[:, N:] == -1)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_deep_k_mfma_route_overflow_and_long_sort(hc, dtype):
    """r06 deep path on the MFMA-prefiltered route (D = 384): k = 10000 (the answers' bitonic
    sort spans 2 LDS chunks + global passes), and k = 2100 with 25000 exact copies of one row --
    more ties than the 16384 admission slots, so the select must tighten the threshold through
    the k-th best kept (score, row) key (ties by id asc) -- against the fp64 oracle."""
    rng = np.random.default_rng(91)
    N, D, B = 60000, 384, 6
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows().astype(np.float64)
        s, i = ix.search(Q, 10000)
        es, ei = O.cosine_topk(Q, R, 10000)
        _check(s, i, es, ei)
    E2 = E.copy()
    E2[30000:55000] = E2[5]
    Q2 = Q.copy()
    Q2[:3] = E2[5] + 0.02 * rng.standard_normal((3, D)).astype(np.float32)
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E2, normalize=True)
        R = ix.get_rows().astype(np.float64)
        s, i = ix.search(Q2, 2100)
        es, ei = O.cosine_topk(Q2, R, 2100)
        _check(s, i, es, ei)
        assert ix.last_stats()["fallback_rounds"] >= 3      # the overflow took extra rounds


@pytest.mark.parametrize("D,dtype", [(768, "f16"), (1024, "bf16")])
def test_deep_k_mfma_route_wide_rows(hc, D, dtype):
    """The deep path on the MFMA-prefiltered route at D = 768 / 1024 (K6h / K6m with 24 / 32
    query fragments, the admission queue rescoring 4 pairs at a time): raw rows, 2 query groups
    (32 + 3), k = 3000, then a row mask and a threshold at k = 4100 -- ids identical to the fp64
    oracle, scores to 1e-12."""
    rng = np.random.default_rng(D + 3)
    N, B = 24000 + 5, 35
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[1] = E[7]
    mask = rng.random(N) < 0.75
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E, normalize=False)
        R = ix.get_rows().astype(np.float64)
        s, i = ix.search(Q, 3000)
        es, ei = O.cosine_topk(Q, R, 3000)
        _check(s, i, es, ei)
        assert ix.last_stats()["fallback_queries"] == B
        ix.set_rowmask(mask)
        s, i = ix.search(Q[:5], 4100, threshold=0.01)
        es, ei = O.cosine_topk(Q[:5], R, 4100, threshold=0.01, rowmask=mask)
        _check(s, i, es, ei)


def test_deep_k_multi_device_sorted_merge(hc):
    """k = 5000 over a 3-shard multi-device index (shards on one device): each shard's deep
    top-k, then the shard merge by one bitonic sort of (score, ~id) keys (g x k > 8192), against the
    unsharded oracle; and hcr_merge_topk_device's sorted path straight on 2 x 3000-deep lists."""
    import ctypes
    import torch
    from hcrag_amd import _lib
    rng = np.random.default_rng(78)
    N, D, B, k = 12000, 128, 5, 5000
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[50:60] = E[3]
    Q = rng.standard_normal((B, D)).astype(np.float32)
    with hc.MultiDeviceIndex(D, [0, 0, 0], dtype="f16") as mx:
        mx.add(E)
        with hc.VectorIndex(D, "f16") as ref:
            ref.add(E)
            R = ref.get_rows()
        s, i = mx.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k)
        _check(s, i, es, ei)
    g, nq, kk = 2, 4, 3000
    S = np.sort(rng.random((g, nq, kk)), axis=2)[:, :, ::-1].copy()
    S[1, :, :10] = S[0, :, :10]                          # cross-shard exact ties
    I = rng.permutation(g * nq * kk).reshape(g, nq, kk).astype(np.int64)
    I[0, :, -5:] = -1
    S[0, :, -5:] = -np.inf
    dev = torch.device("cuda:0")
    ds, di = torch.from_numpy(S).to(dev), torch.from_numpy(I).to(dev)
    os_, oi = torch.empty((nq, kk), dtype=torch.float64, device=dev), torch.empty((nq, kk), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    _lib.check(_lib.lib().hcr_merge_topk_device(ctypes.c_void_p(ds.data_ptr()), ctypes.c_void_p(di.data_ptr()), g,
                                                nq, kk, ctypes.c_void_p(os_.data_ptr()),
                                                ctypes.c_void_p(oi.data_ptr()), None))
    torch.cuda.synchronize()
    for q in range(nq):
        pairs = [(-S[j, q, c], I[j, q, c]) for j in range(g) for c in range(kk) if I[j, q, c] >= 0]
        pairs.sort()
        np.testing.assert_array_equal(oi[q].cpu().numpy(), [p[1] for p in pairs[:kk]])
        np.testing.assert_array_equal(os_[q].cpu().numpy(), [-p[0] for p in pairs[:kk]])
