"""GPU parity: the HIP top-k path (through the C ABI) vs the CPU oracle / sklearn goldens.

Bar (BASELINE.json north_star): identical top-k index sets and cosine scores within 1e-4.
The HIP path re-scores its candidates in fp64 and certifies the candidate set (with an exact
fp64 scan for what the certificate cannot settle), so ids are compared EXACTLY and scores to
1e-12 (both APIs return the fp64 scores).
"""
import glob
import json
import os

import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu

SCORE_TOL_F32 = 1e-12    # host API: fp64 scores (re-scored in fp64 on the GPU)
SCORE_TOL_F64 = 1e-12    # device API: fp64 scores


@pytest.fixture(scope="module")
def hc():
    import hcrag_amd
    if hcrag_amd.device_count() == 0:
        pytest.fail("GPU test collected but no HIP device visible")
    return hcrag_amd


def _check(got_s, got_i, exp_s, exp_i, tol=SCORE_TOL_F32):
    np.testing.assert_array_equal(got_i, exp_i)
    ok = exp_i >= 0
    np.testing.assert_allclose(got_s[ok], exp_s[ok], rtol=0, atol=tol)
    assert np.all(np.isneginf(got_s[~ok]))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(
    os.path.dirname(__file__), "golden", "cos_*.npz"))))
def test_golden_fixtures_f16(hc, path):
    g = np.load(path)
    E, Q, k = g["E"], g["Q"], int(g["k"])
    with hc.VectorIndex(E.shape[1], "f16") as ix:
        ix.add(E, normalize=False)                 # store the fixture's fp16 values exactly
        np.testing.assert_array_equal(ix.get_rows(), E.astype(np.float32))
        s, i = ix.search(Q, k)
        _check(s, i, g["scores"], g["ids"])
        assert ix.last_stats()["uncertified_queries"] == 0


def test_known_answers_gpu(hc, golden_dir):
    ka = json.load(open(os.path.join(golden_dir, "known_answers.json")))
    d = ka["dim"]
    vec = {"ones": np.ones(d), "-ones": -np.ones(d), "random": np.array(ka["random_node"])}
    vec["e0"] = np.eye(1, d, 0)[0]
    vec["e1"] = np.eye(1, d, 1)[0]
    for case in ka["cases"]:
        got = hc.batch_semantic_similarity(vec[case["query"]], [vec[n] for n in case["nodes"]])
        assert len(got) == len(case["nodes"])
        if "tol" in case:
            for gv, e in zip(got, case["expected"]):
                assert abs(gv - e) < case["tol"]
        if "range" in case:
            lo, hi = case["range"]
            assert all(lo <= gv <= hi for gv in got)
            # random node is stored as float32 by the GPU path: 1e-7 vs the fp64 reference
            np.testing.assert_allclose(got, case["expected"], rtol=0, atol=1e-7)
    assert hc.batch_semantic_similarity(np.ones(8), []) == []


@pytest.mark.parametrize("dtype", ["f16", "bf16", "f32"])
@pytest.mark.parametrize("dim", [384, 768, 100])
def test_random_parity_dtypes(hc, dtype, dim):
    rng = np.random.default_rng(dim + len(dtype))
    N, B, k = 5000, 200, 32
    E = rng.standard_normal((N, dim)).astype(np.float32)
    Q = rng.standard_normal((B, dim)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.1 * rng.standard_normal((B // 2, dim)).astype(np.float32)
    with hc.VectorIndex(dim, dtype) as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()                          # decoded stored rows = what is ranked
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k)
        _check(s, i, es, ei)
        st = ix.last_stats()
        assert st["uncertified_queries"] == 0


def test_multiblock_queries_and_partitions(hc):
    rng = np.random.default_rng(7)
    N, D, B, k = 60000, 768, 300, 32
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), k)
        _check(s, i, es, ei)
        st = ix.last_stats()
        assert st["partitions"] > 1 and st["uncertified_queries"] == 0


def test_edge_cases(hc):
    rng = np.random.default_rng(3)
    D = 64
    with hc.VectorIndex(D, "f16") as ix:
        # empty index -> all slots empty
        s, i = ix.search(rng.standard_normal((3, D)), 4)
        assert np.all(i == -1) and np.all(np.isneginf(s))
        E = rng.standard_normal((10, D)).astype(np.float16)
        ix.add(E, normalize=False)
        # k > n: n results then empty slots
        q = rng.standard_normal((2, D)).astype(np.float32)
        s, i = ix.search(q, 16)
        es, ei = O.cosine_topk(q, E.astype(np.float64), 16)
        _check(s, i, es, ei)
        assert np.all(i[:, 10:] == -1)
        # zero query: all cosines 0, ties by row id
        s, i = ix.search(np.zeros((1, D), np.float32), 5)
        np.testing.assert_array_equal(i[0], np.arange(5))
        np.testing.assert_array_equal(s[0], np.zeros(5, np.float32))
        # nq = 0
        s, i = ix.search(np.zeros((0, D), np.float32), 3)
        assert s.shape == (0, 3)
        # dimension mismatch -> ValueError (sklearn raises ValueError)
        with pytest.raises(ValueError):
            ix.search(np.zeros((1, D + 1), np.float32), 3)
        with pytest.raises(ValueError):
            ix.search(q, 0)


def test_threshold_and_unit_mode(hc):
    rng = np.random.default_rng(11)
    D, N = 384, 3000
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = E[:16].astype(np.float32) + 0.3 * rng.standard_normal((16, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        for mode, thr in [(0, 0.3), (1, 0.60), (0, -np.inf), (1, 0.9999)]:
            s, i = ix.search(Q, 10, score_mode=mode, threshold=thr)
            es, ei = O.cosine_topk(Q, E.astype(np.float64), 10, score_mode=mode, threshold=thr)
            _check(s, i, es, ei)


def test_rowmask_category_filter(hc):
    rng = np.random.default_rng(5)
    D, N = 256, 4000
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = rng.standard_normal((20, D)).astype(np.float32)
    mask = rng.random(N) < 0.2
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        ix.set_rowmask(mask)
        s, i = ix.search(Q, 8)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), 8, rowmask=mask)
        _check(s, i, es, ei)
        ix.set_rowmask(None)
        s, i = ix.search(Q, 8)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), 8)
        _check(s, i, es, ei)


def test_duplicate_cluster_forces_widening(hc):
    """300 identical rows tie at the top: the certificate must widen k' and still give the
    reference's answer (lowest row ids among the tie)."""
    rng = np.random.default_rng(9)
    D, N = 128, 2000
    E = rng.standard_normal((N, D)).astype(np.float16)
    dup = rng.choice(N, 300, replace=False)
    E[dup] = E[dup[0]]
    Q = np.repeat(E[dup[0]].astype(np.float32)[None], 3, axis=0)
    Q[1] += 0.001 * rng.standard_normal(D).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        s, i = ix.search(Q, 32)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), 32)
        _check(s, i, es, ei)
        st = ix.last_stats()
        assert st["widened_queries"] > 0 and st["uncertified_queries"] == 0


def test_score_all_matches_oracle(hc):
    rng = np.random.default_rng(4)
    E = rng.standard_normal((257, 384)).astype(np.float32)
    E[5] = 0
    Q = rng.standard_normal((3, 384)).astype(np.float32)
    with hc.VectorIndex(384, "f32") as ix:
        ix.add(E, normalize=False)
        for mode in (0, 1):
            got = ix.score_all(Q, score_mode=mode)
            exp = O.cosine_similarity64(Q, E)
            if mode:
                exp = (exp + 1) / 2
            np.testing.assert_allclose(got, exp, rtol=0, atol=1e-13)


def test_device_api_and_shard_merge(hc):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(21)
    D, N, B, k, g = 768, 9000, 130, 16, 3
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    es, ei = O.cosine_topk(Q, E.astype(np.float64), k)
    dev = torch.device("cuda:0")
    q_t = torch.from_numpy(Q).to(dev)
    bounds = np.linspace(0, N, g + 1).astype(int)
    S = torch.empty((g, B, k), dtype=torch.float64, device=dev)
    I = torch.empty((g, B, k), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for j in range(g):
        with hc.VectorIndex(D, "f16") as ix:
            ix.add(E[bounds[j]:bounds[j + 1]], normalize=False)
            ix.set_id_offset(int(bounds[j]))
            ix.search_device(q_t.data_ptr(), B, k, S[j].data_ptr(), I[j].data_ptr(), stream=stream)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_i = torch.empty((B, k), dtype=torch.int64, device=dev)
    hc.merge_topk_device(S.data_ptr(), I.data_ptr(), g, B, k, out_s.data_ptr(), out_i.data_ptr(),
                         stream=stream)
    torch.cuda.synchronize()
    _check(out_s.cpu().numpy(), out_i.cpu().numpy(), es, ei, tol=SCORE_TOL_F64)


@pytest.mark.parametrize("W,B", [(2, 1024), (8, 1024), (8, 512)])
def test_rank_shapes_of_the_scaling_bench(hc, W, B):
    """The local search each rank of ``bench.py --gpus W`` runs: nq = W x B gathered queries
    (8192 at W = 8, B = 1024; 4096 = configs[3]'s global batch at W = 8, B = 512) over a row
    shard, through the same hip_local_search / hip_merge callables ShardedSearch uses (raw rows:
    the non-UNIT v4 route; test_rank_route_of_configs3 below runs the bench's L2-normalised QW
    route at full query counts); the W shards run one after another on one GPU, the all-to-all is the
    slice [j*B:(j+1)*B] of shard r's result, and the merged lists must equal the unsharded
    oracle exactly."""
    torch = pytest.importorskip("torch")
    from hcrag_amd.distributed import shard_range, hip_local_search, hip_merge
    rng = np.random.default_rng(100 + W)
    D, N, k = 768, 12000, 32
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = rng.standard_normal((W * B, D)).astype(np.float32)
    planted = rng.integers(0, N, W * B // 2)
    Q[::2] = E[planted] + 0.1 * rng.standard_normal((W * B // 2, D))
    dev = torch.device("cuda:0")
    q_all = torch.from_numpy(Q).to(dev)
    S = torch.empty((W, W * B, k), dtype=torch.float64, device=dev)
    I = torch.empty((W, W * B, k), dtype=torch.int64, device=dev)
    for r in range(W):
        r0, r1 = shard_range(N, r, W)
        with hc.VectorIndex(D, "f16", capacity=r1 - r0) as ix:
            ix.add(E[r0:r1], normalize=False)
            ix.set_id_offset(r0)
            s, i = hip_local_search(ix, k)(q_all)
            torch.cuda.synchronize()
            assert ix.last_stats()["uncertified_queries"] == 0
            S[r], I[r] = s, i
    merge = hip_merge(k)
    sub = np.r_[0:64, B - 32:B + 32, W * B - 64:W * B]      # first, a rank boundary, last
    es, ei = O.cosine_topk(Q[sub], E.astype(np.float64), k)
    got_s = np.empty((W * B, k)); got_i = np.empty((W * B, k), dtype=np.int64)
    for j in range(W):                   # rank j receives block j of every shard's result
        ms, mi = merge(S[:, j * B:(j + 1) * B].contiguous(), I[:, j * B:(j + 1) * B].contiguous())
        torch.cuda.synchronize()
        got_s[j * B:(j + 1) * B], got_i[j * B:(j + 1) * B] = ms.cpu().numpy(), mi.cpu().numpy()
    _check(got_s[sub], got_i[sub], es, ei, tol=SCORE_TOL_F64)
    # planted queries find their own row first
    assert np.mean(got_i[::2, 0] == planted) > 0.99


@pytest.mark.parametrize("nq", [4096, 8192])
def test_rank_route_of_configs3(hc, nq):
    """configs[3]'s per-rank production route: a rank of ``bench.py --gpus 8
    --global-batch 4096`` scores all 4096 gathered queries (8192 at --global-batch 8192) on an
    L2-normalised 768-d f16 shard, which routes to QW (score_kernel 6) with 16 / 32 query blocks
    over the row partitions.  >= 100k rows, a shard id offset, half the queries planted (a stored
    row + noise, as bench.make_queries); the queries on both sides of every 256-query block
    boundary are compared with the fp64 oracle (ids exactly, scores to 1e-12), and every planted
    query must find its own row first.  Reference: experiments/main.py:841-844."""
    torch = pytest.importorskip("torch")
    from hcrag_amd.distributed import hip_local_search
    rng = np.random.default_rng(nq)
    D, N, k, off = 768, 131072 + 37, 32, 3 * 1_250_000
    E = rng.standard_normal((N, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16", capacity=N) as ix:
        ix.add(E, normalize=True)
        ix.set_id_offset(off)
        R = ix.get_rows()
        Q = rng.standard_normal((nq, D)).astype(np.float32)
        planted = rng.integers(0, N, nq // 2)
        Q[::2] = R[planted] + 0.05 * rng.standard_normal((nq // 2, D)).astype(np.float32) / D ** 0.5
        s, i = hip_local_search(ix, k)(torch.from_numpy(Q).to("cuda:0"))
        torch.cuda.synchronize()
        st = ix.last_stats()
        assert st["score_kernel"] == 6, st                 # QW, the bench's kernel at this shape
        assert st["uncertified_queries"] == 0, st
    s, i = s.cpu().numpy(), i.cpu().numpy()
    np.testing.assert_array_equal(i[::2, 0], planted + off)
    edges = np.arange(256, nq, 256)
    sub = np.unique(np.r_[0, 1, edges - 1, edges, nq - 1])
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(s[sub], i[sub], es, np.where(ei >= 0, ei + off, -1), tol=SCORE_TOL_F64)


def test_embedding_search_dropin(hc):
    rng = np.random.default_rng(13)
    M = rng.standard_normal((441, 384))            # config 1 scale (Product*.csv rows)
    meta = [{"type": "database_table" if r % 3 else "json_table"} for r in range(441)]
    texts = [f"Record {r}" for r in range(441)]
    srch = hc.EmbeddingSearch(M, texts, meta, dtype="f32")
    q = M[17] + 0.05 * rng.standard_normal(384)
    res = srch.find_similar_content(q, top_k=5, similarity_threshold=0.3)
    ref = O.find_similar_content(q.astype(np.float32), M.astype(np.float32), 5, 0.3)
    assert [r["content"] for r in res] == [texts[i] for i, _ in ref]
    np.testing.assert_allclose([r["similarity_score"] for r in res], [s for _, s in ref], atol=1e-6)
    cat = srch.search_by_category(q, "json_table", top_k=4)
    valid = [i for i, m in enumerate(meta) if m["type"] == "json_table"]
    refc = O.search_by_category(q.astype(np.float32), M.astype(np.float32), valid, 4)
    assert [r["rank"] for r in cat["results"]] == [x[0] for x in refc]
    assert [r["content"] for r in cat["results"]] == [texts[x[2]] for x in refc]
    assert srch.search_by_category(q, "nope")["results"] == []


@pytest.mark.slow
def test_large_planted_recall_and_subset_parity(hc):
    """2M x 768 fp16: planted queries find their source row first (size-independent
    property) and a query subset matches the streamed fp64 oracle exactly."""
    torch = pytest.importorskip("torch")
    N, D, B, k = 2_000_000, 768, 512, 32
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(3)
    E = torch.randn((N, D), generator=gen, device=dev, dtype=torch.float16)
    src = torch.randint(0, N, (B // 2,), generator=gen, device=dev)
    Q = torch.randn((B, D), generator=gen, device=dev, dtype=torch.float32)
    Q[: B // 2] = E[src].float() + 0.05 * torch.randn((B // 2, D), generator=gen, device=dev)
    with hc.VectorIndex(D, "f16", capacity=N) as ix:
        ix.add_device(E.data_ptr(), N, hc.HCR_F16, normalize=False,
                      stream=torch.cuda.current_stream().cuda_stream)
        S = torch.empty((B, k), dtype=torch.float64, device=dev)
        I = torch.empty((B, k), dtype=torch.int64, device=dev)
        ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(),
                         stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        st = ix.last_stats()
        assert st["uncertified_queries"] == 0
        I = I.cpu().numpy()
        assert np.array_equal(I[: B // 2, 0], src.cpu().numpy())
        sub = np.r_[0:4, B // 2:B // 2 + 4]
        Eh = E.cpu().numpy()
        es, ei = O.cosine_topk(Q.cpu().numpy()[sub], Eh, k, chunk_rows=1 << 19)
        _check(S.cpu().numpy()[sub], I[sub], es, ei, tol=SCORE_TOL_F64)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("B", [1, 20, 40, 100, 130, 384, 700])
def test_batch_sizes_both_kernels(hc, dtype, B):
    """Tile shapes 256 x 16 (B <= 16) and 256 x 256 (17-64 queries on small corpora such as
    this one, and > 64; padded query columns at 20, 40, 100 and 130).  256 x 64 (17-64 queries
    on large corpora): test_narrow_tiles_forced."""
    rng = np.random.default_rng(B)
    N, D, k = 20000, 384, 10
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
    with hc.VectorIndex(D, dtype) as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k)
        _check(s, i, es, ei)
        assert ix.last_stats()["uncertified_queries"] == 0


@pytest.mark.parametrize("D", [128, 384, 768])
@pytest.mark.parametrize("B", [17, 200, 256])
@pytest.mark.parametrize("variant", ["unit", "raw", "masked"])
def test_query_stationary_kernels(hc, D, B, variant):
    """The query-stationary kernels (17-256 queries): QS with 1 query block per wave on 256-row
    tiles (any B at KS = 4..24) and 2 blocks per wave on 128-row tiles (B > 128, D <= 384); at
    D = 768 a normalised corpus with B > 128 goes to QW (256 queries per workgroup).  Normalised rows (UNIT epilogue), raw rows
    (inverse norms from LDS; at D = 768 routed to v3/v4), a row mask; N not a multiple of the
    tile (last tile partly past the corpus end) and large enough for several tiles per
    workgroup (candidate compactions, the seeded pre-pass)."""
    rng = np.random.default_rng(D * 1000 + B)
    N, k = 150000 + 77, 10
    E = rng.standard_normal((N, D)).astype(np.float32)
    if variant == "raw":
        E *= rng.uniform(0.5, 2.0, (N, 1)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
    mask = (rng.random(N) < 0.7) if variant == "masked" else None
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=(variant != "raw"))
        if mask is not None:
            ix.set_rowmask(mask)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k, rowmask=mask)
        _check(s, i, es, ei)
        assert ix.last_stats()["uncertified_queries"] == 0


_NARROW = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import hcrag_amd as hc
from oracle import cosine_topk as O
for B in (20, 40, 64):
    rng = np.random.default_rng(B)
    N, D, k = 30000, 384, 10
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        R = ix.get_rows()
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, R, k)
        assert np.array_equal(i, ei), B
        assert np.max(np.abs(s - es)) < 1e-6, B
        assert ix.last_stats()["uncertified_queries"] == 0
print("narrow ok")
"""


@pytest.mark.parametrize("min_tiles", ["1", "32"])
def test_narrow_tiles_forced(min_tiles):
    """The 256 x 64 tiles (17-64 queries on corpora above HCRAG_Q64_ELEMS) forced on a small
    corpus, with and without the pre-pass, in a subprocess (the switches are read once)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HCRAG_Q64_ELEMS="0", HCRAG_PREPASS_MIN_TILES=min_tiles)
    r = subprocess.run([sys.executable, "-c", _NARROW, root, os.path.join(root, "hc-rag_amd")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "narrow ok" in r.stdout


def test_large_batch_mask_and_widening(hc):
    """256x256 kernel: row mask + a duplicate cluster that forces k' widening."""
    rng = np.random.default_rng(17)
    N, D, B, k = 30000, 256, 512, 32
    E = rng.standard_normal((N, D)).astype(np.float16)
    dup = rng.choice(N, 200, replace=False)
    E[dup] = E[dup[0]]
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[:8] = E[dup[0]].astype(np.float32)
    mask = rng.random(N) < 0.5
    mask[dup] = True
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), k)
        _check(s, i, es, ei)
        st = ix.last_stats()
        assert st["widened_queries"] > 0 and st["uncertified_queries"] == 0
        ix.set_rowmask(mask)
        s, i = ix.search(Q, k)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), k, rowmask=mask)
        _check(s, i, es, ei)


def test_ragged_tail_rows(hc):
    """Corpus sizes that end mid-tile (256 and 128 row tiles) and tiny corpora."""
    rng = np.random.default_rng(23)
    D = 192
    for N in (1, 5, 255, 257, 1000, 4097):
        E = rng.standard_normal((N, D)).astype(np.float16)
        Q = rng.standard_normal((400, D)).astype(np.float32)
        with hc.VectorIndex(D, "f16") as ix:
            ix.add(E, normalize=False)
            for qs in (Q[:3], Q):
                s, i = ix.search(qs, 7)
                es, ei = O.cosine_topk(qs, E.astype(np.float64), 7)
                _check(s, i, es, ei)


def test_llama_vector_store_dropin(hc):
    """MI355XVectorStore.query vs the restated llama-index get_top_k_embeddings path."""
    from types import SimpleNamespace
    from hcrag_amd.llama_compat import MI355XVectorStore, TextNodeLite, VectorStoreQuery
    rng = np.random.default_rng(31)
    D, N = 384, 700
    E = rng.standard_normal((N, D))
    nodes = [TextNodeLite(id_=f"n{r}", text=f"t{r}", metadata={"type": "a" if r % 4 else "b"},
                          embedding=E[r].tolist()) for r in range(N)]
    vs = MI355XVectorStore(D, dtype="f32")
    assert vs.add(nodes) == [f"n{r}" for r in range(N)]
    q = E[5] + 0.1 * rng.standard_normal(D)
    res = vs.query(VectorStoreQuery(query_embedding=q.tolist(), similarity_top_k=10))
    sims, ids = O.llama_get_top_k_embeddings(q.astype(np.float32), E.astype(np.float32), 10,
                                             [f"n{r}" for r in range(N)])
    assert res.ids == ids
    np.testing.assert_allclose(res.similarities, sims, atol=1e-12)
    flt = SimpleNamespace(filters=[SimpleNamespace(key="type", value="b", operator="==")])
    res = vs.query(VectorStoreQuery(query_embedding=q.tolist(), similarity_top_k=5, filters=flt))
    keep = [r for r in range(N) if r % 4 == 0]
    sims, ids = O.llama_get_top_k_embeddings(q.astype(np.float32), E[keep].astype(np.float32), 5,
                                             [f"n{r}" for r in keep])
    assert res.ids == ids
    vs.delete("n0")
    res = vs.query(VectorStoreQuery(query_embedding=E[0].tolist(), similarity_top_k=3))
    assert "n0" not in res.ids


@pytest.mark.gpu
def test_property_graph_store_vector_query():
    """PropertyGraphStore.vector_query form of the boundary."""
    from hcrag_amd.llama_compat import MI355XPropertyGraphStore, TextNodeLite, VectorStoreQuery
    rng = np.random.default_rng(11)
    E = rng.standard_normal((300, 64)).astype(np.float32)
    nodes = [TextNodeLite(id_=f"n{i}", embedding=E[i].tolist(), metadata={"type": "t%d" % (i % 3)})
             for i in range(300)]
    gs = MI355XPropertyGraphStore(64, dtype="f32")
    gs.upsert_nodes(nodes)
    assert gs.supports_vector_queries
    q = rng.standard_normal(64).astype(np.float32)
    got_nodes, got_scores = gs.vector_query(VectorStoreQuery(query_embedding=q.tolist(),
                                                             similarity_top_k=7))
    s, ids = O.cosine_topk(q[None].astype(np.float64), E.astype(np.float64), 7)
    assert [n.node_id for n in got_nodes] == [f"n{i}" for i in ids[0]]
    np.testing.assert_allclose(got_scores, s[0], atol=1e-6)
    assert [n.node_id for n in gs.get(ids=["n3", "n5"])] == ["n3", "n5"]


@pytest.mark.parametrize("env", [
    {"HCRAG_PREPASS_MIN_TILES": "1"},                       # estimated seed (default j)
    {"HCRAG_PREPASS_MIN_TILES": "1", "HCRAG_RIGOROUS_SEED": "1"},
    # aggressive seed (the sample's best row): short candidate lists, the seed-aware
    # certificate and the rigorous re-run of what it cannot certify
    {"HCRAG_PREPASS_MIN_TILES": "1", "HCRAG_SAMPLE_STRIDE": "2", "HCRAG_SEED_RANK": "1"},
    {"HCRAG_PREPASS_MIN_TILES": "1", "HCRAG_TEST_DTYPE": "bf16"},
    {"HCRAG_PREPASS_MIN_TILES": "1", "HCRAG_PREPASS_TOPK": "1"},          # the top-k' pre-pass form
    {"HCRAG_NO_PREPASS": "1"}])                  # cold per-workgroup bounds (no seed at all)
def test_prepass_seed_parity(env):
    """The sampling pre-pass forced on small corpora: ids identical to the oracle whatever the
    seed, certificates complete after widening."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "seed_check.py")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "parity ok" in r.stdout


def test_configs4_rank_shape_bf16(hc):
    """configs[4]'s per-rank shape (100M x 1024 bf16 over 8 GPUs, global batch 8192, top-64):
    bf16 rows, D = 1024, k = 64, nq = 8192 on one shard (rows reduced to 40k so the oracle
    finishes; 64 queries of it checked exactly, planted recall on all)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(1024)
    N, D, B, k = 40000, 1024, 8192, 64
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    planted = rng.integers(0, N, B // 2)
    Q[::2] = E[planted] + 0.05 * rng.standard_normal((B // 2, D)).astype(np.float32)
    dev = torch.device("cuda:0")
    with hc.VectorIndex(D, "bf16", capacity=N) as ix:
        ix.add(E, normalize=True)
        ix.set_id_offset(3 * N)                       # a rank's shard offset
        q = torch.from_numpy(Q).to(dev)
        S = torch.empty((B, k), dtype=torch.float64, device=dev)
        I = torch.empty((B, k), dtype=torch.int64, device=dev)
        ix.search_device(q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(),
                         stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        st = ix.last_stats()
        assert st["uncertified_queries"] == 0, st
        assert st["score_kernel"] == 7, st            # QW1, the D = 1024 large-batch kernel
        S, I = S.cpu().numpy(), I.cpu().numpy()
        R = ix.get_rows()
    assert np.mean(I[::2, 0] - 3 * N == planted) > 0.99
    sub = np.r_[0:32, B - 32:B]
    es, ei = O.cosine_topk(Q[sub], R, k)
    _check(S[sub], I[sub] - 3 * N, es, ei, tol=SCORE_TOL_F64)
