"""GPU: the global seed across row shards (hcr_search_sample_device + hcr_search_seeded_device,
DESIGN.md §6) run shard by shard on one device through the callables ShardedSearch uses
(hcrag_amd.distributed.hip_global_seed / hip_merge): every shard's sampled unit maxima gathered,
each shard's dense pass seeded from all of them, the lists merged on the device and certified
at the merge (the merged k-th score must beat every shard's bound).  Certified queries must equal
the unsharded fp64 oracle over the stored rows exactly; the test also requires (nearly) every
query to certify, as the seed rank is chosen for."""
import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hc():
    import hcrag_amd
    if hcrag_amd.device_count() == 0:
        pytest.fail("GPU test collected but no HIP device visible")
    return hcrag_amd


def _run(hc, E, Q, W, k, dtype="f16"):
    import torch
    from hcrag_amd.distributed import hip_global_seed, hip_merge, shard_range
    N, D = E.shape
    B = Q.shape[0]
    dev = torch.device("cuda:0")
    q_all = torch.from_numpy(Q).to(dev)
    n_tiles = (N + 255) // 256
    shards, rows, umaxes, srows = [], [], [], 0
    for r in range(W):
        r0, r1 = shard_range(N, r, W)
        ix = hc.VectorIndex(D, dtype, capacity=r1 - r0)
        ix.add(E[r0:r1], normalize=True)
        ix.set_id_offset(r0)
        shards.append(ix)
        rows.append(ix.get_rows())
        sample, _ = hip_global_seed(ix, k, W, n_tiles)
        u, nr = sample(q_all)
        torch.cuda.synchronize()
        assert u is not None and u.shape[0] > 0, "no sample on this shard's route"
        umaxes.append(u.clone())
        srows += nr
    umax_max = max(u.shape[0] for u in umaxes)
    umax_all = torch.full((W * umax_max, B), float("-inf"), dtype=torch.float32, device=dev)
    for r, u in enumerate(umaxes):
        umax_all[r * umax_max:r * umax_max + u.shape[0]] = u
    S = torch.empty((W, B, k), dtype=torch.float64, device=dev)
    I = torch.empty((W, B, k), dtype=torch.int64, device=dev)
    Bd = torch.empty((W, B), dtype=torch.float64, device=dev)
    for r, ix in enumerate(shards):
        _, seeded = hip_global_seed(ix, k, W, n_tiles)
        s, i, b = seeded(q_all, umax_all, W * umax_max, srows / N)
        torch.cuda.synchronize()
        st = ix.last_stats()
        assert st["uncertified_queries"] == 0 and st["fallback_queries"] == 0, st
        S[r], I[r], Bd[r] = s, i, b
    ms, mi = hip_merge(k)(S, I)
    torch.cuda.synchronize()
    kth = ms[:, k - 1]
    worst = Bd.max(dim=0).values
    cert = ((kth > worst) | torch.isneginf(worst)).cpu().numpy()
    for ix in shards:
        ix.close()
    return (ms.cpu().numpy(), mi.cpu().numpy(), cert, np.concatenate(rows).astype(np.float64),
            Bd.cpu().numpy(), I.cpu().numpy(), S.cpu().numpy())


# (shard sizes: the dense route's pre-pass needs >= 4 stages per partition -- 256 partitions of
# 64-row stages at 256 queries, D = 384)
@pytest.mark.parametrize("W,D,B,k,per", [(3, 768, 512, 32, 40000), (4, 384, 256, 10, 70000),
                                         (2, 768, 1024, 16, 40000)])
def test_global_seed_shards_match_oracle(hc, W, D, B, k, per):
    rng = np.random.default_rng(300 + W + D)
    N = W * per + 123
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[5000:5300] = E[77] + 1e-3 * rng.standard_normal((300, D)).astype(np.float32)   # a cluster
    Q = rng.standard_normal((B, D)).astype(np.float32)
    src = rng.integers(0, N, B // 2)
    Q[::2] = E[src] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
    Q[1] = E[77]
    s, i, cert, R, bounds, shard_ids, shard_s = _run(hc, E, Q, W, k)
    assert cert.mean() >= 0.99, f"only {cert.mean():.3f} of the queries certified"
    sub = np.r_[0:48, B - 16:B]
    sub = sub[cert[sub]]
    es, ei = O.cosine_topk(Q[sub], R, k)
    np.testing.assert_array_equal(i[sub], ei)
    np.testing.assert_allclose(s[sub], es, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(i[0::2][cert[0::2], 0], src[cert[0::2]])
    # the bound is a real bound: every row a shard left out scores at or below it -- or, when
    # the shard returned k rows, at or below its k-th (candidates past its top k: the merge
    # argument) -- exact fp64 cosine of the stored rows, queries 0-7 (random, planted, cluster)
    from hcrag_amd.distributed import shard_range
    qn = Q[:8].astype(np.float64)
    qn /= np.linalg.norm(qn, axis=1, keepdims=True)
    Rn = R / np.linalg.norm(R, axis=1, keepdims=True)
    for r in range(W):
        r0, r1 = shard_range(N, r, W)
        sc = Rn[r0:r1] @ qn.T                          # [rows, 8]
        for q in range(8):
            out = np.ones(r1 - r0, dtype=bool)
            got = shard_ids[r, q][shard_ids[r, q] >= 0] - r0
            out[got] = False
            lim = bounds[r, q]
            if got.size == k:
                lim = max(lim, shard_s[r, q, k - 1])
            if out.any():
                assert sc[out, q].max() <= lim + 1e-9, (r, q)


def test_global_seed_sample_needs_a_sampled_route(hc):
    """A shard too small for the sampling pre-pass reports 0 units (the caller then searches
    every shard the plain way) and the seeded call rejects what it cannot serve."""
    import torch
    from hcrag_amd import HcrError
    rng = np.random.default_rng(9)
    D = 384
    E = rng.standard_normal((500, D)).astype(np.float32)
    q = torch.from_numpy(rng.standard_normal((64, D)).astype(np.float32)).cuda()
    buf = torch.empty((8192, 64), dtype=torch.float32, device="cuda")
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=True)
        u, nr = ix.sample_device(q.data_ptr(), 64, 10, buf.data_ptr(), buf.numel())
        assert (u, nr) == (0, 0)
        s = torch.empty((64, 300), dtype=torch.float64, device="cuda")
        i = torch.empty((64, 300), dtype=torch.int64, device="cuda")
        b = torch.empty((64,), dtype=torch.float64, device="cuda")
        with pytest.raises((ValueError, HcrError)):
            ix.search_seeded_device(q.data_ptr(), 64, 300, buf.data_ptr(), 8, 0.1, s.data_ptr(),
                                    i.data_ptr(), b.data_ptr())
