"""CPU: the row-sharded exchange (all_gather queries -> local top-k -> all_to_all -> merge)
over gloo with world_size 2 and 3 equals the unsharded oracle for every rank's queries.
The local search / merge here are test-side numpy stand-ins for the HIP kernels; the
exchange object (hcrag_amd.distributed.ShardedSearch) is the one the bench runs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np_merge(k):
    def run(s_recv, i_recv):
        W, B, _ = s_recv.shape
        s = s_recv.permute(1, 0, 2).reshape(B, W * k).numpy()
        i = i_recv.permute(1, 0, 2).reshape(B, W * k).numpy()
        os_, oi = np.full((B, k), -np.inf), np.full((B, k), -1, dtype=np.int64)
        for b in range(B):
            ok = i[b] >= 0
            ss, ii = s[b][ok], i[b][ok]
            o = np.lexsort((ii, -ss))[:k]
            os_[b, :o.size], oi[b, :o.size] = ss[o], ii[o]
        return torch.from_numpy(os_), torch.from_numpy(oi)
    return run


def _worker(rank, world, port, N, D, B, k, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hc-rag_amd")]
    from oracle import cosine_topk as O
    from hcrag_amd.distributed import ShardedSearch, shard_range
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rng = np.random.default_rng(5)
    E = rng.standard_normal((N, D))
    E[3] = 0                                          # zero row
    E[N - 1] = E[10]                                  # duplicate across shards
    Qall = rng.standard_normal((world * B, D)).astype(np.float32)
    Qall[0] = E[10]                                   # tie between rows 10 and N-1
    r0, r1 = shard_range(N, rank, world)

    def local_search(q_all):
        s, i = O.cosine_topk(q_all.numpy(), E[r0:r1], k)
        i = np.where(i >= 0, i + r0, -1)
        return torch.from_numpy(s), torch.from_numpy(i)

    ss = ShardedSearch(local_search, _np_merge(k), k)
    q_local = torch.from_numpy(Qall[rank * B:(rank + 1) * B].copy())
    s, i = ss.search(q_local)
    es, ei = O.cosine_topk(Qall[rank * B:(rank + 1) * B], E, k)
    # the plain step is the query all-gather + ONE all-to-all of the packed
    # (scores, ids) lists
    out[rank] = bool(np.array_equal(i.numpy(), ei)) and bool(
        np.allclose(s.numpy()[ei >= 0], es[ei >= 0], rtol=0, atol=1e-12)) and ss.collectives == 2
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_search_matches_unsharded(world):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, port, 1001, 24, 7, 9, out), nprocs=world,
                       join=True, start_method="spawn")
    assert dict(out) == {r: True for r in range(world)}


def test_shard_range_partitions_rows():
    from hcrag_amd.distributed import shard_range
    for N in (0, 1, 7, 1000, 10_000_000):
        for W in (1, 2, 3, 8):
            rs = [shard_range(N, r, W) for r in range(W)]
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(rs[j][1] == rs[j + 1][0] for j in range(W - 1))


def _gs_worker(rank, world, port, N, D, B, k, mode, out):
    """The global-seed protocol (ShardedSearch with local_sample / local_seeded) over gloo: the
    stand-ins follow hcr_search_sample_device / hcr_search_seeded_device's contract -- one-row
    sample units, the seed the j-th best of every rank's units with j from the whole corpus'
    sampled fraction, a rank's top-k among its rows at or above the seed, and the
    bound of the rows it left out."""
    import math
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "hc-rag_amd")]
    from oracle import cosine_topk as O
    from hcrag_amd.distributed import ShardedSearch, shard_range
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rng = np.random.default_rng(7)
    E = rng.standard_normal((N, D))
    E[N - 1] = E[10]                                  # duplicate across shards
    Qall = rng.standard_normal((world * B, D)).astype(np.float32)
    Qall[0] = E[10]
    Qall[1::3] = E[rng.integers(0, N, Qall[1::3].shape[0])] + 0.05 * rng.standard_normal((Qall[1::3].shape[0], D))
    r0, r1 = shard_range(N, rank, world)
    En = E / np.linalg.norm(E, axis=1, keepdims=True)
    aggressive = mode == "aggressive"
    calls = [0]

    def scores(q_all):
        q = q_all.numpy().astype(np.float64)
        q = q / np.linalg.norm(q, axis=1, keepdims=True)
        # (row by row, not a GEMM: its blocking depends on the shard's shape, and a row's score
        # must not -- duplicate rows on two shards tie exactly, as in the oracle)
        return (q[:, None, :] * En[None, r0:r1, :]).sum(-1)          # [WB, rows]

    def local_search(q_all):                         # the plain step (re-runs)
        sc = scores(q_all)
        o = np.argsort(-sc, axis=1, kind="stable")[:, :k]
        return (torch.from_numpy(np.take_along_axis(sc, o, 1)),
                torch.from_numpy((o + r0).astype(np.int64)))

    def local_sample(q_all):
        calls[0] += 1
        stride = 4
        if mode == "stale" and rank == 0 and calls[0] == 2:
            stride = 2                                # more units than the cached shape holds
        if mode == "raise" and rank == world - 1 and calls[0] == 2:
            raise ValueError("over-cap sample")      # as sample_device's HcrError(EINVAL)
        sc = scores(q_all)[:, ::stride]               # [WB, units]
        return torch.from_numpy(np.ascontiguousarray(sc.T).astype(np.float32)), sc.shape[1]

    def local_seeded(q_all, umax_all, units, frac):
        lam = k * frac
        j = 1 if aggressive else int(math.ceil(lam + 5 * math.sqrt(lam) + 3))
        u = umax_all.numpy()[:units].astype(np.float64)          # [U, WB]
        srt = -np.sort(-u, axis=0)
        seed = srt[min(j, units) - 1] if j <= units else np.full(u.shape[1], -np.inf)
        sc = scores(q_all)
        WB = sc.shape[0]
        s_out = np.full((WB, k), -np.inf)
        i_out = np.full((WB, k), -1, dtype=np.int64)
        bound = np.full(WB, -np.inf)
        for q in range(WB):
            cand = np.nonzero(sc[q] >= seed[q] - 1e-7)[0]
            if cand.size < sc.shape[1]:
                bound[q] = seed[q]
            o = cand[np.lexsort((cand, -sc[q][cand]))][:k]
            s_out[q, :o.size] = sc[q][o]
            i_out[q, :o.size] = o + r0
        return torch.from_numpy(s_out), torch.from_numpy(i_out), torch.from_numpy(bound)

    ss = ShardedSearch(local_search, _np_merge(k), k, local_sample=local_sample,
                       local_seeded=local_seeded, n_local=r1 - r0)
    q_local = torch.from_numpy(Qall[rank * B:(rank + 1) * B].copy())
    # expected: the same row-wise scores over the whole corpus, (score desc, id asc); the scores
    # also match the oracle's
    qn = Qall[rank * B:(rank + 1) * B].astype(np.float64)
    qn = qn / np.linalg.norm(qn, axis=1, keepdims=True)
    full = (qn[:, None, :] * En[None, :, :]).sum(-1)
    ei = np.argsort(-full, axis=1, kind="stable")[:, :k]
    es = np.take_along_axis(full, ei, 1)
    os_, _ = O.cosine_topk(Qall[rank * B:(rank + 1) * B], E, k)
    res = []
    for _ in range(3):                                # the shape is cached after the first step
        s, i = ss.search(q_local)
        ok = bool(np.array_equal(i.numpy(), ei)) and bool(np.allclose(s.numpy(), es, rtol=0, atol=0)) \
            and bool(np.allclose(s.numpy(), os_, rtol=0, atol=1e-9))
        res.append((ok, ss.last_global_seed, ss.collectives))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "normal"), (3, "normal"), (2, "aggressive"),
                                        (3, "stale"), (2, "raise")])
def test_sharded_search_global_seed(world, mode):
    """Exact with the global seed; an over-shot seed (the best sampled unit) fails the merge
    certificate for some queries and the step is re-run the plain way -- still exact.
    Collectives per step: the first step 5 (query all-gather, the one-time
    shape all-reduce, maxima all-gather, ONE packed all-to-all, the re-run all-reduce), later
    steps 4; a re-run adds 1 (its all-to-all: the queries are already gathered).
    "stale": rank 0's second sample has more units than the cached shape -- every rank re-runs
    that step the plain way and the third step recomputes the shape; "raise": the last rank's
    second sample raises (an over-cap sample) -- same, without any rank raising."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_gs_worker, args=(world, port, 1201, 24, 9, 5, mode, out),
                       nprocs=world, join=True, start_method="spawn")
    res = dict(out)
    for r in range(world):
        assert all(step[0] for step in res[r]), res   # exact on every step, every rank
    for t in range(3):
        steps = {res[r][t][1:] for r in range(world)}
        assert len(steps) == 1, res                   # every rank took the same branch
        reruns, coll = steps.pop()
        assert reruns is not None, res
        rerun = reruns > 0
        expect = (5 if t == 0 or (t == 2 and mode in ("stale", "raise")) else 4) + (1 if rerun else 0)
        assert coll == expect, (t, res)
        if mode == "aggressive":
            assert rerun
        elif mode in ("stale", "raise") and t == 1:
            assert reruns == world * 9, res          # every query of the step re-runs
        else:
            assert not rerun, (t, res)
