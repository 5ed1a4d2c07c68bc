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
    out[rank] = bool(np.array_equal(i.numpy(), ei)) and bool(
        np.allclose(s.numpy()[ei >= 0], es[ei >= 0], rtol=0, atol=1e-12))
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
