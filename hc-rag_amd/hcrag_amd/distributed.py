"""Row-sharded multi-GPU search: one process per GPU over torch.distributed.

The node-embedding matrix is split into contiguous row shards (rank r owns rows
[r*N//W, (r+1)*N//W), global id = shard offset + local row).  Each rank brings its own batch
of B query embeddings.  One search step:

    all_gather(query embeddings)          B*D*4 bytes per rank      (RCCL over xGMI)
    local exact top-k of all W*B queries  fused MFMA score + top-k' + fp64 rescore on the shard
    all_to_all(per-shard top-k lists)     B*k*16 bytes per rank pair (fp64 score + int64 id)
    merge W lists per own query           on-device K5 (score desc, id asc)

Every rank ends with the exact global top-k of its own queries.  Because each shard's list is
exact (fp64 re-scored), the merge is exact too.

Global seed (``local_sample`` / ``local_seeded`` given): each rank's sampling
pre-pass reports its unit maxima, the ranks all-gather them (units x W*B floats each) and every
rank seeds its dense pass from the whole corpus' sample -- a rank then appends only the rows
above a global estimate of the k-th best instead of its own shard's (~W x fewer), and samples W x
sparser.  A rank may hold fewer than k rows above that seed: it returns what it has plus the
bound every row it left out stays under, and the certificate moves to the merge (the merged k-th
score must beat every rank's bound).  Queries that fail it (rare) are searched again the plain
way, all ranks together, so results stay exact.

``ShardedSearch`` takes the local search and the merge as callables so the exchange logic is
the same object on MI355X (HIP index + RCCL) and in the CPU tests (gloo + a test-side merge).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n_rows: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row block of ``rank`` (the last ranks may hold one row fewer)."""
    return rank * n_rows // world, (rank + 1) * n_rows // world


class ShardedSearch:
    """Exchange logic of the row-sharded search.

    local_search(q_all [W*B, D] fp32) -> (scores [W*B, k] fp64, ids [W*B, k] int64, global ids)
    merge(scores [W, B, k], ids [W, B, k]) -> (scores [B, k], ids [B, k])
    """

    def __init__(self, local_search: Callable, merge: Callable, k: int,
                 group: Optional[dist.ProcessGroup] = None, local_sample: Optional[Callable] = None,
                 local_seeded: Optional[Callable] = None, n_local: int = 0):
        """local_sample(q_all) -> (umax [units, W*B] float32 or None, sampled rows);
        local_seeded(q_all, umax_all [U, W*B], U, sampled fraction) -> (scores, ids, bound [W*B]
        fp64); n_local = the rank's rows.  Both given: the global seed protocol."""
        self.local_search = local_search
        self.merge = merge
        self.k = int(k)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.local_sample = local_sample
        self.local_seeded = local_seeded
        self.n_local = int(n_local)
        self.last_global_seed = None        # None: not tried; else the number of re-run queries
        self._bufs = {}

    def _buf(self, name, shape, dtype, device):
        t = self._bufs.get(name)
        if t is None or t.shape != shape or t.dtype != dtype or t.device != device:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[name] = t
        return t

    def search(self, q_local: torch.Tensor):
        """Exact global top-k of this rank's queries (q_local [B, D] fp32)."""
        W, k = self.world, self.k
        B, D = q_local.shape
        if W == 1:
            return self.local_search(q_local.contiguous())
        dev = q_local.device
        q_all = self._buf("q_all", (W * B, D), q_local.dtype, dev)
        dist.all_gather_into_tensor(q_all, q_local.contiguous(), group=self.group)
        if self.local_sample is not None and self.local_seeded is not None:
            out = self._search_global_seed(q_all, B)
            if out is not None:
                return out
        return self._exchange(self.local_search(q_all), B)

    def _exchange(self, local, B, bound=None):
        W, k = self.world, self.k
        s, i = local
        dev = s.device
        s_recv = self._buf("s_recv", (W, B, k), torch.float64, dev)
        i_recv = self._buf("i_recv", (W, B, k), torch.int64, dev)
        # block j of s (the queries of rank j) goes to rank j; rank r receives [W shards][B][k]
        dist.all_to_all_single(s_recv.view(W * B, k), s.contiguous(), group=self.group)
        dist.all_to_all_single(i_recv.view(W * B, k), i.contiguous(), group=self.group)
        out = self.merge(s_recv, i_recv)
        if bound is None:
            return out
        b_recv = self._buf("b_recv", (W, B), torch.float64, dev)
        dist.all_to_all_single(b_recv.view(W * B), bound.contiguous(), group=self.group)
        return out, b_recv

    def _search_global_seed(self, q_all, B):
        """The global seed step; None when some rank has no sample or a query failed the merge
        certificate (the caller then runs the plain step for the whole batch)."""
        W, k = self.world, self.k
        WB = q_all.shape[0]
        dev = q_all.device
        umax, srows = self.local_sample(q_all)
        units = 0 if umax is None else int(umax.shape[0])
        st = torch.tensor([units, -units, int(srows), self.n_local], dtype=torch.int64, device=dev)
        mx = st[:2].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.group)
        sm = st[2:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM, group=self.group)
        u_max, u_min = int(mx[0]), -int(mx[1])
        srows_tot, n_tot = int(sm[0]), int(sm[1])
        if u_min == 0 or srows_tot <= 0 or n_tot <= 0:
            self.last_global_seed = None
            return None
        mine = self._buf("umax_pad", (u_max, WB), torch.float32, dev)
        mine.fill_(float("-inf"))
        mine[:units].copy_(umax)
        umax_all = self._buf("umax_all", (W * u_max, WB), torch.float32, dev)
        dist.all_gather_into_tensor(umax_all, mine, group=self.group)
        s, i, bound = self.local_seeded(q_all, umax_all, W * u_max, min(1.0, srows_tot / n_tot))
        (ms, mi), b_recv = self._exchange((s, i), B, bound)
        kth = ms[:, k - 1]
        worst = b_recv.max(dim=0).values
        bad = ~((kth > worst) | torch.isneginf(worst))
        nbad = bad.sum().to(torch.int64).reshape(1)
        dist.all_reduce(nbad, op=dist.ReduceOp.SUM, group=self.group)
        self.last_global_seed = int(nbad)
        if int(nbad) > 0:
            return None
        return ms, mi


def hip_local_search(index, k: int, score_mode: int = 0, threshold: float = float("-inf")):
    """local_search callable backed by a ``VectorIndex`` shard (device pointers, same stream)."""
    def run(q_all: torch.Tensor):
        nq = q_all.shape[0]
        s = torch.empty((nq, k), dtype=torch.float64, device=q_all.device)
        i = torch.empty((nq, k), dtype=torch.int64, device=q_all.device)
        index.search_device(q_all.data_ptr(), nq, k, s.data_ptr(), i.data_ptr(), score_mode,
                            threshold, stream=torch.cuda.current_stream(q_all.device).cuda_stream)
        return s, i
    return run


def hip_global_seed(index, k: int, world: int, n_total_tiles: int = 0, min_tiles: int = 300):
    """(local_sample, local_seeded) callables backed by a ``VectorIndex`` shard: the rank samples
    W x sparser than on its own (one stride for all ranks: the largest power of two leaving >=
    min_tiles sampled 256-row tiles over the whole corpus of n_total_tiles)."""
    stride = 16
    if n_total_tiles > 0:
        while stride * 2 <= 4096 and n_total_tiles // (stride * 2) >= min_tiles:
            stride *= 2
    cap_units = 8192

    def sample(q_all: torch.Tensor):
        nq = q_all.shape[0]
        buf = torch.empty((cap_units, nq), dtype=torch.float32, device=q_all.device)
        index.set_option(index.OPT_SAMPLE_STRIDE, stride)
        try:
            units, rows = index.sample_device(q_all.data_ptr(), nq, k, buf.data_ptr(), cap_units * nq,
                                              stream=torch.cuda.current_stream(q_all.device).cuda_stream)
        finally:
            index.set_option(index.OPT_SAMPLE_STRIDE, 0)
        return (buf[:units] if units else None), rows

    def seeded(q_all: torch.Tensor, umax_all: torch.Tensor, units: int, frac: float):
        nq = q_all.shape[0]
        s = torch.empty((nq, k), dtype=torch.float64, device=q_all.device)
        i = torch.empty((nq, k), dtype=torch.int64, device=q_all.device)
        b = torch.empty((nq,), dtype=torch.float64, device=q_all.device)
        index.search_seeded_device(q_all.data_ptr(), nq, k, umax_all.data_ptr(), units, frac,
                                   s.data_ptr(), i.data_ptr(), b.data_ptr(),
                                   stream=torch.cuda.current_stream(q_all.device).cuda_stream)
        return s, i, b

    return sample, seeded


def hip_merge(k: int):
    """merge callable backed by the on-device K5 kernel (hcr_merge_topk_device)."""
    from .index import merge_topk_device

    def run(s_recv: torch.Tensor, i_recv: torch.Tensor):
        W, B, _ = s_recv.shape
        out_s = torch.empty((B, k), dtype=torch.float64, device=s_recv.device)
        out_i = torch.empty((B, k), dtype=torch.int64, device=s_recv.device)
        merge_topk_device(s_recv.data_ptr(), i_recv.data_ptr(), W, B, k, out_s.data_ptr(),
                          out_i.data_ptr(),
                          stream=torch.cuda.current_stream(s_recv.device).cuda_stream)
        return out_s, out_i
    return run


__all__ = ["ShardedSearch", "shard_range", "hip_local_search", "hip_merge", "hip_global_seed"]
