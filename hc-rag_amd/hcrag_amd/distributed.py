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
                 group: Optional[dist.ProcessGroup] = None):
        self.local_search = local_search
        self.merge = merge
        self.k = int(k)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
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
        s, i = self.local_search(q_all)
        s_recv = self._buf("s_recv", (W, B, k), torch.float64, dev)
        i_recv = self._buf("i_recv", (W, B, k), torch.int64, dev)
        # block j of s (the queries of rank j) goes to rank j; rank r receives [W shards][B][k]
        dist.all_to_all_single(s_recv.view(W * B, k), s.contiguous(), group=self.group)
        dist.all_to_all_single(i_recv.view(W * B, k), i.contiguous(), group=self.group)
        return self.merge(s_recv, i_recv)


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


__all__ = ["ShardedSearch", "shard_range", "hip_local_search", "hip_merge"]
