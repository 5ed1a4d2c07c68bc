"""Row-sharded multi-GPU search: one process per GPU over torch.distributed.

The node-embedding matrix is split into contiguous row shards (rank r owns rows
[r*N//W, (r+1)*N//W), global id = shard offset + local row).  Each rank brings its own batch
of B query embeddings.  One search step:

    all_gather(query embeddings)          B*D*4 bytes per rank      (RCCL over xGMI)
    local exact top-k of all W*B queries  fused MFMA score + top-k' + fp64 rescore on the shard
    all_to_all(per-shard top-k lists)     B*k*16 bytes per rank pair (fp64 score + int64 id,
                                          packed into one buffer: one collective)
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

    Collectives per step (``self.collectives`` counts the last call's):
      plain        all_gather(queries) + ONE all_to_all of the packed (scores, ids) lists;
      global seed  all_gather(queries) + all_gather(sampled maxima) + ONE all_to_all of the
                   packed (scores, ids, bound) lists + ONE all_reduce (the re-run decision and a
                   stale-shape flag; its value is the step's one host read).
    The shape of the global seed (every rank's unit count, the sampled fraction, the corpus
    size) depends only on the shard sizes and the stride: one all_reduce the first time (and
    after ``refresh_shape()`` or a step that found it stale), not per step.
    """

    def __init__(self, local_search: Callable, merge: Callable, k: int,
                 group: Optional[dist.ProcessGroup] = None, local_sample: Optional[Callable] = None,
                 local_seeded: Optional[Callable] = None, n_local: int = 0, max_units: int = 16384):
        """local_sample(q_all) -> (umax [units, W*B] float32 or None, sampled rows);
        local_seeded(q_all, umax_all [U, W*B], U, sampled fraction) -> (scores, ids, bound [W*B]
        fp64); n_local = the rank's rows; max_units = the most gathered units local_seeded takes
        (hcr_search_seeded_device: 16384).  Both callables given: the global seed protocol."""
        self.local_search = local_search
        self.merge = merge
        self.k = int(k)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.local_sample = local_sample
        self.local_seeded = local_seeded
        self.n_local = int(n_local)
        self.max_units = int(max_units)
        self.last_global_seed = None        # None: not tried; else the number of re-run queries
        self.collectives = 0                # collectives issued by the last search() call
        self.timing = False                 # CUDA events per phase (bench; device tensors only)
        self.last_phases = None             # event triples of the last timed call
        self._gs_shape = None               # (WB, u_max, sampled fraction) or (WB, 0, 0) = off
        self._sample_error = None           # the last local_sample failure (HcrError, ...)
        self._bufs = {}

    def refresh_shape(self):
        """Forget the global seed's shape (call on every rank after changing any shard)."""
        self._gs_shape = None

    def _buf(self, name, shape, dtype, device):
        t = self._bufs.get(name)
        if t is None or t.shape != shape or t.dtype != dtype or t.device != device:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[name] = t
        return t

    def _ev(self, name):
        if self.timing:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.last_phases[name] = e

    def phase_ms(self):
        """Milliseconds of the last timed search() per phase (synchronises the device):
        gather (query all-gather), local (the shard's own search: sample + seeded, or plain),
        exchange (maxima all-gather, all-to-all, merge, the re-run decision), total."""
        p = self.last_phases
        if not p or "end" not in p:
            return None
        p["end"].synchronize()
        out = {"gather_ms": p["t0"].elapsed_time(p["gathered"]), "total_ms": p["t0"].elapsed_time(p["end"])}
        loc = 0.0
        for a, b in (("ls0", "ls1"), ("ld0", "ld1")):
            if a in p and b in p:
                loc += p[a].elapsed_time(p[b])
        out["local_ms"] = loc
        out["exchange_ms"] = out["total_ms"] - out["gather_ms"] - loc
        return {kk: round(v, 4) for kk, v in out.items()}

    def search(self, q_local: torch.Tensor):
        """Exact global top-k of this rank's queries (q_local [B, D] fp32)."""
        W, k = self.world, self.k
        B, D = q_local.shape
        self.collectives = 0
        if self.timing:
            self.last_phases = {}
        if W == 1:
            return self.local_search(q_local.contiguous())
        dev = q_local.device
        self._ev("t0")
        q_all = self._buf("q_all", (W * B, D), q_local.dtype, dev)
        dist.all_gather_into_tensor(q_all, q_local.contiguous(), group=self.group)
        self.collectives += 1
        self._ev("gathered")
        if self.local_sample is not None and self.local_seeded is not None:
            out = self._search_global_seed(q_all, B)
            if out is not None:
                self._ev("end")
                return out
            if self.timing:                      # the re-run: its local search is what counts
                self.last_phases = {"t0": self.last_phases["t0"], "gathered": self.last_phases["gathered"]}
        self._ev("ld0")
        local = self.local_search(q_all)
        self._ev("ld1")
        out = self._exchange(local, B)
        self._ev("end")
        return out

    def _exchange(self, local, B, bound=None):
        """ONE all_to_all of the packed lists: the block for rank j is [B*k scores (fp64 bits) |
        B*k ids | B bounds] int64 words, so every destination's part is contiguous."""
        W, k = self.world, self.k
        s, i = local
        dev = s.device
        Bk = B * k
        words = 2 * Bk + (B if bound is not None else 0)
        send = self._buf("x_send", (W, words), torch.int64, dev)
        send[:, :Bk].copy_(s.contiguous().view(torch.int64).view(W, Bk))
        send[:, Bk:2 * Bk].copy_(i.contiguous().view(W, Bk))
        if bound is not None:
            send[:, 2 * Bk:].copy_(bound.contiguous().view(torch.int64).view(W, B))
        recv = self._buf("x_recv", (W, words), torch.int64, dev)
        dist.all_to_all_single(recv, send, group=self.group)
        self.collectives += 1
        s_recv = recv[:, :Bk].contiguous().view(torch.float64).view(W, B, k)
        i_recv = recv[:, Bk:2 * Bk].contiguous().view(W, B, k)
        out = self.merge(s_recv, i_recv)
        if bound is None:
            return out
        return out, recv[:, 2 * Bk:].contiguous().view(torch.float64)

    def _shape(self, units, srows, WB, dev):
        """The global seed's shape: one all_reduce, cached (None = the seed is off here)."""
        if self._gs_shape is None or self._gs_shape[0] != WB:
            st = torch.tensor([units, -units, int(srows), self.n_local], dtype=torch.int64, device=dev)
            # (MAX of [u, -u] and SUM of [srows, n] in one call: the sums travel as MAX of a
            # one-hot spread -- W slots each -- so one all_reduce carries both)
            W = self.world
            r = dist.get_rank(self.group)
            pk = torch.zeros(2 + 2 * W, dtype=torch.int64, device=dev)
            pk[:2] = st[:2]
            pk[2 + r] = st[2]
            pk[2 + W + r] = st[3]
            dist.all_reduce(pk, op=dist.ReduceOp.MAX, group=self.group)
            self.collectives += 1
            pk = pk.cpu()
            u_max, u_min = int(pk[0]), -int(pk[1])
            srows_tot, n_tot = int(pk[2:2 + W].sum()), int(pk[2 + W:].sum())
            if u_min <= 0 or srows_tot <= 0 or n_tot <= 0 or W * u_max > self.max_units:
                self._gs_shape = (WB, 0, 0.0)
            else:
                self._gs_shape = (WB, u_max, min(1.0, srows_tot / n_tot))
        return self._gs_shape

    def _search_global_seed(self, q_all, B):
        """The global seed step; None when the seed is off for this shape or some query failed
        the merge certificate (the caller then runs the plain step for the whole batch)."""
        W, k = self.world, self.k
        WB = q_all.shape[0]
        dev = q_all.device
        self._ev("ls0")
        try:
            umax, srows = self.local_sample(q_all)
        except (ValueError, RuntimeError) as e:       # an over-cap sample (HcrError is a
            # RuntimeError): this rank has none -- it must not raise alone, the others would
            # block in the next collective
            umax, srows = None, 0
            self._sample_error = e
        units = 0 if umax is None else int(umax.shape[0])
        self._ev("ls1")
        _, u_max, frac = self._shape(units, srows, WB, dev)
        if u_max == 0:
            self.last_global_seed = None
            return None
        # a rank whose sample no longer fits the shape (its shard changed, or the sample failed):
        # it still takes part in every collective, sends no maxima and an infinite bound -- every
        # query then fails the merge certificate, all ranks re-run the plain way, and the stale
        # flag makes every rank recompute the shape before the next step
        stale = units == 0 or units > u_max
        mine = self._buf("umax_pad", (u_max, WB), torch.float32, dev)
        mine.fill_(float("-inf"))
        if not stale:
            mine[:units].copy_(umax)
        umax_all = self._buf("umax_all", (W * u_max, WB), torch.float32, dev)
        dist.all_gather_into_tensor(umax_all, mine, group=self.group)
        self.collectives += 1
        if self.timing:
            self.last_phases["ld0"] = torch.cuda.Event(enable_timing=True)
            self.last_phases["ld0"].record()
        if stale:
            s = torch.full((WB, k), float("-inf"), dtype=torch.float64, device=dev)
            i = torch.full((WB, k), -1, dtype=torch.int64, device=dev)
            bound = torch.full((WB,), float("inf"), dtype=torch.float64, device=dev)
        else:
            s, i, bound = self.local_seeded(q_all, umax_all, W * u_max, frac)
        self._ev("ld1")
        (ms, mi), b_recv = self._exchange((s, i), B, bound)
        kth = ms[:, k - 1]
        worst = b_recv.max(dim=0).values
        bad = ~((kth > worst) | torch.isneginf(worst))
        flag = torch.stack([bad.sum().to(torch.int64),
                            torch.tensor(1 if stale else 0, dtype=torch.int64, device=dev)])
        dist.all_reduce(flag, op=dist.ReduceOp.SUM, group=self.group)
        self.collectives += 1
        nbad, nstale = (int(x) for x in flag.cpu())
        if nstale:
            self._gs_shape = None
        self.last_global_seed = nbad
        if nbad > 0:
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


def global_seed_stride(n_total_tiles: int, world: int, min_tiles: int = 300, max_units: int = 16384) -> int:
    """One sampling stride for all ranks: the largest power of two in [16, 4096] leaving >=
    min_tiles sampled 256-row tiles over the whole corpus -- raised, if need be, until every
    rank's units (two per sampled tile) fit its 8192-unit buffer and all ranks' together fit the
    seeded call's max_units (a fixed stride overflowed both on large corpora)."""
    if n_total_tiles <= 0:
        raise ValueError("global seed: n_total_tiles must be the whole corpus' 256-row tiles (> 0)")
    stride = 16
    while stride * 2 <= 4096 and n_total_tiles // (stride * 2) >= min_tiles:
        stride *= 2
    per_rank = -(-n_total_tiles // world) + 1
    while stride < (1 << 30) and (2 * -(-per_rank // stride) > 8192
                                  or world * 2 * -(-per_rank // stride) > max_units):
        stride *= 2
    return stride


def hip_global_seed(index, k: int, world: int, n_total_tiles: int, min_tiles: int = 300):
    """(local_sample, local_seeded) callables backed by a ``VectorIndex`` shard: the rank samples
    W x sparser than on its own (``global_seed_stride``: one stride for all ranks, from the whole
    corpus' n_total_tiles 256-row tiles)."""
    stride = global_seed_stride(n_total_tiles, world, min_tiles)
    cap_units = 8192

    def sample(q_all: torch.Tensor):
        nq = q_all.shape[0]
        buf = torch.empty((cap_units, nq), dtype=torch.float32, device=q_all.device)
        # (stride <= 4096 is what the option takes; above it the C side's own bump applies)
        index.set_option(index.OPT_SAMPLE_STRIDE, min(stride, 4096))
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


__all__ = ["ShardedSearch", "shard_range", "hip_local_search", "hip_merge", "hip_global_seed",
           "global_seed_stride"]
