"""The W-GPU strong-scaling step's per-rank search with and without the global seed, emulated on
one GPU: W shard indexes of a ROWS x DIM corpus (bench.make_shard: the rows each
rank of `bench.py --gpus W` holds), the gathered batch of GB queries (bench.make_queries).

    python tools/global_seed_rank.py ROWS DIM GB K W ROUNDS [OPT=V ...]

Per round and shard: the plain per-rank search (hcr_search_device: own pre-pass, own seed) and
the global-seed pair (hcr_search_sample_device at the shared sparser stride, then -- after the
maxima of all shards are gathered, here a device concatenation standing in for the RCCL
all-gather -- hcr_search_seeded_device); wall time per call with its sync.  Then the merged
global-seed lists are certified (merged k-th score > every shard's bound) and compared with the
merged plain lists: ids must be identical for every certified query.  Prints the medians over
shards and rounds."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]
import bench  # noqa: E402
import hcrag_amd  # noqa: E402
from hcrag_amd.distributed import hip_global_seed, hip_merge, shard_range  # noqa: E402

N, D, GB, K, W, R = (int(x) for x in sys.argv[1:7])
dev = torch.device("cuda:0")
shards = []
for r in range(W):
    r0, r1 = shard_range(N, r, W)
    ix = hcrag_amd.VectorIndex(D, "f16", device=0, capacity=r1 - r0)
    bench.make_shard(ix, hcrag_amd, r0, r1, D, "f16", dev, seed=2000)
    ix.set_id_offset(r0)
    for kv in sys.argv[7:]:                  # index options NAME=VALUE (VectorIndex.OPT_NAME)
        name, v = kv.split("=")
        ix.set_option(getattr(ix, "OPT_" + name), int(v))
    shards.append((ix, r0, r1))
ix0, a0, b0 = shards[0]


def rows_fn(idx):
    return torch.stack([torch.from_numpy(ix0.get_rows(i, 1)[0]) for i in idx.tolist()]).to(dev)


Q, _ = bench.make_queries(rows_fn, GB, D, dev, 0, b0 - a0, a0)
n_tiles = (N + 255) // 256
stream = torch.cuda.current_stream().cuda_stream
S = torch.empty((W, GB, K), dtype=torch.float64, device=dev)
I = torch.empty((W, GB, K), dtype=torch.int64, device=dev)
Sg = torch.empty_like(S)
Ig = torch.empty_like(I)
Bd = torch.empty((W, GB), dtype=torch.float64, device=dev)
merge = hip_merge(K)
plain_ms, gs_ms, sample_ms, seeded_ms = [], [], [], []
for rnd in range(R + 1):                     # round 0: warm-up
    for r, (ix, r0, r1) in enumerate(shards):
        for _ in range(2 if rnd == 0 else 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ix.search_device(Q.data_ptr(), GB, K, S[r].data_ptr(), I[r].data_ptr(), stream=stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
        if rnd:
            plain_ms.append((t1 - t0) * 1e3)
    # global seed: every shard's sample, the gather, every shard's seeded pass
    fns = [hip_global_seed(ix, K, W, n_tiles) for ix, _, _ in shards]
    ums, srows, t_s = [], 0, []
    for r, (ix, r0, r1) in enumerate(shards):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        u, nr = fns[r][0](Q)
        torch.cuda.synchronize()
        t_s.append((time.perf_counter() - t0) * 1e3)
        assert u is not None, "no sample"
        ums.append(u.clone())
        srows += nr
    umax = max(u.shape[0] for u in ums)
    umax_all = torch.full((W * umax, GB), float("-inf"), dtype=torch.float32, device=dev)
    for r, u in enumerate(ums):
        umax_all[r * umax:r * umax + u.shape[0]] = u
    for r, (ix, r0, r1) in enumerate(shards):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s, i, b = fns[r][1](Q, umax_all, W * umax, srows / N)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) * 1e3
        Sg[r], Ig[r], Bd[r] = s, i, b
        if rnd:
            sample_ms.append(t_s[r])
            seeded_ms.append(t)
            gs_ms.append(t_s[r] + t)
    ps, pi = merge(S, I)
    gs_s, gs_i = merge(Sg, Ig)
    torch.cuda.synchronize()
    cert = ((gs_s[:, K - 1] > Bd.max(0).values) | torch.isneginf(Bd.max(0).values))
    same = bool(torch.equal(gs_i[cert], pi[cert]))
    print(f"round {rnd}: units {W * umax} (sampled rows {srows}), certified {int(cert.sum())} / {GB}, "
          f"ids identical to the plain path on them: {same}", flush=True)
    assert same
print(f"== {N} x {D}, {GB} queries, k = {K}, W = {W}: per-rank medians over shards and {R} rounds")
print(f"plain per-rank search      {np.median(plain_ms):.4f} ms")
print(f"global seed: sample {np.median(sample_ms):.4f} + seeded {np.median(seeded_ms):.4f} = "
      f"{np.median(gs_ms):.4f} ms (the all-gather of the maxima not included)")
