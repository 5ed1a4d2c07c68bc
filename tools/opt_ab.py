"""Interleaved A/B of per-index tuning options (hcr_index_set_option: results never change) in ONE
process on one synthetic corpus (cdna_hip_programming.md §5.4 rule 24):

    python tools/opt_ab.py ROWS DIM BATCH K ROUNDS ARM [ARM ...]

An ARM is a comma list of NAME=VALUE over VectorIndex.OPT_* (QW1, SAMPLE_STRIDE, QS_FORM, PREPASS,
QW_DM, QW_MIN), or "default".  Per arm and round: 20 timed searches (wall per search, HBM-resident
queries, its host sync included) and the HIP-event score-phase time; ids must be identical to
the first arm's.  Prints one line per (round, arm) and a median summary."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]
import bench  # noqa: E402
import hcrag_amd  # noqa: E402

N, D, B, K, R = (int(x) for x in sys.argv[1:6])
arms = sys.argv[6:]
dev = torch.device("cuda:0")
ix = hcrag_amd.VectorIndex(D, "f16", device=0, capacity=N)
bench.make_shard(ix, hcrag_amd, 0, N, D, "f16", dev, seed=2000)


def rows_fn(idx):
    return torch.stack([torch.from_numpy(ix.get_rows(i, 1)[0]) for i in idx.tolist()]).to(dev)


Q, _ = bench.make_queries(rows_fn, B, D, dev, 0, N, 0)
S = torch.empty((B, K), dtype=torch.float64, device=dev)
I = torch.empty((B, K), dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream().cuda_stream
names = {"QW1": ix.OPT_QW1, "SAMPLE_STRIDE": ix.OPT_SAMPLE_STRIDE, "QS_FORM": ix.OPT_QS_FORM,
         "PREPASS": ix.OPT_PREPASS, "QW_DM": ix.OPT_QW_DM, "QW_MIN": ix.OPT_QW_MIN,
         "QW_STAGGER": ix.OPT_QW_STAGGER, "FLAG_READ": ix.OPT_FLAG_READ}
defaults = {"QW1": -1, "SAMPLE_STRIDE": 0, "QS_FORM": 0, "PREPASS": 0, "QW_DM": -1, "QW_MIN": 0,
            "QW_STAGGER": -1, "FLAG_READ": 0}


def apply(arm):
    for k, v in defaults.items():
        ix.set_option(names[k], v)
    if arm != "default":
        for kv in arm.split(","):
            k, v = kv.split("=")
            ix.set_option(names[k], int(v))


def step():
    ix.search_device(Q.data_ptr(), B, K, S.data_ptr(), I.data_ptr(), stream=stream)


ref_ids = None
res = {a: [] for a in arms}
for r in range(R):
    for a in arms:
        apply(a)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        if ref_ids is None:
            ref_ids = I.cpu().numpy().copy()
        else:
            assert np.array_equal(I.cpu().numpy(), ref_ids), f"ids differ under {a}"
        n = 20
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n * 1e3
        ix.set_timing(True)
        km = 0.0
        for _ in range(n):
            step()
            km += ix.last_stats()["score_kernel_ms"]
        ix.set_timing(False)
        st = ix.last_stats()
        res[a].append((wall, km / n))
        print(f"round {r} {a:40s} wall {wall:.4f} ms  score {km / n:.4f} ms  kernel {st['score_kernel']}"
              f"  widened {st['widened_queries']}  fallback {st['fallback_queries']}", flush=True)
print(f"== {N} x {D}, B = {B}, k = {K}: medians over {R} rounds")
for a in arms:
    w = np.median([x[0] for x in res[a]])
    s = np.median([x[1] for x in res[a]])
    print(f"{a:40s} wall {w:.4f} ms  score {s:.4f} ms")
