"""Deep top-k timing (bench.py configs[1] deep_k point, standalone): 1M x 384 f16 index, 64
queries (half planted), k = 5000 by default.  Prints one JSON line; run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split of the exact deep path.

    python tools/deep_prof.py [--k 5000] [--batch 64] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]
import torch                                    # noqa: E402
import bench                                    # noqa: E402
import hcrag_amd as hc                          # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--k", type=int, default=5000)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, D, B, k = a.rows, a.dim, a.batch, a.k
    ix = hc.VectorIndex(D, "f16", device=0, capacity=N)
    bench.make_shard(ix, hc, 0, N, D, "f16", dev, seed=2000)

    def rows_fn(idx):
        return torch.stack([torch.from_numpy(ix.get_rows(i, 1)[0]) for i in idx.tolist()]).to(dev)
    Q, src = bench.make_queries(rows_fn, B, D, dev, 0, N, 0)
    S = torch.empty((B, k), dtype=torch.float64, device=dev)
    I = torch.empty((B, k), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / a.steps
    st = ix.last_stats()
    ok = bool((S[:, :-1] >= S[:, 1:]).all().item())
    print(json.dumps({"rows": N, "dim": D, "k": k, "batch": B, "ms_per_batch": round(per * 1e3, 3),
                      "fallback_rounds": st["fallback_rounds"], "sorted": ok,
                      "planted_recall_at_1": float((I[: B // 2, 0].cpu() == src.cpu()).float().mean().item())}))
    ix.close()


if __name__ == "__main__":
    main()
