"""Calibration on the GPU box: what the vendor GEMM (torch.matmul -> hipBLASLt) reaches on the
score GEMM shape of the headline config (B = 1024 queries x 768 x N rows, fp16, f32 accumulate)
and on the encoder's projection shapes.  It is the practical ceiling the fused score + top-k'
kernel is compared against (not part of the product path)."""
import json
import sys
import time

import torch


def bench(fn, flops, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, flops / (ms * 1e-3) / 1e12


def main():
    dev = torch.device("cuda", 0)
    out = []
    for dt in (torch.float16, torch.bfloat16):
        # score GEMM: [1024 x 768] x [768 x 1M]  (rows chunk of 1M; fp16 output 2 GB)
        Q = torch.randn(1024, 768, device=dev, dtype=dt)
        E = torch.randn(1_000_000, 768, device=dev, dtype=dt)
        C = torch.empty(1024, 1_000_000, device=dev, dtype=dt)
        ms, tf = bench(lambda: torch.matmul(Q, E.t(), out=C), 2.0 * 1024 * 768 * 1_000_000)
        out.append({"shape": "score 1024x768 . 768x1M", "dtype": str(dt), "ms": ms, "TFLOPs": tf})
        ms, tf = bench(lambda: torch.matmul(E, Q.t()), 2.0 * 1024 * 768 * 1_000_000)
        out.append({"shape": "score^T 1M x768 . 768x1024", "dtype": str(dt), "ms": ms, "TFLOPs": tf})
        del Q, E, C
        # encoder projections at 1024 sequences x 32 tokens (bge-base)
        T = 32768
        for (n, kk) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
            X = torch.randn(T, kk, device=dev, dtype=dt)
            W = torch.randn(n, kk, device=dev, dtype=dt)
            ms, tf = bench(lambda: torch.matmul(X, W.t()), 2.0 * T * n * kk)
            out.append({"shape": f"enc {T}x{kk} . {kk}x{n}", "dtype": str(dt), "ms": ms, "TFLOPs": tf})
        torch.cuda.empty_cache()
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    sys.exit(main())
