"""Profiling driver for the encoder (one shape, one mode): the bench's encoder leg without the
rest of the bench, so a rocprofv3 pass (kernel trace or --pmc) sees only encoder dispatches --
and, with --mm, the vendor GEMM the bench calibrates against (torch.mm fp16 8192^3) in the same
process, for SQ counters side by side.

    python tools/enc_prof.py [--model bge-base] [--mode f32] [--batch 1024] [--seq 32]
                             [--steps 10] [--mm 0]
Prints one JSON line: ms per batch (HIP events) and embeddings/s."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hc-rag_amd"))

import torch  # noqa: E402

import bench  # noqa: E402  (ENC_SHAPES, random_bert_state: the bench's own shapes and weights)
import hcrag_amd as hc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bge-base", choices=list(bench.ENC_SHAPES))
    ap.add_argument("--mode", default="f32")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seq", type=int, default=32)
    ap.add_argument("--seed", type=int, default=77)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mm", type=int, default=0, help="torch.mm fp16 8192^3 calls after the encoder")
    ap.add_argument("--power", action="store_true", help="sample board power / clock (bench.PowerSampler) while timing")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.ENC_SHAPES[a.model]
    enc = hc.BertEncoder(cfg, bench.random_bert_state(cfg), dtype=a.mode, device=0)
    g = torch.Generator(device="cpu").manual_seed(a.seed)
    S, B = a.seq, a.batch
    ids = torch.randint(1000, cfg["vocab_size"], (B, S), generator=g, dtype=torch.int32)
    lens = torch.randint(S // 2, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None, :] < lens[:, None]).to(torch.int32)
    ids = (ids * mask).to(dev)
    mask = mask.to(dev)
    out = torch.empty((B, cfg["hidden"]), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        enc.encode_device(ids, mask, out, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ps = bench.PowerSampler(0) if a.power else None
    if ps:
        ps.start()
    e0.record()
    for _ in range(a.steps):
        enc.encode_device(ids, mask, out, stream)
    e1.record()
    torch.cuda.synchronize()
    pc = ps.stop() if ps else None
    ms = e0.elapsed_time(e1) / a.steps
    res = {"model": a.model, "mode": a.mode, "batch": B, "seq": S, "ms_per_batch": round(ms, 3),
           "embeddings_per_s": round(B / ms * 1e3, 1), "tokens_valid": int(mask.sum().item()),
           "split_dm": os.environ.get("HCRAG_SPLIT_DM", "default"),
           "streams": os.environ.get("HCRAG_ENC_STREAMS", "default"), "power": pc}
    enc.close()
    if a.mm:
        A = torch.randn((8192, 8192), device=dev, dtype=torch.float16)
        Bm = torch.randn((8192, 8192), device=dev, dtype=torch.float16)
        C = torch.empty((8192, 8192), device=dev, dtype=torch.float16)
        t_end = time.perf_counter() + 1.0
        while time.perf_counter() < t_end:
            torch.mm(A, Bm.t(), out=C)
            torch.cuda.synchronize()
        e0.record()
        for _ in range(a.mm):
            torch.mm(A, Bm.t(), out=C)
        e1.record()
        torch.cuda.synchronize()
        mms = e0.elapsed_time(e1) / a.mm
        res["mm_8192_ms"] = round(mms, 3)
        res["mm_8192_TFLOPs"] = round(2.0 * 8192 ** 3 / (mms * 1e-3) / 1e12, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
