"""A/B of the large-batch score kernels in ONE process (cdna_hip_programming.md §5.4 rule 24):
interleaved rounds of HCR_OPT_QW1 = 0 (QW at D = 768 / v4 at D = 1024), 1 (QW1, DMA issue
spread over the MFMA groups) and 2 (QW1, DMA issue at the stage barrier) on the headline corpus
(configs[2]: 10M x 768 f16, B = 1024, k = 32) and the configs[4] per-rank shape (12.5M x 1024
bf16, B = 8192, k = 64).  Prints one JSON line per (shape, variant, round) and a summary.
Usage: python tools/qw1_ab.py [--shapes c2,c4] [--rounds 3] [--variants 0,1,2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

SHAPES = {"c2": (10_000_000, 768, "f16", 1024, 32), "c4": (12_500_000, 1024, "bf16", 8192, 64),
          "c1": (1_000_000, 384, "f16", 256, 10),
          "c2s": (2_000_000, 768, "f16", 1024, 32), "c4s": (2_000_000, 1024, "bf16", 8192, 64),
          "w8": (1_250_000, 768, "f16", 1024, 32), "w4": (2_500_000, 768, "f16", 1024, 32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c2,c4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2",
                    help="HCR_OPT_QW1 values, each optionally ':stride' (HCR_OPT_SAMPLE_STRIDE), "
                         "':qs_form' and ':prepass', e.g. -1:32")
    a = ap.parse_args()
    import hcrag_amd as hc
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    summary = {}
    for sh in a.shapes.split(","):
        N, D, dt, B, k = SHAPES[sh]
        t0 = time.perf_counter()
        ix = hc.VectorIndex(D, dt, device=0, capacity=N)
        bench.make_shard(ix, hc, 0, N, D, dt, dev)
        print(f"[{sh}] built {N} x {D} {dt} in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        g = torch.Generator(device=dev).manual_seed(5)
        Q = torch.randn((B, D), generator=g, device=dev)
        S = torch.empty((B, k), dtype=torch.float64, device=dev)
        I = torch.empty((B, k), dtype=torch.int64, device=dev)
        ref = None
        for r in range(a.rounds):
            for vs in a.variants.split(","):
                v, stride, qsf, pre = (int(x) for x in (vs + ":0:0:0").split(":")[:4])
                ix.set_option(ix.OPT_QW1, v)
                ix.set_option(ix.OPT_SAMPLE_STRIDE, stride)
                ix.set_option(ix.OPT_QS_FORM, qsf)
                ix.set_option(ix.OPT_PREPASS, pre)
                ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)
                torch.cuda.synchronize()
                ix.set_timing(True)
                kms, walls = [], []
                for _ in range(a.reps):
                    ts = time.perf_counter()
                    ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)
                    torch.cuda.synchronize()
                    walls.append((time.perf_counter() - ts) * 1e3)
                    kms.append(ix.last_stats()["score_kernel_ms"])
                ix.set_timing(False)
                st = ix.last_stats()
                ids = I.cpu()
                same = True if ref is None else bool(torch.equal(ids, ref))
                if ref is None:
                    ref = ids
                fl = 2.0 * B * N * D
                rec = {"shape": sh, "variant": vs, "round": r, "score_kernel": st["score_kernel"],
                       "score_ms": round(min(kms), 4), "score_ms_med": round(sorted(kms)[len(kms) // 2], 4),
                       "wall_ms": round(min(walls), 4), "wall_ms_med": round(sorted(walls)[len(walls) // 2], 4), "mfma_frac": round(fl / (min(kms) * 1e-3) / 2.5e15, 4),
                       "wg": st["workgroups"], "P": st["partitions"], "unit": st["unit_kernel"], "widened": st["widened_queries"],
                       "fallback": st["fallback_queries"], "ids_equal_first": same}
                print(json.dumps(rec), flush=True)
                summary.setdefault((sh, vs), []).append((min(kms), min(walls)))
        ix.close()
        del Q, S, I
        torch.cuda.empty_cache()
    for (sh, v), xs in summary.items():
        ks, ws = sorted(x[0] for x in xs), sorted(x[1] for x in xs)
        print(json.dumps({"summary": sh, "variant": v, "score_ms_min": round(ks[0], 4),
                          "score_ms_med": round(ks[len(ks) // 2], 4), "wall_ms_min": round(ws[0], 4),
                          "wall_ms_med": round(ws[len(ws) // 2], 4)}), flush=True)


if __name__ == "__main__":
    main()
