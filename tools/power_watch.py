"""Board power and clocks while a score kernel runs back to back (is the headline's dense pass
power-capped?).  The parent never touches the GPU: it starts the workload as a child process and
samples `amd-smi metric` (fallback: `rocm-smi`) every ~0.2 s, tagging each sample with the
phase the child last reported on stderr.

    python tools/power_watch.py [--shape c2] [--variants 0,1] [--seconds 6]

Output: gpurun_out/power_watch.log (raw SMI text per sample) and one JSON summary line per
variant on stdout (median power / clocks over the variant's phase)."""
import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, time, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/hc-rag_amd']
import bench, hcrag_amd as hc
SH = {"c2": (10_000_000, 768, "f16", 1024, 32), "c4": (12_500_000, 1024, "bf16", 8192, 64),
      "c1": (1_000_000, 384, "f16", 256, 10)}
N, D, dt, B, k = SH[sys.argv[2]]
secs = float(sys.argv[4])
dev = torch.device("cuda", 0)
ix = hc.VectorIndex(D, dt, device=0, capacity=N)
bench.make_shard(ix, hc, 0, N, D, dt, dev)
g = torch.Generator(device=dev).manual_seed(5)
Q = torch.randn((B, D), generator=g, device=dev)
S = torch.empty((B, k), dtype=torch.float64, device=dev)
I = torch.empty((B, k), dtype=torch.int64, device=dev)
st = torch.cuda.current_stream().cuda_stream
for v in sys.argv[3].split(","):
    ix.set_option(ix.OPT_QW1, int(v))
    ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=st)
    torch.cuda.synchronize()
    print("PHASE", v, flush=True, file=sys.stderr)
    t0 = time.perf_counter(); n = 0
    while time.perf_counter() - t0 < secs:
        ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=st)
        n += 1
    torch.cuda.synchronize()
    dt_ = time.perf_counter() - t0
    print("DONE", v, n, dt_, flush=True, file=sys.stderr)
    print("PHASE idle", flush=True, file=sys.stderr)
    time.sleep(1.5)
print("END", flush=True, file=sys.stderr)
"""

# Vendor-GEMM ceiling under the same power cap: torch.mm (hipBLASLt / rocBLAS) on the headline's
# GEMM shape (1024 queries x 768 . 768 x 131072-row chunks, fp16 in, fp16 out) and on a square
# 8192^3 fp16 GEMM, each run back to back for the phase (reported as TFLOP/s in DONE lines).
CHILD_GEMM = r"""
import sys, time, torch
secs = float(sys.argv[4])
dev = torch.device("cuda", 0)
shapes = {"g_head": (1024, 131072, 768), "g_sq": (8192, 8192, 8192), "g_head_t": (131072, 1024, 768)}
for v in sys.argv[3].split(","):
    M, N, K = shapes[v]
    A = torch.randn((M, K), device=dev, dtype=torch.float16)
    B = torch.randn((N, K), device=dev, dtype=torch.float16)
    C = torch.empty((M, N), device=dev, dtype=torch.float16)
    torch.mm(A, B.t(), out=C); torch.cuda.synchronize()
    print("PHASE", v, flush=True, file=sys.stderr)
    t0 = time.perf_counter(); n = 0
    while time.perf_counter() - t0 < secs:
        for _ in range(8):
            torch.mm(A, B.t(), out=C)
        torch.cuda.synchronize()
        n += 8
    dt_ = time.perf_counter() - t0
    print("DONE", v, n, dt_, flush=True, file=sys.stderr)
    print("TFLOPS", v, round(2.0 * M * N * K * n / dt_ / 1e12, 1), flush=True, file=sys.stderr)
    del A, B, C
    torch.cuda.empty_cache()
    print("PHASE idle", flush=True, file=sys.stderr)
    time.sleep(1.5)
print("END", flush=True, file=sys.stderr)
"""


def smi_sample():
    for cmd in (["amd-smi", "metric", "--power", "--clock", "--json"],
                ["rocm-smi", "--showpower", "--showgpuclocks", "--json"]):
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=5)
            if r.returncode == 0 and r.stdout.strip():
                return " ".join(cmd[:1]), r.stdout
        except (OSError, subprocess.TimeoutExpired):
            continue
    return "none", ""


def numbers(txt, keys):
    """First numeric value following each key (case-insensitive) in the SMI text."""
    out = {}
    for k in keys:
        m = re.search(k + r'[^0-9\-]{0,40}?(-?\d+(?:\.\d+)?)', txt, re.I)
        if m:
            out[k] = float(m.group(1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c2")
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--gemm", action="store_true", help="vendor GEMM phases (CHILD_GEMM)")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log = open(os.path.join(ROOT, "gpurun_out", "power_watch.log"), "w")
    p = subprocess.Popen([sys.executable, "-c", CHILD_GEMM if a.gemm else CHILD, ROOT, a.shape, a.variants, str(a.seconds)],
                         stderr=subprocess.PIPE, text=True)
    os.set_blocking(p.stderr.fileno(), False)
    phase, buf, samples, done = "build", "", [], {}
    while p.poll() is None:
        try:
            chunk = p.stderr.read()
        except (BlockingIOError, TypeError):
            chunk = None
        if chunk:
            buf += chunk
            *lines, buf = buf.split("\n")
            for ln in lines:
                if ln.startswith("PHASE"):
                    phase = ln.split()[1]
                elif ln.startswith("DONE"):
                    _, v, n, dt = ln.split()
                    done[v] = {"searches": int(n), "ms_per_search": 1e3 * float(dt) / int(n)}
                print(ln, flush=True)
        tool, txt = smi_sample()
        t = time.time()
        log.write(f"=== {t:.3f} phase={phase} tool={tool}\n{txt}\n")
        log.flush()
        vals = numbers(txt, ["socket_power", "power", "gfx_0", "gfxclk", "sclk", "uclk", "fclk"])
        samples.append((phase, vals))
        time.sleep(0.2)
    for v in a.variants.split(","):
        ph = [s for ph_, s in samples if ph_ == v and s]
        summ = {"variant": v, "samples": len(ph), **done.get(v, {})}
        for key in ("socket_power", "power", "gfx_0", "gfxclk", "sclk", "uclk"):
            xs = sorted(s[key] for s in ph if key in s)
            if xs:
                summ[key + "_med"] = xs[len(xs) // 2]
                summ[key + "_max"] = xs[-1]
        print(json.dumps(summ), flush=True)
    idle = [s for ph_, s in samples if ph_ == "idle" and s]
    if idle:
        print(json.dumps({"variant": "idle", "samples": len(idle), **idle[len(idle) // 2]}), flush=True)
    return p.returncode


if __name__ == "__main__":
    sys.exit(main())
