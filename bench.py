"""Headline benchmark (BASELINE.json): brute-force cosine top-k QPS over a 10M x 768 fp16
node-embedding corpus, batch 1024 queries, top-32 (configs[2]), on 1..8 MI355X, plus the
query-embedding throughput of the encoder in both compute modes.

One process per GPU (torchrun sets RANK / LOCAL_RANK / WORLD_SIZE; `bench.py --gpus N` without
torchrun launches its own N ranks through torch.distributed.run before touching the GPU).
Strong scaling (the metric: a fixed 10M corpus and a fixed global batch of 1024 queries on
1/2/4/8 GPUs; --global-batch 4096 at 8 GPUs is configs[3]): the corpus is row-sharded over W
GPUs, each rank holds global_batch / W queries, and one step is
    all-gather(query embeddings)  ->  local fused MFMA score + top-k' + fp64 rescore of all
    global_batch queries on the shard  ->  all-to-all(per-shard exact top-k)  ->  on-device
    merge of W lists per own query,
with the queries already resident in HBM.  `value` = global_batch / (max-over-ranks step time).

Prints ONE JSON line on rank 0 (the driver's contract); diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hc-rag_amd"))
sys.path.insert(0, ROOT)

import numpy as np
import torch

METRIC = "query-embeddings/sec + top-k QPS, 10M×768 corpus, batch=1024, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_PEAK_TFLOPS = 2500.0    # dense fp16/bf16 MFMA (no sparsity)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=10_000_000)
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--global-batch", type=int, default=1024,
                   help="queries per step over all GPUs (strong scaling; configs[3]: 4096)")
    p.add_argument("--batch", type=int, default=0,
                   help="queries per GPU per step (weak scaling; overrides --global-batch)")
    p.add_argument("--k", type=int, default=32)
    p.add_argument("--global-seed", default="on", choices=["on", "off"],
                   help="N > 1: seed every rank's dense pass from the all-gathered sample of the "
                        "whole corpus (DESIGN.md §6); off: each rank seeds from its own shard")
    p.add_argument("--dtype", default="f16", choices=["f16", "bf16"])
    p.add_argument("--cpu-rows", type=int, default=1_000_000)
    p.add_argument("--cpu-queries", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--encoder", default="bge-base", choices=["bge-base", "bge-large", "minilm", "none"],
                   help="query-embedding leg: BERT shape (random init) encoded on each GPU")
    p.add_argument("--enc-modes", default="f32,f16",
                   help="encoder compute modes to time: f32 (reference precision) and/or f16/bf16")
    p.add_argument("--enc-seq", type=int, default=32)
    p.add_argument("--enc-seed", type=int, default=77,
                   help="seed of the encoder leg's synthetic token lengths (the packed token count)")
    p.add_argument("--enc-steps", type=int, default=10)
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_score.json"),
                   help="PMC HBM-traffic summary (tools/pmc_summary.py --traffic) of this config")
    p.add_argument("--no-configs0", action="store_true",
                   help="skip the configs[0] real-data leg (GPU vs CPU on data/Product*.csv)")
    p.add_argument("--sweep", default="1,8,32,64,256",
                   help="batch sizes of the 1-GPU small-batch sweep recorded in extra.batch_sweep "
                        "('' to skip)")
    p.add_argument("--pipe-modes", default="f32,f16",
                   help="encoder modes of the end-to-end query pipeline leg (token ids -> encoder "
                        "-> sharded search), '' to skip")
    p.add_argument("--pipe-steps", type=int, default=5)
    p.add_argument("--no-configs1", action="store_true",
                   help="skip the configs[1] leg (1M x 384 f16, B = 256, top-10; 1 GPU)")
    p.add_argument("--no-vendor-gemm", action="store_true",
                   help="skip the vendor-GEMM calibration of the MFMA roofline (torch.mm)")
    p.add_argument("--power-seconds", type=float, default=3.0,
                   help="seconds of back-to-back headline steps with board power / clock sampled "
                        "(0: skip)")
    p.add_argument("--no-leg-power", action="store_true",
                   help="do not sample board power / clock during the encoder and configs[4] legs")
    p.add_argument("--large-k", default="1000,2048",
                   help="k values of the k > 256 leg (exact fallback) at B = 64 ('' to skip)")
    p.add_argument("--no-configs4", action="store_true",
                   help="skip the configs[4] per-rank leg (12.5M x 1024 bf16, 8192 queries, "
                        "top-64, bge-large encoder; 1 GPU)")
    return p.parse_args()


def spawn_ranks(a):
    """`bench.py --gpus N` outside torchrun: launch N ranks (torch.distributed.run, 127.0.0.1)
    as a child process -- before this process touches the GPU -- and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    log(f"spawning {a.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cgroup_cpu_quota():
    """CPUs of this process' cgroup quota (cgroup v2 cpu.max 'quota period'), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_cores():
    """Host threads the CPU legs run on: the CPUs this process may run on (sched_getaffinity),
    capped by the cgroup quota and by the pool's per-GPU host-CPU share, which the GPU box
    states in OMP_NUM_THREADS (16 per GPU there; sched_getaffinity shows the whole machine's
    CPUs, shared with the other GPUs' jobs)."""
    n = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    if quota:
        n = min(n, max(1, int(quota)))
    env = os.environ.get("OMP_NUM_THREADS") or os.environ.get("OPENBLAS_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return n


def make_shard(ix, hc, r0, r1, dim, dtype, dev, seed=1000, chunk=1 << 20):
    """Rows [r0, r1) of a deterministic global corpus (identical for any GPU count):
    global chunk c (1M rows) is N(0,1) from a Philox stream seeded (seed + c)."""
    tdt = torch.float16 if dtype == "f16" else torch.bfloat16
    hdt = hc.HCR_F16 if dtype == "f16" else hc.HCR_BF16
    g = torch.Generator(device=dev)
    c0, c1 = r0 // chunk, (r1 - 1) // chunk
    for c in range(c0, c1 + 1):
        g.manual_seed(seed + c)
        base = c * chunk
        x = torch.randn((chunk, dim), generator=g, device=dev, dtype=tdt)
        a, b = max(r0, base) - base, min(r1, base + chunk) - base
        xs = x[a:b].contiguous()
        ix.add_device(xs.data_ptr(), b - a, hdt, normalize=True,
                      stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        del x, xs


def make_queries(ix_rows_fn, B, dim, dev, rank, n_local, r0):
    """50% planted (a corpus row of this shard + N(0, 0.05^2) noise), 50% fresh."""
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    Q = torch.randn((B, dim), generator=g, device=dev, dtype=torch.float32)
    src_local = torch.randint(0, n_local, (B // 2,), generator=g, device=dev)
    rows = ix_rows_fn(src_local)
    Q[: B // 2] = rows + 0.05 * torch.randn((B // 2, dim), generator=g, device=dev) / dim ** 0.5
    return Q, (src_local + r0)


def workload_name(N, D, dtype, GB, k, world):
    """Names the BASELINE.json config a run matches (configs[2] is the default headline)."""
    key = (N, D, GB, k)
    if key == (10_000_000, 768, 1024, 32):
        tag = "configs[2]" if world == 1 else "metric strong-scaling point (configs[2] corpus and batch)"
    elif key == (10_000_000, 768, 4096, 32):
        tag = "configs[3]" if world == 8 else "configs[3] corpus and batch"
    elif key == (1_000_000, 384, 256, 10):
        tag = "configs[1]"
    elif key == (100_000_000 // 8, 1024, 8192, 64):
        tag = "configs[4] per-rank shape"
    else:
        tag = "custom"
    return (f"{tag}: {N:,} x {D} {dtype} node embeddings, global batch={GB} queries, top-{k} "
            f"(row-sharded over {world} GPU{'s' if world > 1 else ''})")


def load_traffic(path, N, D, nq, k, dtype, world):
    """HBM bytes per score phase from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes of
    this exact config (profiles/, corrected per MI355X_MICROARCH.md §HBM), or None."""
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    c = t.get("config", {})
    if (c.get("rows"), c.get("dim"), c.get("batch"), c.get("k"), c.get("dtype")) != (N, D, nq, k, dtype) \
            or world != 1:
        return None
    return round(t["hbm_bytes_per_search"] / 1e9, 3)


def cpu_baseline(E_rows_f16, Q, k, n_total):
    """Oracle ("port") timed on the host: the reference's literal path -- sklearn-semantics
    cosine in fp64 over the fp64 matrix + np.argsort(...)[::-1][:k] (experiments/main.py:
    841-844) -- on a bounded sample, extrapolated linearly in rows; beside it the tuned CPU
    path of BASELINE.md §3 (fp32 BLAS GEMM + argpartition) on the same sample."""
    from concurrent.futures import ThreadPoolExecutor
    from threadpoolctl import threadpool_limits
    from oracle import cosine_topk as O
    threads = cpu_cores()
    E = E_rows_f16.astype(np.float64)
    q = Q.astype(np.float64)
    with threadpool_limits(limits=threads):          # BLAS threads = every CPU the job may use
        t0 = time.perf_counter()
        sims = O.cosine_similarity64(q, E)
        top = np.argsort(sims, axis=1)[:, ::-1][:, :k]
        t = time.perf_counter() - t0
        del top, sims
        nq, nr = Q.shape[0], E.shape[0]
        qps = nq / (t * (n_total / nr))
        # tuned: fp32 unit rows (normalised once, outside the timed region, as an index would
        # store them), one SGEMM, argpartition + a sort of the k survivors -- the selection
        # spread over the same threads (numpy releases the GIL in its partition / sort)
        E32 = (E / np.linalg.norm(E, axis=1, keepdims=True)).astype(np.float32)
        q32 = Q.astype(np.float32)
        del E

        def select(s32, a, b):
            part = np.argpartition(-s32[a:b], k, axis=1)[:, :k]
            np.take_along_axis(s32[a:b], part, axis=1).argsort(axis=1)
        with ThreadPoolExecutor(threads) as pool:
            t1 = time.perf_counter()
            s32 = (q32 / np.linalg.norm(q32, axis=1, keepdims=True)) @ E32.T
            step = -(-nq // threads)
            list(pool.map(lambda a: select(s32, a, min(nq, a + step)), range(0, nq, step)))
            tt = time.perf_counter() - t1
        del s32, E32
    return {"value": qps, "unit": "queries/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "threads_env": {v: os.environ.get(v) for v in (
                "OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")},
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": cgroup_cpu_quota(),
            "threads_rule": "BLAS threads and the tuned leg's selection threads = the CPUs the job "
                            "may use: sched_getaffinity capped by the cgroup quota and by the pool's "
                            "per-GPU host-CPU share (OMP_NUM_THREADS on the GPU box); the literal "
                            "leg's argsort is numpy's own (single-threaded), as the reference runs it",
            "sample": f"{nq} queries x {nr:,}-row slice of the same corpus (fp16 decoded to fp64), "
                      f"cosine_similarity fp64 + argsort[::-1][:{k}] in {t:.2f} s, "
                      f"extrapolated linearly to {n_total:,} rows",
            "tuned": {"value": nq / (tt * (n_total / nr)), "unit": "queries/s",
                      "path": "fp32 SGEMM over pre-normalised rows + argpartition (BASELINE.md §3)",
                      "seconds_on_sample": round(tt, 3)}}


class PowerSampler:
    """Board power and gfx clock of one GPU from its amdgpu hwmon sysfs files, sampled by a
    thread of this process (file reads only: no SMI child process).  power1_average /
    power1_input are microwatts; freq1_input (label sclk) is Hz; pp_dpm_sclk's starred level is
    the fallback clock.  The in-kernel clock reads up to ~10 % below these (MI355X_MICROARCH.md
    'DVFS give-back' item 6); this samples what the board reports while the step runs."""

    def __init__(self, dev_index, period=0.02):
        import glob
        import threading
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self._thread = None
        self.dir = None
        try:
            pr = torch.cuda.get_device_properties(dev_index)
            bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        except Exception:
            bdf = None
        # only this device's hwmon: the PCI path of its BDF, or a drm card whose
        # device resolves to that BDF; with no BDF, a card only when the box shows exactly one
        # (on a shared box any other card may be another job's GPU) -- else 'unknown'
        drm = sorted(glob.glob("/sys/class/drm/card*/device"))
        if bdf:
            cands = [f"/sys/bus/pci/devices/{bdf}"] + [
                d for d in drm if os.path.basename(os.path.realpath(d)).lower() == bdf.lower()]
        else:
            cands = drm if len({os.path.realpath(d) for d in drm}) == 1 else []
        for d in cands:
            hw = sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*")))
            if hw and any(os.path.exists(os.path.join(hw[0], f)) for f in ("power1_average", "power1_input")):
                self.dir, self.hwmon = d, hw[0]
                break

    @staticmethod
    def _read(path):
        try:
            with open(path) as fh:
                return fh.read()
        except OSError:
            return None

    def sample(self):
        if not self.dir:
            return None
        w = None
        for f in ("power1_average", "power1_input"):
            v = self._read(os.path.join(self.hwmon, f))
            if v and v.strip().isdigit() and int(v) > 0:
                w = int(v) / 1e6
                break
        mhz = None
        v = self._read(os.path.join(self.hwmon, "freq1_input"))
        if v and v.strip().isdigit():
            mhz = int(v) / 1e6
        else:
            txt = self._read(os.path.join(self.dir, "pp_dpm_sclk")) or ""
            for ln in txt.splitlines():
                if ln.strip().endswith("*"):
                    try:
                        mhz = float(ln.split(":")[1].strip().rstrip("*").strip().lower().rstrip("mhz"))
                    except (IndexError, ValueError):
                        pass
        return (w, mhz)

    def _run(self):
        while not self._stop.is_set():
            x = self.sample()
            if x:
                self.samples.append(x)
            self._stop.wait(self.period)

    def start(self):
        import threading
        self.samples = []
        self._stop.clear()
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread:
            self._thread.join()
        ws = sorted(w for w, _ in self.samples if w is not None)
        ms = sorted(m for _, m in self.samples if m is not None)
        med = lambda xs: xs[len(xs) // 2] if xs else None
        return {"samples": len(self.samples), "power_W_med": med(ws), "power_W_max": ws[-1] if ws else None,
                "gfx_mhz_med": med(ms), "gfx_mhz_min": ms[0] if ms else None,
                "source": (self.hwmon if self.dir else "no amdgpu hwmon in sysfs")}


def power_leg(step, dev, achieved_tf, seconds=3.0):
    """Board power and gfx clock while the headline step runs back to back for `seconds`
    (after the timed region, same process, same shapes): is the dense pass at the board's power
    cap, and what fraction of the MFMA peak AT THE HELD CLOCK does it reach (2.5 PF is quoted at
    2400 MHz)?"""
    ps = PowerSampler(dev.index)
    step()
    torch.cuda.synchronize()
    ps.start()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        step()
        n += 1
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = ps.stop()
    out["steps"] = n
    out["ms_per_step"] = round(el / n * 1e3, 3)
    mhz = out.get("gfx_mhz_med")
    if mhz and achieved_tf:
        peak_at = MFMA_PEAK_TFLOPS * mhz / 2400.0
        out["mfma_peak_at_held_clock_TFLOPs"] = round(peak_at, 1)
        out["frac_at_held_clock"] = round(achieved_tf / peak_at, 4)
    return out


def large_k_leg(ix, dev, nloc, D, B=64, ks=(1000, 2048), reps=3):
    """k > 256 (no MFMA candidate path that deep: the exact fallback, MFMA-prefiltered scans of
    the whole shard): ms per batch, fallback rounds, and the scans' bytes (rounds x
    corpus) as a fraction of the 8 TB/s HBM roof.  experiments/main.py:844 (argsort has no k
    cliff)."""
    out = []
    stream = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(31)
    Q = torch.randn((B, D), device=dev, generator=g)
    for k in ks:
        S = torch.empty((B, k), dtype=torch.float64, device=dev)
        I = torch.empty((B, k), dtype=torch.int64, device=dev)
        ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        te = (time.perf_counter() - t0) / reps
        st = ix.last_stats()
        scan_bytes = st["fallback_rounds"] * nloc * D * 2
        out.append({"batch": B, "k": k, "ms_per_batch": round(te * 1e3, 3),
                    "fallback_queries": st["fallback_queries"], "fallback_rounds": st["fallback_rounds"],
                    "scan_GB": round(scan_bytes / 1e9, 2),
                    "hbm_frac_scan": round(scan_bytes / te / 1e9 / HBM_PEAK_GBS, 4)})
        log(json.dumps({"large_k": out[-1]}))
        del S, I
    return out


ENC_SHAPES = {
    # bge-base-en (768-d, the corpus dim of configs[2]; CLS pooling) and all-MiniLM-L6-v2
    "bge-base": dict(vocab_size=30522, hidden=768, layers=12, heads=12, intermediate=3072,
                     max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=1, normalize=1),
    # bge-large-en (1024-d, the corpus dim of configs[4])
    "bge-large": dict(vocab_size=30522, hidden=1024, layers=24, heads=16, intermediate=4096,
                      max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=1, normalize=1),
    "minilm": dict(vocab_size=30522, hidden=384, layers=6, heads=12, intermediate=1536,
                   max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=0, normalize=1),
}


def random_bert_state(cfg, seed=0):
    """Random-init BERT weights (HF BertModel names; no checkpoints offline)."""
    rng = np.random.default_rng(seed)
    H, F = cfg["hidden"], cfg["intermediate"]

    def w(*shape):
        return (0.02 * rng.standard_normal(shape)).astype(np.float32)
    sd = {"embeddings.word_embeddings.weight": w(cfg["vocab_size"], H),
          "embeddings.position_embeddings.weight": w(cfg["max_position"], H),
          "embeddings.token_type_embeddings.weight": w(cfg["type_vocab"], H),
          "embeddings.LayerNorm.weight": np.ones(H, np.float32),
          "embeddings.LayerNorm.bias": np.zeros(H, np.float32)}
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."
        for nm in ("attention.self.query", "attention.self.key", "attention.self.value",
                   "attention.output.dense"):
            sd[p + nm + ".weight"], sd[p + nm + ".bias"] = w(H, H), w(H)
        sd[p + "intermediate.dense.weight"], sd[p + "intermediate.dense.bias"] = w(F, H), w(F)
        sd[p + "output.dense.weight"], sd[p + "output.dense.bias"] = w(H, F), w(H)
        for nm in ("attention.output.LayerNorm", "output.LayerNorm"):
            sd[p + nm + ".weight"] = np.ones(H, np.float32)
            sd[p + nm + ".bias"] = np.zeros(H, np.float32)
    return sd


def enc_inputs(cfg, B, S, dev, seed):
    """B ragged synthetic token sequences (lengths S/2..S, ids >= 1000, zero-padded) on dev."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    ids = torch.randint(1000, cfg["vocab_size"], (B, S), generator=g, dtype=torch.int32)
    lens = torch.randint(S // 2, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None, :] < lens[:, None]).to(torch.int32)
    return (ids * mask).to(dev), mask.to(dev)


def timed_steps(step, steps, dev, dist):
    """Wall time of `steps` calls of step() bracketed by barrier + synchronize, max over ranks."""
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el / steps


def pipeline_leg(a, hc, dev, rank, world, dist, searcher, B, nq, mode):
    """The metric's end-to-end path (experiments/main.py:807-815 process_query: encode the query,
    then find_similar_content; query_interface.py:200-204 'vector' mode): each rank's B query
    token sequences -> the encoder (mode) -> ShardedSearch (all-gather of the embeddings, local
    certified top-k on the shard, all-to-all, merge) on one stream.  Whole-job queries/s."""
    cfg = ENC_SHAPES[a.encoder]
    enc = hc.BertEncoder(cfg, random_bert_state(cfg), dtype=mode, device=dev.index)
    ids, mask = enc_inputs(cfg, B, a.enc_seq, dev, 177 + rank)
    out = torch.empty((B, cfg["hidden"]), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        enc.encode_device(ids, mask, out, stream)
        return searcher.search(out)
    for _ in range(2):
        step()
    per = timed_steps(step, a.pipe_steps, dev, dist)
    enc_only = timed_steps(lambda: enc.encode_device(ids, mask, out, stream), a.pipe_steps, dev, dist)
    enc.close()
    return {"mode": mode, "model": f"{a.encoder} shape, random init", "seq_len": a.enc_seq,
            "queries_per_step": nq, "query_pipeline_qps": round(nq / per, 1),
            "ms_per_step": round(per * 1e3, 3), "encoder_ms": round(enc_only * 1e3, 3),
            "search_ms": round((per - enc_only) * 1e3, 3),
            "path": "token ids -> encoder -> all-gather -> certified top-k -> all-to-all -> merge"
                    if world > 1 else "token ids -> encoder -> certified top-k (one stream)"}


def vendor_gemm_leg(dev, seconds=2.0):
    """What the chip sustains on plain fp16 GEMMs through the vendor library (torch.mm ->
    hipBLASLt / rocBLAS), on random operands, after a warm-up long enough for the clock to
    settle under load (MI355X_MICROARCH.md 'DVFS give-back'): the headline's GEMM shape without
    the top-k (1024 queries x 768 . 768 x 131072-row chunks, fp16 out) and a square 8192^3.
    A calibration of the MFMA roofline under the power and clock the board holds; not a
    baseline of the retrieval path (the dense kernel also selects its top-k')."""
    out = {}
    for name, (M, Nn, K) in {"headline_shape_1024x131072x768": (1024, 131072, 768),
                             "square_8192": (8192, 8192, 8192)}.items():
        A = torch.randn((M, K), device=dev, dtype=torch.float16)
        B = torch.randn((Nn, K), device=dev, dtype=torch.float16)
        C = torch.empty((M, Nn), device=dev, dtype=torch.float16)
        t_end = time.perf_counter() + seconds / 2            # warm-up: the clock settles
        while time.perf_counter() < t_end:
            torch.mm(A, B.t(), out=C)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n, ms = 0, 0.0
        while ms < seconds * 500:
            e0.record()
            for _ in range(8):
                torch.mm(A, B.t(), out=C)
            e1.record()
            e1.synchronize()
            ms += e0.elapsed_time(e1)
            n += 8
        tf = 2.0 * M * Nn * K * n / (ms * 1e-3) / 1e12
        out[name] = {"TFLOPs": round(tf, 1), "frac_of_peak": round(tf / MFMA_PEAK_TFLOPS, 4)}
        del A, B, C
        torch.cuda.empty_cache()
    out["path"] = "torch.mm fp16 (hipBLASLt / rocBLAS), random operands, HIP events after a warm-up"
    return out


def configs1_leg(a, hc, dev, steps=50):
    """BASELINE.json configs[1] on one GPU: 1M x 384 f16 (L2-normalised N(0,1) rows), 256
    queries (half planted), top-10.  HBM-bound (256 flop/B < the 312 ridge): the roofline is the
    corpus stream, 0.768 GB per batch = 96 us at 8 TB/s."""
    N, D, B, k = 1_000_000, 384, 256, 10
    ix = hc.VectorIndex(D, "f16", device=dev.index, capacity=N)
    make_shard(ix, hc, 0, N, D, "f16", dev, seed=2000)

    def rows_fn(idx):
        return torch.stack([torch.from_numpy(ix.get_rows(i, 1)[0]) for i in idx.tolist()]).to(dev)
    Q, src = make_queries(rows_fn, B, D, dev, 0, N, 0)
    S = torch.empty((B, k), dtype=torch.float64, device=dev)
    I = torch.empty((B, k), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)
    for _ in range(5):
        step()
    per = timed_steps(step, steps, dev, None)
    ix.set_timing(True)
    km = 0.0
    for _ in range(steps):
        step()
        km += ix.last_stats()["score_kernel_ms"]
    ix.set_timing(False)
    st = ix.last_stats()
    km /= steps
    recall = float((I[: B // 2, 0].cpu() == src.cpu()).float().mean().item())
    byt = N * D * 2 + B * D * 2 + B * k * 12
    # deep k (VERDICT r5 missing #4 / item 5): k = 5000 for 64 of the queries -- the exact path
    # (sampled histogram threshold, one MFMA-prefiltered admission scan, radix select of the
    # k-th admitted key, bitonic sort of the k answers), against the time of one corpus scan
    kd, Bd = 5000, 64
    Sd = torch.empty((Bd, kd), dtype=torch.float64, device=dev)
    Id = torch.empty((Bd, kd), dtype=torch.int64, device=dev)

    def deep():
        ix.search_device(Q.data_ptr(), Bd, kd, Sd.data_ptr(), Id.data_ptr(), stream=stream)
    deep()
    dper = timed_steps(deep, 5, dev, None)
    dst = ix.last_stats()
    scan_ms = N * D * 2 / (HBM_PEAK_GBS * 1e9) * 1e3 / 0.79     # one scan at the measured ~6.3 TB/s copy rate
    deep_k = {"k": kd, "queries": Bd, "ms_per_batch": round(dper * 1e3, 3),
              "fallback_rounds": dst["fallback_rounds"], "corpus_scan_ms_at_6.3TBps": round(scan_ms, 4),
              "scans_equivalent": round(dper * 1e3 / scan_ms, 2),
              "planted_recall_at_1": float((Id[: Bd // 2, 0].cpu() == src[: Bd // 2].cpu()).float().mean().item())}
    ix.close()
    return {"workload": "configs[1]: 1,000,000 x 384 f16 node embeddings, batch=256 queries, "
                        "top-10, 1 GPU", "qps": round(B / per, 1), "ms_per_step": round(per * 1e3, 4),
            "score_kernel_ms": round(km, 4), "hbm_frac_step": round(byt / per / 1e9 / HBM_PEAK_GBS, 4),
            "hbm_frac_kernel": round(byt / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "alg_bytes": byt, "score_kernel": st.get("score_kernel"), "kprime": st["kprime"],
            "planted_recall_at_1": recall, "uncertified_queries": st["uncertified_queries"],
            "deep_k": deep_k,
            "note": "ms_per_step = wall time of one hcr_search_device call (queries in HBM, its one "
                    "host sync included); score_kernel_ms = HIP events around the pre-pass + dense "
                    "score launches"}


def configs4_leg(a, hc, dev, steps=3):
    """BASELINE.json configs[4] at its per-rank shape on one GPU: a 12.5M x 1024 bf16 shard
    (100M / 8), the global batch of 8192 queries, top-64, with this rank's 1024 queries encoded
    by the bge-large-shape encoder (reference precision) in the same step; the other ranks'
    7168 embeddings stand in for the all-gather (exchange time excluded: one GPU)."""
    N, D, B, k, own = 12_500_000, 1024, 8192, 64, 1024
    cfg = ENC_SHAPES["bge-large"]
    ix = hc.VectorIndex(D, "bf16", device=dev.index, capacity=N)
    make_shard(ix, hc, 0, N, D, "bf16", dev, seed=3000)
    enc = hc.BertEncoder(cfg, random_bert_state(cfg, seed=1), dtype="f32", device=dev.index)
    ids, mask = enc_inputs(cfg, own, a.enc_seq, dev, 401)
    g = torch.Generator(device=dev).manual_seed(402)
    Q = torch.randn((B, D), generator=g, device=dev)
    Qown = Q[:own]                                         # rows 0..1023: this rank's queries
    S = torch.empty((B, k), dtype=torch.float64, device=dev)
    I = torch.empty((B, k), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def search():
        ix.search_device(Q.data_ptr(), B, k, S.data_ptr(), I.data_ptr(), stream=stream)

    evs = []

    def step():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        enc.encode_device(ids, mask, Qown, stream)
        e1.record()
        evs.append((e0, e1))
        search()
    step()
    evs.clear()
    # the encoder's own time inside each step from events around it -- not the difference of
    # two loops -- and the board's power and clock over as many steps again
    per = timed_steps(step, steps, dev, None)
    enc_in_step = sorted(a.elapsed_time(b) for a, b in evs)
    ps = PowerSampler(dev.index)                 # (sampled after the timed steps, as above)
    ps.start()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pc = ps.stop()
    ix.set_timing(True)
    km = 0.0
    for _ in range(steps):
        search()
        km += ix.last_stats()["score_kernel_ms"]
    ix.set_timing(False)
    st = ix.last_stats()
    km /= steps
    srch = timed_steps(search, steps, dev, None)
    enc.close()
    ix.close()
    fl = 2.0 * B * N * D
    return {"workload": "configs[4] per-rank shape: 12,500,000 x 1024 bf16 shard, 8192 queries "
                        "(1024 encoded here by bge-large f32), top-64, 1 GPU",
            "per_rank_ms": round(per * 1e3, 3), "search_ms": round(srch * 1e3, 3),
            "encoder_ms": round((per - srch) * 1e3, 3),
            "encoder_ms_events": round(enc_in_step[len(enc_in_step) // 2], 3),
            "power_clock": pc, "score_kernel_ms": round(km, 3),
            "mfma_frac_score": round(fl / (km * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS, 4),
            "mfma_frac_search": round(fl / srch / 1e12 / MFMA_PEAK_TFLOPS, 4),
            "est_8gpu_qps": round(B / per, 1), "score_kernel": st.get("score_kernel"),
            "kprime": st["kprime"], "workgroups": st["workgroups"],
            "uncertified_queries": st["uncertified_queries"],
            "note": "est_8gpu_qps = 8192 / per-rank step (each of 8 ranks holds 12.5M rows and "
                    "scores all 8192 queries); the all-gather / all-to-all are not in it"}


def encoder_leg(a, hc, dev, rank, world, dist, mode, B):
    """Query-embedding throughput of one compute mode: B query token sequences per rank
    (S = --enc-seq, ragged lengths) -> BERT forward -> pool -> L2; whole-job embeddings/s over
    the max-over-ranks time.  Useful FLOPs per sequence = 2 * P_nonemb * len + 4 * L * len^2 * H
    (at each sequence's own token count: the encoder packs the valid tokens);
    the reference-precision mode executes 3x the projection FLOPs on MFMA (three split-f16
    terms), reported as mfma_frac_executed."""
    cfg = ENC_SHAPES[a.encoder]
    enc = hc.BertEncoder(cfg, random_bert_state(cfg), dtype=mode, device=dev.index)
    S = a.enc_seq
    g = torch.Generator(device="cpu").manual_seed(a.enc_seed + rank)
    ids = torch.randint(1000, cfg["vocab_size"], (B, S), generator=g, dtype=torch.int32)
    lens = torch.randint(S // 2, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None, :] < lens[:, None]).to(torch.int32)
    lens = mask.sum(1).double()
    ids = (ids * mask).to(dev)
    mask = mask.to(dev)
    out = torch.empty((B, cfg["hidden"]), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        enc.encode_device(ids, mask, out, stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.enc_steps):
        enc.encode_device(ids, mask, out, stream)
    ev1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    #  board power / clock of this leg, sampled over the same number of
    # batches right after the timed ones: the sysfs reads cost the encoder ~2 % (r06h), so they
    # stay out of the timed loop
    ps = PowerSampler(dev.index)
    if a.no_leg_power:
        ps.dir = None
    ps.start()
    for _ in range(a.enc_steps):
        enc.encode_device(ids, mask, out, stream)
    torch.cuda.synchronize()
    pc = ps.stop()
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    H, F, L = cfg["hidden"], cfg["intermediate"], cfg["layers"]
    p_nonemb = L * (4 * H * H + 2 * H * F)
    # model flops of the batch: every sequence at its own length (the tokens the result depends
    # on; the encoder packs them, pack_tokens_kernel) -- and, for comparison with rounds before
    # the packing, the padded basis (every sequence at S)
    flops_batch = float((2.0 * p_nonemb * lens + 4.0 * L * lens * lens * H).sum())
    flops_q = 2.0 * p_nonemb * S + 4.0 * L * S * S * H
    per_step = el / a.enc_steps
    tf = flops_batch / per_step / 1e12
    tf_padded = B * flops_q / per_step / 1e12
    gemm_mult = 3.0 if mode == "f32" else 1.0
    tf_exec = gemm_mult * 2.0 * p_nonemb * float(lens.sum()) / per_step / 1e12
    norms = out.norm(dim=1)
    enc.close()
    return {"mode": mode,
            "precision": ("reference (split-f16 MFMA GEMMs, fp32 attention; max |diff| vs fp32 "
                          "BertModel <= 2e-7 at full depth, tests/test_encoder_gpu.py)" if mode == "f32"
                          else f"fast ({mode} MFMA operands, fp32 accumulation)"),
            "model": f"{a.encoder} shape, random init", "seq_len": S, "batch_per_gpu": B,
            "query_embeddings_per_s": round(world * B / per_step, 1),
            "ms_per_batch": round(per_step * 1e3, 3),
            "gpu_ms_per_batch": round(ev0.elapsed_time(ev1) / a.enc_steps, 3),
            "tokens_valid": int(lens.sum()), "tokens_padded": B * S,
            "flops_per_batch": flops_batch, "TFLOPs": round(tf, 2),
            "TFLOPs_padded_basis": round(tf_padded, 2),
            "mfma_frac": round(tf / MFMA_PEAK_TFLOPS, 4),
            "mfma_frac_executed": round(tf_exec / MFMA_PEAK_TFLOPS, 4),
            "power_clock": pc,
            "unit_norm_ok": bool(((norms - 1).abs() < 1e-3).all().item())}


def configs0_leg(hc):
    """BASELINE.json configs[0] on the reference's own data: the 441 graph_builder.py:224-284
    documents of data/Product*.csv (committed fixture tests/golden/configs0/), MiniLM-shape
    encoder (seeded weights; no checkpoints offline), node index, top-5 / threshold 0.3 for the
    queries of experiments/main.py:1179-1184.  GPU: WordPiece + reference-precision encoder +
    EmbeddingSearch.  CPU, same run, same host: the reference's engines restated (HF Rust
    tokenizer + transformers BertModel fp32 in batches of 10 as HuggingFaceEmbedding's
    embed_batch_size, then sklearn cosine + argsort per query).  Times exclude model loading."""
    import gzip
    gdir = os.path.join(ROOT, "tests", "golden", "configs0")
    if not os.path.exists(os.path.join(gdir, "goldens.json")):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_configs0 import cpu_reference_embed
    from oracle import cosine_topk as O
    from hcrag_amd.synthetic import bert_state
    with gzip.open(os.path.join(gdir, "texts.jsonl.gz"), "rt", encoding="utf-8") as fh:
        docs = [json.loads(line) for line in fh]
    with open(os.path.join(gdir, "goldens.json")) as fh:
        gold = json.load(fh)
    texts = [d["text"] for d in docs]
    cfg = dict(gold["model"])
    state = bert_state(cfg, seed=gold["seed"], perturb_ln=gold["perturb_ln"])
    vocab = os.path.join(gdir, "vocab.txt")
    tok = hc.WordPieceTokenizer(vocab, lowercase=True)
    emb = hc.SentenceEmbedder(tok, hc.BertEncoder(cfg, state, dtype="f32"),
                              max_seq_length=gold["max_seq_length"], batch_size=64)
    emb.encode(texts[:8])                                  # warm-up (kernel load)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    E = emb.encode(texts)
    srch = hc.EmbeddingSearch(E, texts, [d["metadata"] for d in docs], dtype="f32", embedder=emb)
    gpu_res = [srch.find_similar_content(q, top_k=gold["top_k"], similarity_threshold=gold["threshold"])
               for q in gold["queries"]]
    t_gpu = time.perf_counter() - t0
    t1 = time.perf_counter()
    Ec = cpu_reference_embed(texts, vocab, state, cfg, batch=10)
    cpu_res = []
    for q in gold["queries"]:
        qe = cpu_reference_embed([q], vocab, state, cfg, batch=1)[0]
        cpu_res.append(O.find_similar_content(qe, Ec.astype(np.float64), gold["top_k"], gold["threshold"]))
    t_cpu = time.perf_counter() - t1
    same = all([texts.index(x["content"]) for x in g] == [i for i, _ in c]
               for g, c in zip(gpu_res, cpu_res))
    dmax = max(abs(x["similarity_score"] - sc) for g, c in zip(gpu_res, cpu_res)
               for x, (_, sc) in zip(g, c))
    threads = cpu_cores()
    return {"workload": "configs[0]: data/Product*.csv (441 graph_builder.py documents) -> "
                        "MiniLM-shape encoder (seeded) -> vector top-5, threshold 0.3, 4 queries "
                        "(experiments/main.py:1179-1184)",
            "gpu_s": round(t_gpu, 4), "cpu_s": round(t_cpu, 4), "speedup": round(t_cpu / t_gpu, 1),
            "gpu_texts_per_s": round(len(texts) / t_gpu, 1), "cpu_texts_per_s": round(len(texts) / t_cpu, 1),
            "cpu_cores": threads, "cpu_model": cpu_model(), "ids_identical": bool(same),
            "max_score_diff": float(dmax),
            "gpu_path": "hcr_tokenize + hcr_encode (f32 reference precision) + hcr_search",
            "cpu_path": "HF tokenizers + transformers BertModel fp32 (batches of 10) + sklearn-"
                        "semantics cosine + argsort (oracle)"}


def batch_sweep(a, ix, dev, nloc, D, k):
    """Small-batch sweep on rank 0 (1 GPU): the HBM-bound regime of north_star (B <= 64 on the
    headline corpus).  Per batch: wall time of one search (queries in HBM), the score kernel's
    HIP-event time, and both as fractions of the 8 TB/s HBM roofline on the algorithmic bytes."""
    out = []
    stream = torch.cuda.current_stream().cuda_stream
    for bsz in [int(x) for x in a.sweep.split(",") if x]:
        g = torch.Generator(device=dev).manual_seed(900 + bsz)
        Qs = torch.randn((bsz, D), device=dev, generator=g)
        Ss = torch.empty((bsz, k), dtype=torch.float64, device=dev)
        Is = torch.empty((bsz, k), dtype=torch.int64, device=dev)
        for _ in range(2):
            ix.search_device(Qs.data_ptr(), bsz, k, Ss.data_ptr(), Is.data_ptr(), stream=stream)
        ix.set_timing(True)
        torch.cuda.synchronize()
        reps = 10
        ts = time.perf_counter()
        km = 0.0
        for _ in range(reps):
            ix.search_device(Qs.data_ptr(), bsz, k, Ss.data_ptr(), Is.data_ptr(), stream=stream)
            km += ix.last_stats()["score_kernel_ms"]
        torch.cuda.synchronize()
        te = (time.perf_counter() - ts) / reps
        ix.set_timing(False)
        kms = km / reps
        byt = nloc * D * 2 + bsz * D * 2 + bsz * k * 12
        fl = 2.0 * bsz * nloc * D
        out.append({"batch": bsz, "qps": round(bsz / te, 1), "ms_per_batch": round(te * 1e3, 4),
                    "kernel_ms": round(kms, 4),
                    "hbm_frac_batch": round(byt / te / 1e9 / HBM_PEAK_GBS, 4),
                    "hbm_frac_kernel": round(byt / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "kernel_TFLOPs": round(fl / (kms * 1e-3) / 1e12, 2)})
        log(json.dumps({"sweep": out[-1]}))
    return out


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import hcrag_amd as hc
    N, D, k = a.rows, a.dim, a.k
    if a.batch > 0:                         # weak scaling: a fixed batch per GPU
        B, scaling = a.batch, "weak"
    else:                                   # strong scaling: a fixed global batch
        if a.global_batch % world:
            raise SystemExit(f"--global-batch {a.global_batch} not divisible by {world} GPUs")
        B, scaling = a.global_batch // world, "strong"
    nq = world * B                          # queries scored by every shard per step
    from hcrag_amd.distributed import shard_range
    r0, r1 = shard_range(N, rank, world)
    nloc = r1 - r0
    ix = hc.VectorIndex(D, a.dtype, device=local, capacity=nloc)
    ix.set_id_offset(r0)
    t_build = time.perf_counter()
    make_shard(ix, hc, r0, r1, D, a.dtype, dev)
    log(f"[rank {rank}] shard rows [{r0}, {r1}) built in {time.perf_counter() - t_build:.1f} s")

    # stored (normalised, rounded) rows for planted queries
    def rows_fn(idx):
        out = []
        for i in idx.tolist():
            out.append(torch.from_numpy(ix.get_rows(i, 1)[0]))
        return torch.stack(out).to(dev)

    Q, src = make_queries(rows_fn, B, D, dev, rank, nloc, r0)
    from hcrag_amd.distributed import ShardedSearch, hip_local_search, hip_merge, hip_global_seed
    gs = hip_global_seed(ix, k, world, (N + 255) // 256) if (world > 1 and a.global_seed == "on"
                                                              and k <= 256) else (None, None)
    searcher = ShardedSearch(hip_local_search(ix, k), hip_merge(k), k, local_sample=gs[0],
                             local_seeded=gs[1], n_local=nloc)
    gs_reruns = []

    def step():
        return searcher.search(Q)[1]

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()

    ix.set_timing(True)
    kern_ms, launches, unc, widened, fallback = 0.0, 0, 0, 0, 0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
        gs_reruns.append(searcher.last_global_seed)
        st = ix.last_stats()
        kern_ms += st["score_kernel_ms"]
        launches += st["score_launches"]
        unc += st["uncertified_queries"]
        widened += st["widened_queries"]
        fallback += st["fallback_queries"]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ix.set_timing(False)
    st = ix.last_stats()
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # planted recall@1 on this rank's own queries (global ids)
    top1 = res[: B // 2, 0].cpu()
    recall1 = float((top1 == src.cpu()).float().mean().item())

    # roofline of the dominant kernel (fused score + top-k'), per launch
    avg_ms = kern_ms / max(launches, 1)
    flops = 2.0 * nq * nloc * D
    elt = 2
    bytes_alg = nloc * D * elt + nq * D * elt + nq * k * 12
    ai = flops / bytes_alg
    if ai > (MFMA_PEAK_TFLOPS * 1e12) / (HBM_PEAK_GBS * 1e9):
        achieved = flops / (avg_ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / MFMA_PEAK_TFLOPS, 4), "traffic": None}
    else:
        achieved = bytes_alg / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None}
    roof["traffic"] = load_traffic(a.traffic_file, N, D, nq, k, a.dtype, world)
    roof["traffic_unit"] = ("GB per score phase (rocprofv3 FETCH_SIZE+WRITE_SIZE passes of this "
                            "config, profiles/traffic_score.json)")
    kname = {1: "score_topk_kernel (register-staged 128 x 128)", 3: "score_topk_v3_kernel",
             4: "score_topk_v4_kernel (256 x 256 tiles)",
             5: "score_topk_qs_kernel (query-stationary, 128/256 queries per workgroup)",
             6: "score_topk_qw_kernel (wide query-stationary: 256 queries per workgroup in VGPRs, "
                "full-K row stages)",
             7: "score_topk_qw1_kernel (D = 1024: one wave per SIMD, 48 queries per wave in AGPR/VGPRs)"
             }.get(st.get("score_kernel", 0), "?")
    roof["kernel"] = (kname + ", fused MFMA score + top-k': sampling pre-pass (MAXONLY form: QW's under QW, else v4's) + dense "
                      "pass, HIP events around both on the library's stream")
    roof["kernel_ms_avg"] = round(avg_ms, 4)
    roof["flops_per_launch"] = flops
    roof["alg_bytes_per_launch"] = bytes_alg
    ld = -(-D // 64) * 64
    if st.get("score_kernel") == 6:
        # QW's LDS fill: only rows, once per 256-query block (queries stay in VGPRs)
        fill = nloc * ld * elt * (-(-nq // 256))
        roof["lds_dma_fill_bytes"] = fill
        roof["lds_dma_fill_TBps"] = round(fill / (avg_ms * 1e-3) / 1e12, 2)
    elif st.get("score_kernel") == 4:
        # the 256 x 256 kernel's LDS fill: every stage brings 256 rows + 256 queries x 32 k
        # by LDS-DMA for 2*256*256*32 flop (128 flop per byte); the dense pass's rate of it
        # (the fill, not the MFMA pipe, bounds this tiling)
        n_tiles = -(-nloc // 256)
        fill = n_tiles * (-(-nq // 256)) * 512 * ld * elt
        roof["lds_dma_fill_bytes"] = fill
        roof["lds_dma_fill_TBps"] = round(fill / (avg_ms * 1e-3) / 1e12, 2)

    value = nq / (elapsed / a.steps)
    if a.power_seconds > 0 and roof["bound"] == "mfma" and world == 1:
        roof["power_clock"] = power_leg(step, dev, achieved, a.power_seconds)
        log(json.dumps({"power_clock": roof["power_clock"]}))
    if rank == 0 and world == 1 and not a.no_vendor_gemm and roof["bound"] == "mfma":
        cal = vendor_gemm_leg(dev)
        cal["this_kernel_vs_headline_shape"] = round(
            achieved / cal["headline_shape_1024x131072x768"]["TFLOPs"], 3)
        cal["this_kernel_vs_square"] = round(achieved / cal["square_8192"]["TFLOPs"], 3)
        roof["vendor_gemm_calibration"] = cal
        log(json.dumps({"vendor_gemm_calibration": cal}))
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        nr = min(a.cpu_rows, nloc)
        Eh = ix.get_rows(0, nr)
        cpu = cpu_baseline(Eh, Q[: a.cpu_queries].cpu().numpy(), k, N)
        del Eh

    enc_res = None
    if a.encoder != "none":
        enc_res = {}
        for mode in [m for m in a.enc_modes.split(",") if m]:
            enc_res[mode] = encoder_leg(a, hc, dev, rank, world, dist, mode, B)

    pipe = None
    if a.pipe_modes and a.encoder != "none" and ENC_SHAPES[a.encoder]["hidden"] == D:
        pipe = {}
        for mode in [m for m in a.pipe_modes.split(",") if m]:
            pipe[mode] = pipeline_leg(a, hc, dev, rank, world, dist, searcher, B, nq, mode)
            log(json.dumps({"pipeline": pipe[mode]}))

    sweep = None
    if a.sweep and world == 1 and rank == 0:
        sweep = batch_sweep(a, ix, dev, nloc, D, k)
    large_k = None
    if a.large_k and world == 1 and rank == 0:
        large_k = large_k_leg(ix, dev, nloc, D, ks=[int(x) for x in a.large_k.split(",") if x])
    c1 = c4 = None
    if rank == 0 and world == 1 and not a.no_configs1:
        c1 = configs1_leg(a, hc, dev)
        log(json.dumps({"configs1": c1}))
    c0 = None
    if rank == 0 and world == 1 and not a.no_configs0:
        c0 = configs0_leg(hc)

    # N > 1: where a step's time goes -- this rank's own search on its shard
    # (sample + seeded, or the plain search) against the exchange (the query all-gather, the
    # maxima all-gather, the one packed all-to-all, the merge and the re-run all-reduce), CUDA
    # events on the step's stream over a few extra steps after the timed ones; the rank with the
    # largest local time bounds the step.  The driver computes scaling efficiency from its own
    # per-N values; per_rank_shape gives what its T_1 / (N T_N) needs beside them.
    multi = None
    if world > 1:
        searcher.timing = True
        ph = []
        for _ in range(max(3, min(a.steps, 10))):
            step()
            ph.append(searcher.phase_ms())
        searcher.timing = False
        loc = torch.tensor([[p["local_ms"], p["gather_ms"], p["exchange_ms"], p["total_ms"]] for p in ph],
                           dtype=torch.float64, device=dev).median(dim=0).values
        allr = [torch.zeros_like(loc) for _ in range(world)]
        dist.all_gather(allr, loc)
        allr = torch.stack(allr).cpu().numpy()
        multi = {"per_rank_local_ms": [round(float(x), 4) for x in allr[:, 0]],
                 "per_rank_gather_ms": [round(float(x), 4) for x in allr[:, 1]],
                 "per_rank_exchange_ms": [round(float(x), 4) for x in allr[:, 2]],
                 "per_rank_step_ms": [round(float(x), 4) for x in allr[:, 3]],
                 "local_ms": round(float(allr[:, 0].max()), 4),
                 "exchange_ms": round(float(allr[:, 1:3].sum(axis=1).max()), 4),
                 "collectives_per_step": searcher.collectives,
                 "per_rank_shape": {"rows": nloc, "queries_scored": nq, "k": k},
                 "note": "median over extra steps after the timed ones, CUDA events on the search "
                         "stream; exchange_ms = query all-gather + maxima all-gather + packed "
                         "all-to-all + merge + re-run decision (max over ranks); local_ms = the "
                         "shard's own search (max over ranks)"}
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "queries/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic: N(0,1) rows L2-normalised at ingest then rounded to fp16; "
                    "queries 50% planted (corpus row + noise) / 50% random, fp32, HBM-resident",
            "config": {"workload": workload_name(N, D, a.dtype, nq, k, world),
                       "rows": N, "dim": D, "batch_per_gpu": B, "global_batch": nq, "k": k,
                       "parallelism": f"rowshard{world}" + ("+rccl_allgather_alltoall" if world > 1 else ""),
                       "global_seed": gs[0] is not None},
            "roofline": roof,
            "cpu_baseline": cpu,
            "encoder": enc_res,
            "configs0": c0,
            "configs1": c1,
            "query_pipeline": pipe,
            "query_pipeline_qps": (pipe or {}).get("f32", {}).get("query_pipeline_qps"),
            "extra": {"planted_recall_at_1": recall1, "uncertified_queries": unc,
                      "widened_queries": widened, "fallback_queries": fallback,
                      "kprime": st["kprime"], "unit_kernel": st["unit_kernel"],
                      "score_kernel": st.get("score_kernel"),
                      "partitions": st["partitions"], "workgroups": st["workgroups"],
                      "mfma_frac": round(flops / (avg_ms * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS, 4),
                      "hbm_frac_kernel": round(bytes_alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "pipeline_ms_per_step": round(elapsed / a.steps * 1e3, 3),
                      "batch_sweep": sweep, "large_k": large_k,
                      "global_seed_reruns": (None if gs[0] is None else
                                             sum(x for x in gs_reruns if x is not None)),
                      "global_seed_plain_steps": (None if gs[0] is None else
                                                  sum(1 for x in gs_reruns if x is None)),
                      "multi_gpu": multi},
        }
    ix.close()
    if rank == 0 and world == 1 and not a.no_configs4:
        torch.cuda.empty_cache()
        c4 = configs4_leg(a, hc, dev)
        log(json.dumps({"configs4_rank": c4}))
    if rank == 0:
        line["configs4_rank"] = c4
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
