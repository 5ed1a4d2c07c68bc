"""Where the QW score kernel's dense launch spends a stage, from the stamps build (Makefile target
`stamps_qw`):

    HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so python tools/qw_stamps.py ROWS DIM BATCH [K] [OPT=V ...]

Runs a few searches on a synthetic L2-normalised corpus, then reads the per-wave s_memtime sums
of the last dense QW launch: stage wait (vmcnt + barrier), DMA issue + bound reads, MFMA groups
(issue), epilogue; prints cycles per stage for all waves and for each half of the workgroup
(waves 0-3 / 4-7: the two waves of each SIMD).  The stamps' own lgkmcnt waits change the timing:
read shares, not absolute lengths."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]
import bench  # noqa: E402
import hcrag_amd  # noqa: E402
from hcrag_amd import _lib  # noqa: E402

N, D, B = (int(x) for x in sys.argv[1:4])
K = int(sys.argv[4]) if len(sys.argv) > 4 else 32
dev = torch.device("cuda:0")
ix = hcrag_amd.VectorIndex(D, "f16", device=0, capacity=N)
bench.make_shard(ix, hcrag_amd, 0, N, D, "f16", dev)
for kv in sys.argv[5:]:                    # index options NAME=VALUE (VectorIndex.OPT_NAME)
    name, v = kv.split("=")
    ix.set_option(getattr(ix, "OPT_" + name), int(v))
Q = np.random.default_rng(1).standard_normal((B, D)).astype(np.float32)
for _ in range(3):
    ix.search(Q, K)
st = ix.last_stats()
fn = _lib.lib().hcr_debug_qw_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
n = 4096 * 8 * 8
buf = (ctypes.c_ulonglong * n)()
assert fn(buf, n) == 0
raw = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8, 8)
a = raw.astype(np.float64)
o4 = raw[:, :, 4]
a[:, :, 4] = (o4 & np.uint64(0xFFFFFF)).astype(np.float64)          # stages
pro = ((o4 >> np.uint64(24)) & np.uint64(0xFFFFF)).astype(np.float64) / 100.0   # us
fin = (o4 >> np.uint64(44)).astype(np.float64) / 100.0
parts = ["wait+barrier", "dma+bounds", "mfma groups", "epilogue"]
live0 = a[:, :, 6] > 0
ghz = np.median(a[:, :, 5][live0] / a[:, :, 6][live0]) * 0.1 if live0.any() else 0.0
print(f"score_kernel {st['score_kernel']} workgroups {st['workgroups']}  in-kernel clock {ghz:.3f} GHz "
      f"(median over waves: s_memtime / s_memrealtime)")
for name, sel in (("all waves", slice(0, 8)), ("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
    sub = a[:, sel, :]
    live = sub[:, :, 4] > 0
    stages = sub[:, :, 4][live]
    tot = sum(sub[:, :, i][live].sum() for i in range(4))
    print(f"{name}: {live.sum()} waves, {stages.mean():.0f} stages per wave, "
          f"{tot / stages.sum():.0f} cycles per stage")
    for i, nm in enumerate(parts):
        x = sub[:, :, i][live] / stages
        print(f"  {nm:14s} {x.mean():8.0f} cycles/stage (p10 {np.percentile(x, 10):7.0f}, "
              f"p90 {np.percentile(x, 90):7.0f})  share {sub[:, :, i][live].sum() / tot:.3f}")
# the launch's time line per wave (100 MHz ticks -> us): entry skew, prologue (query fragments,
# ring primed), the stage loop, the final lists
live = a[:, :, 4] > 0
if live.any():
    e0 = raw[:, :, 7][live].astype(np.float64) / 100.0
    loop = a[:, :, 6][live] / 100.0
    p_, f_ = pro[live], fin[live]
    t0 = e0.min()
    end = e0 - t0 + p_ + loop + f_
    print(f"time line (us, median / p90 / max over waves): entry skew {np.median(e0 - t0):.1f} / "
          f"{np.percentile(e0 - t0, 90):.1f} / {(e0 - t0).max():.1f}; prologue {np.median(p_):.1f} / "
          f"{np.percentile(p_, 90):.1f} / {p_.max():.1f}; loop {np.median(loop):.1f} / "
          f"{np.percentile(loop, 90):.1f} / {loop.max():.1f}; final lists {np.median(f_):.1f} / "
          f"{np.percentile(f_, 90):.1f} / {f_.max():.1f}; last wave ends at {end.max():.1f}")
