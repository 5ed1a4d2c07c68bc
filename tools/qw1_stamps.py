"""Where the QW1 score kernel's time goes, from the stamps build (Makefile target `stamps_qw1`):

    HCRAG_LIB=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so python tools/qw1_stamps.py ROWS DIM BATCH [OPT SHAPE]

Runs a few searches on a synthetic L2-normalised corpus, then reads the per-wave s_memtime sums
of the last QW1 launch: stage wait (vmcnt + barrier), DMA issue + first reads, MFMA groups,
epilogue; prints cycles per stage and shares (the stamps' own waits change the timing: read
shares, not lengths)."""
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
opt = int(sys.argv[4]) if len(sys.argv) > 4 else 1
shape = 0
dev = torch.device("cuda:0")
ix = hcrag_amd.VectorIndex(D, "f16", device=0, capacity=N)
bench.make_shard(ix, hcrag_amd, 0, N, D, "f16", dev)
ix.set_option(ix.OPT_QW1, opt)
Q = np.random.default_rng(1).standard_normal((B, D)).astype(np.float32)
for _ in range(3):
    ix.search(Q, 32)
st = ix.last_stats()
fn = _lib.lib().hcr_debug_qw1_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
n = 4096 * 8 * 8
buf = (ctypes.c_ulonglong * n)()
assert fn(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8, 8).astype(np.float64)
live = a[:, :, 4] > 0
stages = a[:, :, 4][live]
parts = ["wait+barrier", "dma+first reads", "mfma groups", "epilogue"]
tot = sum(a[:, :, i][live].sum() for i in range(4))
print(f"score_kernel {st['score_kernel']} opt {opt} shape {shape}: {live.sum()} waves, "
      f"{stages.mean():.0f} stages per wave")
for i, nm in enumerate(parts):
    x = a[:, :, i][live] / stages
    print(f"  {nm:18s} {x.mean():8.0f} cycles/stage (p10 {np.percentile(x, 10):7.0f}, "
          f"p90 {np.percentile(x, 90):7.0f})  share {a[:, :, i][live].sum() / tot:.3f}")
