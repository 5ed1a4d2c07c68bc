"""Where the merge + rescore kernel (finish_kernel, B <= 512) spends its time, from the stamps
build (Makefile target `stamps_fin`):

    HCRAG_LIB=hc-rag_amd/lib/stamps_fin/libhcrag_hip.so python tools/finish_stamps.py ROWS DIM BATCH [K]

Runs a few searches on a synthetic L2-normalised corpus, then reads the per-block (query)
s_memrealtime stamps of the last finish launch: entry, after the merge of the partition lists,
after the candidates' norm gather, after the fp64 dot products, after the pair sort, end."""
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
Q = np.random.default_rng(1).standard_normal((B, D)).astype(np.float32)
for _ in range(3):
    ix.search(Q, K)
fn = _lib.lib().hcr_debug_finish_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
n = 4096 * 8
buf = (ctypes.c_ulonglong * n)()
assert fn(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8)[:B].astype(np.float64) / 100.0   # us
live = a[:, 0] > 0
a = a[live]
t0 = a[:, 0].min()
names = ["merge (lists -> sorted k')", "norm64 gather", "fp64 dots", "pair sort", "certificate + outputs"]
print(f"{live.sum()} blocks; entry skew median {np.median(a[:, 0] - t0):.1f} us, max {(a[:, 0] - t0).max():.1f} us")
for i, nm in enumerate(names):
    d = a[:, i + 1] - a[:, i]
    print(f"  {nm:28s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f}")
print(f"  block total median {np.median(a[:, 5] - a[:, 0]):.2f} us; last block ends at {(a[:, 5] - t0).max():.2f} us")
