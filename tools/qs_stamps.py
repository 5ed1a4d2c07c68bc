"""Where the QS score kernel's time goes, from the stamps build (Makefile target `stamps`).

    HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py ROWS DIM BATCH [QS_FORM [STRIDE]]

Runs a few searches, then reads the per-wave s_memtime sums of the last launch: stage wait
(vmcnt + barrier), stage issue (DMA + fragment reads + MFMAs), tile epilogue; prints them per
tile and as shares (the stamps' own fences change the timing: read shares, not lengths)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hc-rag_amd"))
import hcrag_amd  # noqa: E402
from hcrag_amd import _lib  # noqa: E402

N, D, B = (int(x) for x in sys.argv[1:4])
QSF = int(sys.argv[4]) if len(sys.argv) > 4 else 0
STRIDE = int(sys.argv[5]) if len(sys.argv) > 5 else 0
dev = torch.device("cuda:0")
torch.manual_seed(0)
ix = hcrag_amd.VectorIndex(D, "f16", device=0)
chunk = 1 << 20
for a in range(0, N, chunk):
    b = min(N, a + chunk)
    xs = torch.randn(b - a, D, device=dev, dtype=torch.float32)
    torch.cuda.synchronize()
    ix.add_device(xs.data_ptr(), b - a, _lib.HCR_F32, normalize=True)
torch.cuda.synchronize()
ix.set_option(ix.OPT_QS_FORM, QSF)
ix.set_option(ix.OPT_SAMPLE_STRIDE, STRIDE)
Q = np.random.default_rng(1).standard_normal((B, D)).astype(np.float32)
for _ in range(20):        # back to back: the clock settles under load
    ix.search(Q, 10)
print("score_kernel", ix.last_stats()["score_kernel"])
lib = _lib.lib()
fn = lib.hcr_debug_qs_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
n = 4096 * 8 * 8
buf = (ctypes.c_ulonglong * n)()
assert fn(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8, 8).astype(np.float64)
live = a[:, :, 3] > 0
w, c, e, t = (a[:, :, i][live] for i in range(4))
tiles = t.sum()
print(f"rows={N} dim={D} batch={B} waves={live.sum()} tiles/wave={t.mean():.1f}")
print(f"per tile (s_memtime ticks, 100 MHz): wait {w.sum() / tiles:.1f}  issue {c.sum() / tiles:.1f}  "
      f"epilogue {e.sum() / tiles:.1f}")
f, sn = a[:, :, 4][live], a[:, :, 5][live]
print(f"epilogue split: max/test part {f.sum() / tiles:.1f} per tile; slow path entered on "
      f"{sn.sum() / tiles:.3f} of the tiles, {(e.sum() - f.sum()) / max(sn.sum(), 1):.1f} ticks per entry")
tot = w.sum() + c.sum() + e.sum()
print(f"shares: wait {w.sum() / tot:.3f}  issue {c.sum() / tot:.3f}  epilogue {e.sum() / tot:.3f}")
clk, rt = a[:, :, 6][live], a[:, :, 7][live]
print(f"in-kernel clock over the tile loop: {np.median(clk / np.maximum(rt, 1)) * 100:.0f} MHz (median over waves)")
for wv in range(8):
    m = a[:, wv, 3] > 0
    if not m.any():
        continue
    print(f"  wave {wv}: wait {a[m, wv, 0].sum() / a[m, wv, 3].sum():.1f} issue {a[m, wv, 1].sum() / a[m, wv, 3].sum():.1f} "
          f"epi {a[m, wv, 2].sum() / a[m, wv, 3].sum():.1f}")
