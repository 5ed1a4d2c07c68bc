"""Diagnostic: norm deviation of stored normalised f16 rows (bench corpus) vs the UNIT bound."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "hc-rag_amd"))
import numpy as np, torch
import hcrag_amd as hc
import bench
dev = torch.device("cuda:0")
ix = hc.VectorIndex(768, dtype="f16", capacity=1 << 21)
bench.make_shard(ix, hc, 0, 1 << 21, 768, "f16", dev)
dmax, worst = 0.0, -1
for r0 in range(0, len(ix), 1 << 18):
    R = ix.get_rows(r0, min(1 << 18, len(ix) - r0)).astype(np.float64)
    nr = np.linalg.norm(R, axis=1)
    d = np.abs(nr - 1)
    if d.max() > dmax:
        dmax, worst = float(d.max()), r0 + int(d.argmax())
print("max |norm-1| over stored rows:", dmax, "row", worst, flush=True)
R = ix.get_rows(worst, 1)[0]
print("worst row: min|x| nonzero", np.abs(R[R != 0]).min(), "max|x|", np.abs(R).max(), "zeros", int((R == 0).sum()))
g = torch.Generator(device=dev); c = worst >> 20; g.manual_seed(1000 + c)
x = torch.randn((1 << 20, 768), generator=g, device=dev, dtype=torch.float16)[worst - (c << 20)].double().cpu().numpy()
print("input row norm", np.linalg.norm(x), "max|x|", np.abs(x).max(), "finite", np.isfinite(x).all())
xn = x / np.linalg.norm(x)
print("stored vs round(normalised input): max diff", np.abs(R - xn.astype(np.float16).astype(np.float32)).max(),
      "ratio stored/xn median", np.median(R / xn))
for r in (worst - 1, worst + 1, (c << 20), (c << 20) + 5):
    Rr = ix.get_rows(r, 1)[0].astype(np.float64); print("row", r, "norm", np.linalg.norm(Rr))
q = np.random.default_rng(0).standard_normal((1024, 768)).astype(np.float32)
os.environ["HCRAG_DEBUG_UNIT"] = "1"
ix.search(q, 32)
