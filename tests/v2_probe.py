"""Tiny standalone probe of the 224x256 score kernel (run in its own process on the GPU box)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]
import numpy as np
import hcrag_amd as hc
from oracle import cosine_topk as O
rng = np.random.default_rng(0)
for (N, D, B) in [(1000, 128, 400), (50000, 768, 1024)]:
    E = rng.standard_normal((N, D)).astype(np.float16)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    with hc.VectorIndex(D, "f16") as ix:
        ix.add(E, normalize=False)
        s, i = ix.search(Q, 16)
        es, ei = O.cosine_topk(Q, E.astype(np.float64), 16)
        print(N, D, B, "ids equal:", bool(np.array_equal(i, ei)), "max ds:", float(np.max(np.abs(s - es))), ix.last_stats(), flush=True)
