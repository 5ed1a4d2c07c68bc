import sys, os, numpy as np
sys.path[:0] = ['.', 'hc-rag_amd']
import hcrag_amd as hc
from oracle import cosine_topk as O
rng = np.random.default_rng(77)
N, D, B, k = 3000, 192, 2, 2100
E = rng.standard_normal((N, D)).astype(np.float32)
Q = rng.standard_normal((B, D)).astype(np.float32)
with hc.VectorIndex(D, "f16") as ix:
    ix.add(E, normalize=False)
    R = ix.get_rows().astype(np.float64)
    s, i = ix.search(Q, k)
    print("stats", ix.last_stats())
    es, ei = O.cosine_topk(Q, R, k)
    print("got s", s[0, :5], s[0, -3:], "i", i[0, :5], i[0, -3:])
    print("exp s", es[0, :5], "i", ei[0, :5])
    print("ids equal", np.array_equal(i, ei), "n zero ids", int((i == 0).sum()), "n -1", int((i == -1).sum()))
