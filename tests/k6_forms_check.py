"""Parity of the exact fallback's MFMA-prefiltered admission scan in its three forms (the
process-wide hooks are read once per process, hence a subprocess of tests/test_exact_gpu.py):
HCRAG_K6_INLINE (every admitted pair rescored by the scanning wave, K6m), the default two-launch
form (K6c compacts the coarse-admitted pairs, K6r rescores them), and the two-launch form with a
pair list too small for any group (HCRAG_K6_PCAP: every group overflows and the inline K6m
launched after K6r rescans it).  Deep k (radix select + bitonic sort), k in the fallback's LDS
select, exact duplicates, a row mask, against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]

import numpy as np  # noqa: E402

import hcrag_amd as hc  # noqa: E402
from oracle import cosine_topk as O  # noqa: E402


def check(s, i, es, ei):
    np.testing.assert_array_equal(i, ei)
    ok = ei >= 0
    np.testing.assert_allclose(s[ok], es[ok], rtol=0, atol=1e-12)


def main():
    rng = np.random.default_rng(606)
    N, D, B = 24000, 384, 70            # three query groups of 32, the last one partial
    E = rng.standard_normal((N, D)).astype(np.float32)
    E[300:700] = E[11]                  # 401 exact duplicates
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[0] = E[11]
    Q[1] = E[5] + 0.05 * rng.standard_normal(D).astype(np.float32)
    for dtype in ("f16", "bf16"):
        with hc.VectorIndex(D, dtype) as ix:
            ix.add(E, normalize=True)
            R = ix.get_rows().astype(np.float64)
            for k in (3000, 700):
                s, i = ix.search(Q, k)
                es, ei = O.cosine_topk(Q, R, k)
                check(s, i, es, ei)
                assert ix.last_stats()["fallback_queries"] == B
            # two whole groups (no partial group)
            s, i = ix.search(Q[:64], 3000)
            es, ei = O.cosine_topk(Q[:64], R, 3000)
            check(s, i, es, ei)
            mask = rng.random(N) < 0.6
            ix.set_rowmask(mask)
            s, i = ix.search(Q[:40], 2500)
            es, ei = O.cosine_topk(Q[:40], R, 2500, rowmask=mask)
            check(s, i, es, ei)
    print("parity ok", os.environ.get("HCRAG_K6_INLINE"), os.environ.get("HCRAG_K6_PCAP"))


if __name__ == "__main__":
    main()
