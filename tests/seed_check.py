"""Parity of the score kernels under the process-wide test hooks (read once per process, hence a
subprocess of tests/test_search_gpu.py): the forced sampling pre-pass and its estimated /
aggressive seeds: UNIT path (L2-normalised corpus), inverse-norm path (raw corpus), row mask
and k' widening, against the oracle."""
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
    dt = os.environ.get("HCRAG_TEST_DTYPE", "f16")      # storage dtype of the indexes
    rng = np.random.default_rng(5)
    N, D, B, k = 40000, 256, 512, 32
    E = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((B, D)).astype(np.float32)
    Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.1 * rng.standard_normal((B // 2, D)).astype(np.float32)
    for normalize, want_unit in ((True, 1), (False, 0)):
        with hc.VectorIndex(D, dt) as ix:
            ix.add(E, normalize=normalize)
            R = ix.get_rows()
            s, i = ix.search(Q, k)
            es, ei = O.cosine_topk(Q, R, k)
            check(s, i, es, ei)
            st = ix.last_stats()
            assert st["unit_kernel"] == want_unit, st
            assert st["uncertified_queries"] == 0, st
            mask = rng.random(N) < 0.3
            ix.set_rowmask(mask)
            s, i = ix.search(Q, k)
            es, ei = O.cosine_topk(Q, R, k, rowmask=mask)
            check(s, i, es, ei)
    # duplicate cluster: forces widening (k' x 4, CAP 1024 instantiation)
    Ed = rng.standard_normal((N, D)).astype(np.float16)
    dup = rng.choice(N, 300, replace=False)
    Ed[dup] = Ed[dup[0]]
    Qd = rng.standard_normal((B, D)).astype(np.float32)
    Qd[:8] = Ed[dup[0]].astype(np.float32)
    with hc.VectorIndex(D, dt) as ix:
        ix.add(Ed, normalize=False)
        s, i = ix.search(Qd, k)
        es, ei = O.cosine_topk(Qd, ix.get_rows().astype(np.float64), k)
        check(s, i, es, ei)
        assert ix.last_stats()["widened_queries"] > 0
    print("parity ok")


if __name__ == "__main__":
    main()
