"""The fused last-merge-level + rescore kernel (finish_kernel, topk_kernels.h) against the separate
merge_lists_kernel + rescore_kernel launches (HCRAG_NO_FINISH, run in a child process): results
must be bit-identical (same keys, same fp64 summation order), and both equal to the fp64 oracle.
Shapes: configs[1]'s QS batch (P = 256 lists of k' = 64: one 16384-key level), a QW batch with
a multi-level merge (k' = 512: G = 32 lists per level), and QW1 at D = 1024 (192-query blocks);
all <= 512 queries (kFinishMaxQueries: larger batches take the separate
launches).  Reference: experiments/main.py:841-844."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import cosine_topk as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(384, 150_000 + 77, 256, 10, -1), (768, 60_000 + 5, 512, 200, -1), (1024, 40_000 + 1, 300, 32, -1)]

_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import hcrag_amd as hc
from oracle import cosine_topk as O
D, N, B, k, opt = (int(x) for x in sys.argv[3:8])
rng = np.random.default_rng(D + B + k)
E = rng.standard_normal((N, D)).astype(np.float32)
Q = rng.standard_normal((B, D)).astype(np.float32)
Q[: B // 2] = E[rng.integers(0, N, B // 2)] + 0.2 * rng.standard_normal((B // 2, D)).astype(np.float32)
with hc.VectorIndex(D, "f16") as ix:
    if opt >= 0:
        ix.set_option(ix.OPT_QW1, opt)
    ix.add(E, normalize=True)
    s, i = ix.search(Q, k)
    st = ix.last_stats()
    R = ix.get_rows()
sub = np.r_[0:8, B // 2:B // 2 + 8, B - 8:B]
es, ei = O.cosine_topk(Q[sub], R, k)
assert np.array_equal(i[sub], ei)
assert np.max(np.abs(s[sub] - es)) <= 1e-12
np.savez(sys.argv[8], s=s, i=i, kernel=st["score_kernel"], unc=st["uncertified_queries"])
"""


def _run(tmp_path, case, no_finish):
    env = dict(os.environ)
    if no_finish:
        env["HCRAG_NO_FINISH"] = "1"
    else:
        env.pop("HCRAG_NO_FINISH", None)
    out = str(tmp_path / f"r{int(no_finish)}.npz")
    subprocess.run([sys.executable, "-c", _CHILD, ROOT, os.path.join(ROOT, "hc-rag_amd"),
                    *(str(x) for x in case), out], env=env, check=True, timeout=240)
    return np.load(out)


@pytest.mark.parametrize("case", CASES, ids=["qs_c1", "qw_k200", "qw1_d1024"])
def test_finish_matches_separate_launches(tmp_path, case):
    a = _run(tmp_path, case, False)
    b = _run(tmp_path, case, True)
    np.testing.assert_array_equal(a["i"], b["i"])
    np.testing.assert_array_equal(a["s"], b["s"])
    assert int(a["kernel"]) == int(b["kernel"])
