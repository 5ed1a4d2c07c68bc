"""Diagnostic: repeat the MiniLM-shape encode in one process, report min cosine vs the fp32
torch reference per repetition and whether outputs are bitwise identical across repetitions."""
import os, sys, subprocess
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "hc-rag_amd"))
import test_encoder_gpu as T


def run(reps, fresh):
    conf, m = T._hf_model(T.MINILM, 2)
    rng = np.random.default_rng(1)
    ids, mask = T._batch(rng, 24, 128, T.MINILM["vocab_size"])
    ref = T._ref_embed(m, ids, mask)
    out = []
    enc = T._encoder(conf, m, "f16")
    first = None
    for r in range(reps):
        if fresh:
            enc = T._encoder(conf, m, "f16")
        o = enc.encode_ids(ids, mask)
        cos = np.sum(o * ref, 1) / (np.linalg.norm(o, axis=1) * np.linalg.norm(ref, axis=1))
        if first is None:
            first = o
        bad = np.nonzero(cos < 0.9999)[0]
        out.append(f"{cos.min():.5f}{'=' if np.array_equal(o, first) else '!'}{list(bad)[:6] if len(bad) else ''}")
    print(os.environ.get("TAG", "main"), "fresh" if fresh else "reuse", " ".join(out), flush=True)


if __name__ == "__main__":
    run(int(sys.argv[1]), sys.argv[2] == "fresh")
    if len(sys.argv) > 3:
        for tag, env in [("child", {}), ("child_v1", {"HCRAG_GEMM_V1": "1"}),
                         ("child_scal_att", {"HCRAG_SCALAR_ATTENTION": "1"}),
                         ("child_ln_scalar", {"HCRAG_LN_SCALAR": "1"})]:
            for fresh in ("reuse", "fresh"):
                subprocess.run([sys.executable, __file__, sys.argv[1], fresh],
                               env=dict(os.environ, TAG=tag, **env), timeout=300, check=True)
