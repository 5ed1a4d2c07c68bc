"""Synthetic BERT weights (no checkpoints can be downloaded here): deterministic random-init
state dicts under HF ``BertModel`` names, for the benchmarks and the configs[0] parity fixture.

numpy PCG64 streams (stable across numpy versions and machines), so the same seed gives the
same model in this container and on the GPU box.  Shapes of the reference's models:
all-MiniLM-L6-v2 (experiments/embedding_generator.py:21, graph_builder.py:146-149 via
config.EMBEDDING_MODEL), bge-base-en and bge-large-en (the 768-d / 1024-d corpora of
BASELINE.json configs[2]-[4]).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

SHAPES = {
    "minilm": dict(vocab_size=30522, hidden=384, layers=6, heads=12, intermediate=1536,
                   max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=0, normalize=1),
    "bge-base": dict(vocab_size=30522, hidden=768, layers=12, heads=12, intermediate=3072,
                     max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=1, normalize=1),
    "bge-large": dict(vocab_size=30522, hidden=1024, layers=24, heads=16, intermediate=4096,
                      max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=1, normalize=1),
}


def bert_state(cfg: dict, seed: int = 0, perturb_ln: bool = False) -> Dict[str, np.ndarray]:
    """HF BertModel state dict (fp32) for an ``hcr_bert_config``-style dict: N(0, 0.02)
    matrices and biases (HF's initializer_range), LayerNorm gamma 1 / beta 0, or -- with
    ``perturb_ln`` -- gamma 1 + N(0, 0.1) and beta N(0, 0.02) so the affine terms matter."""
    rng = np.random.default_rng(seed)
    H, F = cfg["hidden"], cfg["intermediate"]

    def w(*shape):
        return (0.02 * rng.standard_normal(shape)).astype(np.float32)

    def ln(prefix, sd):
        if perturb_ln:
            sd[prefix + ".weight"] = (1.0 + 0.1 * rng.standard_normal(H)).astype(np.float32)
            sd[prefix + ".bias"] = w(H)
        else:
            sd[prefix + ".weight"] = np.ones(H, np.float32)
            sd[prefix + ".bias"] = np.zeros(H, np.float32)

    sd = {"embeddings.word_embeddings.weight": w(cfg["vocab_size"], H),
          "embeddings.position_embeddings.weight": w(cfg["max_position"], H),
          "embeddings.token_type_embeddings.weight": w(cfg["type_vocab"], H)}
    ln("embeddings.LayerNorm", sd)
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."
        for nm in ("attention.self.query", "attention.self.key", "attention.self.value",
                   "attention.output.dense"):
            sd[p + nm + ".weight"], sd[p + nm + ".bias"] = w(H, H), w(H)
        sd[p + "intermediate.dense.weight"], sd[p + "intermediate.dense.bias"] = w(F, H), w(F)
        sd[p + "output.dense.weight"], sd[p + "output.dense.bias"] = w(H, F), w(H)
        ln(p + "attention.output.LayerNorm", sd)
        ln(p + "output.LayerNorm", sd)
    return sd


def hf_config(cfg: dict) -> dict:
    """The matching transformers ``BertConfig`` kwargs (erf GELU, no dropout)."""
    return dict(vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden"],
                num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
                intermediate_size=cfg["intermediate"], max_position_embeddings=cfg["max_position"],
                type_vocab_size=cfg["type_vocab"], layer_norm_eps=cfg["layer_norm_eps"],
                hidden_act="gelu", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)


__all__ = ["SHAPES", "bert_state", "hf_config"]
