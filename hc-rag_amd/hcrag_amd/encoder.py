"""Sentence-embedding forward on MI355X.

``BertEncoder`` binds the C-ABI encoder of libhcrag_hip.so (``hcr_encoder_*``,
include/hcrag.h); ``SentenceEmbedder`` mirrors the call surface the reference uses:

* ``SentenceTransformer('all-MiniLM-L6-v2').encode(texts)`` —
  experiments/embedding_generator.py:21,124,197,337 and experiments/main.py:807,869:
  tokenise (WordPiece, truncation to ``max_seq_length``), BertModel forward, mean pooling over
  the attention mask, L2 normalise; length-sorted batches, results in input order.
* ``HuggingFaceEmbedding(model_name=...)`` — graph_builder.py:146-149,
  query_interface.py:136-137: ``get_text_embedding``, ``get_text_embedding_batch``,
  ``get_query_embedding`` (llama-index BaseEmbedding surface).

Weights come from a local directory (``config.json`` + ``model.safetensors`` or
``pytorch_model.bin`` + ``vocab.txt``: the layout of a sentence-transformers / HF snapshot) or
from an in-memory state dict; there is no network here.  No CPU fallback: without the HIP
library these classes raise.
"""
from __future__ import annotations

import ctypes
import json
import os
from ctypes import c_void_p
from typing import Dict, List, Mapping, Optional, Sequence

import numpy as np

from ._lib import BertConfig, check, lib
from .tokenizer import WordPieceTokenizer

HCR_F16, HCR_BF16, HCR_F32 = 0, 1, 2
# "f32": reference precision (split-f16 MFMA GEMMs, fp32 attention / LayerNorm; the reference
# encodes in fp32 torch, experiments/embedding_generator.py:124) -- the default.
# "f16" / "bf16": fast modes (16-bit MFMA operands, fp32 accumulation).
_DTYPES = {"f32": HCR_F32, "fp32": HCR_F32, "float32": HCR_F32,
           "f16": HCR_F16, "fp16": HCR_F16, "float16": HCR_F16,
           "bf16": HCR_BF16, "bfloat16": HCR_BF16}

# all-MiniLM-L6-v2 (the reference's model, experiments/embedding_generator.py:21)
MINILM_L6_V2 = dict(vocab_size=30522, hidden=384, layers=6, heads=12, intermediate=1536,
                    max_position=512, type_vocab=2, layer_norm_eps=1e-12, pooling=0, normalize=1)


def config_from_hf(cfg: Mapping, pooling: str = "mean", normalize: bool = True) -> dict:
    """HF ``BertConfig`` dict (config.json) -> ``hcr_bert_config`` fields."""
    act = cfg.get("hidden_act", "gelu")
    if act not in ("gelu", "gelu_python"):
        raise ValueError(f"hidden_act {act!r} not supported (BERT 'gelu' = erf GELU)")
    pet = cfg.get("position_embedding_type", "absolute")
    if pet != "absolute":
        raise ValueError(f"position_embedding_type {pet!r} not supported")
    return dict(vocab_size=int(cfg["vocab_size"]), hidden=int(cfg["hidden_size"]),
                layers=int(cfg["num_hidden_layers"]), heads=int(cfg["num_attention_heads"]),
                intermediate=int(cfg["intermediate_size"]),
                max_position=int(cfg.get("max_position_embeddings", 512)),
                type_vocab=int(cfg.get("type_vocab_size", 2)),
                layer_norm_eps=float(cfg.get("layer_norm_eps", 1e-12)),
                pooling={"mean": 0, "cls": 1}[pooling], normalize=int(bool(normalize)))


class BertEncoder:
    """BertModel + Pooling + Normalize on one GPU.

    ``state_dict``: mapping name -> array-like (numpy or torch tensor), HF BertModel names
    with any prefix (``bert.``, ``0.auto_model.``).
    """

    def __init__(self, config: Mapping, state_dict: Mapping, dtype: str = "f32", device: int = 0):
        if dtype not in _DTYPES:
            raise ValueError(f"unknown encoder dtype {dtype!r} (f32 | f16 | bf16)")
        self.config = dict(config)
        self.hidden = int(self.config["hidden"])
        self.max_position = int(self.config["max_position"])
        self.vocab_size = int(self.config["vocab_size"])
        self.device = int(device)
        self.dtype = dtype
        c = BertConfig(**{k: self.config[k] for k, _ in BertConfig._fields_})
        self._h = c_void_p()
        check(lib().hcr_encoder_create(self.device, ctypes.byref(c), _DTYPES[dtype],
                                       ctypes.byref(self._h)))
        for name, t in state_dict.items():
            a = _as_f32(t)
            check(lib().hcr_encoder_set_weight(self._h, name.encode(), a.ctypes.data, a.size))
        check(lib().hcr_encoder_finalize(self._h))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().hcr_encoder_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode_ids(self, ids: np.ndarray, mask: np.ndarray) -> np.ndarray:
        """[n, S] int32 ids / mask (host) -> [n, hidden] fp32 (host)."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        mask = np.ascontiguousarray(mask, dtype=np.int32)
        if ids.shape != mask.shape or ids.ndim != 2:
            raise ValueError("ids and mask must both be [n, S]")
        n, S = ids.shape
        out = np.zeros((n, self.hidden), dtype=np.float32)
        if n:
            check(lib().hcr_encode(self._h, ids.ctypes.data, mask.ctypes.data, n, S,
                                   out.ctypes.data))
        return out

    def encode_device(self, ids, mask, out, stream: Optional[int] = None) -> None:
        """Device tensors (torch, int32 [n, S] / fp32 [n, hidden]) on ``stream`` (a raw
        hipStream_t handle, default: torch's current stream).  The call reads the packed token
        count back once (hcr_encode_device), then enqueues the layers asynchronously."""
        n, S = ids.shape
        if tuple(mask.shape) != (n, S) or tuple(out.shape) != (n, self.hidden):
            raise ValueError("shape mismatch")
        for t, dt in ((ids, "int32"), (mask, "int32"), (out, "float32")):
            if str(t.dtype).split(".")[-1] != dt or not t.is_contiguous() or not t.is_cuda:
                raise ValueError(f"expected contiguous {dt} device tensors")
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(out.device).cuda_stream
        check(lib().hcr_encode_device(self._h, ids.data_ptr(), mask.data_ptr(), n, S,
                                      out.data_ptr(), stream))


def _as_f32(t) -> np.ndarray:
    if hasattr(t, "detach"):
        t = t.detach().to("cpu").float().numpy()
    return np.ascontiguousarray(np.asarray(t, dtype=np.float32))


def _load_state_dict(path: str) -> Dict[str, np.ndarray]:
    st = os.path.join(path, "model.safetensors")
    if os.path.exists(st):
        from safetensors.numpy import load_file
        return load_file(st)
    pt = os.path.join(path, "pytorch_model.bin")
    if os.path.exists(pt):
        import torch
        return torch.load(pt, map_location="cpu", weights_only=True)
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path}")


class SentenceEmbedder:
    """``SentenceTransformer.encode`` / ``HuggingFaceEmbedding`` drop-in on the HIP path."""

    def __init__(self, tokenizer: WordPieceTokenizer, encoder: BertEncoder,
                 max_seq_length: int = 256, batch_size: int = 32):
        self.tokenizer = tokenizer
        self.encoder = encoder
        self.max_seq_length = min(int(max_seq_length), encoder.max_position)
        self.batch_size = int(batch_size)

    @classmethod
    def from_pretrained(cls, path: str, dtype: str = "f32", device: int = 0,
                        max_seq_length: Optional[int] = None, batch_size: int = 32,
                        pooling: str = "mean", normalize: bool = True) -> "SentenceEmbedder":
        """Local sentence-transformers / HF snapshot directory (no download)."""
        with open(os.path.join(path, "config.json")) as f:
            hf = json.load(f)
        # sentence-transformers keeps max_seq_length / pooling beside the model
        stc = os.path.join(path, "sentence_bert_config.json")
        if max_seq_length is None and os.path.exists(stc):
            with open(stc) as f:
                max_seq_length = json.load(f).get("max_seq_length")
        pc = os.path.join(path, "1_Pooling", "config.json")
        if os.path.exists(pc):
            with open(pc) as f:
                pj = json.load(f)
            pooling = "cls" if pj.get("pooling_mode_cls_token") else "mean"
        lower = True
        tc = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(tc):
            with open(tc) as f:
                lower = bool(json.load(f).get("do_lower_case", True))
        tok = WordPieceTokenizer(os.path.join(path, "vocab.txt"), lowercase=lower)
        enc = BertEncoder(config_from_hf(hf, pooling, normalize), _load_state_dict(path),
                          dtype=dtype, device=device)
        return cls(tok, enc, max_seq_length or 512, batch_size)

    # --- SentenceTransformer.encode surface -------------------------------------------
    def encode(self, sentences, batch_size: Optional[int] = None, convert_to_numpy: bool = True,
               show_progress_bar: bool = False, normalize_embeddings: bool = False, **_):
        single = isinstance(sentences, str)
        texts = [sentences] if single else list(sentences)
        bs = int(batch_size or self.batch_size)
        out = np.zeros((len(texts), self.encoder.hidden), dtype=np.float32)
        if texts:
            ids, mask, lens = self.tokenizer.encode(texts, self.max_seq_length, pad_to_longest=False)
            order = np.argsort(-lens, kind="stable")          # length-sorted batches
            for s in range(0, len(texts), bs):
                sel = order[s:s + bs]
                L = int(lens[sel].max())
                out[sel] = self.encoder.encode_ids(ids[sel, :L], mask[sel, :L])
        if normalize_embeddings:
            out /= np.maximum(np.linalg.norm(out, axis=1, keepdims=True), 1e-12)
        if not convert_to_numpy:
            import torch
            out = torch.from_numpy(out)
        return out[0] if single else out

    # --- llama-index BaseEmbedding surface (HuggingFaceEmbedding) ----------------------
    def get_text_embedding(self, text: str) -> List[float]:
        return self.encode([text])[0].tolist()

    def get_query_embedding(self, query: str) -> List[float]:
        return self.get_text_embedding(query)

    def get_text_embedding_batch(self, texts: Sequence[str], **_) -> List[List[float]]:
        return self.encode(list(texts)).tolist()

    def get_agg_embedding_from_queries(self, queries: Sequence[str]) -> List[float]:
        return np.mean(self.encode(list(queries)), axis=0).tolist()


class MI355XEmbedding(SentenceEmbedder):
    """``HuggingFaceEmbedding`` field/method surface (SURVEY.md §8(a) a9;
    graph_builder.py:146-149, query_interface.py:136-137): ``model_name``,
    ``embed_batch_size`` (llama-index default 10), embeddings always L2-normalised
    (``normalize_embeddings=True``), optional query / text instruction prefixes (bge-*-en)."""

    def __init__(self, model_name: str, embed_batch_size: int = 10, dtype: str = "f32",
                 device: int = 0, max_length: Optional[int] = None,
                 query_instruction: Optional[str] = None, text_instruction: Optional[str] = None,
                 pooling: str = "mean"):
        base = SentenceEmbedder.from_pretrained(model_name, dtype=dtype, device=device,
                                                max_seq_length=max_length,
                                                batch_size=embed_batch_size, pooling=pooling)
        super().__init__(base.tokenizer, base.encoder, base.max_seq_length, embed_batch_size)
        self.model_name = model_name
        self.embed_batch_size = int(embed_batch_size)
        self.query_instruction = query_instruction
        self.text_instruction = text_instruction

    def _fmt(self, text: str, instr: Optional[str]) -> str:
        return f"{instr} {text}".strip() if instr else text

    def _get_query_embedding(self, query: str) -> List[float]:
        return self.encode([self._fmt(query, self.query_instruction)],
                           normalize_embeddings=True)[0].tolist()

    def _get_text_embedding(self, text: str) -> List[float]:
        return self.encode([self._fmt(text, self.text_instruction)],
                           normalize_embeddings=True)[0].tolist()

    def _get_text_embeddings(self, texts: List[str]) -> List[List[float]]:
        return self.encode([self._fmt(t, self.text_instruction) for t in texts],
                           normalize_embeddings=True).tolist()

    get_query_embedding = _get_query_embedding
    get_text_embedding = _get_text_embedding

    def get_text_embedding_batch(self, texts: Sequence[str], show_progress: bool = False,
                                 **_) -> List[List[float]]:
        return self._get_text_embeddings(list(texts))

    def get_agg_embedding_from_queries(self, queries: Sequence[str], agg_fn=None) -> List[float]:
        """llama-index BaseEmbedding semantics: each query through get_query_embedding (query
        instruction applied), then the mean (or ``agg_fn``)."""
        embs = [self._get_query_embedding(q) for q in queries]
        if agg_fn is not None:
            return agg_fn(embs)
        return np.mean(np.asarray(embs), axis=0).tolist()
