"""hcrag_amd — MI355X-native embedding + vector-retrieval core for HC-RAG's hot path.

Host package over libhcrag_hip.so (HIP, gfx950).  See DESIGN.md for the architecture and
INTEGRATION.md for the drop-in points in the reference (graph_builder.py:146-161,
query_interface.py:136-139,172-204, experiments/main.py:831-905,
experiments/isRelevant.py:197-210).
"""
from ._lib import (HCR_BF16, HCR_F16, HCR_F32, HCR_SCORE_COSINE, HCR_SCORE_UNIT, HcrError,
                   device_count, lib)
from .index import MultiDeviceIndex, VectorIndex, merge_topk_device
from .retrieval import EmbeddingSearch, batch_semantic_similarity
from .tokenizer import WordPieceTokenizer
from .encoder import MINILM_L6_V2, BertEncoder, MI355XEmbedding, SentenceEmbedder, config_from_hf
from .ingest import BatchedEmbeddingGenerator, EmbeddingStore
from . import relevance
from . import graph_relevance

__version__ = "0.3.0"

__all__ = ["VectorIndex", "MultiDeviceIndex", "merge_topk_device", "EmbeddingSearch", "batch_semantic_similarity",
           "WordPieceTokenizer", "BertEncoder", "SentenceEmbedder", "MI355XEmbedding", "config_from_hf",
           "MINILM_L6_V2", "device_count", "lib", "HcrError", "HCR_F16", "HCR_BF16", "HCR_F32",
           "HCR_SCORE_COSINE", "HCR_SCORE_UNIT", "BatchedEmbeddingGenerator", "EmbeddingStore",
           "relevance", "graph_relevance"]
