"""Batched ingestion + on-disk store (experiments/embedding_generator.py).

CPU: text construction worked by hand from embedding_generator.py:28-104 / :152-215 on small
synthetic tables (parity with the reference's own outputs unpinned: the module needs
sentence_transformers, absent here), metadata (:130-145), store round trip with no pickle,
and one encode call per table.  GPU: the same through the MI355X encoder into a VectorIndex.
"""
import json

import numpy as np
import pandas as pd
import pytest

from hcrag_amd.ingest import (BatchedEmbeddingGenerator, EmbeddingStore, analyze_data_patterns,
                              flatten_json_to_text, smart_text)


class CountingEmbedder:
    def __init__(self, dim=8):
        self.dim, self.calls = dim, []

    def encode(self, texts):
        self.calls.append(len(texts))
        out = np.zeros((len(texts), self.dim), np.float32)
        for i, t in enumerate(texts):
            out[i, hash(t) % self.dim] = 1.0
        return out


def _table(tmp_path):
    df = pd.DataFrame({
        "ProductID": [1, 2, 3, 4],
        "Name": ["Mountain-100 Silver, 38 frame", "Road-150 Red, 62 frame",
                 "Touring-1000 Blue, 46 frame", "HL Road Frame - Black, 58"],
        "Color": ["Silver", "Red", "Blue", "Black"],
        "Size": ["38", "62", "46", "58"],
        "Class": ["H", "H", None, "L"],
    })
    p = tmp_path / "Product.csv"
    df.to_csv(p, sep=";", index=False)
    return df, p


def test_field_importance_and_text(tmp_path):
    df, _ = _table(tmp_path)
    a = analyze_data_patterns(df)
    # unique ratio 1.0 and avg length > 20 -> high; unique > 0.8 -> medium; else low (:44-52)
    assert a["Name"]["importance"] == "high"
    assert a["ProductID"]["importance"] == "medium" and a["Color"]["importance"] == "medium"
    assert a["Class"]["importance"] == "low"                 # 2 unique of 3, short
    t = smart_text(df.iloc[2], a, "Product")
    # "Table: ..", high fields, first 3 medium (ProductID, Color, Size), low fields (NaN skipped)
    assert t == ("Table: Product. Name: Touring-1000 Blue, 46 frame. ProductID: 3. "
                 "Color: Blue. Size: 46")
    assert smart_text(df.iloc[0], a, "Product").endswith("Size: 38. Class: H")


def test_json_flatten():
    obj = {"a": 1, "b": {"c": [1, {"d": "x"}]}, "e": []}
    assert flatten_json_to_text(obj) == ["a: 1", "b.c[0]: 1", "b.c[1].d: x"]
    assert flatten_json_to_text([1, [2]]) == ["item_0: 1", "item_1[0]: 2"]
    assert flatten_json_to_text(5) == ["5"]


def test_generator_batches_and_store_round_trip(tmp_path):
    df, p = _table(tmp_path)
    (tmp_path / "doc.json").write_text(json.dumps({"title": "Spec", "parts": ["frame", "fork"]}))
    emb = CountingEmbedder()
    g = BatchedEmbeddingGenerator(emb)
    g.process_all_data(tmp_path)
    assert emb.calls == [4, 1]                   # one encode call per table / document
    md = g.embeddings_data["metadata"]
    assert md[0] == {"id": "Product_0", "type": "database_table", "table_name": "Product",
                     "row_index": 0, "source_file": str(p), "entity_id": 1}
    assert md[4]["type"] == "json_table" and md[4]["json_keys"] == ["title", "parts"]
    assert g.embeddings_data["texts"][4].startswith("Document: doc. Contains structured information. title: Spec")
    st = g.get_statistics()
    assert st["total_embeddings"] == 5 and st["content_types"] == {"database_table": 4, "json_table": 1}
    out = g.save_embeddings(str(tmp_path / "store"))
    data = EmbeddingStore.load(out)
    assert data["embeddings"].dtype == np.float16 and data["embeddings"].shape == (5, 8)
    np.testing.assert_array_equal(np.asarray(data["embeddings"], np.float32), g.embeddings_matrix())
    assert data["texts"] == g.embeddings_data["texts"] and data["metadata"] == md
    assert data["generation_info"]["total_entries"] == 5
    g2 = BatchedEmbeddingGenerator(emb)
    g2.load_embeddings(out)
    assert g2.get_statistics() == st


def test_store_rejects_mismatched_lengths(tmp_path):
    with pytest.raises(ValueError):
        EmbeddingStore.save(str(tmp_path / "s"), np.zeros((2, 4)), ["a"], [{}, {}])


@pytest.mark.gpu
def test_gpu_ingest_into_index(tmp_path):
    """CSV rows -> one batched MI355X encode -> store -> VectorIndex: every row finds itself."""
    import hcrag_amd as hc
    from hcrag_amd.encoder import BertEncoder, SentenceEmbedder, WordPieceTokenizer
    from test_encoder_gpu import TINY, _hf_model
    from hcrag_amd import config_from_hf
    conf, m = _hf_model(TINY, 4)
    chars = sorted(set("abcdefghijklmnopqrstuvwxyz0123456789-:,.;"))
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "table", "name", "product", "color"] + \
        chars + ["##" + c for c in chars]
    vocab = vocab[: TINY["vocab_size"]]
    tok = WordPieceTokenizer(vocab_tokens=vocab)
    enc = BertEncoder(config_from_hf(conf.to_dict(), "mean", True), m.state_dict(), dtype="f16")
    emb = SentenceEmbedder(tok, enc, max_seq_length=64, batch_size=16)
    df, p = _table(tmp_path)
    g = BatchedEmbeddingGenerator(emb)
    g.process_csv_table(p)
    data = EmbeddingStore.load(g.save_embeddings(str(tmp_path / "store")))
    E = np.asarray(data["embeddings"], np.float32)
    ref = emb.encode(data["texts"])
    np.testing.assert_allclose(E, ref, rtol=0, atol=2e-3)      # fp16 storage rounding
    with hc.VectorIndex(E.shape[1], "f16") as ix:
        ix.add(E, normalize=False)
        _, ids = ix.search(ref.astype(np.float32), 1)
        assert list(ids[:, 0]) == list(range(len(E)))
