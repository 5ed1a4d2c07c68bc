"""Batched ingestion + on-disk store (experiments/embedding_generator.py).

CPU: text construction worked by hand from embedding_generator.py:28-104 / :152-215 on small
synthetic tables; the product's texts and metadata over the reference's own data/ (CSV tables and
IngestedDocuments JSON) against the independent restatement of tests/golden/make_ingest_f1.py
(the reference module itself needs sentence_transformers, absent here); chunk_text (:278-305);
store round trip with no pickle; one encode call per table / document.  GPU: the same data
through the reference-precision MI355X encoder against the fixture's CPU BertModel fp32
embeddings (<= 1e-4), then into a VectorIndex.
"""
import gzip
import json
import os
import shutil

import numpy as np
import pandas as pd
import pytest

from hcrag_amd.ingest import (BatchedEmbeddingGenerator, EmbeddingStore, analyze_data_patterns,
                              chunk_text, flatten_json_to_text, smart_text)

F1 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "f1")


def _f1_data(tmp_path):
    """The fixture's copy of the reference's data/ decompressed to tmp_path/data."""
    src = os.path.join(F1, "data")
    for dirpath, _, files in os.walk(src):
        for f in files:
            rel = os.path.relpath(os.path.join(dirpath, f), src)[:-3]       # strip .gz
            dst = tmp_path / "data" / rel
            dst.parent.mkdir(parents=True, exist_ok=True)
            with gzip.open(os.path.join(dirpath, f), "rb") as fi, open(dst, "wb") as fo:
                shutil.copyfileobj(fi, fo)
    with gzip.open(os.path.join(F1, "expected.jsonl.gz"), "rt", encoding="utf-8") as fh:
        expected = [json.loads(line) for line in fh]
    return tmp_path / "data", expected


def _relative_meta(metas, root):
    out = []
    for m in metas:
        m = dict(m)
        m["source_file"] = os.path.relpath(m["source_file"], root)
        out.append(m)
    return out


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
    (tmp_path / "IngestedDocuments").mkdir()
    (tmp_path / "IngestedDocuments" / "doc.json").write_text(
        json.dumps({"title": "Spec", "parts": ["frame", "fork"]}))
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


def test_reference_data_texts_match_restatement(tmp_path):
    """The reference's data/ (573 CSV rows of 7 tables + 6 IngestedDocuments JSON tables):
    texts and metadata identical, in order, to the independent restatement's fixture; one
    encode call per table / document."""
    root, expected = _f1_data(tmp_path)
    emb = CountingEmbedder()
    g = BatchedEmbeddingGenerator(emb)
    g.process_all_data(root)
    assert g.embeddings_data["texts"] == [e["text"] for e in expected]
    assert _relative_meta(g.embeddings_data["metadata"], tmp_path) == [e["metadata"] for e in expected]
    assert len(emb.calls) == 7 + 6 and sum(emb.calls) == len(expected)
    kinds = g.get_statistics()["content_types"]
    assert kinds == {"database_table": 573, "json_table": 6}
    parents = {e["metadata"]["parent_document"] for e in expected if e["metadata"]["type"] == "json_table"}
    assert "Mountain Bike Manual" in parents


def test_chunk_text_matches_restatement():
    """chunk_text (:278-305) on the fixture's long document: identical chunks; the PDF item
    texts / metadata of process_text_document (:307-364) identical too."""
    with open(os.path.join(F1, "chunks.json"), encoding="utf-8") as fh:
        fx = json.load(fh)
    doc = fx["document"]
    ch = chunk_text(doc, fx["chunk_size"], fx["overlap"])
    prefix = f"PDF Document: {fx['document_name']}. "
    assert [prefix + c for c in ch] == [it["text"] for it in fx["items"]]
    emb = CountingEmbedder()
    g = BatchedEmbeddingGenerator(emb)
    n = g.process_text_document(doc, fx["document_name"], fx["items"][0]["metadata"]["source_file"], 0)
    assert n == len(ch) and emb.calls == [n]                 # all chunks in one encode call
    assert g.embeddings_data["metadata"] == [it["metadata"] for it in fx["items"]]
    # edge cases of the reference loop
    assert chunk_text("short.", 800, 100) == ["short."]
    t = "a" * 1750                                           # no sentence end: hard cuts
    assert [len(c) for c in chunk_text(t, 800, 100)] == [800, 800, 350]
    t = ("x" * 30 + ". ") * 40                               # boundary search backs up to a '.'
    assert all(c.endswith(".") for c in chunk_text(t, 800, 100)[:-1])


def test_pdf_without_extractor_embeds_the_failure_text(tmp_path):
    """No pdfplumber / PyPDF2 here: process_pdf_document embeds the reference's own
    extraction-failure sentence (:270-272), as one chunk; an extractor callable is used when
    given."""
    pdf = tmp_path / "Manual.pdf"
    pdf.write_bytes(b"%PDF-1.4 not really")
    emb = CountingEmbedder()
    g = BatchedEmbeddingGenerator(emb)
    assert g.process_pdf_document(pdf) == 1
    assert g.embeddings_data["texts"] == ["PDF Document: Manual. PDF Document: Manual. Text "
                                          "extraction failed - may be image-based PDF or corrupted."]
    assert g.embeddings_data["metadata"][0]["file_size"] == pdf.stat().st_size
    assert g.process_pdf_document(pdf, "M2", extract_text=lambda p: "Page 1: hello. " * 80) == 2


def test_pdf_page_errors_skip_only_that_page(tmp_path, monkeypatch):
    """embedding_generator.py:242-252: pdfplumber pages are read one by one and a page whose
    extract_text raises is skipped, the others kept (one bad page emptied the PDF);
    a PDF that cannot be opened falls through to PyPDF2, then to ""."""
    import sys
    import types
    from hcrag_amd.ingest import extract_pdf_text

    class Page:
        def __init__(self, t):
            self.t = t

        def extract_text(self):
            if self.t is None:
                raise ValueError("bad page")
            return self.t

    class Doc:
        pages = [Page("first  page\ntext"), Page(None), Page("third"), Page("   ")]

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False
    fake = types.ModuleType("pdfplumber")
    fake.open = lambda path: Doc()
    monkeypatch.setitem(sys.modules, "pdfplumber", fake)
    assert extract_pdf_text(tmp_path / "x.pdf") == "Page 1: first page text\nPage 3: third"

    def boom(path):
        raise OSError("cannot open")
    fake.open = boom
    monkeypatch.setitem(sys.modules, "PyPDF2", None)   # (import fails: neither reads it)
    assert extract_pdf_text(tmp_path / "x.pdf") == ""


def test_store_rejects_mismatched_lengths(tmp_path):
    with pytest.raises(ValueError):
        EmbeddingStore.save(str(tmp_path / "s"), np.zeros((2, 4)), ["a"], [{}, {}])


@pytest.mark.gpu
def test_gpu_ingest_reference_data_matches_cpu_bert(tmp_path):
    """The reference's data/ through BatchedEmbeddingGenerator.process_all_data on the MI355X
    encoder in reference precision (f32: split-f16 MFMA GEMMs, fp32 attention): every embedding
    within 1e-4 of the fixture's CPU transformers BertModel fp32 (the configs[0] MiniLM-shape
    seeded model), the long document's chunks too; then store -> VectorIndex, each row its own
    nearest neighbour."""
    import hcrag_amd as hc
    from hcrag_amd.synthetic import bert_state
    root, expected = _f1_data(tmp_path)
    g0dir = os.path.join(os.path.dirname(F1), "configs0")
    with open(os.path.join(g0dir, "goldens.json")) as fh:
        g0 = json.load(fh)
    cfg = dict(g0["model"])
    state = bert_state(cfg, seed=g0["seed"], perturb_ln=g0["perturb_ln"])
    tok = hc.WordPieceTokenizer(os.path.join(g0dir, "vocab.txt"), lowercase=True)
    emb = hc.SentenceEmbedder(tok, hc.BertEncoder(cfg, state, dtype="f32"),
                              max_seq_length=g0["max_seq_length"], batch_size=128)
    ref = np.load(os.path.join(F1, "embeddings.npz"))
    g = BatchedEmbeddingGenerator(emb)
    g.process_all_data(root)
    assert g.embeddings_data["texts"] == [e["text"] for e in expected]
    E = g.embeddings_matrix()
    assert E.shape == ref["items"].shape
    assert float(np.max(np.abs(E - ref["items"]))) <= 1e-4
    with open(os.path.join(F1, "chunks.json"), encoding="utf-8") as fh:
        fx = json.load(fh)
    g2 = BatchedEmbeddingGenerator(emb)
    g2.process_text_document(fx["document"], fx["document_name"])
    assert float(np.max(np.abs(g2.embeddings_matrix() - ref["chunks"]))) <= 1e-4
    data = EmbeddingStore.load(g.save_embeddings(str(tmp_path / "store"), dtype="f32"))
    with hc.VectorIndex(E.shape[1], "f32") as ix:
        ix.add(np.asarray(data["embeddings"], np.float32), normalize=False)
        _, ids = ix.search(E[:64], 1)
        assert list(ids[:, 0]) == list(range(64))
