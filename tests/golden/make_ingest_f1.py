"""Generate the SURVEY.md §8(f) rank-1 fixture (batched corpus ingestion) from the reference's own
data.  Run HERE (it reads /root/reference/data, which the GPU box does not have):

    python tests/golden/make_ingest_f1.py

This script is the ORACLE of the ingestion text path, written independently of the product
(hcrag_amd.ingest): it restates experiments/embedding_generator.py literally, row by row --
    :28-61    field importance (avg length / unique ratio of the first 10 non-null values),
              recomputed for EVERY row as create_smart_text_representation does (:67);
    :63-104   "Table: name", the high fields, the first 3 medium, the first 2 low, ". "-joined;
    :106-150  process_csv_table (';'-separated, metadata id / type / table_name / row_index /
              source_file, entity_id from the first column whose name contains "id");
    :152-175  flatten_json_to_text; :177-216 process_json_table ("Document: ..", the first 20
              flattened fields, metadata json_keys);
    :278-305  chunk_text (800 / 100 for PDFs, sentence-boundary search, trailing overlap chunk);
    :307-364  process_pdf_document's per-chunk "PDF Document: {name}. " prefix and metadata;
    :366-401  process_all_data (CSV files, then IngestedDocuments/*.json with the parent document
              taken from " Table " in the file name, then the PDFs).
File order: sorted by name (the reference iterates Path.glob, i.e. directory-listing order).
PDF text extraction (pdfplumber / PyPDF2, :218-272) is absent here: the chunk leg runs on a
synthetic long document (the ProductDescription texts joined), and the PDFs take the
reference's own extraction-failure text (:270-272) -- what the reference embeds for a PDF it
cannot read.

Writes tests/golden/f1/:
  data/*.csv.gz, data/IngestedDocuments/*.json.gz  the reference's input data files (data, not
                   source), decompressed by the tests into a temporary directory;
  expected.jsonl.gz  one record per embedded item, in order: text + metadata;
  chunks.json      the synthetic long document and its expected chunk texts;
  embeddings.npz   CPU fp32 embeddings of every text (HF Rust WordPiece + transformers
                   BertModel fp32 + mean pooling + L2 = SentenceTransformer.encode, :124), with
                   the configs[0] MiniLM-shape seeded model and corpus vocabulary
                   (tests/golden/configs0/).
"""
import gzip
import json
import os
import shutil
import sys
from pathlib import Path

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd"), HERE]

SRC = Path("/root/reference/data")
OUT = Path(HERE) / "f1"
PDF_CHUNK, PDF_OVERLAP = 800, 100


# ---- the oracle restatement (see the module docstring for the reference lines) ----------
def field_importance(df):
    import pandas as pd  # noqa: F401
    res = {}
    for col in df.columns:
        present = df[col].dropna()
        vals = present.head(10).astype(str).tolist()
        if len(vals) == 0:
            continue
        mean_len = np.mean([len(str(v)) for v in vals])
        ratio = len(present.unique()) / len(present) if len(present) > 0 else 0
        if ratio > 0.9 and mean_len > 20:
            level = "high"
        elif ratio > 0.8 or mean_len > 10:
            level = "medium"
        else:
            level = "low"
        res[col] = level
    return res


def row_text(row, df, table):
    import pandas as pd
    levels = field_importance(df)               # per row, as the reference does
    buckets = {"high": [], "medium": [], "low": []}
    for col, level in levels.items():
        v = row.get(col)
        if pd.notna(v) and str(row[col]).strip():
            buckets[level].append(f"{col}: {str(row[col]).strip()}")
    pieces = []
    if table:
        pieces.append(f"Table: {table}")
    pieces += buckets["high"]
    pieces += buckets["medium"][:3]
    pieces += buckets["low"][:2]
    return ". ".join(pieces)


def csv_items(path):
    import pandas as pd
    df = pd.read_csv(path, sep=";")
    table = Path(path).stem
    idcols = [c for c in df.columns if "id" in c.lower() or "ID" in c]
    items = []
    for idx, row in df.iterrows():
        text = row_text(row, df, table)
        if not text.strip():
            continue
        meta = {"id": f"{table}_{idx}", "type": "database_table", "table_name": table,
                "row_index": int(idx), "source_file": str(path)}
        if idcols:
            ev = row.get(idcols[0])
            if pd.notna(ev):
                meta["entity_id"] = int(ev) if str(ev).isdigit() else str(ev)
        items.append({"text": text, "metadata": meta})
    return items


def flatten(obj, prefix=""):
    parts = []
    if isinstance(obj, dict):
        for key, val in obj.items():
            p = f"{prefix}.{key}" if prefix else key
            parts += flatten(val, p) if isinstance(val, (dict, list)) else [f"{p}: {val}"]
    elif isinstance(obj, list):
        for i, val in enumerate(obj):
            p = f"{prefix}[{i}]" if prefix else f"item_{i}"
            parts += flatten(val, p) if isinstance(val, (dict, list)) else [f"{p}: {val}"]
    else:
        parts.append(f"{prefix}: {obj}" if prefix else str(obj))
    return parts


def json_item(path, parent):
    with open(path, encoding="utf-8") as fh:
        data = json.load(fh)
    name = Path(path).stem
    text = f"Document: {parent or name}. Contains structured information. " + ". ".join(flatten(data)[:20])
    return {"text": text, "metadata": {"id": f"json_{name}", "type": "json_table", "filename": name,
                                       "parent_document": parent, "source_file": str(path),
                                       "json_keys": list(data.keys()) if isinstance(data, dict) else []}}


def chunks_of(text, size, overlap):
    if len(text) <= size:
        return [text]
    out, start = [], 0
    while start < len(text):
        end = start + size
        if end < len(text):
            for i in range(end, max(start + size // 2, end - 200), -1):
                if text[i] in ".!?":
                    end = i + 1
                    break
        piece = text[start:end].strip()
        if piece:
            out.append(piece)
        start = end - overlap
        if start >= len(text):
            break
    return out


def pdf_items(text, doc_name, source, file_size):
    chunks = chunks_of(text, PDF_CHUNK, PDF_OVERLAP)
    return [{"text": f"PDF Document: {doc_name}. " + c,
             "metadata": {"id": f"pdf_{doc_name}_chunk_{j}", "type": "pdf_document",
                          "document_name": doc_name, "source_file": source, "chunk_index": j,
                          "total_chunks": len(chunks), "text_length": len(c), "file_size": file_size}}
            for j, c in enumerate(chunks)]


def all_items(data_dir):
    """process_all_data over data_dir (paths as they are under data_dir)."""
    d = Path(data_dir)
    items = []
    for p in sorted(d.glob("*.csv")):
        items += csv_items(p)
    jd = d / "IngestedDocuments"
    if jd.exists():
        for p in sorted(jd.glob("*.json")):
            parent = p.stem.split(" Table ")[0] if " Table " in p.stem else None
            items.append(json_item(p, parent))
        for p in sorted(jd.glob("*.pdf")):
            failed = f"PDF Document: {p.stem}. Text extraction failed - may be image-based PDF or corrupted."
            items += pdf_items(failed, p.stem, str(p), p.stat().st_size)
    return items


def main():
    from make_configs0 import cpu_reference_embed, model_cfg
    from hcrag_amd.synthetic import bert_state
    if OUT.exists():
        shutil.rmtree(OUT)
    (OUT / "data" / "IngestedDocuments").mkdir(parents=True)
    for p in sorted(SRC.glob("*.csv")) + sorted((SRC / "IngestedDocuments").glob("*.json")):
        rel = p.relative_to(SRC)
        with open(p, "rb") as fi, open(OUT / "data" / (str(rel) + ".gz"), "wb") as fo:
            fo.write(gzip.compress(fi.read(), mtime=0))      # reproducible bytes
    # the items as a test sees them: data decompressed under a directory named "data"
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        root = Path(td) / "data"
        (root / "IngestedDocuments").mkdir(parents=True)
        for p in sorted(SRC.glob("*.csv")) + sorted((SRC / "IngestedDocuments").glob("*.json")):
            shutil.copy(p, root / p.relative_to(SRC))
        items = all_items(root)
        for it in items:                          # paths relative to the data directory
            it["metadata"]["source_file"] = os.path.relpath(it["metadata"]["source_file"], td)
    # no PDFs are committed (binary, unreadable here): the PDF leg is the chunk fixture below
    long_doc = " ".join(it["text"] for it in items
                        if it["metadata"].get("table_name") == "ProductDescription")[:6000]
    doc_items = pdf_items(long_doc, "Synthetic Manual", "data/IngestedDocuments/Synthetic Manual.pdf", 0)
    with gzip.open(OUT / "expected.jsonl.gz", "wt", encoding="utf-8") as fh:
        for it in items:
            fh.write(json.dumps(it, ensure_ascii=False) + "\n")
    with open(OUT / "chunks.json", "w", encoding="utf-8") as fh:
        json.dump({"document": long_doc, "document_name": "Synthetic Manual",
                   "chunk_size": PDF_CHUNK, "overlap": PDF_OVERLAP, "items": doc_items}, fh,
                  ensure_ascii=False, indent=0)
    with open(os.path.join(HERE, "configs0", "goldens.json")) as fh:
        g0 = json.load(fh)
    cfg = model_cfg(g0["model"]["vocab_size"])
    state = bert_state(cfg, seed=g0["seed"], perturb_ln=g0["perturb_ln"])
    vocab = os.path.join(HERE, "configs0", "vocab.txt")
    E = cpu_reference_embed([it["text"] for it in items], vocab, state, cfg)
    C = cpu_reference_embed([it["text"] for it in doc_items], vocab, state, cfg)
    np.savez_compressed(OUT / "embeddings.npz", items=E, chunks=C)
    kinds = {}
    for it in items:
        kinds[it["metadata"]["type"]] = kinds.get(it["metadata"]["type"], 0) + 1
    print(f"{len(items)} items {kinds}, {len(doc_items)} chunks of a {len(long_doc)}-char document")


if __name__ == "__main__":
    main()
