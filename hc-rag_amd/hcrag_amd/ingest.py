"""Batched corpus ingestion and an on-disk embedding store.

Replaces experiments/embedding_generator.py's ``DynamicEmbeddingGenerator`` ingestion path:
  * the reference encodes one row at a time (``self.model.encode([text])[0]``, :124, :197)
    and re-runs ``analyze_data_patterns`` over the whole table for every row (:67, O(rows^2));
    here a table's texts are built with the analysis computed once per table (same result:
    the DataFrame does not change between rows) and encoded in ONE call of the MI355X encoder
    (length-sorted batches on the GPU, ``SentenceEmbedder.encode``);
  * the reference stores Python-float lists in a pickle (:127, :422-437); here the store is a
    directory: ``embeddings.npy`` (fp16 by default: the index's storage dtype, loaded
    memory-mapped), ``texts.jsonl``, ``metadata.jsonl``, ``generation_info.json``.  Loading
    executes nothing from the files.

The text representation follows :28-104 (field importance from avg length / unique ratio,
"Table: name" then high / first 3 medium / first 2 low fields, joined by ". ") and the metadata
:130-145 (``id``, ``type``, ``table_name``, ``row_index``, ``source_file``, ``entity_id`` from
the first column whose name contains "id").  JSON documents follow :152-215 (the parent document
from " Table " in the file name, :385-389).  PDF documents follow :278-364: the extracted text is
cut by ``chunk_text`` (800 characters, 100 overlap, sentence-boundary search) and every chunk,
prefixed "PDF Document: {name}. ", is encoded in ONE batched call (the reference: one encode per
chunk, :326-337).  Text extraction itself (:218-276, pdfplumber / PyPDF2) is the caller's: pass
``extract_text`` (a callable) or already-extracted ``text``; pdfplumber / PyPDF2 are used when
importable, and otherwise the reference's own extraction-failure text is embedded (:270-272).
Parity: tests/golden/make_ingest_f1.py restates these lines independently over the reference's
data/ and its fixture pins texts, metadata and (CPU BertModel fp32) embeddings.
"""
from __future__ import annotations

import datetime
import json
import os
from pathlib import Path
from typing import Any, Dict, List, Optional

import numpy as np


class EmbeddingStore:
    """On-disk embedding store: a directory of plain files, nothing unpickled on load."""

    @staticmethod
    def save(path: str, embeddings: np.ndarray, texts: List[str], metadata: List[dict],
             generation_info: Optional[dict] = None, dtype: str = "f16") -> str:
        E = np.asarray(embeddings)
        if E.ndim != 2 or len(texts) != E.shape[0] or len(metadata) != E.shape[0]:
            raise ValueError("embeddings [n, D], texts [n] and metadata [n] must agree")
        os.makedirs(path, exist_ok=True)
        np.save(os.path.join(path, "embeddings.npy"),
                E.astype(np.float16 if dtype == "f16" else np.float32))
        with open(os.path.join(path, "texts.jsonl"), "w", encoding="utf-8") as f:
            for t in texts:
                f.write(json.dumps(t, ensure_ascii=False) + "\n")
        with open(os.path.join(path, "metadata.jsonl"), "w", encoding="utf-8") as f:
            for m in metadata:
                f.write(json.dumps(m, ensure_ascii=False, default=str) + "\n")
        info = dict(generation_info or {})
        info.setdefault("total_entries", int(E.shape[0]))
        info.setdefault("embedding_dimension", int(E.shape[1]) if E.shape[0] else 0)
        info["storage_dtype"] = dtype
        with open(os.path.join(path, "generation_info.json"), "w") as f:
            json.dump(info, f, indent=1, default=str)
        return path

    @staticmethod
    def load(path: str, mmap: bool = True) -> Dict[str, Any]:
        """The reference's ``embeddings_data`` shape: embeddings (ndarray [n, D]), texts,
        metadata, generation_info."""
        E = np.load(os.path.join(path, "embeddings.npy"), mmap_mode="r" if mmap else None,
                    allow_pickle=False)
        with open(os.path.join(path, "texts.jsonl"), encoding="utf-8") as f:
            texts = [json.loads(line) for line in f]
        with open(os.path.join(path, "metadata.jsonl"), encoding="utf-8") as f:
            metadata = [json.loads(line) for line in f]
        with open(os.path.join(path, "generation_info.json")) as f:
            info = json.load(f)
        if len(texts) != E.shape[0] or len(metadata) != E.shape[0]:
            raise ValueError(f"corrupt store {path}: {E.shape[0]} rows, {len(texts)} texts, "
                             f"{len(metadata)} metadata")
        return {"embeddings": E, "texts": texts, "metadata": metadata, "generation_info": info}


def analyze_data_patterns(df) -> Dict[str, dict]:
    """Field importance per column (embedding_generator.py:28-61)."""
    out = {}
    for col in df.columns:
        nn = df[col].dropna()
        sample = nn.head(10).astype(str).tolist()
        if not sample:
            continue
        avg_len = float(np.mean([len(str(v)) for v in sample]))
        uniq = len(nn.unique()) / len(nn) if len(nn) > 0 else 0
        if uniq > 0.9 and avg_len > 20:
            imp = "high"
        elif uniq > 0.8:
            imp = "medium"
        elif avg_len > 10:
            imp = "medium"
        else:
            imp = "low"
        out[col] = {"importance": imp, "avg_length": avg_len, "unique_ratio": uniq,
                    "sample_values": sample[:3]}
    return out


def smart_text(row, analysis: Dict[str, dict], table_name: Optional[str] = None) -> str:
    """embedding_generator.py:63-104 with the table analysis precomputed."""
    import pandas as pd
    hi, me, lo = [], [], []
    for col, a in analysis.items():
        v = row.get(col)
        if pd.notna(v) and str(v).strip():
            info = f"{col}: {str(v).strip()}"
            (hi if a["importance"] == "high" else me if a["importance"] == "medium" else lo).append(info)
    parts = [f"Table: {table_name}"] if table_name else []
    parts += hi + me[:3] + lo[:2]
    return ". ".join(parts)


def flatten_json_to_text(obj, prefix: str = "") -> List[str]:
    """embedding_generator.py:152-175."""
    out: List[str] = []
    if isinstance(obj, (dict, list)):
        items = obj.items() if isinstance(obj, dict) else enumerate(obj)
        for k, v in items:
            if isinstance(obj, dict):
                p = f"{prefix}.{k}" if prefix else k
            else:
                p = f"{prefix}[{k}]" if prefix else f"item_{k}"
            if isinstance(v, (dict, list)):
                out.extend(flatten_json_to_text(v, p))
            else:
                out.append(f"{p}: {v}")
    else:
        out.append(f"{prefix}: {obj}" if prefix else str(obj))
    return out


def chunk_text(text: str, max_chunk_size: int = 1000, overlap: int = 100) -> List[str]:
    """embedding_generator.py:278-305: windows of max_chunk_size characters, each ended at the
    last '.', '!' or '?' found scanning back from the window end (at most 200 characters and not
    into the window's first half), the next window starting `overlap` characters before the
    previous end -- including the reference's short trailing window when the last end overshoots
    the text by less than `overlap`."""
    n = len(text)
    if n <= max_chunk_size:
        return [text]
    out: List[str] = []
    start = 0
    while start < n:
        end = start + max_chunk_size
        if end < n:
            lo = max(start + max_chunk_size // 2, end - 200)
            for i in range(end, lo, -1):
                if text[i] in ".!?":
                    end = i + 1
                    break
        piece = text[start:end].strip()
        if piece:
            out.append(piece)
        start = end - overlap
        if start >= n:
            break
    return out


def extract_pdf_text(pdf_path) -> str:
    """embedding_generator.py:218-276 when pdfplumber / PyPDF2 are importable ("Page n: ..."
    lines; pdfplumber first, whitespace-collapsed); "" when neither reads the file.  As there, a
    page whose extraction raises is skipped (:229-231, :250-252) and the pages read so far are
    kept; only a failure to open the file empties the method's result."""
    def pdfplumber_pages():
        out: List[str] = []
        try:
            import pdfplumber
            with pdfplumber.open(pdf_path) as pdf:
                for i, page in enumerate(pdf.pages):
                    try:
                        t = page.extract_text()
                    except Exception:                   # noqa: BLE001 -- this page only
                        continue
                    if t and t.strip():
                        out.append(f"Page {i + 1}: " + " ".join(t.split()))
        except Exception:                               # noqa: BLE001 -- open / import failed
            return []
        return out

    def pypdf2_pages():
        out: List[str] = []
        try:
            import PyPDF2
            with open(pdf_path, "rb") as fh:
                for i, page in enumerate(PyPDF2.PdfReader(fh).pages):
                    try:
                        t = page.extract_text()
                    except Exception:                   # noqa: BLE001 -- this page only
                        continue
                    if t.strip():
                        out.append(f"Page {i + 1}: {t.strip()}")
        except Exception:                               # noqa: BLE001
            return []
        return out

    pages = pdfplumber_pages()
    if not "\n".join(pages).strip():
        pages = pypdf2_pages()
    return "\n".join(pages)


def read_csv_like_graph_builder(path):
    """graph_builder.py:228-248: the first (separator, encoding) among ``, ; \\t |`` x
    ``utf-8 latin-1 cp1252`` that pandas parses into more than one column (the reference tries
    "," first, so a ";"-separated file with decimal commas is split on its commas), else None."""
    import pandas as pd
    df = None
    for sep in (",", ";", "\t", "|"):
        for enc in ("utf-8", "latin-1", "cp1252"):
            try:
                df = pd.read_csv(path, sep=sep, encoding=enc)
                if len(df.columns) > 1:
                    break
            except Exception:
                continue
        if df is not None and len(df.columns) > 1:
            break
    if df is None or len(df.columns) <= 1:
        return None
    return df


def csv_record_documents(path, file_name: Optional[str] = None) -> List[Dict[str, Any]]:
    """The documents ``GraphBuilder._process_csv_content`` makes of a CSV (graph_builder.py:
    224-284): per row "Record from {file}:" then "col: value" for every non-null, non-blank
    cell, joined by ". ", with metadata source / source_type / row_index / columns and id
    ``{file}_row_{idx}``.  These texts are what ``PropertyGraphIndex.from_documents`` embeds into
    the SimplePropertyGraphStore path of BASELINE.json configs[0]."""
    import pandas as pd
    name = file_name or Path(path).name
    df = read_csv_like_graph_builder(path)
    if df is None:
        return []
    docs = []
    for idx, row in df.iterrows():
        parts = [f"Record from {name}:"]
        for col, value in row.items():
            if pd.notna(value) and str(value).strip():
                parts.append(f"{col}: {value}")
        if len(parts) > 1:
            docs.append({"id": f"{name}_row_{idx}", "text": ". ".join(parts),
                         "metadata": {"source": name, "source_type": "csv", "row_index": int(idx),
                                      "columns": [str(c) for c in row.keys()]}})
    return docs


class BatchedEmbeddingGenerator:
    """``DynamicEmbeddingGenerator`` surface with batched GPU encoding.

    ``embedder``: object with ``encode(List[str]) -> ndarray [n, D]`` (``SentenceEmbedder`` /
    ``MI355XEmbedding``-backed, or any SentenceTransformer-like model)."""

    def __init__(self, embedder, model_name: str = "all-MiniLM-L6-v2"):
        self.model = embedder
        self.model_name = model_name
        self.embeddings_data = {"embeddings": [], "metadata": [], "texts": []}
        self._chunks: List[np.ndarray] = []

    # the reference's per-table helpers, as methods for drop-in callers
    def analyze_data_patterns(self, df):
        return analyze_data_patterns(df)

    def create_smart_text_representation(self, row, df, table_name=None):
        return smart_text(row, analyze_data_patterns(df), table_name)

    def flatten_json_to_text(self, json_obj, prefix=""):
        return flatten_json_to_text(json_obj, prefix)

    def _append(self, texts: List[str], metas: List[dict]) -> None:
        if not texts:
            return
        E = np.asarray(self.model.encode(texts), dtype=np.float32)
        if E.shape[0] != len(texts):
            raise ValueError("embedder returned a wrong number of rows")
        self._chunks.append(E)
        self.embeddings_data["texts"].extend(texts)
        self.embeddings_data["metadata"].extend(metas)

    def process_csv_table(self, csv_path, related_data=None, sep: str = ";") -> int:
        """embedding_generator.py:106-150, one encode call per table."""
        import pandas as pd
        df = pd.read_csv(csv_path, sep=sep)
        table = Path(csv_path).stem
        analysis = analyze_data_patterns(df)
        id_cols = [c for c in df.columns if "id" in c.lower() or "ID" in c]
        texts, metas = [], []
        for idx, row in df.iterrows():
            text = smart_text(row, analysis, table)
            if not text.strip():
                continue
            m = {"id": f"{table}_{idx}", "type": "database_table", "table_name": table,
                 "row_index": int(idx), "source_file": str(csv_path)}
            if id_cols:
                v = row.get(id_cols[0])
                if pd.notna(v):
                    m["entity_id"] = int(v) if str(v).isdigit() else str(v)
            texts.append(text)
            metas.append(m)
        self._append(texts, metas)
        return len(texts)

    def process_json_table(self, json_path, parent_document=None) -> int:
        """embedding_generator.py:177-215."""
        with open(json_path, "r", encoding="utf-8") as f:
            data = json.load(f)
        name = Path(json_path).stem
        text = f"Document: {parent_document or name}. Contains structured information. "
        text += ". ".join(flatten_json_to_text(data)[:20])
        self._append([text], [{"id": f"json_{name}", "type": "json_table", "filename": name,
                               "parent_document": parent_document, "source_file": str(json_path),
                               "json_keys": list(data.keys()) if isinstance(data, dict) else []}])
        return 1

    def process_text_document(self, text: str, document_name: str, source_file: str = "",
                              file_size: int = 0, max_chunk_size: int = 800,
                              overlap: int = 100) -> int:
        """embedding_generator.py:307-364 after text extraction: chunk_text, the
        "PDF Document: {name}. " prefix and per-chunk metadata, all chunks in ONE encode call."""
        if not text.strip():
            return 0
        chunks = chunk_text(text, max_chunk_size, overlap)
        ctx = f"PDF Document: {document_name}. "
        metas = [{"id": f"pdf_{document_name}_chunk_{j}", "type": "pdf_document",
                  "document_name": document_name, "source_file": source_file, "chunk_index": j,
                  "total_chunks": len(chunks), "text_length": len(c), "file_size": file_size}
                 for j, c in enumerate(chunks)]
        self._append([ctx + c for c in chunks], metas)
        return len(chunks)

    def process_pdf_document(self, pdf_path, document_name=None, text: Optional[str] = None,
                             extract_text=None) -> int:
        """embedding_generator.py:307-364.  The text is `text`, else `extract_text(pdf_path)`,
        else extract_pdf_text (pdfplumber / PyPDF2 when importable); when none yields any,
        the reference's extraction-failure sentence (:270-272) is what gets embedded."""
        p = Path(pdf_path)
        name = document_name or p.stem
        if text is None:
            text = extract_text(pdf_path) if extract_text is not None else extract_pdf_text(pdf_path)
        if not text.strip():
            text = (f"PDF Document: {p.stem}. Text extraction failed - may be image-based PDF "
                    f"or corrupted.")
        size = p.stat().st_size if p.exists() else 0
        return self.process_text_document(text, name, str(pdf_path), size)

    def process_all_data(self, data_directory, extract_text=None) -> None:
        """embedding_generator.py:366-401: the directory's ';'-separated CSV tables, then
        IngestedDocuments/*.json (parent document = the file name before " Table "), then
        IngestedDocuments/*.pdf.  Files in name order (the reference: directory-listing order)."""
        d = Path(data_directory)
        for p in sorted(d.glob("*.csv")):
            self.process_csv_table(p)
        jd = d / "IngestedDocuments"
        if jd.exists():
            for p in sorted(jd.glob("*.json")):
                parent = p.stem.split(" Table ")[0] if " Table " in p.stem else None
                self.process_json_table(p, parent)
            for p in sorted(jd.glob("*.pdf")):
                self.process_pdf_document(p, p.stem, extract_text=extract_text)

    def embeddings_matrix(self) -> np.ndarray:
        if not self._chunks:
            return np.zeros((0, 0), np.float32)
        if len(self._chunks) > 1:
            self._chunks = [np.concatenate(self._chunks)]
        return self._chunks[0]

    def save_embeddings(self, output_path: str = "knowledge_graph_embeddings", dtype: str = "f16") -> str:
        """Directory store instead of the reference's pickle (:422-437)."""
        E = self.embeddings_matrix()
        info = {"model_name": self.model_name, "total_entries": len(self.embeddings_data["texts"]),
                "embedding_dimension": int(E.shape[1]) if E.size else 0,
                "generation_timestamp": datetime.datetime.now().isoformat()}
        return EmbeddingStore.save(output_path, E, self.embeddings_data["texts"],
                                   self.embeddings_data["metadata"], info, dtype)

    def load_embeddings(self, input_path: str = "knowledge_graph_embeddings") -> Dict[str, Any]:
        data = EmbeddingStore.load(input_path)
        self._chunks = [np.asarray(data["embeddings"], dtype=np.float32)]
        self.embeddings_data = {"embeddings": [], "texts": data["texts"],
                                "metadata": data["metadata"],
                                "generation_info": data["generation_info"]}
        return {**self.embeddings_data, "embeddings": data["embeddings"]}

    def get_statistics(self):
        """embedding_generator.py:449-466."""
        E = self.embeddings_matrix()
        if E.size == 0:
            return "No embeddings generated yet"
        types: Dict[str, int] = {}
        for m in self.embeddings_data["metadata"]:
            types[m["type"]] = types.get(m["type"], 0) + 1
        return {"total_embeddings": int(E.shape[0]), "embedding_dimension": int(E.shape[1]),
                "content_types": types}


__all__ = ["EmbeddingStore", "BatchedEmbeddingGenerator", "analyze_data_patterns", "smart_text",
           "flatten_json_to_text", "csv_record_documents", "read_csv_like_graph_builder",
           "chunk_text", "extract_pdf_text"]
