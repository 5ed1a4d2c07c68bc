"""Generate the configs[0] fixture (BASELINE.json: data/Product*.csv -> SimplePropertyGraphStore,
all-MiniLM-L6-v2 CPU embeddings, vector top-5).  Run HERE (it reads /root/reference/data, which
the GPU box does not have):

    python tests/golden/make_configs0.py

Writes tests/golden/configs0/:
  texts.jsonl.gz  the documents graph_builder.py:224-284 builds from data/Product*.csv (441 rows,
                  "Record from {file}:. col: value. ..."), via hcrag_amd.ingest.csv_record_documents
                  -- data, not reference source;
  vocab.txt       a WordPiece vocabulary trained on those texts (HF `tokenizers` BertWordPiece
                  trainer, lowercase): the real all-MiniLM-L6-v2 vocab/weights cannot be
                  downloaded here, so the model is MiniLM-shaped with seeded random weights
                  (hcrag_amd.synthetic.bert_state(seed=SEED, perturb_ln=True));
  goldens.json    the CPU path the reference runs (HF Rust tokenizer, transformers BertModel fp32,
                  mean pooling over the mask + L2 normalise = SentenceTransformer.encode; sklearn
                  cosine + argsort top-5 + >= 0.3 threshold = experiments/main.py:831-857) for the
                  queries of experiments/main.py:1179-1184: query embeddings, top-5 ids / scores,
                  the score gaps around each rank, and corpus-embedding checksums.

Parity status: the text construction and the CPU path are restated (llama_index and
sentence-transformers are not installed, so graph_builder.py itself cannot run here); the
encoder arithmetic is pinned to the installed transformers BertModel.
"""
import gzip
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hc-rag_amd")]

DATA = "/root/reference/data"
FILES = ["Product.csv", "ProductCategory.csv", "ProductDescription.csv", "ProductModel.csv",
         "ProductModelProductDescription.csv"]
QUERIES = ["Find information about mountain bikes", "Show me black bicycle components",
           "What products are available in red color?", "Find bike frames with size 58"]
SEED = 0
MAX_SEQ = 256          # all-MiniLM-L6-v2 max_seq_length
TOP_K, THRESHOLD = 5, 0.3
VOCAB_SIZE = 3000
OUT = os.path.join(HERE, "configs0")


def cpu_reference_embed(texts, vocab_path, state, cfg, batch=32):
    """SentenceTransformer.encode restated: HF Rust WordPiece (truncate to MAX_SEQ, pad to
    longest), BertModel fp32, mean pooling over the attention mask, L2 normalise."""
    import torch
    import transformers
    from tokenizers import BertWordPieceTokenizer
    from hcrag_amd.synthetic import hf_config
    tok = BertWordPieceTokenizer(vocab_path, lowercase=True)
    tok.enable_truncation(MAX_SEQ)
    m = transformers.BertModel(transformers.BertConfig(**hf_config(cfg)), add_pooling_layer=False).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()}, strict=False)
    out = np.zeros((len(texts), cfg["hidden"]), np.float32)
    with torch.no_grad():
        for s in range(0, len(texts), batch):
            enc = tok.encode_batch(texts[s:s + batch])
            L = max(len(e.ids) for e in enc)
            ids = torch.zeros((len(enc), L), dtype=torch.int64)
            mask = torch.zeros((len(enc), L), dtype=torch.int64)
            for i, e in enumerate(enc):
                ids[i, :len(e.ids)] = torch.tensor(e.ids)
                mask[i, :len(e.ids)] = 1
            h = m(input_ids=ids, attention_mask=mask).last_hidden_state
            mm = mask.unsqueeze(-1).float()
            v = (h * mm).sum(1) / mm.sum(1).clamp(min=1e-9)
            out[s:s + batch] = torch.nn.functional.normalize(v, p=2, dim=1).numpy()
    return out


def model_cfg(vocab_size):
    from hcrag_amd.synthetic import SHAPES
    return dict(SHAPES["minilm"], vocab_size=vocab_size)


def main():
    from tokenizers import BertWordPieceTokenizer
    from hcrag_amd.ingest import csv_record_documents
    from hcrag_amd.synthetic import bert_state
    from oracle import cosine_topk as O
    os.makedirs(OUT, exist_ok=True)
    docs = []
    for f in FILES:
        docs += csv_record_documents(os.path.join(DATA, f), f)
    with gzip.open(os.path.join(OUT, "texts.jsonl.gz"), "wt", encoding="utf-8") as fh:
        for d in docs:
            fh.write(json.dumps(d, ensure_ascii=False) + "\n")
    texts = [d["text"] for d in docs]
    # corpus-derived WordPiece vocabulary
    with tempfile.TemporaryDirectory() as td:
        corpus = os.path.join(td, "corpus.txt")
        with open(corpus, "w", encoding="utf-8") as fh:
            fh.write("\n".join(texts + QUERIES) + "\n")
        trainer = BertWordPieceTokenizer(lowercase=True)
        trainer.train([corpus], vocab_size=VOCAB_SIZE, min_frequency=1, show_progress=False)
        trainer.save_model(td)
        with open(os.path.join(td, "vocab.txt"), encoding="utf-8") as fh:
            vocab = fh.read()
    vocab_path = os.path.join(OUT, "vocab.txt")
    with open(vocab_path, "w", encoding="utf-8") as fh:
        fh.write(vocab)
    nvocab = sum(1 for line in vocab.splitlines() if line)
    cfg = model_cfg(nvocab)
    state = bert_state(cfg, seed=SEED, perturb_ln=True)
    E = cpu_reference_embed(texts, vocab_path, state, cfg)
    Qe = cpu_reference_embed(QUERIES, vocab_path, state, cfg)
    results = []
    for qi, q in enumerate(QUERIES):
        sims = O.cosine_similarity64(Qe[qi:qi + 1], E.astype(np.float64))[0]
        top = O.find_similar_content(Qe[qi], E.astype(np.float64), TOP_K, THRESHOLD)
        order = O.topk_order(sims, TOP_K + 1)
        gaps = [float(sims[order[r]] - sims[order[r + 1]]) for r in range(TOP_K)]
        results.append({"query": q, "ids": [i for i, _ in top], "scores": [s for _, s in top],
                        "gaps_to_next": gaps})
    gold = {"files": FILES, "queries": QUERIES, "seed": SEED, "perturb_ln": True,
            "max_seq_length": MAX_SEQ, "top_k": TOP_K, "threshold": THRESHOLD,
            "model": {k: v for k, v in cfg.items()}, "n_texts": len(texts),
            "query_embeddings": Qe.tolist(), "results": results,
            "corpus_checksums": {"sum": float(E.astype(np.float64).sum()),
                                 "abs_sum": float(np.abs(E.astype(np.float64)).sum()),
                                 "rows_0_2": E[:3].tolist()}}
    with open(os.path.join(OUT, "goldens.json"), "w") as fh:
        json.dump(gold, fh, indent=1)
    for r in results:
        print(r["query"], r["ids"], ["%.6f" % s for s in r["scores"]],
              "min gap %.2e" % min(r["gaps_to_next"]))


if __name__ == "__main__":
    main()
