"""CPU: the C++ WordPiece tokenizer vs the installed HF `tokenizers` Rust engine (the engine
the reference reaches through SentenceTransformer.encode; pinned 0.21.1, installed 0.22.2),
on a synthetic vocab (the real all-MiniLM-L6-v2 vocab is not available offline)."""
import os
import tempfile

import numpy as np
import pytest

tokenizers = pytest.importorskip("tokenizers")

TEXTS = [
    "Record from Product.csv: ProductID: 680; Name: HL Road Frame - Black, 58; ListPrice: 1431,50",
    "Mountain Bike Frame - HL Mountain Frame, Black, 42",
    "red helmet", "mountain bike frame", "",
    "Café naïve résumé Ångström ÉLAN œuvre Straße",
    "北京欢迎你 tokyo 東京",
    "Hello!!! (test) [x] {y} «quote» — dash… ¿qué? ¡sí!",
    "tabs\tand\nnewlines\r\nand  spaces nbsp　ideo",
    "ctrl\x00chars\x07here​zw﻿bom",
    "a" * 150 + " long",
    "emoji 🚲 bikes 🚲🚲",
    "한국어 텍스트", "Ελληνικά ΚΕΦΑΛΑΙΑ", "İstanbul DİYARBAKIR",
    "combining é and à marks ́alone",
    "unaffable unaffordable running runner 2024-01-01 3.14 $19.99",
    "UPPER lower MiXeD 12345 abc123def",
]


def _vocab():
    from tokenizers.normalizers import BertNormalizer
    from tokenizers.pre_tokenizers import BertPreTokenizer
    norm, pre = BertNormalizer(lowercase=True), BertPreTokenizer()
    words = []
    for t in TEXTS:
        words += [w for w, _ in pre.pre_tokenize_str(norm.normalize_str(t))]
    chars = sorted({c for w in words for c in w})
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    vocab += chars + ["##" + c for c in chars]
    whole = sorted({w for w in words if 1 < len(w) < 12})[::2]      # some words whole
    vocab += whole + ["##able", "##ford", "##ning", "##ner", "un", "##aff", "run", "moun",
                      "##tain", "##ike", "fra", "##me"]
    seen, out = set(), []
    for v in vocab:
        if v not in seen:
            seen.add(v)
            out.append(v)
    return out


@pytest.mark.parametrize("max_len", [8, 32, 256])
def test_tokenizer_matches_hf_rust_engine(max_len):
    from hcrag_amd.tokenizer import WordPieceTokenizer
    vocab = _vocab()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "vocab.txt")
        with open(path, "w", encoding="utf-8") as f:
            f.write("\n".join(vocab) + "\n")
        ref = tokenizers.BertWordPieceTokenizer(path, lowercase=True, clean_text=True,
                                                handle_chinese_chars=True)
        ref.enable_truncation(max_len)
        mine = WordPieceTokenizer(vocab_path=path)
        ids, mask, lens = mine.encode(TEXTS, max_len=max_len, pad_to_longest=False)
        for r, t in enumerate(TEXTS):
            exp = ref.encode(t).ids
            got = ids[r, :lens[r]].tolist()
            assert got == exp, (t, got, exp)
            assert mask[r].sum() == lens[r]
            assert np.all(ids[r, lens[r]:] == vocab.index("[PAD]"))
        mine2 = WordPieceTokenizer(vocab_tokens=vocab)
        ids2, _, lens2 = mine2.encode(TEXTS, max_len=max_len)
        assert ids2.shape[1] == lens2.max()
        np.testing.assert_array_equal(ids2, ids[:, :ids2.shape[1]])


def test_tokenizer_errors():
    from hcrag_amd.tokenizer import WordPieceTokenizer
    from hcrag_amd._lib import HcrError
    with pytest.raises(HcrError):
        WordPieceTokenizer(vocab_path="/nonexistent/vocab.txt")
    with pytest.raises(HcrError):
        WordPieceTokenizer(vocab_tokens=["a", "b"])          # no [CLS]/[SEP]/[UNK]
