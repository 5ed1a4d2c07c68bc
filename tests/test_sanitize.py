"""Host sanitizers ("Host ASan/UBSan build of the C++ library"): the WordPiece
tokenizer -- the library's parser of arbitrary input text -- built with
-fsanitize=address,undefined as a standalone driver (Makefile target `san`, no HIP, no
preloading), run over the configs[0] corpus (ids compared with the HF Rust engine) and over
random byte strings (invalid UTF-8, control / multi-byte characters, over-long words).  Any
sanitizer report aborts the driver, failing the test."""
import gzip
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "hc-rag_amd", "lib", "san", "tok_driver")
VOCAB = os.path.join(ROOT, "tests", "golden", "configs0", "vocab.txt")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def driver():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "hc-rag_amd", "csrc"), "san"],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stdout[-2000:] + r.stderr[-2000:])
    return DRIVER


def test_sanitized_tokenizer_matches_hf(driver, tmp_path):
    tokenizers = pytest.importorskip("tokenizers")
    with gzip.open(os.path.join(ROOT, "tests", "golden", "configs0", "texts.jsonl.gz"), "rt",
                   encoding="utf-8") as fh:
        texts = [json.loads(line)["text"] for line in fh]
    texts += ["Café 中文 naïve ¿Qué?", "", "   ", "é" * 300,
              "ProductID: 680. Weight: 1016.04"]
    f = tmp_path / "texts.bin"
    f.write_bytes(b"\0".join(t.encode("utf-8") for t in texts))
    r = subprocess.run([driver, VOCAB, "128", str(f)], capture_output=True, text=True, env=ENV,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    got = [list(map(int, line.split())) for line in r.stdout.split("\n")[:len(texts)]]
    hf = tokenizers.BertWordPieceTokenizer(VOCAB, lowercase=True)
    hf.enable_truncation(128)
    exp = [e.ids for e in hf.encode_batch(texts)]
    assert got == exp


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sanitized_tokenizer_fuzz(driver, seed):
    r = subprocess.run([driver, VOCAB, "64", "--fuzz", "3000", str(seed)], capture_output=True,
                       text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("fuzz ok 3000")
