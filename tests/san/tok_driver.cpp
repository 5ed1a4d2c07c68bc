// tok_driver.cpp — host-only driver of the C++ WordPiece tokenizer (hc-rag_amd/csrc/wordpiece.cpp)
// for the ASan + UBSan build (Makefile target `san`; tests/test_sanitize.py).  No HIP.
//
//   tok_driver VOCAB MAX_LEN TEXTS_FILE       texts separated by NUL bytes; prints one line of
//                                             token ids per text
//   tok_driver VOCAB MAX_LEN --fuzz N SEED    N random byte strings (invalid UTF-8, control and
//                                             multi-byte characters, long words); prints a checksum
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "hcrag.h"

static int run(const hcr_tok* tok, const std::vector<std::string>& texts, int max_len, bool print,
               uint64_t* sum) {
  const int64_t n = (int64_t)texts.size();
  std::vector<const char*> ptrs(n);
  std::vector<int64_t> lens(n);
  for (int64_t i = 0; i < n; ++i) { ptrs[i] = texts[i].data(); lens[i] = (int64_t)texts[i].size(); }
  std::vector<int32_t> ids((size_t)n * max_len), mask((size_t)n * max_len), tl(n);
  const int rc = hcr_tokenize(tok, ptrs.data(), lens.data(), n, max_len, ids.data(), mask.data(), tl.data());
  if (rc != HCR_OK) { fprintf(stderr, "tokenize: %s\n", hcr_last_error()); return rc; }
  for (int64_t i = 0; i < n; ++i) {
    for (int j = 0; j < tl[i]; ++j) {
      if (print) printf(j ? " %d" : "%d", ids[(size_t)i * max_len + j]);
      *sum = *sum * 1000003u + (uint64_t)ids[(size_t)i * max_len + j];
    }
    if (print) printf("\n");
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: tok_driver VOCAB MAX_LEN TEXTS | --fuzz N SEED\n"); return 2; }
  hcr_tok* tok = nullptr;
  if (hcr_wordpiece_create(argv[1], 1, -1, &tok) != HCR_OK) { fprintf(stderr, "%s\n", hcr_last_error()); return 2; }
  const int max_len = atoi(argv[2]);
  uint64_t sum = 0;
  int rc = 0;
  if (std::string(argv[3]) == "--fuzz") {
    const int n = argc > 4 ? atoi(argv[4]) : 1000;
    std::mt19937_64 rng(argc > 5 ? strtoull(argv[5], nullptr, 10) : 1);
    const char* pieces[] = {"bike", " ", "\xC3\xA9", "\xE4\xB8\xAD", "\xF0\x9F\x9A\xB2", "\t", "\x01",
                            ",", "##", "[CLS]", "\xC3", "\xE4\xB8", "\xFF", "\x80", "aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa"};
    std::vector<std::string> texts;
    for (int i = 0; i < n; ++i) {
      std::string t;
      const int parts = (int)(rng() % 64);
      for (int p = 0; p < parts; ++p) {
        if (rng() % 4 == 0) t.push_back((char)(rng() & 0xFF));
        else t += pieces[rng() % (sizeof(pieces) / sizeof(pieces[0]))];
      }
      texts.push_back(t);
    }
    rc = run(tok, texts, max_len, false, &sum);
    printf("fuzz ok %d %llu\n", n, (unsigned long long)sum);
  } else {
    std::ifstream f(argv[3], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string all = ss.str();
    std::vector<std::string> texts;
    size_t s = 0;
    for (size_t i = 0; i <= all.size(); ++i)
      if (i == all.size() || all[i] == '\0') {
        if (i > s || i < all.size()) texts.push_back(all.substr(s, i - s));
        s = i + 1;
      }
    rc = run(tok, texts, max_len, true, &sum);
  }
  hcr_wordpiece_destroy(tok);
  return rc;
}
