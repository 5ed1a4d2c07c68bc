// wordpiece.cpp — BERT uncased WordPiece tokenizer on the host.
//
// Replaces the Rust HF tokenizers 0.21.1 BertNormalizer + BertPreTokenizer + WordPiece model
// reached through SentenceTransformer.encode (experiments/embedding_generator.py:124) and
// HuggingFaceEmbedding (graph_builder.py:146-149).  Semantics follow the published BERT
// tokenizer (transformers tokenization_bert.py BasicTokenizer + WordpieceTokenizer):
//   clean text (drop NUL / U+FFFD / control chars, whitespace -> ' '), pad CJK ideographs
//   with spaces, whitespace split, lowercase + NFD accent strip, split on punctuation,
//   greedy longest-match-first WordPiece with "##" continuations, words longer than 100
//   chars -> [UNK]; [CLS] ... [SEP], truncation to max_len, [PAD] = vocab id of "[PAD]".
// Unicode properties come from unicode_tables.h (generated from Python's unicodedata).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "hcrag.h"
#include "unicode_tables.h"

extern int hcr_set_error(int code, const char* msg);   // errors.cpp

namespace {

bool in_ranges(const uint32_t (*r)[2], int n, uint32_t cp) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < r[mid][0]) hi = mid - 1;
    else if (cp > r[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}

// mapping table lookup: number of output code points (>= 0, 0 = maps to nothing) or -1
int lookup_map(const uint32_t (*idx)[3], int n, const uint32_t* data, uint32_t cp,
               const uint32_t** out) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < idx[mid][0]) hi = mid - 1;
    else if (cp > idx[mid][0]) lo = mid + 1;
    else { *out = data + idx[mid][1]; return (int)idx[mid][2]; }
  }
  return -1;
}

bool is_whitespace(uint32_t c) {
  if (c == ' ' || c == '\t' || c == '\n' || c == '\r') return true;
  return in_ranges(hcr_uni::kSpaceZs, hcr_uni::kSpaceZsN, c);
}
bool is_control(uint32_t c) {
  if (c == '\t' || c == '\n' || c == '\r') return false;
  return in_ranges(hcr_uni::kControl, hcr_uni::kControlN, c);
}
bool is_punct(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126))
    return true;
  return in_ranges(hcr_uni::kPunct, hcr_uni::kPunctN, c);
}
bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) ||
         (c >= 0x20000 && c <= 0x2A6DF) || (c >= 0x2A700 && c <= 0x2B73F) ||
         (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B820 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

// UTF-8 decode (invalid bytes -> U+FFFD, which clean_text then drops, as Python's
// errors="replace" decoding followed by BasicTokenizer would)
void utf8_decode(const char* s, size_t n, std::vector<uint32_t>& out) {
  size_t i = 0;
  while (i < n) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp = 0xFFFD;
    int len = 1;
    if (c < 0x80) { cp = c; }
    else if ((c >> 5) == 6 && i + 1 < n) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); len = 2; }
    else if ((c >> 4) == 14 && i + 2 < n) {
      cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); len = 3;
    } else if ((c >> 3) == 30 && i + 3 < n) {
      cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
      len = 4;
    }
    out.push_back(cp);
    i += len;
  }
}
void utf8_append(std::string& s, uint32_t cp) {
  if (cp < 0x80) s += (char)cp;
  else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) {
    s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
  } else {
    s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 0x3F));
    s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
  }
}

}  // namespace

struct hcr_tok {
  std::unordered_map<std::string, int32_t> vocab;
  int32_t cls = -1, sep = -1, pad = 0, unk = -1;
  bool lower = true, strip = true;
  int max_chars_per_word = 100;

  // BasicTokenizer: text -> list of words (code point vectors)
  void basic(const std::string& text, std::vector<std::vector<uint32_t>>& words) const {
    std::vector<uint32_t> cps;
    utf8_decode(text.data(), text.size(), cps);
    std::vector<uint32_t> clean;
    clean.reserve(cps.size() + 8);
    for (uint32_t c : cps) {          // _clean_text + _tokenize_chinese_chars
      if (c == 0 || c == 0xFFFD || is_control(c)) continue;
      if (is_whitespace(c)) { clean.push_back(' '); continue; }
      if (is_cjk(c)) { clean.push_back(' '); clean.push_back(c); clean.push_back(' '); continue; }
      clean.push_back(c);
    }
    std::vector<uint32_t> tok;
    auto flush_token = [&]() {
      if (tok.empty()) return;
      std::vector<uint32_t> t = tok, t2;
      if (lower) {
        t2.clear();
        for (uint32_t c : t) {
          const uint32_t* m;
          const int k = lookup_map(hcr_uni::kLowerIdx, hcr_uni::kLowerN, hcr_uni::kLowerData, c, &m);
          if (k >= 0) t2.insert(t2.end(), m, m + k); else t2.push_back(c);
        }
        t.swap(t2);
      }
      if (strip) {
        t2.clear();
        for (uint32_t c : t) {
          const uint32_t* m;
          const int k = lookup_map(hcr_uni::kStripIdx, hcr_uni::kStripN, hcr_uni::kStripData, c, &m);
          if (k >= 0) t2.insert(t2.end(), m, m + k); else t2.push_back(c);
        }
        t.swap(t2);
      }
      // _run_split_on_punc
      std::vector<uint32_t> cur;
      for (uint32_t c : t) {
        if (is_punct(c)) {
          if (!cur.empty()) { words.push_back(cur); cur.clear(); }
          words.push_back(std::vector<uint32_t>{c});
        } else {
          cur.push_back(c);
        }
      }
      if (!cur.empty()) words.push_back(cur);
      tok.clear();
    };
    for (uint32_t c : clean) {
      if (c == ' ') flush_token(); else tok.push_back(c);
    }
    flush_token();
    // a lone combining mark left after stripping yields an empty word: drop empties
    words.erase(std::remove_if(words.begin(), words.end(),
                               [](const std::vector<uint32_t>& w) { return w.empty(); }),
                words.end());
  }

  void wordpiece(const std::vector<uint32_t>& w, std::vector<int32_t>& ids) const {
    if ((int)w.size() > max_chars_per_word) { ids.push_back(unk); return; }
    std::vector<int32_t> sub;
    size_t start = 0;
    std::string piece;
    while (start < w.size()) {
      size_t end = w.size();
      int32_t found = -1;
      while (start < end) {
        piece.clear();
        if (start > 0) piece = "##";
        for (size_t i = start; i < end; ++i) utf8_append(piece, w[i]);
        auto it = vocab.find(piece);
        if (it != vocab.end()) { found = it->second; break; }
        --end;
      }
      if (found < 0) { ids.push_back(unk); return; }
      sub.push_back(found);
      start = end;
    }
    ids.insert(ids.end(), sub.begin(), sub.end());
  }
};

static int load_vocab(hcr_tok* t, std::istream& in) {
  std::string line;
  int32_t id = 0;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    // transformers load_vocab: token = line.rstrip("\n"); duplicates keep the last id
    t->vocab[line] = id++;
  }
  auto get = [&](const char* s) { auto it = t->vocab.find(s); return it == t->vocab.end() ? -1 : it->second; };
  t->cls = get("[CLS]"); t->sep = get("[SEP]"); t->unk = get("[UNK]");
  const int32_t p = get("[PAD]");
  t->pad = p < 0 ? 0 : p;
  if (t->cls < 0 || t->sep < 0 || t->unk < 0) return -1;
  return 0;
}

extern "C" int hcr_wordpiece_create(const char* vocab_path, int lowercase, int strip_accents,
                                    hcr_tok** out) {
  if (!out || !vocab_path) return hcr_set_error(HCR_EINVAL, "NULL argument");
  *out = nullptr;
  std::ifstream f(vocab_path);
  if (!f) return hcr_set_error(HCR_EIO, (std::string("cannot open vocab ") + vocab_path).c_str());
  hcr_tok* t = new hcr_tok();
  t->lower = lowercase != 0;
  t->strip = strip_accents < 0 ? t->lower : strip_accents != 0;   // BERT: strip follows lower
  if (load_vocab(t, f) != 0) {
    delete t;
    return hcr_set_error(HCR_EIO, "vocab lacks [CLS]/[SEP]/[UNK]");
  }
  *out = t;
  return HCR_OK;
}

extern "C" int hcr_wordpiece_create_from_buffer(const char* data, int64_t len, int lowercase,
                                                int strip_accents, hcr_tok** out) {
  if (!out || !data || len < 0) return hcr_set_error(HCR_EINVAL, "NULL argument");
  *out = nullptr;
  std::istringstream in(std::string(data, (size_t)len));
  hcr_tok* t = new hcr_tok();
  t->lower = lowercase != 0;
  t->strip = strip_accents < 0 ? t->lower : strip_accents != 0;
  if (load_vocab(t, in) != 0) {
    delete t;
    return hcr_set_error(HCR_EIO, "vocab lacks [CLS]/[SEP]/[UNK]");
  }
  *out = t;
  return HCR_OK;
}

extern "C" int hcr_wordpiece_destroy(hcr_tok* t) {
  delete t;
  return HCR_OK;
}

extern "C" int32_t hcr_wordpiece_vocab_size(const hcr_tok* t) { return t ? (int32_t)t->vocab.size() : -1; }

extern "C" int hcr_tokenize(const hcr_tok* t, const char* const* texts, const int64_t* text_lens,
                            int64_t n, int max_len, int32_t* ids, int32_t* mask,
                            int32_t* lengths) {
  if (!t) return hcr_set_error(HCR_EINVAL, "tokenizer is NULL");
  if (n < 0 || max_len < 2) return hcr_set_error(HCR_EINVAL, "need n >= 0 and max_len >= 2");
  if (n == 0) return HCR_OK;
  if (!texts || !ids || !mask || !lengths) return hcr_set_error(HCR_EINVAL, "NULL buffer");
  std::vector<std::vector<uint32_t>> words;
  std::vector<int32_t> toks;
  for (int64_t r = 0; r < n; ++r) {
    words.clear();
    toks.clear();
    const char* tx = texts[r];
    const size_t tl = !tx ? 0 : (text_lens ? (size_t)text_lens[r] : strlen(tx));
    t->basic(tx ? std::string(tx, tl) : std::string(), words);
    for (const auto& w : words) {
      t->wordpiece(w, toks);
      if ((int)toks.size() >= max_len - 2) break;   // truncation (tokens past it are dropped)
    }
    const int keep = std::min<int>((int)toks.size(), max_len - 2);
    int32_t* row = ids + r * max_len;
    int32_t* mrow = mask + r * max_len;
    row[0] = t->cls;
    for (int i = 0; i < keep; ++i) row[1 + i] = toks[i];
    row[1 + keep] = t->sep;
    const int L = keep + 2;
    for (int i = 0; i < max_len; ++i) mrow[i] = i < L ? 1 : 0;
    for (int i = L; i < max_len; ++i) row[i] = t->pad;
    lengths[r] = L;
  }
  return HCR_OK;
}
