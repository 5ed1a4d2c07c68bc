// encoder.hip — host side of the BERT sentence-embedding C ABI (include/hcrag.h).
//
// Replaces SentenceTransformer('all-MiniLM-L6-v2').encode(...) (experiments/
// embedding_generator.py:21,124,197,337; experiments/main.py:807,869) and
// HuggingFaceEmbedding(model_name=...) (graph_builder.py:146-149, query_interface.py:136-137):
// BertModel forward (transformers modeling_bert: embeddings -> N x [self-attention ->
// dense+residual+LayerNorm -> dense+GELU -> dense+residual+LayerNorm]) followed by the
// sentence-transformers Pooling (mean over the attention mask, or CLS) and Normalize.
//
// Compute modes (hcr_encoder_create's compute_dtype):
//   HCR_F16 / HCR_BF16  fast: MFMA operands in f16 / bf16, fp32 accumulation, LayerNorm,
//                       softmax and residual stream;
//   HCR_F32             reference precision (the reference encodes in fp32 torch,
//                       experiments/embedding_generator.py:124): every projection GEMM as the
//                       three-term split-f16 product on the same MFMA kernel (~22-bit operands,
//                       fp32 accumulation), fp32 attention, library erff / expf.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "encoder_kernels.h"
#include "gemm_v4.h"
#define HCR_TOPK_TEMPLATES_ONLY   // (gemm_ws.h reaches topk_kernels.h: its kernels live in hcrag_index.hip)
#include "gemm_ws.h"
#include "hcrag.h"
#include "host_common.h"

using namespace hcr;

struct EncLayer {
  DevBuf wqkv, bqkv, wo, bo, ln1g, ln1b, wi, bi, wo2, bo2, ln2g, ln2b;
  // GEMM output scales (reference-precision mode: undo the weights' power-of-two scale and
  // the split's 2^11; 1 in the fast modes)
  float sqkv = 1.f, so = 1.f, si = 1.f, so2 = 1.f;
};

// One sub-batch's activations and the stream its layers run on (hcr_encode_device splits a
// batch over kEncSplits streams: the GEMMs' partly filled last rounds of one sub-batch are then
// filled by the other's workgroups).
struct EncWork {
  DevBuf x, xh, qkv, ctx, inter, y;
  DevBuf pk_off, pk_map, pk_ok, pk_tot;   // token packing (pack_tokens_kernel)
  DevBuf split_ws, split_cnt;             // split GEMM last-round K-split: chunk slabs and a
                                          // ticket counter per tile (zeroed once, reset by use)
  hipStream_t st = nullptr;               // (split sub-batches only; the first runs unsplit
  hipEvent_t done = nullptr;              //  batches on the caller's stream)
  bool whole_tiles = false;               // split GEMM in whole-tile rounds only: set when the
                                          // other sub-batch's stream fills the partly filled
                                          // last rounds (reference-precision mode, r06)
  void release() {
    DevBuf* b[] = {&x, &xh, &qkv, &ctx, &inter, &y, &pk_off, &pk_map, &pk_ok, &pk_tot, &split_ws, &split_cnt};
    for (DevBuf* d : b) d->release();
  }
};
static constexpr int kEncSplits = 2;
// reference-precision default (HCRAG_ENC_STREAMS overrides): two sub-batches on two streams with
// whole-tile GEMM rounds, each stream's partly filled last rounds filled by the other's
// workgroups instead of K-split -- r06 A/B with DM 4: 13.83 -> 13.06 ms per 1024 x 32 batch
// (r04a measured the split slower, before the K-split remainder and with it on)
static constexpr int kF32Streams = 2;
static constexpr int64_t kEncSplitMinSeqs = 128;   // smaller batches run on one stream

struct hcr_encoder {
  int device = 0;
  hcr_bert_config cfg{};
  int dtype = HCR_F16;           // HCR_F16 / HCR_BF16 (fast) or HCR_F32 (split-f16 reference precision)
  hipStream_t stream = nullptr;
  std::map<std::string, std::vector<float>> host;   // weights until finalize
  bool ready = false;
  DevBuf wemb, pemb, temb, embg, embb;
  std::vector<EncLayer> layers;
  // workspace
  DevBuf ids, mask, out;
  EncWork work[kEncSplits];
  hipEvent_t ev_in = nullptr;             // the caller's stream reached the batch
  size_t att_lds_limit = 64 * 1024;
  int ncu = 256;                          // compute units (stream-K grid of the split GEMM)
};

static int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Test hooks (read once): HCRAG_GEMM_FT=256|192 forces the GEMM feature tile; HCRAG_LN_SCALAR
// forces the scalar LayerNorm kernels (used for widths the vectorised ones do not cover);
// HCRAG_ENC_NO_WS keeps the fast modes' QKV / FFN1 projections on gemm_v4 (A/B of gemm_ws).
// HCRAG_ENC_PADDED runs every token position, padding included (A/B and parity of the packing).
// HCRAG_SPLIT_NONE=1: the split GEMM in whole-tile rounds only (no K-split of the last round;
// A/B and bit-identity tests of the other paths).
// HCRAG_ENC_STREAMS=1: one stream per batch (no sub-batch split; A/B of the split).
// HCRAG_SPLIT_DM=0|4: the split GEMM's stage pipeline (gemm_split_kernel's DM; A/B; default 4).
// HCRAG_LN_WITHX=1: the reference-precision LayerNorms also write the fp32 residual stream x
// (r06 default: only the split activations xh, from which the O / FFN2 epilogues read the
// residual as h + l 2^-11 -- one 4-byte-per-element write less per LayerNorm; the last layer's
// second LayerNorm writes x for the pooling either way).
struct EncHooks { int gemm_ft = 0; bool ln_scalar = false, gelu_liberf = false, no_ws = false, padded = false,
                  no_split = false, ln_withx = false; int streams = 0; int split_dm = -1; };
static const EncHooks& enc_hooks() {
  static const EncHooks h = [] {
    EncHooks t;
    if (const char* e = getenv("HCRAG_GEMM_FT")) t.gemm_ft = atoi(e);
    t.ln_scalar = getenv("HCRAG_LN_SCALAR") != nullptr;
    // reference-precision FFN1 GELU with the library erff instead of erf_as
    t.gelu_liberf = getenv("HCRAG_GELU_LIBERF") != nullptr;
    t.no_ws = getenv("HCRAG_ENC_NO_WS") != nullptr;
    t.padded = getenv("HCRAG_ENC_PADDED") != nullptr;
    t.no_split = getenv("HCRAG_SPLIT_NONE") != nullptr;
    if (const char* v = getenv("HCRAG_ENC_STREAMS")) t.streams = atoi(v);
    if (const char* v = getenv("HCRAG_SPLIT_DM")) t.split_dm = atoi(v);
    t.ln_withx = getenv("HCRAG_LN_WITHX") != nullptr;
    return t;
  }();
  return h;
}

extern "C" int hcr_encoder_create(int device, const hcr_bert_config* cfg, int compute_dtype,
                                  hcr_encoder** out) {
  if (!out || !cfg) return hcr_set_error(HCR_EINVAL, "NULL argument");
  *out = nullptr;
  const hcr_bert_config& c = *cfg;
  if (c.hidden <= 0 || c.hidden % 64 || c.hidden > 4096)
    return hcr_set_errorf(HCR_EINVAL, "hidden must be a positive multiple of 64 (<= 4096), got %d", c.hidden);
  if (c.heads <= 0 || c.hidden % c.heads) return hcr_set_error(HCR_EINVAL, "hidden % heads != 0");
  if (c.intermediate <= 0 || c.intermediate % 64) return hcr_set_error(HCR_EINVAL, "intermediate must be a multiple of 64");
  if (c.layers <= 0 || c.vocab_size <= 0 || c.max_position <= 0 || c.type_vocab <= 0)
    return hcr_set_error(HCR_EINVAL, "bad config sizes");
  if (c.pooling != 0 && c.pooling != 1) return hcr_set_error(HCR_EINVAL, "pooling must be 0 (mean) or 1 (cls)");
  if (compute_dtype != HCR_F16 && compute_dtype != HCR_BF16 && compute_dtype != HCR_F32)
    return hcr_set_error(HCR_EINVAL, "compute dtype must be HCR_F16, HCR_BF16 or HCR_F32");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (device < 0 || device >= ndev)
    return hcr_set_errorf(HCR_EINVAL, "device %d not available (%d HIP devices)", device, ndev);
  HIPC(hipSetDevice(device));
  hcr_encoder* e = new hcr_encoder();
  e->device = device;
  e->cfg = c;
  e->dtype = compute_dtype;
  if (hipDeviceGetAttribute(&e->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || e->ncu <= 0)
    e->ncu = 256;
  hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (he != hipSuccess) {
    delete e;
    return hcr_set_errorf(HCR_EHIP, "hipStreamCreate: %s", hipGetErrorString(he));
  }
  *out = e;
  return HCR_OK;
}

extern "C" int hcr_encoder_destroy(hcr_encoder* e) {
  if (!e) return HCR_OK;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  DevBuf* bufs[] = {&e->wemb, &e->pemb, &e->temb, &e->embg, &e->embb, &e->ids, &e->mask, &e->out};
  for (DevBuf* b : bufs) b->release();
  for (EncWork& w : e->work) {
    if (w.st) (void)hipStreamSynchronize(w.st);
    w.release();
    if (w.done) (void)hipEventDestroy(w.done);
    if (w.st) (void)hipStreamDestroy(w.st);
  }
  if (e->ev_in) (void)hipEventDestroy(e->ev_in);
  for (auto& L : e->layers) {
    DevBuf* lb[] = {&L.wqkv, &L.bqkv, &L.wo, &L.bo, &L.ln1g, &L.ln1b, &L.wi, &L.bi, &L.wo2, &L.bo2, &L.ln2g, &L.ln2b};
    for (DevBuf* b : lb) b->release();
  }
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return HCR_OK;
}

extern "C" int hcr_encoder_compute_dtype(const hcr_encoder* e) { return e ? e->dtype : -1; }

// HF BertModel state-dict name, any prefix before "embeddings." / "encoder." is ignored
// (sentence-transformers checkpoints use "0.auto_model." or none; BertForX uses "bert.").
extern "C" int hcr_encoder_set_weight(hcr_encoder* e, const char* name, const float* data,
                                      int64_t numel) {
  if (!e || !name || (!data && numel > 0) || numel < 0) return hcr_set_error(HCR_EINVAL, "bad argument");
  std::string n(name);
  size_t p = n.find("embeddings.");
  size_t q = n.find("encoder.");
  if (q != std::string::npos && (p == std::string::npos || q < p)) p = q;
  if (p == std::string::npos) return HCR_OK;    // pooler / heads: not used by the path
  n = n.substr(p);
  e->host[n].assign(data, data + numel);
  e->ready = false;
  return HCR_OK;
}

// Projection weights [rows][cols] fp32 -> device, rows padded with zeros to rows_pad.
// Fast modes: MFMA dtype [rows_pad][cols].  Reference-precision mode: split f16
// [rows_pad][3 cols] scaled by a power of two (max |W| -> ~16); *oscale receives the factor
// that the GEMM epilogue applies.
template <typename TM, bool SPLIT>
static int upload_weights(DevBuf& dst, const std::vector<float>& src, int64_t rows, int64_t cols,
                          int64_t rows_pad, float* oscale, hipStream_t st) {
  const int w = SPLIT ? 3 : 1;
  CHECK(dst.ensure((size_t)rows_pad * cols * w * sizeof(TM)));
  DevBuf tmp;
  CHECK(tmp.ensure((size_t)rows * cols * 4));
  HIPC(hipMemcpyAsync(tmp.p, src.data(), (size_t)rows * cols * 4, hipMemcpyHostToDevice, st));
  const int64_t tot = rows_pad * cols;
  const dim3 grid((unsigned)((tot + 255) / 256));
  if constexpr (SPLIT) {
    float mx = 0.f;
    for (size_t i = 0; i < (size_t)(rows * cols); ++i) mx = std::max(mx, std::fabs(src[i]));
    const int e2 = mx > 0.f ? (int)std::floor(std::log2(16.0 / mx)) : 0;
    const float scale = std::ldexp(1.f, e2);
    hipLaunchKernelGGL(to_split_weights, grid, dim3(256), 0, st, tmp.as<const float>(), rows,
                       rows_pad, (int)cols, scale, dst.as<_Float16>());
    *oscale = 1.f / (scale * kSplitLo);
  } else {
    hipLaunchKernelGGL((to_mfma_dtype<TM>), grid, dim3(256), 0, st, tmp.as<const float>(), rows,
                       rows_pad, (int)cols, dst.as<TM>());
    *oscale = 1.f;
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(st));
  tmp.release();
  return HCR_OK;
}

static int upload_f32(DevBuf& dst, const float* src, size_t n, size_t n_pad, hipStream_t st) {
  CHECK(dst.ensure(n_pad * 4));
  HIPC(hipMemsetAsync(dst.p, 0, n_pad * 4, st));
  HIPC(hipMemcpyAsync(dst.p, src, n * 4, hipMemcpyHostToDevice, st));
  return HCR_OK;
}

template <typename TM, bool SPLIT>
static int finalize_t(hcr_encoder* e) {
  const auto& c = e->cfg;
  const int H = c.hidden, F = c.intermediate;
  auto need = [&](const std::string& n, size_t numel, const std::vector<float>** out) -> int {
    auto it = e->host.find(n);
    if (it == e->host.end()) return hcr_set_errorf(HCR_EINVAL, "missing weight %s", n.c_str());
    if (it->second.size() != numel)
      return hcr_set_errorf(HCR_EINVAL, "weight %s has %zu elements, expected %zu", n.c_str(),
                            it->second.size(), numel);
    *out = &it->second;
    return HCR_OK;
  };
  const std::vector<float> *we, *pe, *te, *eg, *eb;
  CHECK(need("embeddings.word_embeddings.weight", (size_t)c.vocab_size * H, &we));
  CHECK(need("embeddings.position_embeddings.weight", (size_t)c.max_position * H, &pe));
  CHECK(need("embeddings.token_type_embeddings.weight", (size_t)c.type_vocab * H, &te));
  CHECK(need("embeddings.LayerNorm.weight", H, &eg));
  CHECK(need("embeddings.LayerNorm.bias", H, &eb));
  hipStream_t st = e->stream;
  CHECK(upload_f32(e->wemb, we->data(), we->size(), we->size(), st));
  CHECK(upload_f32(e->pemb, pe->data(), pe->size(), pe->size(), st));
  CHECK(upload_f32(e->temb, te->data(), te->size(), te->size(), st));
  CHECK(upload_f32(e->embg, eg->data(), H, H, st));
  CHECK(upload_f32(e->embb, eb->data(), H, H, st));
  e->layers.clear();
  e->layers.resize(c.layers);
  for (int l = 0; l < c.layers; ++l) {
    const std::string pfx = "encoder.layer." + std::to_string(l) + ".";
    const std::vector<float> *wq, *bq, *wk, *bk, *wv, *bv, *wo, *bo, *g1, *b1, *wi, *bi, *wo2, *bo2, *g2, *b2;
    CHECK(need(pfx + "attention.self.query.weight", (size_t)H * H, &wq));
    CHECK(need(pfx + "attention.self.query.bias", H, &bq));
    CHECK(need(pfx + "attention.self.key.weight", (size_t)H * H, &wk));
    CHECK(need(pfx + "attention.self.key.bias", H, &bk));
    CHECK(need(pfx + "attention.self.value.weight", (size_t)H * H, &wv));
    CHECK(need(pfx + "attention.self.value.bias", H, &bv));
    CHECK(need(pfx + "attention.output.dense.weight", (size_t)H * H, &wo));
    CHECK(need(pfx + "attention.output.dense.bias", H, &bo));
    CHECK(need(pfx + "attention.output.LayerNorm.weight", H, &g1));
    CHECK(need(pfx + "attention.output.LayerNorm.bias", H, &b1));
    CHECK(need(pfx + "intermediate.dense.weight", (size_t)F * H, &wi));
    CHECK(need(pfx + "intermediate.dense.bias", F, &bi));
    CHECK(need(pfx + "output.dense.weight", (size_t)H * F, &wo2));
    CHECK(need(pfx + "output.dense.bias", H, &bo2));
    CHECK(need(pfx + "output.LayerNorm.weight", H, &g2));
    CHECK(need(pfx + "output.LayerNorm.bias", H, &b2));
    EncLayer& L = e->layers[l];
    std::vector<float> wqkv((size_t)3 * H * H), bqkv((size_t)3 * H);
    std::memcpy(wqkv.data(), wq->data(), (size_t)H * H * 4);
    std::memcpy(wqkv.data() + (size_t)H * H, wk->data(), (size_t)H * H * 4);
    std::memcpy(wqkv.data() + (size_t)2 * H * H, wv->data(), (size_t)H * H * 4);
    std::memcpy(bqkv.data(), bq->data(), H * 4);
    std::memcpy(bqkv.data() + H, bk->data(), H * 4);
    std::memcpy(bqkv.data() + 2 * H, bv->data(), H * 4);
    CHECK((upload_weights<TM, SPLIT>(L.wqkv, wqkv, 3 * H, H, rup(3 * H, 768), &L.sqkv, st)));
    CHECK(upload_f32(L.bqkv, bqkv.data(), 3 * H, rup(3 * H, 768), st));
    CHECK((upload_weights<TM, SPLIT>(L.wo, *wo, H, H, rup(H, 768), &L.so, st)));
    CHECK(upload_f32(L.bo, bo->data(), H, rup(H, 768), st));
    CHECK(upload_f32(L.ln1g, g1->data(), H, H, st));
    CHECK(upload_f32(L.ln1b, b1->data(), H, H, st));
    CHECK((upload_weights<TM, SPLIT>(L.wi, *wi, F, H, rup(F, 768), &L.si, st)));
    CHECK(upload_f32(L.bi, bi->data(), F, rup(F, 768), st));
    CHECK((upload_weights<TM, SPLIT>(L.wo2, *wo2, H, F, rup(H, 768), &L.so2, st)));
    CHECK(upload_f32(L.bo2, bo2->data(), H, rup(H, 768), st));
    CHECK(upload_f32(L.ln2g, g2->data(), H, H, st));
    CHECK(upload_f32(L.ln2b, b2->data(), H, H, st));
  }
  HIPC(hipStreamSynchronize(st));
  return HCR_OK;
}

extern "C" int hcr_encoder_finalize(hcr_encoder* e) {
  if (!e) return hcr_set_error(HCR_EINVAL, "encoder is NULL");
  HIPC(hipSetDevice(e->device));
  int rc = e->dtype == HCR_F16    ? finalize_t<_Float16, false>(e)
           : e->dtype == HCR_BF16 ? finalize_t<__bf16, false>(e)
                                  : finalize_t<_Float16, true>(e);
  if (rc != HCR_OK) return rc;
  e->host.clear();
  e->ready = true;
  return HCR_OK;
}

// C = oscale * X . W^T + bias (+ epilogue) on the LDS-DMA ring GEMM (gemm_v4.h).  K is the
// operand row length (3 x the model width in the reference-precision mode).
// The weight-stationary GEMM (gemm_ws.h) for 16-bit outputs at K = 384 / 768: nft 256-feature
// tiles x P token partitions filling one round of 256 workgroups (one per CU: its LDS).
template <typename TM, int EPI, int KS>
static void launch_ws_ks(const TM* W, const TM* X, int K, int N, int T, const float* bias, TM* out_h,
                         int ldo, float oscale, hipStream_t st) {
  const int sr = ws_sr(KS);
  const int ntiles = (int)(rup(T, 256) / sr);
  const int nft = (int)(rup(N, WS_FT) / WS_FT);
  const int P = std::max(1, std::min(ntiles, 256 / nft));
  hipLaunchKernelGGL((gemm_ws_kernel<TM, EPI, KS>), dim3((unsigned)(nft * P)), dim3(V3_NT), 0, st, W, X, K, N,
                     T, nft, P, ntiles, bias, out_h, ldo, oscale);
}
template <typename TM, int EPI>
static bool launch_ws(const TM* W, const TM* X, int K, int N, int T, const float* bias, TM* out_h, int ldo,
                      float oscale, hipStream_t st) {
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
    if (enc_hooks().no_ws || N > 256 * 64) return false;
    if (K == 768) { launch_ws_ks<TM, EPI, 24>(W, X, K, N, T, bias, out_h, ldo, oscale, st); return true; }
    if (K == 384) { launch_ws_ks<TM, EPI, 12>(W, X, K, N, T, bias, out_h, ldo, oscale, st); return true; }
  }
  return false;
}

template <typename TM, int EPI>
static int launch_gemm(const TM* W, const TM* X, int K, int N, int T, const float* bias,
                       const float* resid, TM* out_h, float* out_f, int ldo, float oscale,
                       hipStream_t st) {
  if (K % V3_BK) return hcr_set_errorf(HCR_EINVAL, "internal: GEMM K=%d not a multiple of %d", K, V3_BK);
  if (N % 8) return hcr_set_errorf(HCR_EINVAL, "internal: GEMM N=%d not a multiple of 8", N);
  if (launch_ws<TM, EPI>(W, X, K, N, T, bias, out_h, ldo, oscale, st)) {
    HIPC(hipGetLastError());
    return HCR_OK;
  }
  // feature tile: 192 when it fills the last round of 256-CU workgroups better than 256
  // (N = 768 at T = 32768: 512 tiles = 2 full rounds vs 384 = 1.5); weights are padded to
  // a multiple of 768 rows so either tile reads whole rows.
  const int ntt = (int)(rup(T, G4_T) / G4_T);
  auto rounds = [&](int ft) {            // rounds of 256 resident workgroups
    const int64_t tiles = rup(N, ft) / ft * (int64_t)ntt;
    return (double)((tiles + 255) / 256);
  };
  // a 192-feature tile takes ~0.94x the time of a 256-feature one (r01c: QKV 183 vs 163 us
  // at 6 vs 5 rounds), not 0.75x: it pays only where it removes a mostly-empty round
  const int force_ft = enc_hooks().gemm_ft;
  const bool ft192 = force_ft ? force_ft == 192 : (rounds(192) * 0.94 < rounds(256));
  if (ft192) {
    const int nft = (int)(rup(N, 192) / 192);
    hipLaunchKernelGGL((gemm_v4_kernel<TM, EPI, 4, 192>), dim3((unsigned)(nft * ntt)), dim3(V3_NT),
                       0, st, W, X, K, N, T, nft, bias, resid, out_h, out_f, ldo, oscale);
  } else {
    const int nft = (int)(rup(N, G4_T) / G4_T);
    hipLaunchKernelGGL((gemm_v4_kernel<TM, EPI, 4, 256>), dim3((unsigned)(nft * ntt)), dim3(V3_NT),
                       0, st, W, X, K, N, T, nft, bias, resid, out_h, out_f, ldo, oscale);
  }
  HIPC(hipGetLastError());
  return HCR_OK;
}

// Reference-precision projection: C = oscale * (Xh.Wh 2^11 + Xh.Wl 2^11 + Xl 2^11.Wh) + bias (+
// epilogue) from the split operands (row length 3 K), on gemm_split_kernel (4 distinct tiles
// per stage instead of the concatenated GEMM's 6).  Weights are padded to 768-row multiples (a
// whole number of 256- or 192-feature tiles), T padded to 256.
//
// Decomposition: whole 256- or 192-feature x 256-token tiles in rounds of one workgroup per CU
// (the LDS ring holds one per CU), then the R tiles of a partly filled last round split into s
// K-chunks each (s = ncu / R, <= 8, one round; gemm_split_kernel<SPLIT>).  The width and the
// split are chosen by estimated time: tile-times per CU (a 192-wide tile costs 0.86 of a 256
// one: r04n whole-tile traces, 51.8 vs 60 us at K = 768; r02: 0.86) plus the split launch's
// overhead over its chunks' MFMA time (slab stores, the last arriver reading s 256-KiB slabs:
// ~9 + 4.3 s us, r04q traces: 17 us at s = 2, 43 at s = 8).  Measured (r04q, one box, A/B):
// f32 encoder 67.1k -> 69.8k embeddings/s, f32 query pipeline 36.1k -> 36.7k queries/s.
// Stream-K over a linear (tile, k) order was built
// first and measured neutral to negative (r04n/r04o): its split ranges put the
// workgroups that share a token tile's activations at different K offsets.
struct SplitPlan { int ft, nft, full, rem, nsplit; };
static constexpr int kSplitDM = 4;     // gemm_split_kernel's default stage pipeline (r06 A/B)
static SplitPlan split_plan(int N, int K, int T, int ncu, bool can192, int force_ft, bool split_on) {
  const int ntt = (int)(rup(T, G4_T) / G4_T);
  const int nsteps = K / V3_BK;
  const double t256 = 60.0 * K / 768.0;                  // us per 256-wide tile round
  SplitPlan best{};
  double best_us = 1e30;
  // (a forced width the epilogue cannot take -- 192 for FFN1 -- falls back to 256)
  const int forced = (force_ft == 192 && !can192) ? G4_T : force_ft;
  for (int ft : {192, G4_T}) {
    if (ft == 192 && !can192) continue;
    if (forced && ft != forced) continue;
    SplitPlan p{};
    p.ft = ft;
    p.nft = (int)(rup(N, ft) / ft);
    const int nt = p.nft * ntt;
    p.full = nt / ncu * ncu;
    p.rem = nt - p.full;
    p.nsplit = p.rem ? std::min({ncu / p.rem, nsteps, 8}) : 0;
    const double w = ft == 192 ? 0.86 : 1.0;
    double us;
    if (!split_on || p.nsplit < 2) {
      p.full = nt; p.rem = 0; p.nsplit = 0;
      us = (double)((nt + ncu - 1) / ncu) * w * t256;
    } else {
      us = ((double)(p.full / ncu) + 1.0 / p.nsplit) * w * t256 + 9.0 + 4.3 * p.nsplit;
    }
    if (us < best_us) { best_us = us; best = p; }
  }
  return best;
}

template <int EPI>
static int launch_gemm_split(EncWork& w, int ncu, const _Float16* W, const _Float16* X, int K, int N, int T,
                             const float* bias, const float* resid, _Float16* out_h, float* out_f,
                             int ldo, float oscale, hipStream_t st) {
  if (K % V3_BK) return hcr_set_errorf(HCR_EINVAL, "internal: GEMM K=%d not a multiple of %d", K, V3_BK);
  if (N % 8) return hcr_set_errorf(HCR_EINVAL, "internal: GEMM N=%d not a multiple of 8", N);
  // (FFN1's epilogue stages 64-feature halves: 256-feature tiles only)
  constexpr bool can192 = EPI != EPI_BIAS_GELU_SPLIT;
  const SplitPlan p = split_plan(N, K, T, ncu, can192, enc_hooks().gemm_ft, !enc_hooks().no_split && !w.whole_tiles);
  float* ws = nullptr;
  uint32_t* cnt = nullptr;
  if (p.nsplit) {
    // s slabs of a tile's fp32 accumulators per remainder tile (rem x nsplit <= ncu), a counter each
    CHECK(w.split_ws.ensure((size_t)ncu * G4_T * G4_T * 4));
    CHECK(w.split_cnt.ensure((size_t)ncu * 4));
    ws = w.split_ws.as<float>();
    cnt = w.split_cnt.as<uint32_t>();
  }
  const int dm = enc_hooks().split_dm >= 0 ? enc_hooks().split_dm : kSplitDM;
#define HCR_SPLIT_DM(FT_, LIB_, SP_, GRID_, DM_)                                                    \
  hipLaunchKernelGGL((gemm_split_kernel<EPI, FT_, LIB_, SP_, DM_>), dim3((unsigned)(GRID_)), dim3(V3_NT), 0, st, \
                     W, X, K, N, T, p.nft, bias, resid, out_h, out_f, ldo, oscale, p.full, p.nsplit, ws, cnt)
#define HCR_SPLIT(FT_, LIB_, SP_, GRID_)                                                            \
  do {                                                                                              \
    if (dm == 4) HCR_SPLIT_DM(FT_, LIB_, SP_, GRID_, 4);                                            \
    else HCR_SPLIT_DM(FT_, LIB_, SP_, GRID_, 0);                                                    \
  } while (0)
#define HCR_SPLIT_FT(FT_, LIB_)                                                                     \
  do {                                                                                              \
    if (p.full > 0) HCR_SPLIT(FT_, LIB_, false, p.full);                                            \
    if (p.nsplit > 0) HCR_SPLIT(FT_, LIB_, true, p.rem * p.nsplit);                                 \
  } while (0)
  if constexpr (!can192) {
    if (enc_hooks().gelu_liberf) HCR_SPLIT_FT(G4_T, true);
    else HCR_SPLIT_FT(G4_T, false);
  } else if (p.ft == 192) {
    HCR_SPLIT_FT(192, false);
  } else {
    HCR_SPLIT_FT(G4_T, false);
  }
#undef HCR_SPLIT_FT
#undef HCR_SPLIT
#undef HCR_SPLIT_DM
  HIPC(hipGetLastError());
  return HCR_OK;
}

template <typename TM, int DH, int KB>
static int launch_attention_mfma(hcr_encoder* e, EncWork& w, const int32_t* d_mask, const int32_t* seq_off, int64_t n, int S,
                                 hipStream_t st) {
  const size_t lds = attention_mfma_lds<TM, DH>(S);
  if (lds > 64 * 1024)
    HIPC(hipFuncSetAttribute((const void*)attention_mfma_kernel<TM, DH, KB>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipLaunchKernelGGL((attention_mfma_kernel<TM, DH, KB>), dim3((unsigned)(n * e->cfg.heads)),
                     dim3(256), lds, st, w.qkv.as<const TM>(), d_mask, seq_off, S, e->cfg.hidden,
                     e->cfg.heads, w.ctx.as<TM>());
  HIPC(hipGetLastError());
  return HCR_OK;
}

// Fast modes: MFMA attention for head dims 32 / 64 up to 512 keys, the scalar kernel otherwise.
template <typename TM>
static int launch_attention(hcr_encoder* e, EncWork& w, const int32_t* d_mask, const int32_t* seq_off, int64_t n, int S,
                            hipStream_t st) {
  const int dh = e->cfg.hidden / e->cfg.heads;
  const int Sp = (S + 31) & ~31;
  if ((dh == 32 || dh == 64) && Sp <= 512) {
    if (dh == 32) return Sp <= 128 ? launch_attention_mfma<TM, 32, 8>(e, w, d_mask, seq_off, n, S, st)
                                   : launch_attention_mfma<TM, 32, 32>(e, w, d_mask, seq_off, n, S, st);
    return Sp <= 128 ? launch_attention_mfma<TM, 64, 8>(e, w, d_mask, seq_off, n, S, st)
                     : launch_attention_mfma<TM, 64, 32>(e, w, d_mask, seq_off, n, S, st);
  }
  const size_t lds = (size_t)(5 * S + 4 * dh) * 4 + (size_t)2 * S * dh * sizeof(TM);
  if (lds > 160 * 1024) return hcr_set_errorf(HCR_EINVAL, "sequence length %d too long for attention LDS", S);
  if (lds > 64 * 1024)
    HIPC(hipFuncSetAttribute((const void*)attention_kernel<TM>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipLaunchKernelGGL((attention_kernel<TM>), dim3((unsigned)(n * e->cfg.heads)), dim3(256), lds, st,
                     w.qkv.as<const TM>(), d_mask, seq_off, S, e->cfg.hidden, e->cfg.heads, w.ctx.as<TM>());
  HIPC(hipGetLastError());
  return HCR_OK;
}

// Reference-precision mode: fp32 attention, K/V in LDS when the sequence fits.
static int launch_attention_f32(hcr_encoder* e, EncWork& w, const int32_t* d_mask, const int32_t* seq_off, int64_t n, int S,
                                hipStream_t st) {
  const int dh = e->cfg.hidden / e->cfg.heads;
  if (S <= 64 && (dh == 32 || dh == 64)) {      // short sequences: f32 MFMA tiles
    const int nt = (S + 15) / 16;
    const size_t lds = attention_f32_mfma_lds(nt, dh);
    const unsigned grid = (unsigned)(n * e->cfg.heads);
#define HCR_ATT_MFMA(DH_, NT_)                                                                    \
  hipLaunchKernelGGL((attention_f32_mfma_kernel<DH_, NT_>), dim3(grid), dim3(64), lds, st,        \
                     w.qkv.as<const float>(), d_mask, seq_off, S, e->cfg.hidden, e->cfg.heads,            \
                     w.ctx.as<_Float16>())
    if (dh == 64) {
      switch (nt) { case 1: HCR_ATT_MFMA(64, 1); break; case 2: HCR_ATT_MFMA(64, 2); break;
                    case 3: HCR_ATT_MFMA(64, 3); break; default: HCR_ATT_MFMA(64, 4); break; }
    } else {
      switch (nt) { case 1: HCR_ATT_MFMA(32, 1); break; case 2: HCR_ATT_MFMA(32, 2); break;
                    case 3: HCR_ATT_MFMA(32, 3); break; default: HCR_ATT_MFMA(32, 4); break; }
    }
#undef HCR_ATT_MFMA
    HIPC(hipGetLastError());
    return HCR_OK;
  }
  const bool kv_lds = attention_f32_lds(S, dh, true) <= 160 * 1024;
  const size_t lds = attention_f32_lds(S, dh, kv_lds);
  if (lds > 160 * 1024) return hcr_set_errorf(HCR_EINVAL, "sequence length %d too long for attention LDS", S);
  const void* fn = kv_lds ? (const void*)attention_f32_kernel<true> : (const void*)attention_f32_kernel<false>;
  if (lds > 64 * 1024) HIPC(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  if (kv_lds)
    hipLaunchKernelGGL((attention_f32_kernel<true>), dim3((unsigned)(n * e->cfg.heads)), dim3(256), lds, st,
                       w.qkv.as<const float>(), d_mask, seq_off, S, e->cfg.hidden, e->cfg.heads, w.ctx.as<_Float16>());
  else
    hipLaunchKernelGGL((attention_f32_kernel<false>), dim3((unsigned)(n * e->cfg.heads)), dim3(256), lds, st,
                       w.qkv.as<const float>(), d_mask, seq_off, S, e->cfg.hidden, e->cfg.heads, w.ctx.as<_Float16>());
  HIPC(hipGetLastError());
  return HCR_OK;
}

template <typename TM, bool SPLIT>
static int encode_t(hcr_encoder* e, EncWork& w, const int32_t* d_ids, const int32_t* d_mask, int64_t n, int S,
                    float* d_out, hipStream_t st) {
  const auto& c = e->cfg;
  const int H = c.hidden, F = c.intermediate;
  const int aw = SPLIT ? 3 : 1;                       // activation row width factor
  int64_t T = n * (int64_t)S;
  if (T > (int64_t)1 << 30) return hcr_set_error(HCR_EINVAL, "batch too large");
  // Token packing (pack_tokens_kernel): only the tokens the result depends on run through the
  // layers.  The packed row count is read back once (one stream synchronisation per batch):
  // every grid below is sized by it.
  const int32_t* tok_map = nullptr;
  const int32_t* seq_off = nullptr;
  const int32_t* key_mask = d_mask;                   // per-row key bits: padded mask or packed
  if (!enc_hooks().padded) {
    CHECK(w.pk_off.ensure((size_t)(n + 1) * 4));
    CHECK(w.pk_map.ensure((size_t)T * 4));
    CHECK(w.pk_ok.ensure((size_t)T * 4));
    CHECK(w.pk_tot.ensure(4));
    hipLaunchKernelGGL(pack_tokens_kernel, dim3(1), dim3(1024), 0, st, d_mask, n, S, c.pooling == 1 ? 1 : 0,
                       w.pk_off.as<int32_t>(), w.pk_map.as<int32_t>(), w.pk_ok.as<int32_t>(),
                       w.pk_tot.as<int32_t>());
    HIPC(hipGetLastError());
    int32_t tot = 0;
    HIPC(hipMemcpyAsync(&tot, w.pk_tot.p, 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    T = tot;
    tok_map = w.pk_map.as<const int32_t>();
    seq_off = w.pk_off.as<const int32_t>();
    key_mask = w.pk_ok.as<const int32_t>();
  }
  if (T == 0) {                  // no token reaches the output (mean pooling, every mask 0)
    hipLaunchKernelGGL(pool_normalize_kernel, dim3((unsigned)n), dim3(256), 0, st, w.x.as<const float>(),
                       key_mask, seq_off, S, H, c.pooling, c.normalize, d_out);
    HIPC(hipGetLastError());
    return HCR_OK;
  }
  const int64_t Tp = rup(T, 256);
  CHECK(w.x.ensure((size_t)Tp * H * 4));
  CHECK(w.y.ensure((size_t)Tp * H * 4));
  CHECK(w.xh.ensure((size_t)Tp * H * aw * sizeof(TM)));
  CHECK(w.ctx.ensure((size_t)Tp * H * aw * sizeof(TM)));
  CHECK(w.qkv.ensure((size_t)Tp * 3 * H * (SPLIT ? 4 : sizeof(TM))));
  CHECK(w.inter.ensure((size_t)Tp * F * aw * sizeof(TM)));
  const unsigned gT = (unsigned)((T + 3) / 4);
  // vectorised LayerNorm kernels when H % 4 == 0 and H <= 1024 (all BERT widths here)
  const bool ln4 = (H % 4 == 0) && H <= 1024 && !enc_hooks().ln_scalar;
  // reference precision: the residual stream lives in xh only (EPI_BIAS_RESID_XH), x is written
  // by the last LayerNorm for the pooling
  const bool nox = SPLIT && ln4 && !enc_hooks().ln_withx;
  auto layer_norm = [&](const DevBuf& g, const DevBuf& bb, bool last) {
    if (ln4)
      hipLaunchKernelGGL((layernorm4_kernel<TM, SPLIT>), dim3(gT), dim3(256), 0, st, w.y.as<const float>(),
                         (int)T, H, g.as<const float>(), bb.as<const float>(), c.layer_norm_eps,
                         (nox && !last) ? nullptr : w.x.as<float>(), w.xh.as<TM>());
    else
      hipLaunchKernelGGL((layernorm_kernel<TM, SPLIT>), dim3(gT), dim3(256), 0, st, w.y.as<const float>(),
                         (int)T, H, g.as<const float>(), bb.as<const float>(), c.layer_norm_eps,
                         w.x.as<float>(), w.xh.as<TM>());
  };
  if (ln4)
    hipLaunchKernelGGL((embed_ln4_kernel<TM, SPLIT>), dim3(gT), dim3(256), 0, st, d_ids, tok_map, (int)T, S, H,
                       e->wemb.as<const float>(), e->pemb.as<const float>(),
                       e->temb.as<const float>(), e->embg.as<const float>(),
                       e->embb.as<const float>(), c.layer_norm_eps, nox ? nullptr : w.x.as<float>(),
                       w.xh.as<TM>());
  else
    hipLaunchKernelGGL((embed_ln_kernel<TM, SPLIT>), dim3(gT), dim3(256), 0, st, d_ids, tok_map, (int)T, S, H,
                       e->wemb.as<const float>(), e->pemb.as<const float>(),
                       e->temb.as<const float>(), e->embg.as<const float>(),
                       e->embb.as<const float>(), c.layer_norm_eps, w.x.as<float>(), w.xh.as<TM>());
  HIPC(hipGetLastError());
  for (int l = 0; l < c.layers; ++l) {
    const EncLayer& L = e->layers[l];
    if constexpr (SPLIT) {
      CHECK((launch_gemm_split<EPI_BIAS_F32>(w, e->ncu, L.wqkv.as<const _Float16>(), w.xh.as<const _Float16>(), H,
                                             3 * H, (int)T, L.bqkv.as<const float>(), nullptr, nullptr,
                                             w.qkv.as<float>(), 3 * H, L.sqkv, st)));
      CHECK(launch_attention_f32(e, w, key_mask, seq_off, n, S, st));
    } else {
      CHECK((launch_gemm<TM, EPI_BIAS>(L.wqkv.as<const TM>(), w.xh.as<const TM>(), H, 3 * H, (int)T,
                                       L.bqkv.as<const float>(), nullptr, w.qkv.as<TM>(), nullptr,
                                       3 * H, L.sqkv, st)));
      CHECK(launch_attention<TM>(e, w, key_mask, seq_off, n, S, st));
    }
    if constexpr (SPLIT) {
      if (nox)
        CHECK((launch_gemm_split<EPI_BIAS_RESID_XH>(w, e->ncu, L.wo.as<const _Float16>(), w.ctx.as<const _Float16>(), H,
                                                    H, (int)T, L.bo.as<const float>(),
                                                    reinterpret_cast<const float*>(w.xh.p), nullptr, w.y.as<float>(),
                                                    H, L.so, st)));
      else
        CHECK((launch_gemm_split<EPI_BIAS_RESID>(w, e->ncu, L.wo.as<const _Float16>(), w.ctx.as<const _Float16>(), H,
                                                 H, (int)T, L.bo.as<const float>(), w.x.as<const float>(),
                                                 nullptr, w.y.as<float>(), H, L.so, st)));
    }
    else
      CHECK((launch_gemm<TM, EPI_BIAS_RESID>(L.wo.as<const TM>(), w.ctx.as<const TM>(), H, H,
                                             (int)T, L.bo.as<const float>(), w.x.as<const float>(),
                                             nullptr, w.y.as<float>(), H, L.so, st)));
    layer_norm(L.ln1g, L.ln1b, false);
    HIPC(hipGetLastError());
    if constexpr (SPLIT)
      CHECK((launch_gemm_split<EPI_BIAS_GELU_SPLIT>(w, e->ncu, L.wi.as<const _Float16>(), w.xh.as<const _Float16>(),
                                                    H, F, (int)T, L.bi.as<const float>(), nullptr,
                                                    (_Float16*)w.inter.as<TM>(), nullptr, F, L.si, st)));
    else
      CHECK((launch_gemm<TM, EPI_BIAS_GELU>(L.wi.as<const TM>(), w.xh.as<const TM>(), H, F, (int)T,
                                            L.bi.as<const float>(), nullptr, w.inter.as<TM>(),
                                            nullptr, F, L.si, st)));
    if constexpr (SPLIT) {
      if (nox)
        CHECK((launch_gemm_split<EPI_BIAS_RESID_XH>(w, e->ncu, L.wo2.as<const _Float16>(), w.inter.as<const _Float16>(),
                                                    F, H, (int)T, L.bo2.as<const float>(),
                                                    reinterpret_cast<const float*>(w.xh.p), nullptr, w.y.as<float>(),
                                                    H, L.so2, st)));
      else
        CHECK((launch_gemm_split<EPI_BIAS_RESID>(w, e->ncu, L.wo2.as<const _Float16>(), w.inter.as<const _Float16>(), F,
                                                 H, (int)T, L.bo2.as<const float>(), w.x.as<const float>(),
                                                 nullptr, w.y.as<float>(), H, L.so2, st)));
    }
    else
      CHECK((launch_gemm<TM, EPI_BIAS_RESID>(L.wo2.as<const TM>(), w.inter.as<const TM>(), F, H,
                                             (int)T, L.bo2.as<const float>(), w.x.as<const float>(),
                                             nullptr, w.y.as<float>(), H, L.so2, st)));
    layer_norm(L.ln2g, L.ln2b, l == c.layers - 1);
    HIPC(hipGetLastError());
  }
  hipLaunchKernelGGL(pool_normalize_kernel, dim3((unsigned)n), dim3(256), 0, st,
                     w.x.as<const float>(), key_mask, seq_off, S, H, c.pooling, c.normalize, d_out);
  HIPC(hipGetLastError());
  return HCR_OK;
}

extern "C" int hcr_encode_device(hcr_encoder* e, const int32_t* d_ids, const int32_t* d_mask,
                                 int64_t n, int S, float* d_out, void* stream) {
  if (!e) return hcr_set_error(HCR_EINVAL, "encoder is NULL");
  if (!e->ready) return hcr_set_error(HCR_EINVAL, "encoder weights not finalized");
  if (n < 0 || S <= 0) return hcr_set_error(HCR_EINVAL, "need n >= 0 and S > 0");
  if (S > e->cfg.max_position) return hcr_set_errorf(HCR_EINVAL, "S=%d exceeds max_position %d", S, e->cfg.max_position);
  if (n == 0) return HCR_OK;
  if (!d_ids || !d_mask || !d_out) return hcr_set_error(HCR_EINVAL, "NULL buffer");
  HIPC(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;   // the caller's stream (NULL = legacy default)
  auto run = [&](EncWork& w, int64_t s0, int64_t ns, hipStream_t ws) -> int {
    const int32_t* ids = d_ids + s0 * S;
    const int32_t* mask = d_mask + s0 * S;
    float* out = d_out + s0 * e->cfg.hidden;
    if (e->dtype == HCR_F16) return encode_t<_Float16, false>(e, w, ids, mask, ns, S, out, ws);
    if (e->dtype == HCR_BF16) return encode_t<__bf16, false>(e, w, ids, mask, ns, S, out, ws);
    return encode_t<_Float16, true>(e, w, ids, mask, ns, S, out, ws);
  };
  // r04a A/B (bge-base, 1024 x S = 32 ragged, one box): f16 142.3k -> 149.7-152.0k embeddings/s
  // with the split, the f32 mode 66.2k -> 63.9k (its split GEMMs hold 128 KiB of LDS per
  // workgroup and thrash each other's weights): split by default in the fast modes only
  const int want = enc_hooks().streams > 0 ? enc_hooks().streams : (e->dtype == HCR_F32 ? kF32Streams : kEncSplits);
  const int splits = (want <= 1 || n < kEncSplitMinSeqs) ? 1 : kEncSplits;
  for (EncWork& w : e->work) w.whole_tiles = splits > 1 && e->dtype == HCR_F32;
  if (splits == 1) return run(e->work[0], 0, n, st);
  // Sub-batches of n / splits sequences, each on a stream of its own (ordered after the caller's
  // work through ev_in; the caller's stream waits for every sub-batch's `done` event): every
  // kernel of a sub-batch is a small grid whose partly filled last round of workgroups the other
  // sub-batch's kernels fill, instead of leaving CUs idle.  Row-wise work and attention within a
  // sequence do not depend on the split, so the embeddings are the same bits.
  if (!e->ev_in) HIPC(hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming));
  HIPC(hipEventRecord(e->ev_in, st));
  for (int i = 0; i < splits; ++i) {
    EncWork& w = e->work[i];
    if (!w.st) {
      // high-priority streams: the runtime spreads normal-priority streams over its hardware
      // queues (GPU_MAX_HW_QUEUES, 4) by use count, and in a process that already holds other
      // streams both sub-batches can land on one queue and run one after the other (r06h trace
      // of bench.py: both on queue 4, 15.0 ms against 13.1); the high-priority queues are a
      // separate pool that nothing else in the process draws from
      int lo = 0, hi = 0;
      HIPC(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPC(hipStreamCreateWithPriority(&w.st, hipStreamNonBlocking, hi));
    }
    if (!w.done) HIPC(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    HIPC(hipStreamWaitEvent(w.st, e->ev_in, 0));
    const int64_t s0 = n * i / splits, s1 = n * (i + 1) / splits;
    CHECK(run(w, s0, s1 - s0, w.st));
    HIPC(hipEventRecord(w.done, w.st));
  }
  for (int i = 0; i < splits; ++i) HIPC(hipStreamWaitEvent(st, e->work[i].done, 0));
  return HCR_OK;
}

extern "C" int hcr_encode(hcr_encoder* e, const int32_t* ids, const int32_t* mask, int64_t n, int S,
                          float* out) {
  if (!e) return hcr_set_error(HCR_EINVAL, "encoder is NULL");
  if (n == 0) return HCR_OK;
  if (!ids || !mask || !out) return hcr_set_error(HCR_EINVAL, "NULL buffer");
  if (n < 0 || S <= 0) return hcr_set_error(HCR_EINVAL, "need n >= 0 and S > 0");
  HIPC(hipSetDevice(e->device));
  const size_t T = (size_t)n * S;
  CHECK(e->ids.ensure(T * 4));
  CHECK(e->mask.ensure(T * 4));
  CHECK(e->out.ensure((size_t)n * e->cfg.hidden * 4));
  HIPC(hipMemcpyAsync(e->ids.p, ids, T * 4, hipMemcpyHostToDevice, e->stream));
  HIPC(hipMemcpyAsync(e->mask.p, mask, T * 4, hipMemcpyHostToDevice, e->stream));
  // ids must index the vocabulary: check on the host (an out-of-range id would read past the
  // embedding table)
  for (size_t i = 0; i < T; ++i)
    if (ids[i] < 0 || ids[i] >= e->cfg.vocab_size)
      return hcr_set_errorf(HCR_EINVAL, "token id %d out of range [0, %d)", ids[i], e->cfg.vocab_size);
  CHECK(hcr_encode_device(e, e->ids.as<const int32_t>(), e->mask.as<const int32_t>(), n, S,
                          e->out.as<float>(), e->stream));
  HIPC(hipMemcpyAsync(out, e->out.p, (size_t)n * e->cfg.hidden * 4, hipMemcpyDeviceToHost, e->stream));
  HIPC(hipStreamSynchronize(e->stream));
  return HCR_OK;
}
