// hcrag_index.hip — host side of the node-embedding index C ABI (include/hcrag.h).
//
// Replaces, for HC-RAG's vector path:
//   experiments/main.py:762       embeddings_matrix = np.array(pickled embeddings)   -> hcr_index_add
//   experiments/main.py:841-849   cosine_similarity + argsort[::-1][:k] + threshold  -> hcr_search
//   experiments/main.py:872-889   category filter + the same search                 -> rowmask
//   experiments/isRelevant.py:197-210  batch_semantic_similarity (all scores)        -> hcr_score_all
//   llama-index SimpleVectorStore.query / get_top_k_embeddings (query_interface.py:200-204)
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hcrag.h"
#include "host_common.h"
#include "topk_kernels.h"
#include "score_v3.h"
#include "score_v4.h"
#include "score_qs_launch.h"

using namespace hcr;

#define set_err hcr_set_errorf     // errors.cpp: thread-local message + status code

extern "C" const char* hcr_version(void) { return "hcrag-mi355x 0.3.0 (gfx950)"; }
extern "C" int hcr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ---------------------------------------------------------------------------------------
// index object
// ---------------------------------------------------------------------------------------
struct hcr_index {
  // global seed across shards (hcr_search_sample_device / hcr_search_seeded_device), set for one
  // call: the sampling pass only (report the unit maxima), or the dense pass seeded from every
  // shard's maxima with the per-query bound of the rows left out
  bool gs_sample_only = false;
  int gs_sample_units = 0, gs_sample_nqpad = 0;
  int64_t gs_sample_rows = 0;
  const float* gs_umax = nullptr;
  int gs_units = 0;
  double gs_frac = 0.0;
  double* gs_bound = nullptr;
  const float* gs_prep_q = nullptr;   // queries the last sample call prepared (the seeded call
  int gs_prep_nq = 0;                 // right after it, same queries, skips the prep kernel) --
  uint64_t gs_prep_gen = 0;           // valid only while `gen` is unchanged
  // bumped by every call that changes what a search's prep depends on (rows, rho, the unit
  // deviation, the row mask, the route options): a prep left by a sample call is reused by the
  // seeded call only if nothing changed in between
  uint64_t gen = 1;
  bool test_plant_bad_key = false;    // hcr_index_test_hook(HCR_TEST_PLANT_BAD_KEY)
  int device = 0;
  int dim = 0;
  int ld = 0;           // row stride in elements (dim rounded up to 64, zero padded)
  int dtype = HCR_F16;  // storage dtype
  int64_t n = 0;
  int64_t cap = 0;      // allocated rows (multiple of 128)
  int64_t id_offset = 0;
  DevBuf rows, norm64, inv32, maskbits, rho;
  DevBuf idmap;                 // int64 global id per row (only once hcr_index_add_ids was used)
  bool has_idmap = false;
  bool has_mask = false;
  bool rho_dirty = true;
  double rho_host = 0.0;
  double unit_dev_host = 1.0;   // max_r |1/inv32_r - 1| (UNIT score kernels when <= kUnitDevMax)
  hipStream_t stream = nullptr;
  // search workspace
  DevBuf w_qin, w_qhat, w_qnorm, w_eps, w_taug, w_buf, w_part, w_merged, w_outs, w_outi,
      w_unc, w_cnt, w_tauest, w_umax, w_sk, w_pcnt, w_mcnt;
  // exact fallback workspace (K6/K7)
  DevBuf f_idx, f_q, f_qn, f_thh, f_thl, f_act, f_cnt, f_bufh, f_bufl, f_again, f_hlo, f_hhi,
      f_hcnt, f_hmin, f_qhat, f_eps, f_ch, f_tmp, f_est, f_sorth, f_sortl, f_pairs, f_pcnt;
  hcr_search_stats stats{};
  int opt_qw1 = -1;             // HCR_OPT_QW1
  int opt_stride = 0;           // HCR_OPT_SAMPLE_STRIDE (0: the heuristic)
  int opt_qs = 0;               // HCR_OPT_QS_FORM (0: the heuristic)
  int opt_prepass = 0;          // HCR_OPT_PREPASS (0: the heuristic)
  int opt_qw_dm = -1;           // HCR_OPT_QW_DM (-1: the default)
  int opt_qw_min = 0;           // HCR_OPT_QW_MIN (0: the heuristic)
  int opt_qw_stagger = -1;      // HCR_OPT_QW_STAGGER (-1: the default)
  int opt_flag_read = 0;        // HCR_OPT_FLAG_READ (0: the default)
  // the pass's certificate flags as the device leaves them in host memory (pinned, coherent,
  // mapped): [0] sequence number, [1] uncertified queries, [2] out-of-index keys
  int* h_flag = nullptr;
  int* h_flag_dev = nullptr;
  int flag_seq = 0;
  int* pass_hflag = nullptr;          // set for the pass's finish / rescore launch: its last block
  int pass_seq = 0;                   // stores the flags (HCR_OPT_FLAG_READ 3 / 4)
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // ingest from a caller's stream (hcr_index_add_device): recorded there, waited on before
  // anything reads the rows, norms or rho
  hipEvent_t ev_ingest = nullptr;
  bool ingest_pending = false;
};

// Host-side wait for the last device ingest (ordering against the caller's stream).
static int wait_ingest(hcr_index* ix) {
  if (!ix->ingest_pending) return HCR_OK;
  HIPC(hipEventSynchronize(ix->ev_ingest));
  ix->ingest_pending = false;
  return HCR_OK;
}

static size_t dtype_size(int dt) { return dt == HCR_F32 ? 4 : 2; }
static constexpr int64_t kSlackRows = 512;
static int hcr_reserve_internal(hcr_index* ix, int64_t want_rows);
static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

extern "C" int hcr_index_create(int device, int dim, int dtype, int64_t capacity_rows,
                                hcr_index** out) {
  if (!out) return set_err(HCR_EINVAL, "out is NULL");
  *out = nullptr;
  if (dim <= 0 || dim > 4096) return set_err(HCR_EINVAL, "dim must be in [1, 4096], got %d", dim);
  if (dtype != HCR_F16 && dtype != HCR_BF16 && dtype != HCR_F32)
    return set_err(HCR_EINVAL, "unknown storage dtype %d", dtype);
  if (capacity_rows < 0) return set_err(HCR_EINVAL, "negative capacity");
  int ndev = hcr_device_count();
  if (device < 0 || device >= ndev)
    return set_err(HCR_EINVAL, "device %d not available (%d HIP devices)", device, ndev);
  HIPC(hipSetDevice(device));
  hcr_index* ix = new hcr_index();
  ix->device = device;
  ix->dim = dim;
  ix->ld = (int)round_up(dim, BK);
  ix->dtype = dtype;
  hipError_t e = hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete ix;
    return set_err(HCR_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  int rc = ix->rho.ensure(16);            // zero-filled (DevBuf::ensure)
  if (rc != HCR_OK) {
    hcr_index_destroy(ix);
    return rc;
  }
  *out = ix;
  if (capacity_rows > 0) {
    // reserve by growing to the capacity (rows stay empty)
    rc = hcr_reserve_internal(ix, capacity_rows);
    if (rc != HCR_OK) {
      hcr_index_destroy(ix);
      *out = nullptr;
      return rc;
    }
  }
  return HCR_OK;
}

extern "C" int hcr_index_destroy(hcr_index* ix) {
  if (!ix) return HCR_OK;
  (void)hipSetDevice(ix->device);
  if (ix->stream) (void)hipStreamSynchronize(ix->stream);
  DevBuf* all[] = {&ix->rows, &ix->norm64, &ix->inv32, &ix->maskbits, &ix->rho, &ix->idmap,
                   &ix->w_qin, &ix->w_qhat, &ix->w_qnorm, &ix->w_eps, &ix->w_taug,
                   &ix->w_buf, &ix->w_part, &ix->w_merged, &ix->w_outs, &ix->w_outi,
                   &ix->w_unc, &ix->w_cnt, &ix->w_tauest, &ix->w_umax, &ix->w_sk,
                   &ix->w_pcnt, &ix->w_mcnt,
                   &ix->f_idx, &ix->f_q, &ix->f_qn, &ix->f_thh, &ix->f_thl, &ix->f_act,
                   &ix->f_cnt, &ix->f_bufh, &ix->f_bufl, &ix->f_again, &ix->f_hlo, &ix->f_hhi,
                   &ix->f_hcnt, &ix->f_hmin, &ix->f_qhat, &ix->f_eps, &ix->f_ch, &ix->f_tmp, &ix->f_est, &ix->f_sorth, &ix->f_sortl,
                   &ix->f_pairs, &ix->f_pcnt};
  for (DevBuf* b : all) b->release();
  if (ix->h_flag) (void)hipHostFree(ix->h_flag);
  if (ix->ev_ingest) (void)hipEventDestroy(ix->ev_ingest);
  if (ix->ev0) (void)hipEventDestroy(ix->ev0);
  if (ix->ev1) (void)hipEventDestroy(ix->ev1);
  if (ix->stream) (void)hipStreamDestroy(ix->stream);
  delete ix;
  return HCR_OK;
}

extern "C" int hcr_index_reset(hcr_index* ix) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  HIPC(hipStreamSynchronize(ix->stream));
  ix->n = 0;
  ix->has_mask = false;
  ix->has_idmap = false;
  ix->rho_dirty = true;
  ++ix->gen;
  // on the index stream: a null-stream memset does not order against it
  HIPC(hipMemsetAsync(ix->rho.p, 0, 16, ix->stream));
  if (ix->cap > 0)
    HIPC(hipMemsetAsync(ix->maskbits.p, 0xFF, (size_t)((ix->cap + kSlackRows) / 32) * 4, ix->stream));
  return HCR_OK;
}

static int hcr_reserve_internal(hcr_index* ix, int64_t want_rows) {
  if (want_rows <= ix->cap) return HCR_OK;
  CHECK(wait_ingest(ix));        // the copy below reads rows a device ingest may still write
  int64_t ncap = std::max<int64_t>(want_rows, ix->cap + ix->cap / 2);
  ncap = round_up(std::max<int64_t>(ncap, 256), 256);
  // kSlackRows past the capacity: the score kernels read whole tiles (and DMA whole 1 KiB
  // inverse-norm slots), so every allocation covers the last tile plus slack.
  const int64_t arows = ncap + kSlackRows;
  const size_t es = dtype_size(ix->dtype);
  DevBuf nrows, nn64, ninv, nmask, nidm;
  CHECK(nrows.ensure((size_t)arows * ix->ld * es));
  if (ix->has_idmap) CHECK(nidm.ensure((size_t)arows * 8));
  CHECK(nn64.ensure((size_t)arows * 8));
  CHECK(ninv.ensure((size_t)arows * 4));
  CHECK(nmask.ensure((size_t)(arows / 32) * 4));
  HIPC(hipMemsetAsync(nrows.p, 0, (size_t)arows * ix->ld * es, ix->stream));
  HIPC(hipMemsetAsync(ninv.p, 0, (size_t)arows * 4, ix->stream));
  HIPC(hipMemsetAsync(nmask.p, 0xFF, (size_t)(arows / 32) * 4, ix->stream));
  if (ix->n > 0) {
    HIPC(hipMemcpyAsync(nrows.p, ix->rows.p, (size_t)ix->n * ix->ld * es, hipMemcpyDeviceToDevice, ix->stream));
    HIPC(hipMemcpyAsync(nn64.p, ix->norm64.p, (size_t)ix->n * 8, hipMemcpyDeviceToDevice, ix->stream));
    HIPC(hipMemcpyAsync(ninv.p, ix->inv32.p, (size_t)ix->n * 4, hipMemcpyDeviceToDevice, ix->stream));
    if (ix->has_mask)
      HIPC(hipMemcpyAsync(nmask.p, ix->maskbits.p, (size_t)(ix->cap / 32) * 4, hipMemcpyDeviceToDevice, ix->stream));
    if (ix->has_idmap)
      HIPC(hipMemcpyAsync(nidm.p, ix->idmap.p, (size_t)ix->n * 8, hipMemcpyDeviceToDevice, ix->stream));
  }
  HIPC(hipStreamSynchronize(ix->stream));
  ix->rows.release(); ix->norm64.release(); ix->inv32.release(); ix->maskbits.release();
  ix->rows = nrows; ix->norm64 = nn64; ix->inv32 = ninv; ix->maskbits = nmask;
  nrows.p = nn64.p = ninv.p = nmask.p = nullptr;   // ownership moved
  if (ix->has_idmap) {
    ix->idmap.release();
    ix->idmap = nidm;
    nidm.p = nullptr;
  }
  ix->cap = ncap;
  return HCR_OK;
}

template <typename TIN, typename TS>
static void launch_ingest(hcr_index* ix, const void* d_in, int64_t n, int normalize,
                          hipStream_t st) {
  TS* dst = ix->rows.as<TS>() + ix->n * ix->ld;
  const unsigned grid = (unsigned)((n + 3) / 4);
  hipLaunchKernelGGL((ingest_kernel<TIN, TS>), dim3(grid), dim3(256), 0, st,
                     reinterpret_cast<const TIN*>(d_in), n, ix->dim, ix->ld, normalize, dst,
                     ix->norm64.as<double>() + ix->n, ix->inv32.as<float>() + ix->n,
                     ix->rho.as<unsigned int>());
}

static int ingest_device(hcr_index* ix, const void* d_rows, int64_t n, int in_dt, int normalize,
                         hipStream_t st) {
  if (in_dt != HCR_F16 && in_dt != HCR_BF16 && in_dt != HCR_F32)
    return set_err(HCR_EINVAL, "unknown rows dtype %d", in_dt);
#define ING(TIN, TS) launch_ingest<TIN, TS>(ix, d_rows, n, normalize, st)
  const int sd = ix->dtype;
  if (in_dt == HCR_F32) {
    if (sd == HCR_F16) ING(float, _Float16); else if (sd == HCR_BF16) ING(float, __bf16); else ING(float, float);
  } else if (in_dt == HCR_F16) {
    if (sd == HCR_F16) ING(_Float16, _Float16); else if (sd == HCR_BF16) ING(_Float16, __bf16); else ING(_Float16, float);
  } else {
    if (sd == HCR_F16) ING(__bf16, _Float16); else if (sd == HCR_BF16) ING(__bf16, __bf16); else ING(__bf16, float);
  }
#undef ING
  HIPC(hipGetLastError());
  if (ix->has_idmap) {            // plain adds after id-mapped ones: id_offset + row
    hipLaunchKernelGGL(iota_ids_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       ix->idmap.as<int64_t>() + ix->n, n, ix->id_offset + ix->n);
    HIPC(hipGetLastError());
  }
  ix->n += n;
  ix->rho_dirty = true;
  ++ix->gen;
  return HCR_OK;
}

extern "C" int hcr_index_add_device(hcr_index* ix, const void* d_rows, int64_t n, int rows_dtype,
                                    int normalize, void* stream) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (n < 0) return set_err(HCR_EINVAL, "negative row count");
  if (n == 0) return HCR_OK;
  if (!d_rows) return set_err(HCR_EINVAL, "rows is NULL");
  if (ix->n + n > (int64_t)0xFFFFFFFEll) return set_err(HCR_EINVAL, "index limited to 2^32-2 rows per shard");
  HIPC(hipSetDevice(ix->device));
  CHECK(hcr_reserve_internal(ix, ix->n + n));
  // NULL = the legacy default stream (as every *_device entry point): the caller's work on
  // it (e.g. torch's default stream producing the input) is ordered before ours
  hipStream_t st = (hipStream_t)stream;
  if (st != ix->stream) HIPC(hipStreamSynchronize(ix->stream));
  CHECK(ingest_device(ix, d_rows, n, rows_dtype, normalize, st));
  if (st != ix->stream) {
    // later reads of the rows / norms / rho (search, reserve, get_rows) wait for this event
    if (!ix->ev_ingest) HIPC(hipEventCreateWithFlags(&ix->ev_ingest, hipEventDisableTiming));
    HIPC(hipEventRecord(ix->ev_ingest, st));
    ix->ingest_pending = true;
  }
  return HCR_OK;
}

extern "C" int hcr_index_add(hcr_index* ix, const void* rows, int64_t n, int rows_dtype,
                             int normalize) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (n < 0) return set_err(HCR_EINVAL, "negative row count");
  if (n == 0) return HCR_OK;
  if (!rows) return set_err(HCR_EINVAL, "rows is NULL");
  if (rows_dtype != HCR_F16 && rows_dtype != HCR_BF16 && rows_dtype != HCR_F32)
    return set_err(HCR_EINVAL, "unknown rows dtype %d", rows_dtype);
  if (ix->n + n > (int64_t)0xFFFFFFFEll) return set_err(HCR_EINVAL, "index limited to 2^32-2 rows per shard");
  HIPC(hipSetDevice(ix->device));
  CHECK(hcr_reserve_internal(ix, ix->n + n));
  const size_t rb = (size_t)ix->dim * dtype_size(rows_dtype);
  const int64_t chunk = std::max<int64_t>(1, (int64_t)((256u << 20) / rb));
  for (int64_t r0 = 0; r0 < n; r0 += chunk) {
    const int64_t m = std::min(chunk, n - r0);
    CHECK(ix->w_qin.ensure((size_t)m * rb));
    HIPC(hipMemcpyAsync(ix->w_qin.p, (const char*)rows + (size_t)r0 * rb, (size_t)m * rb,
                        hipMemcpyHostToDevice, ix->stream));
    CHECK(ingest_device(ix, ix->w_qin.p, m, rows_dtype, normalize, ix->stream));
  }
  HIPC(hipStreamSynchronize(ix->stream));
  return HCR_OK;
}

extern "C" int hcr_index_add_ids(hcr_index* ix, const void* rows, int64_t n, int rows_dtype,
                                 int normalize, const int64_t* ids) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (n < 0) return set_err(HCR_EINVAL, "negative row count");
  if (n == 0) return HCR_OK;
  if (!ids) return set_err(HCR_EINVAL, "ids is NULL");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  const int64_t n0 = ix->n;
  CHECK(hcr_reserve_internal(ix, n0 + n));
  if (!ix->has_idmap) {           // first id-mapped add: the existing rows keep their ids
    CHECK(ix->idmap.ensure((size_t)(ix->cap + kSlackRows) * 8));
    if (n0 > 0) {
      hipLaunchKernelGGL(iota_ids_kernel, dim3((unsigned)((n0 + 255) / 256)), dim3(256), 0,
                         ix->stream, ix->idmap.as<int64_t>(), n0, ix->id_offset);
      HIPC(hipGetLastError());
    }
    ix->has_idmap = true;
  }
  CHECK(hcr_index_add(ix, rows, n, rows_dtype, normalize));
  // the plain add above wrote id_offset + row for the new rows; overwrite with the given ids
  HIPC(hipMemcpyAsync(ix->idmap.as<int64_t>() + n0, ids, (size_t)n * 8, hipMemcpyHostToDevice,
                      ix->stream));
  HIPC(hipStreamSynchronize(ix->stream));
  return HCR_OK;
}

extern "C" int64_t hcr_index_size(const hcr_index* ix) { return ix ? ix->n : -1; }

int hcr_index_truncate_internal(hcr_index* ix, int64_t n) {
  if (!ix || n < 0 || n > ix->n) return set_err(HCR_EINVAL, "bad truncation");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  HIPC(hipStreamSynchronize(ix->stream));
  ix->n = n;
  ix->rho_dirty = true;           // unit deviation re-measured over the rows that remain
  ++ix->gen;
  return HCR_OK;
}
extern "C" int hcr_index_dim(const hcr_index* ix) { return ix ? ix->dim : -1; }
extern "C" int hcr_index_dtype(const hcr_index* ix) { return ix ? ix->dtype : -1; }

extern "C" int hcr_index_set_id_offset(hcr_index* ix, int64_t off) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (off < 0) return set_err(HCR_EINVAL, "negative id offset");
  // once an id map exists the rows already in it keep the ids they were given; a new offset
  // would apply only to later plain adds -- two numbering rules in one index, so refused
  if (ix->has_idmap && off != ix->id_offset)
    return set_err(HCR_EINVAL, "id offset cannot change after hcr_index_add_ids (ids are explicit)");
  ix->id_offset = off;
  return HCR_OK;
}

static float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000) << 16;
  uint32_t e = (h >> 10) & 0x1F, m = h & 0x3FF;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) bits = s;
    else {
      int sh = 0;
      while (!(m & 0x400)) { m <<= 1; ++sh; }
      m &= 0x3FF;
      bits = s | ((uint32_t)(127 - 15 - sh + 1) << 23) | (m << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7F800000u | (m << 13);
  } else {
    bits = s | ((e - 15 + 127) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

extern "C" int hcr_index_get_rows(const hcr_index* ix, int64_t row0, int64_t n, float* out) {
  if (!ix || !out) return set_err(HCR_EINVAL, "NULL argument");
  if (row0 < 0 || n < 0 || row0 + n > ix->n) return set_err(HCR_EINVAL, "row range out of bounds");
  if (n == 0) return HCR_OK;
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(const_cast<hcr_index*>(ix)));
  const size_t es = dtype_size(ix->dtype);
  std::vector<char> tmp((size_t)n * ix->ld * es);
  HIPC(hipStreamSynchronize(ix->stream));
  HIPC(hipMemcpy(tmp.data(), (const char*)ix->rows.p + (size_t)row0 * ix->ld * es, tmp.size(),
                 hipMemcpyDeviceToHost));
  for (int64_t r = 0; r < n; ++r) {
    for (int d = 0; d < ix->dim; ++d) {
      const size_t i = (size_t)r * ix->ld + d;
      float v;
      if (ix->dtype == HCR_F32) memcpy(&v, tmp.data() + i * 4, 4);
      else {
        uint16_t h;
        memcpy(&h, tmp.data() + i * 2, 2);
        if (ix->dtype == HCR_F16) v = half_to_float(h);
        else { uint32_t b = (uint32_t)h << 16; memcpy(&v, &b, 4); }
      }
      out[(size_t)r * ix->dim + d] = v;
    }
  }
  return HCR_OK;
}

extern "C" int hcr_index_set_rowmask(hcr_index* ix, const uint8_t* mask, int64_t n) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  HIPC(hipSetDevice(ix->device));
  ++ix->gen;
  if (!mask) { ix->has_mask = false; return HCR_OK; }
  if (n != ix->n) return set_err(HCR_EINVAL, "mask length %lld != index size %lld", (long long)n, (long long)ix->n);
  if (ix->cap == 0) { ix->has_mask = false; return HCR_OK; }
  CHECK(wait_ingest(ix));
  // rows appended after the mask is set are visible (their bits are 1, as in a fresh or
  // regrown allocation); rows past the size are never scored either way
  std::vector<uint32_t> bits((size_t)((ix->cap + kSlackRows) / 32), 0xFFFFFFFFu);
  for (int64_t i = 0; i < n; ++i)
    if (!mask[i]) bits[(size_t)(i >> 5)] &= ~(1u << (i & 31));
  HIPC(hipMemcpyAsync(ix->maskbits.p, bits.data(), bits.size() * 4, hipMemcpyHostToDevice, ix->stream));
  HIPC(hipStreamSynchronize(ix->stream));
  ix->has_mask = true;
  return HCR_OK;
}

extern "C" int hcr_index_set_timing(hcr_index* ix, int enable) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  HIPC(hipSetDevice(ix->device));
  if (enable && !ix->ev0) {
    // timing only (read after the pass's own stream sync): no system-scope fence, whose cache
    // write-back + invalidate idled the GPU ~6 us at each record (configs[1] kernel trace, r05ev)
    HIPC(hipEventCreateWithFlags(&ix->ev0, hipEventDisableSystemFence));
    HIPC(hipEventCreateWithFlags(&ix->ev1, hipEventDisableSystemFence));
  }
  ix->timing = enable != 0;
  return HCR_OK;
}

extern "C" int hcr_index_set_option(hcr_index* ix, int option, int value) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  // every option but the sample stride can change the route, hence the prep (UNIT or not); the
  // stride only decides which tiles the sampling pass reads (set around a sample call by
  // distributed.hip_global_seed, between the sample and the seeded call)
  if (option != HCR_OPT_SAMPLE_STRIDE) ++ix->gen;
  switch (option) {
    case HCR_OPT_QW1:
      if (value < -1 || value > 1) return set_err(HCR_EINVAL, "HCR_OPT_QW1 value %d not in [-1, 1]", value);
      ix->opt_qw1 = value;
      return HCR_OK;
    case HCR_OPT_SAMPLE_STRIDE:
      if (value != 0 && (value < 2 || value > 4096))
        return set_err(HCR_EINVAL, "HCR_OPT_SAMPLE_STRIDE value %d not 0 or in [2, 4096]", value);
      ix->opt_stride = value;
      return HCR_OK;
    case HCR_OPT_PREPASS:
      if (value < 0 || value > 2) return set_err(HCR_EINVAL, "HCR_OPT_PREPASS value %d not in [0, 2]", value);
      ix->opt_prepass = value;
      return HCR_OK;
    case HCR_OPT_QW_DM:
      if (value != -1 && value != 0 && value != 3)
        return set_err(HCR_EINVAL, "HCR_OPT_QW_DM value %d not -1, 0 or 3", value);
      ix->opt_qw_dm = value;
      return HCR_OK;
    case HCR_OPT_QW_STAGGER:
      if (value < -1 || value > 2) return set_err(HCR_EINVAL, "HCR_OPT_QW_STAGGER value %d not in [-1, 2]", value);
      ix->opt_qw_stagger = value;
      return HCR_OK;
    case HCR_OPT_QW_MIN:
      if (value < 0) return set_err(HCR_EINVAL, "HCR_OPT_QW_MIN value %d negative", value);
      ix->opt_qw_min = value;
      return HCR_OK;
    case HCR_OPT_QS_FORM:
      if (value != 0 && value != 1 && value != 3)
        return set_err(HCR_EINVAL, "HCR_OPT_QS_FORM value %d not 0, 1 or 3", value);
      ix->opt_qs = value;
      return HCR_OK;
    case HCR_OPT_FLAG_READ:
      if (value < 0 || value > 4) return set_err(HCR_EINVAL, "HCR_OPT_FLAG_READ value %d not in [0, 4]", value);
      ix->opt_flag_read = value;
      return HCR_OK;
    default:
      return set_err(HCR_EINVAL, "unknown index option %d", option);
  }
}

extern "C" int hcr_index_test_hook(hcr_index* ix, int hook, int value) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (hook != HCR_TEST_PLANT_BAD_KEY) return set_err(HCR_EINVAL, "unknown test hook %d", hook);
  ix->test_plant_bad_key = value != 0;
  return HCR_OK;
}

extern "C" int hcr_index_last_stats(const hcr_index* ix, hcr_search_stats* out) {
  if (!ix || !out) return set_err(HCR_EINVAL, "NULL argument");
  *out = ix->stats;
  return HCR_OK;
}

// ---------------------------------------------------------------------------------------
// search pipeline
// ---------------------------------------------------------------------------------------
static int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }
static constexpr int kMaxKprime = 512;
static constexpr int kMergeMaxKeys = 16384;     // keys per merge_lists_kernel block (128 KiB of
                                                // LDS): one level for P x k' <= 256 x 64
static constexpr int kQueryChunk = 16384;       // queries per pipeline pass (bounds workspace)
static constexpr int kMaxDevices = 64;          // per-device once-only kernel attributes
static constexpr size_t kLdsBytes = 160 * 1024;  // LDS per CU (gfx950) = a block's dynamic limit

static int choose_kprime(int k) { return std::max(64, next_pow2(2 * k)); }

// Raise a kernel's dynamic-LDS limit once per device (a per-device attribute; hcr_multi_search
// runs shards of several devices concurrently).  `done` is the call site's own flag array: a
// failure is returned to this caller and the next caller tries again (a once_flag
// marked the attribute done even when setting it failed).
static int raise_lds_limit(const void* fn, int bytes, int device, bool (&done)[kMaxDevices]) {
  if (device < 0 || device >= kMaxDevices) return set_err(HCR_EINVAL, "device %d", device);
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  if (done[device]) return HCR_OK;
  HIPC(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done[device] = true;
  return HCR_OK;
}

template <typename TS, typename TM, int CAP>
static void launch_score(hcr_index* ix, int nqb, int P, int ntiles, int kp, hipStream_t st) {
  const int nwg = nqb * P;
  hipLaunchKernelGGL((score_topk_kernel<TS, TM, CAP>), dim3(nwg), dim3(NT), 0, st,
                     ix->rows.as<const TS>(), ix->ld, ix->n, ix->ld / BK, ix->inv32.as<const float>(),
                     ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,
                     ix->w_qhat.as<const TM>(), nqb, P, ntiles, ix->w_buf.as<uint64_t>(),
                     ix->w_taug.as<uint32_t>(), ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), kp);
}

template <typename TS, typename TM>
static int dispatch_score(hcr_index* ix, int nqb, int P, int ntiles, int kp, int cap, hipStream_t st) {
  switch (cap) {
    case 256: launch_score<TS, TM, 256>(ix, nqb, P, ntiles, kp, st); break;
    case 512: launch_score<TS, TM, 512>(ix, nqb, P, ntiles, kp, st); break;
    case 1024: launch_score<TS, TM, 1024>(ix, nqb, P, ntiles, kp, st); break;
    default: return set_err(HCR_EINVAL, "internal: unsupported candidate capacity %d", cap);
  }
  HIPC(hipGetLastError());
  return HCR_OK;
}

// ---- K2 v3 (score_v3.h): tile configurations by batch size ----
static constexpr int64_t kQ64WideMaxElems = 1500000000;   // rows x ld, see v3_cfg

// Test hooks, read once per process.  They force paths the default heuristics only take at
// scale (or rarely) so that the parity tests reach them on small corpora; they never change
// results, only which exact path produces them.
//   HCRAG_Q64_ELEMS         corpus-size threshold of the 256 x 64 tiles (17-64 queries)
//   HCRAG_NO_PREPASS        no sampling pre-pass (cold per-workgroup bounds)
//   HCRAG_PREPASS_MIN_TILES dense tiles per workgroup from which the pre-pass runs
//   HCRAG_SAMPLE_STRIDE     pre-pass sampling stride
//   HCRAG_RIGOROUS_SEED     seed rank j = k' (rigorous) instead of the estimate
//   HCRAG_SEED_RANK         force seed rank j (aggressive seeds exercise the re-runs)
//   HCRAG_PREPASS_TOPK      the top-k' pre-pass form instead of MAXONLY
//   HCRAG_QS_MAX            largest batch on the query-stationary kernel (0: off)
//   HCRAG_QW_MIN            smallest batch on the wide query-stationary kernel
//   HCRAG_QW1               default of HCR_OPT_QW1 (one-wave-per-SIMD large-batch kernel)
struct TestHooks {
  int64_t q64_elems = kQ64WideMaxElems;
  int qs_max = 256;
  int qw_min = 0;                    // 0: the measured default (v3_cfg)
  int qw1 = -1;                      // HCR_OPT_QW1 default (-1: the heuristic)
  bool no_prepass = false, rigorous_seed = false, prepass_topk = false, debug_cfg = false;
  bool no_finish = false;            // HCRAG_NO_FINISH: separate merge + rescore launches
  bool no_mfma_filter = false;       // HCRAG_NO_MFMA_FILTER: the fallback's scans on K6 (fp64 only)
  bool k6_inline = false;            // HCRAG_K6_INLINE: K6m rescoring inline (no K6c / K6r)
  int64_t k6_pcap = 0;               // HCRAG_K6_PCAP: pair slots per group (tests: force overflow)
  int k6_chunks = 0;                 // HCRAG_K6_CHUNKS: K6 scan blocks per query group (A/B)
  int k6r_blocks = 0;                // HCRAG_K6R_BLOCKS: K6r blocks per query group (A/B)
  bool k6_qb1 = false;               // HCRAG_K6_QB1: K6h / K6c with one query half per wave (A/B)
  int k6h_ratio = 0;                 // HCRAG_K6H_RATIO: K6h sampling rule (A/B)
  int prepass_min_tiles = 0, sample_stride = 0, seed_rank = 0;
};
static const TestHooks& hooks() {
  static const TestHooks h = [] {
    TestHooks t;
    if (const char* e = getenv("HCRAG_Q64_ELEMS")) t.q64_elems = (int64_t)atoll(e);
    if (const char* e = getenv("HCRAG_QS_MAX")) t.qs_max = atoi(e);
    if (const char* e = getenv("HCRAG_QW_MIN")) t.qw_min = std::max(1, atoi(e));
    if (const char* e = getenv("HCRAG_QW1")) t.qw1 = std::min(1, std::max(-1, atoi(e)));
    t.no_prepass = getenv("HCRAG_NO_PREPASS") != nullptr;
    t.debug_cfg = getenv("HCRAG_DEBUG_CFG") != nullptr;
    t.no_finish = getenv("HCRAG_NO_FINISH") != nullptr;
    t.no_mfma_filter = getenv("HCRAG_NO_MFMA_FILTER") != nullptr;
    t.k6_inline = getenv("HCRAG_K6_INLINE") != nullptr;
    if (const char* e = getenv("HCRAG_K6_PCAP")) t.k6_pcap = std::max<int64_t>(1, atoll(e));
    if (const char* e = getenv("HCRAG_K6_CHUNKS")) t.k6_chunks = std::max(8, atoi(e));
    if (const char* e = getenv("HCRAG_K6R_BLOCKS")) t.k6r_blocks = std::max(1, atoi(e));
    t.k6_qb1 = getenv("HCRAG_K6_QB1") != nullptr;
    if (const char* e = getenv("HCRAG_K6H_RATIO")) t.k6h_ratio = std::max(1, atoi(e));
    t.rigorous_seed = getenv("HCRAG_RIGOROUS_SEED") != nullptr;
    t.prepass_topk = getenv("HCRAG_PREPASS_TOPK") != nullptr;
    if (const char* e = getenv("HCRAG_PREPASS_MIN_TILES")) t.prepass_min_tiles = std::max(1, atoi(e));
    if (const char* e = getenv("HCRAG_SAMPLE_STRIDE")) t.sample_stride = std::max(2, atoi(e));
    if (const char* e = getenv("HCRAG_SEED_RANK")) t.seed_rank = std::max(1, atoi(e));
    return t;
  }();
  return h;
}

// qs: query-stationary kernel (score_qs.h); qw: its 256-query form (score_qw.h); qw1: the
// one-wave-per-SIMD form at D = 1024 (score_qw1.h)
struct V3Cfg { int rt, qt, nst; bool qs, qw = false, qw1 = false; int hs = 2; };
// qw_ok / qw1_ok: a UNIT-capable corpus without a row mask and k' small enough for the
// QW / QW1 candidate buffers; opt_qw1: HCR_OPT_QW1; opt_qs: HCR_OPT_QS_FORM
static V3Cfg v3_cfg(int nq, int64_t n_rows, int ld, bool unit_ok, bool qw_ok, bool qw1_ok, int opt_qw1,
                    int opt_qs = 0, int opt_qw_min = 0) {
  if (nq <= 16) return {256, 16, 8, false};
  // > 256 queries (MFMA-bound): 256 queries per workgroup held in VGPRs, only rows streamed
  // through LDS -- half of v4's LDS-DMA fill per flop (score_qw.h)
  // From 129 queries at D = 768 (r02 sweeps at 10M x 768: B = 160 3.64 vs 4.48 ms on QS,
  // B = 256 3.73 vs 4.61) and at D = 384 (r05c, 1M x 384, B = 256 -- configs[1] --, interleaved
  // in one process: QW with its stage DMA spread over the MFMA groups 0.323 ms per search, QS
  // 0.330; QW with DMA at the barrier 0.335).
  const int qw_from = opt_qw_min > 0 ? opt_qw_min : hooks().qw_min > 0 ? hooks().qw_min : 129;
  // QW1: 48 queries per wave at one wave per SIMD, D = 1024 only.  D = 1024 has no other
  // query-stationary kernel (256 queries x 1024 do not fit QW's waves), so it takes QW1 from 257
  // queries unless HCR_OPT_QW1 = 0 (v4 then).
  if (opt_qw1 != 0 && unit_ok && qw1_ok && qw1_supported(ld) && nq >= 257)
    return {qw1_rows(ld), qw1_queries(ld), 0, false, false, true};
  if (nq >= qw_from && unit_ok && qw_ok && qw_supported(ld))
    return {qw_rows(ld, (nq + kQwQueries - 1) / kQwQueries), kQwQueries, kQwStages, false, true};
  // 17-256 queries: the query-stationary kernel (queries in VGPRs, only rows streamed through
  // LDS; 129-256 as two 128-query blocks per row partition).  Score ms, QS vs v3/v4
  // (profiles/r02/qs_ab.txt): 10M x 768 B = 32 2.75 vs 3.67, B = 128 2.82 vs 4.32, B = 160 4.42
  // vs 4.45, B = 256 4.52 vs 4.59; 1M x 384 B = 32 0.187 vs 0.295, B = 256 0.290 vs 0.331.
  if (nq <= hooks().qs_max) {
    // 129-256 queries with KS <= 12: one 256-query block on 128-row tiles (each row filled
    // into LDS once instead of once per 128-query block)
    if (nq > 128 && qs_supported(ld, 2)) {
      V3Cfg c{128, 256, 8, true};
      // KS = 12 (D = 384, configs[1]): 128-deep ring stages by default -- 3 barriers per 128-row
      // tile instead of 6 (r03 A/B, 1M x 384, B = 256, score ms: 64-deep 0.2694, 128-deep
      // 0.2536, 192-deep 0.2559; stamps: 14.1k -> 12.2k cycles per tile); HCR_OPT_QS_FORM 1:
      // 64-deep
      if (ld / V3_BK == 12 && opt_qs != 1) c.hs = 4;
      return c;
    }
    // (KS = 24 without the UNIT epilogue spills VGPRs in its tile loop: v3/v4 then)
    if (qs_supported(ld, 1) && (unit_ok || ld / V3_BK < 24)) return {kQsRowTile, 128, 4, true};
  }
  // 17-64 queries: 256 x 256 on small corpora (MAXONLY pre-pass), 256 x 64 on large ones.
  // r01g (profiles/r01g/q64_sweeps.jsonl, score kernel ms at B = 48): 1M x 384 0.29 vs 0.36,
  // 1M x 768 0.49 vs 0.52, 2.5M x 768 1.11 vs 1.08, 5M x 768 2.13 vs 1.98, 10M x 768 4.13 vs
  // 3.73 -> the crossover is between 0.8e9 and 1.9e9 corpus elements (the cost of either tile
  // shape is flat in the batch within its range).
  if (nq <= 64 && n_rows * (int64_t)ld <= hooks().q64_elems) return {256, 256, 4, false};
  if (nq <= 64) return {256, 64, 7, false};
  // 65+ queries: the 256 x 256 kernel (v4), also for 65-128 where half its query columns are
  // padding (MAXONLY pre-pass + UNIT epilogue; r01g sweeps: 10M x 768 B = 200 4.51 ms vs
  // B = 128 4.74 ms on 256 x 128; 1M x 384 0.31 vs 0.57 ms)
  return V3Cfg{256, 256, 4, false};
}
// the tile-slot rings (inverse norms, mask words, global bounds) need a tile's slot to
// outlive NST-1 stages of look-ahead
static bool v3_fits(const hcr_index* ix, V3Cfg c) {
  if (c.qs || c.qw || c.qw1) return true;         // QS sizes its own slot rings (QsLayout::NIS)
  return (V3_NIS - 1) * (ix->ld / V3_BK) > c.nst - 1;
}

struct V3Launch { int nqb, P, nvt, tstride, kp; bool unit; };

// Largest deviation of a stored row's norm from 1, as max_r |1/inv32_r - 1| (fp64, positive
// doubles order like their bit patterns): the certificate widening of the UNIT score kernels.
__global__ void unit_dev_kernel(const float* __restrict__ inv32, int64_t n,
                                unsigned long long* __restrict__ out) {
  double m = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    m = fmax(m, fabs(1.0 / (double)inv32[i] - 1.0));
  m = wave_max_f64(m);
  if ((threadIdx.x & 63) == 0 && m > 0.0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}
// UNIT kernels for L2-normalised corpora when max_r |1/inv32_r - 1| <= 2^-9 (f16 rows: ~5e-5;
// bf16 rows after the ingest's scale search: < 1e-3)
static constexpr double kUnitDevMax = 1.0 / 512;

template <typename TM, int CAP, int RT, int QT, int WM, int WN, int NST>
static void launch_v3_t(hcr_index* ix, V3Launch a, hipStream_t st) {
  hipLaunchKernelGGL((score_topk_v3_kernel<TM, CAP, RT, QT, WM, WN, NST>), dim3(a.nqb * a.P),
                     dim3(V3_NT), 0, st, ix->rows.as<const TM>(), ix->ld, ix->n, ix->ld / V3_BK,
                     ix->inv32.as<const float>(),
                     ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,
                     ix->w_qhat.as<const TM>(), a.nqb, a.P, a.nvt, a.tstride,
                     ix->w_buf.as<uint64_t>(), ix->w_taug.as<uint32_t>(),
                     ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), a.kp);
}

static int launch_qs_ix(hcr_index* ix, V3Cfg c, V3Launch a, hipStream_t st) {
  QsArgs q{ix->rows.p, ix->ld, ix->n, ix->inv32.as<const float>(),
           ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr, ix->w_qhat.p, a.nqb, a.P,
           a.nvt, a.tstride, ix->w_buf.as<uint64_t>(), ix->w_taug.as<uint32_t>(),
           ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), a.kp, qs_cap(a.kp), a.unit,
           c.qt == 256 ? 2 : 1, c.hs};
  return launch_qs(ix->dtype, q, st);
}

static int launch_qw1_ix(hcr_index* ix, V3Launch a, int cap, hipStream_t st) {
  QsArgs q{ix->rows.p, ix->ld, ix->n, ix->inv32.as<const float>(), nullptr, ix->w_qhat.p, a.nqb,
           a.P, a.nvt, 1, ix->w_buf.as<uint64_t>(), ix->w_taug.as<uint32_t>(),
           ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), a.kp, cap, true, 0};
  return launch_qw1(ix->dtype, q, st);
}

// Row partitions of a QW1 launch (one workgroup per CU, LDS-bound): the smallest P >= 256 / nqb
// whose nqb x P workgroups fill their last round of 256 CUs to >= 97 % (nq = 8192 at D = 1024:
// 43 query blocks x 29 partitions = 1247 workgroups in 5 rounds), else the best fill up to 256.
static int qw1_partitions(int nqb, int ntiles) {
  constexpr int kCus = 256;
  const int p0 = std::max(1, kCus / nqb);
  int best = p0;
  double best_fill = 0.0;
  for (int P = p0; P <= std::max(p0, std::min(256, ntiles)); ++P) {
    const int64_t nwg = (int64_t)nqb * P;
    const double fill = (double)nwg / (double)(((nwg + kCus - 1) / kCus) * kCus);
    if (fill >= 0.97) return P;
    if (fill > best_fill + 1e-9) { best_fill = fill; best = P; }
  }
  return best;
}

static int launch_qw_ix(hcr_index* ix, V3Launch a, int cap, hipStream_t st) {
  QsArgs q{ix->rows.p, ix->ld, ix->n, ix->inv32.as<const float>(), nullptr, ix->w_qhat.p, a.nqb,
           a.P, a.nvt, 1, ix->w_buf.as<uint64_t>(), ix->w_taug.as<uint32_t>(),
           ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), a.kp, cap, true, 0};
  q.dm = ix->opt_qw_dm;
  q.stagger = ix->opt_qw_stagger;
  return launch_qw(ix->dtype, q, st);
}

template <typename TM, int CAP>
static int launch_v3_cap(hcr_index* ix, V3Cfg c, V3Launch a, hipStream_t st) {
  if (c.qt == 256) {
    if (a.unit)
      hipLaunchKernelGGL((score_topk_v4_kernel<TM, CAP, 4, true>), dim3(a.nqb * a.P), dim3(V3_NT), 0, st,
                         ix->rows.as<const TM>(), ix->ld, ix->n, ix->ld / V3_BK,
                         ix->inv32.as<const float>(),
                         ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,
                         ix->w_qhat.as<const TM>(), a.nqb, a.P, a.nvt, a.tstride,
                         ix->w_buf.as<uint64_t>(), ix->w_taug.as<uint32_t>(),
                         ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), a.kp);
    else
      hipLaunchKernelGGL((score_topk_v4_kernel<TM, CAP, 4, false>), dim3(a.nqb * a.P), dim3(V3_NT), 0, st,
                         ix->rows.as<const TM>(), ix->ld, ix->n, ix->ld / V3_BK,
                         ix->inv32.as<const float>(),
                         ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,
                         ix->w_qhat.as<const TM>(), a.nqb, a.P, a.nvt, a.tstride,
                         ix->w_buf.as<uint64_t>(), ix->w_taug.as<uint32_t>(),
                         ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), a.kp);
  }
  else if (c.qt == 64) launch_v3_t<TM, CAP, 256, 64, 4, 2, 7>(ix, a, st);
  else launch_v3_t<TM, CAP, 256, 16, 8, 1, 8>(ix, a, st);
  HIPC(hipGetLastError());
  return HCR_OK;
}

// sampling pre-pass: v4 in MAXONLY mode, unit maxima into ix->w_umax
template <typename TM>
static int launch_v4_maxonly(hcr_index* ix, V3Launch a, hipStream_t st) {
  if (a.unit)
    hipLaunchKernelGGL((score_topk_v4_kernel<TM, 512, 4, true, true>), dim3(a.nqb * a.P), dim3(V3_NT), 0,
                       st, ix->rows.as<const TM>(), ix->ld, ix->n, ix->ld / V3_BK,
                       ix->inv32.as<const float>(),
                       ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,
                       ix->w_qhat.as<const TM>(), a.nqb, a.P, a.nvt, a.tstride,
                       ix->w_umax.as<uint64_t>(), ix->w_taug.as<uint32_t>(), nullptr, nullptr, a.kp);
  else
    hipLaunchKernelGGL((score_topk_v4_kernel<TM, 512, 4, false, true>), dim3(a.nqb * a.P), dim3(V3_NT), 0,
                       st, ix->rows.as<const TM>(), ix->ld, ix->n, ix->ld / V3_BK,
                       ix->inv32.as<const float>(),
                       ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,
                       ix->w_qhat.as<const TM>(), a.nqb, a.P, a.nvt, a.tstride,
                       ix->w_umax.as<uint64_t>(), ix->w_taug.as<uint32_t>(), nullptr, nullptr, a.kp);
  HIPC(hipGetLastError());
  return HCR_OK;
}

template <typename TM>
static int dispatch_v3(hcr_index* ix, V3Cfg c, V3Launch a, int cap, hipStream_t st) {
  if (c.qs) return launch_qs_ix(ix, c, a, st);              // CAP chosen in score_qs.hip
  if (c.qw) return launch_qw_ix(ix, a, cap, st);
  if (c.qw1) return launch_qw1_ix(ix, a, cap, st);
  switch (cap) {
    case 512: return launch_v3_cap<TM, 512>(ix, c, a, st);
    case 1024: return launch_v3_cap<TM, 1024>(ix, c, a, st);
    default: return set_err(HCR_EINVAL, "internal: unsupported candidate capacity %d", cap);
  }
}

template <typename TS>
static void launch_rescore(hcr_index* ix, const uint64_t* merged, const float* d_q, int nq, int kp, int k, int mode,
                           double thr, double* out_s, int64_t* out_i, hipStream_t st) {
  const size_t lds = (size_t)ix->dim * 8 + (size_t)kp * 32 + 16;
  hipLaunchKernelGGL((rescore_kernel<TS>), dim3(nq), dim3(256), lds, st, merged,
                     kp, d_q, ix->dim, ix->w_qnorm.as<const double>(), ix->w_eps.as<const double>(),
                     ix->rows.as<const TS>(), ix->ld, ix->n, ix->norm64.as<const double>(), k, mode, thr,
                     ix->id_offset, out_s, out_i, ix->w_unc.as<int>(), ix->w_cnt.as<int>(),
                     ix->w_tauest.as<const uint32_t>(), ix->w_sk.as<uint64_t>(),
                     ix->has_idmap ? ix->idmap.as<const int64_t>() : nullptr, ix->gs_bound, ix->pass_hflag,
                     ix->pass_seq);
}

// Merge of the last <= G lists + rescore in one launch (finish_kernel); false when its LDS
// (the merge's keys + the fp64 query + the candidates) exceeds the CU's 160 KiB.
static constexpr size_t kFinishDynLds = kLdsBytes - 4096;   // (its static LDS: the scan, histogram)
static constexpr int kFinishMaxQueries = 512;     // (1024 fused: slower, r05v)
static size_t finish_lds(int np, int kp, int dim) {
  return (size_t)next_pow2(std::max(np * kp, kp)) * 8 + (size_t)dim * 8 + (size_t)kp * 24 + 16;
}
template <typename TS>
static int launch_finish(hcr_index* ix, const uint64_t* lists, const int* cnt, int np, const float* d_q,
                         int nq, int kp, int k, int mode, double thr, double* out_s, int64_t* out_i,
                         hipStream_t st) {
  static bool lds_done[kMaxDevices];
  CHECK(raise_lds_limit((const void*)finish_kernel<TS>, (int)kFinishDynLds, ix->device, lds_done));
  const int M = next_pow2(std::max(np * kp, kp));
  hipLaunchKernelGGL((finish_kernel<TS>), dim3(nq), dim3(256), finish_lds(np, kp, ix->dim), st, lists, cnt,
                     np, M, kp, d_q, ix->dim, ix->w_qnorm.as<const double>(), ix->w_eps.as<const double>(),
                     ix->rows.as<const TS>(), ix->ld, ix->n, ix->norm64.as<const double>(), k, mode, thr,
                     ix->id_offset, out_s, out_i, ix->w_unc.as<int>(), ix->w_cnt.as<int>(),
                     ix->w_tauest.as<const uint32_t>(), ix->w_sk.as<uint64_t>(),
                     ix->has_idmap ? ix->idmap.as<const int64_t>() : nullptr, ix->gs_bound, ix->pass_hflag,
                     ix->pass_seq);
  HIPC(hipGetLastError());
  return HCR_OK;
}

static constexpr int kSampleStrideDefault = 512;  // pre-pass samples 1 row tile in 512
                                                  // (estimated seed, r01d sweep at 10M x 768,
                                                  // B = 1024: 64 -> 512 saves ~0.5 ms)
// MAXONLY pre-pass stride: the largest power of two in [16, 128] that keeps >= 150 row tiles
// (~38k rows) in the sample.  The seed's global rank is ~j / (sampled fraction) (j = 8-25, see
// search_pass): a small corpus needs a denser sample for a seed tight enough to keep the dense
// pass's appends rare, a large one reaches it at 128.  r03 A/B (tools/rounds/r03_seed.sh, score ms):
// 1M x 384 B = 256 stride 64 0.270 / 32 0.264 / 16 0.260 (QS4); 1.25M x 768 B = 1024 (the W = 8
// rank shape) 64 1.746 / 32 1.712 / 16 1.723 / 8 1.873; 2.5M x 768 64 3.427 / 32 3.431 / 16
// 3.635; 10M x 768 128 13.20 / 64 13.23 / 32 13.48.
static constexpr int kSampleMinTiles = 150;
static constexpr int kSampleStrideMin = 16, kSampleStrideMaxAll = 128;
static int maxonly_stride(int64_t ntiles) {
  int s = kSampleStrideMin;
  while (s * 2 <= kSampleStrideMaxAll && ntiles / (s * 2) >= kSampleMinTiles) s *= 2;
  return s;
}
static constexpr int kPrepassMinTilesPerWg = 4;   // ... when each dense workgroup has >= 4 tiles
                                                  // (r01g, configs[1] 1M x 384 B = 256: 15 tiles
                                                  // per workgroup; seeded 0.32 ms vs cold 1.84 ms)

// tau_g[q] = ord32 score of the k'-th best key of the sample's merged list (0 if short)
// rank < kp: an ESTIMATED bound (not a k'-th of any row set); it is also written to tau_est
// so that the rescore certificate accounts for the rows it excluded
__global__ void seed_tau_kernel(const uint64_t* __restrict__ merged, int nq, int kp,
                                uint32_t* __restrict__ tau_g, int rank = 0,
                                uint32_t* __restrict__ tau_est = nullptr) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const uint64_t kth = merged[(size_t)q * kp + (rank > 0 ? rank : kp) - 1];
  tau_g[q] = kth ? (uint32_t)(kth >> 32) : 0u;
  if (tau_est) tau_est[q] = kth ? (uint32_t)(kth >> 32) : 0u;
}

// Seed from the sampling pre-pass's unit maxima ([U][nqpad] floats, one per 128-row half tile
// and query): the j-th largest of a query's U maxima is the score of j distinct rows, so
// j = k' gives a rigorous bound and a smaller j an estimate (tau_est).
__global__ void __launch_bounds__(256)
seed_from_maxima_kernel(const float* __restrict__ umax, int U, int nqpad, int j, int M,
                        uint32_t* __restrict__ tau_g, uint32_t* __restrict__ tau_est) {
  extern __shared__ uint64_t sv[];
  const int q = blockIdx.x;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const float v = i < U ? umax[(size_t)i * nqpad + q] : -INFINITY;
    sv[i] = (v == v && v > -INFINITY) ? (uint64_t)ord32(v) : 0ull;   // NaN / -inf: no row
  }
  __syncthreads();
  block_sort_desc_u64_fast(sv, M);
  if (threadIdx.x == 0) {
    const uint32_t t = j <= U ? (uint32_t)sv[j - 1] : 0u;
    tau_g[q] = t;
    if (tau_est) tau_est[q] = t;
  }
}

// The same seed with one wave per query and the U maxima in registers (E per lane, U <= 64 E):
// the j-th largest ordered key is the largest t with #{v >= t} >= j, found bit by bit from the
// top with ballot counts -- no LDS, no block barriers (the block sort above: 45 barrier-separated
// stages for U = 306; r03 kernel trace at the W = 8 rank shape, 1024 queries: 16 us).  Invalid
// maxima (NaN, -inf) are key 0, as there; fewer than j valid ones give 0.
template <int E>
__global__ void __launch_bounds__(256)
seed_select_kernel(const float* __restrict__ umax, int U, int nqpad, int nq, int j,
                   uint32_t* __restrict__ tau_g, uint32_t* __restrict__ tau_est) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  uint32_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = e * 64 + lane;
    const float x = i < U ? umax[(size_t)i * nqpad + q] : -INFINITY;
    v[e] = (x == x && x > -INFINITY) ? ord32(x) : 0u;
  }
  // The answer is a valid key between the smallest and largest valid one (when >= j are
  // valid; else 0), so it shares their common prefix: the search starts below it, two bits a
  // step (three independent ballot counts each).
  uint32_t mx = 0u, mn = 0xFFFFFFFFu;
  int nv = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (v[e]) { mx = v[e] > mx ? v[e] : mx; mn = v[e] < mn ? v[e] : mn; }
    nv += __popcll(__ballot(v[e] != 0u));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint32_t a = (uint32_t)__shfl_xor((int)mx, m), b = (uint32_t)__shfl_xor((int)mn, m);
    mx = a > mx ? a : mx;
    mn = b < mn ? b : mn;
  }
  uint32_t t = 0u;
  if (nv >= j) {
    const uint32_t d = mx ^ mn;
    int bit = d ? 31 - __clz(d) : -1;        // highest bit where the valid keys differ
    t = bit < 0 ? mx : (mx & ~((2u << bit) - 1u));
    for (; bit >= 1; bit -= 2) {
      const uint32_t c1 = t | (1u << (bit - 1)), c2 = t | (2u << (bit - 1)), c3 = t | (3u << (bit - 1));
      int n1 = 0, n2 = 0, n3 = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        n1 += __popcll(__ballot(v[e] >= c1));
        n2 += __popcll(__ballot(v[e] >= c2));
        n3 += __popcll(__ballot(v[e] >= c3));
      }
      t = n3 >= j ? c3 : n2 >= j ? c2 : n1 >= j ? c1 : t;
    }
    if (bit == 0) {
      int n = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) n += __popcll(__ballot(v[e] >= (t | 1u)));
      if (n >= j) t |= 1u;
    }
  }
  if (lane == 0) {
    tau_g[q] = t;
    if (tau_est) tau_est[q] = t;
  }
}

#ifdef HCR_FINISH_STAMPS
extern "C" int hcr_debug_finish_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hcr::hcr_fin_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif

__global__ void fill_f64(double* __restrict__ p, int64_t n, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// HCR_TEST_PLANT_BAD_KEY (hcr_index_test_hook): slot 0 of query 0's first list := the key (score 2.0, row)
__global__ void plant_key_kernel(uint64_t* __restrict__ list, int* __restrict__ cnt, uint32_t row) {
  if (threadIdx.x == 0) {
    list[0] = ((uint64_t)ord32(2.0f) << 32) | (uint64_t)(0xFFFFFFFFu - row);
    if (cnt && cnt[0] < 1) cnt[0] = 1;
  }
}

// Tree merge of the per-partition lists in ix->w_part ([q][P][kp] slots, counts in w_pcnt)
// into one sorted top-kp list per query ([q][kp] at the front of w_merged); G lists per block
// (G x kp <= kMergeMaxKeys: one level for P x kp <= 256 x 64), intermediate levels
// ping-ponging behind it.
// With out_cnt / out_p set, the levels stop once at most G lists per query remain (the caller's
// finish_kernel merges those): *out / *out_cnt / *out_p are then the remaining lists.
static int merge_groups(int kp) { return std::min(256, std::max(2, kMergeMaxKeys / kp)); }
static int merge_lists(hcr_index* ix, int nq, int nqpad, int P, int kp, hipStream_t st,
                       const uint64_t** out, const int** out_cnt = nullptr, int* out_p = nullptr) {
  // the dynamic-LDS limit is a per-device attribute: raised once per device, by whichever
  // thread gets there first (hcr_multi_search runs shards of several devices concurrently)
  static bool lds_done[kMaxDevices];
  CHECK(raise_lds_limit((const void*)merge_lists_kernel, kMergeMaxKeys * 8, ix->device, lds_done));
  const int G = merge_groups(kp);
  const int P2 = (P + G - 1) / G;
  const uint64_t* src = ix->w_part.as<const uint64_t>();
  const int* cnt = ix->w_pcnt.as<const int>();
  uint64_t* final_dst = ix->w_merged.as<uint64_t>();
  uint64_t* bufs[2] = {final_dst + (size_t)nqpad * kp, final_dst + (size_t)nqpad * kp * (1 + P2)};
  int* cbufs[2] = {ix->w_mcnt.as<int>(), ix->w_mcnt.as<int>() + (size_t)nqpad * P2};
  int which = 0, pin = P;
  while (true) {
    if (out_cnt && pin <= G) {
      *out = src;
      *out_cnt = cnt;
      *out_p = pin;
      return HCR_OK;
    }
    const int pout = (pin + G - 1) / G;
    const int M = next_pow2(std::min(G, pin) * kp);
    uint64_t* dst = pout == 1 ? final_dst : bufs[which];
    int* dcnt = pout == 1 ? nullptr : cbufs[which];
    hipLaunchKernelGGL(merge_lists_kernel, dim3(nq, pout), dim3(256), (size_t)M * 8, st, src, cnt,
                       pin, G, kp, dst, dcnt);
    HIPC(hipGetLastError());
    if (pout == 1) break;
    src = dst;
    cnt = dcnt;
    which ^= 1;
    pin = pout;
  }
  *out = final_dst;
  return HCR_OK;
}

// workspace keys of merge_lists: the final [nqpad][kp] list + two ping-pong levels
static size_t merge_workspace_keys(int nqpad, int P, int kp) {
  const int G = merge_groups(kp);
  const size_t P2 = (size_t)((P + G - 1) / G);
  return (size_t)nqpad * kp * (1 + (P2 > 1 ? 2 * P2 : 0));
}

// The corpus' norm statistics (rho, unit deviation): recomputed after an add.
static int refresh_norm_stats(hcr_index* ix) {
  if (!ix->rho_dirty) return HCR_OK;
  unsigned int rho_bits = 0;
  HIPC(hipStreamSynchronize(ix->stream));
  HIPC(hipMemcpy(&rho_bits, ix->rho.p, 4, hipMemcpyDeviceToHost));
  float rho_f;
  memcpy(&rho_f, &rho_bits, 4);
  ix->rho_host = (double)rho_f;
  unsigned long long* ud = reinterpret_cast<unsigned long long*>(ix->rho.as<char>() + 8);
  HIPC(hipMemsetAsync(ud, 0, 8, ix->stream));
  hipLaunchKernelGGL(unit_dev_kernel, dim3(1024), dim3(256), 0, ix->stream, ix->inv32.as<const float>(),
                     ix->n, ud);
  HIPC(hipGetLastError());
  unsigned long long ud_bits = 0;
  HIPC(hipStreamSynchronize(ix->stream));
  HIPC(hipMemcpy(&ud_bits, ud, 8, hipMemcpyDeviceToHost));
  memcpy(&ix->unit_dev_host, &ud_bits, 8);
  ix->rho_dirty = false;
  return HCR_OK;
}

// rigorous fp32 accumulation bound of a K-deep MFMA dot: gamma_{ld+1} + 4u (u = 2^-24)
static double accum_gamma(int ld) {
  const double u = std::ldexp(1.0, -24);
  const double nu = (ld + 1) * u;
  return nu / (1.0 - nu) + 4.0 * u;
}

// The pass's one host read (the certificate count and the bounds-check flag, w_cnt[0..1]); the
// stream's work is complete when it returns.  HCR_OPT_FLAG_READ: 1 = hipMemcpyAsync into pageable
// memory + hipStreamSynchronize (r05), 2 = the same into pinned memory, 3 / 4 = the last block of
// the pass's finish / rescore launch stores the flags and a sequence number into pinned coherent
// host memory (flags_prepare sets it up before that launch) and the host spins on the sequence
// number (no copy engine, no runtime wait, no extra launch), checking the stream for an error
// every 4096 polls; 3 then synchronises the stream (idle by then), 4 (the default) does not: the
// store comes after every other write of the pass.
static int flag_mode(const hcr_index* ix) { return ix->opt_flag_read == 0 ? 4 : ix->opt_flag_read; }
static int flags_prepare(hcr_index* ix) {
  ix->pass_hflag = nullptr;
  if (flag_mode(ix) == 1) return HCR_OK;
  if (!ix->h_flag) {
    void* h = nullptr;
    HIPC(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    memset(h, 0, 64);
    void* dp = nullptr;
    hipError_t e = hipHostGetDevicePointer(&dp, h, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(h);
      return set_err(HCR_EHIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    ix->h_flag = static_cast<int*>(h);
    ix->h_flag_dev = static_cast<int*>(dp);
  }
  if (flag_mode(ix) >= 3) {
    ix->pass_seq = ix->flag_seq = (ix->flag_seq % 0x3FFFFFFF) + 1;
    ix->pass_hflag = ix->h_flag_dev;
  }
  return HCR_OK;
}
static int read_pass_flags(hcr_index* ix, hipStream_t st, int* out) {
  const int mode = flag_mode(ix);
  ix->pass_hflag = nullptr;
  if (mode == 1) {
    HIPC(hipMemcpyAsync(out, ix->w_cnt.p, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    return HCR_OK;
  }
  if (mode == 2) {
    HIPC(hipMemcpyAsync(ix->h_flag + 1, ix->w_cnt.p, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    out[0] = ix->h_flag[1];
    out[1] = ix->h_flag[2];
    return HCR_OK;
  }
  const int seq = ix->pass_seq;
  for (unsigned it = 1;; ++it) {
    if (__atomic_load_n(ix->h_flag, __ATOMIC_ACQUIRE) == seq) break;
    if ((it & 4095u) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {                // (done: the stores are visible by now)
        if (__atomic_load_n(ix->h_flag, __ATOMIC_ACQUIRE) == seq) break;
        return set_err(HCR_EINTERNAL, "internal: the pass's finish launch completed without its flag store");
      }
      if (q != hipErrorNotReady) return set_err(HCR_EHIP, "search stream: %s", hipGetErrorString(q));
    }
    // (past ~0.3 ms of polling -- the large batches' searches take milliseconds -- the thread
    // yields its core between polls instead of spinning on it)
    if (it > 16384u) sched_yield();
    else __builtin_ia32_pause();
  }
  out[0] = __atomic_load_n(ix->h_flag + 1, __ATOMIC_RELAXED);
  out[1] = __atomic_load_n(ix->h_flag + 2, __ATOMIC_RELAXED);
  if (mode == 3) HIPC(hipStreamSynchronize(st));
  return HCR_OK;
}

// One pipeline pass over nq (<= kQueryChunk) device queries at candidate depth kp.
// Returns the number of uncertified queries in *n_unc (stream is synchronised).
static int search_pass(hcr_index* ix, const float* d_q, int nq, int k, int mode, double thr,
                       double* d_out_s, int64_t* d_out_i, int kp, hipStream_t st, int* n_unc,
                       std::vector<int>* unc_list, bool rigorous_seed = false) {
  const uint64_t* merged_ptr = nullptr;
  // kernel choice: v3/v4 (deep LDS-DMA ring, tile shape by batch size) for 16-bit rows;
  // v1 (register-staged 128 x 128, converts fp32 rows to bf16 on the way into LDS) for fp32
  // rows and for rows too narrow for the v3 tile-slot rings.
  CHECK(refresh_norm_stats(ix));
  const bool qwable = !ix->has_mask && ix->dtype != HCR_F32;
  const V3Cfg c3 = v3_cfg(nq, ix->n, ix->ld, ix->unit_dev_host <= kUnitDevMax,
                          qwable && qw_cap(kp, ix->ld, (nq + kQwQueries - 1) / kQwQueries) > 0, qwable && qw1_cap(kp, ix->ld) > 0,
                          ix->opt_qw1 >= 0 ? ix->opt_qw1 : hooks().qw1, ix->opt_qs, ix->opt_qw_min);
  const int ver = (ix->dtype == HCR_F32 || !v3_fits(ix, c3)) ? 1 : 3;
  if (hooks().debug_cfg)
    fprintf(stderr, "[hcrag] search_pass nq=%d n=%lld ld=%d kp=%d unit_dev=%.3g rho=%.3g mask=%d "
                    "qw1_opt=%d -> ver=%d rt=%d qt=%d qs=%d qw=%d qw1=%d\n", nq, (long long)ix->n,
            ix->ld, kp, ix->unit_dev_host, ix->rho_host, (int)ix->has_mask,
            ix->opt_qw1 >= 0 ? ix->opt_qw1 : hooks().qw1, ver, c3.rt, c3.qt, (int)c3.qs,
            (int)c3.qw, (int)c3.qw1);
  const int tq = ver == 3 ? c3.qt : BQ, tr = ver == 3 ? c3.rt : BR;
  const bool qs = ver == 3 && c3.qs, qw = ver == 3 && c3.qw, qw1 = ver == 3 && c3.qw1;
  // QS batches are padded to 256 queries for their MAXONLY pre-pass on the 256 x 256 kernel
  // (QW1's 192-query blocks: to both)
  const int nqpad = (int)(qw1 ? round_up(round_up(nq, tq), 256) : round_up(nq, qs ? 256 : tq));
  const int nqb = (int)round_up(nq, tq) / tq;
  const int ntiles = (int)((ix->n + tr - 1) / tr);
  const int cap = qs ? qs_cap(kp) : qw ? qw_cap(kp, ix->ld, nqb) : qw1 ? qw1_cap(kp, ix->ld) : next_pow2(kp + tr);
  const int wg_target = ver == 1 ? 512 : 256;
  // (QW: one workgroup per CU -- its LDS -- so at most 256 workgroups: one round)
  int P = qw1 ? qw1_partitions(nqb, ntiles)
               : qw ? std::max(1, wg_target / nqb) : std::max(1, (wg_target + nqb - 1) / nqb);
  P = std::min(P, ntiles);
  const int nwg = nqb * P;
  const int PL = P;                     // final lists per query: one per partition
  const bool tm_f16 = ix->dtype == HCR_F16;
  const size_t tms = 2;

  CHECK(ix->w_qhat.ensure((size_t)nqpad * ix->ld * tms));
  CHECK(ix->w_qnorm.ensure((size_t)nqpad * 8));
  CHECK(ix->w_eps.ensure((size_t)nqpad * 8));
  CHECK(ix->w_taug.ensure((size_t)nqpad * 4));
  CHECK(ix->w_buf.ensure((size_t)nwg * tq * cap * 8));
  CHECK(ix->w_part.ensure((size_t)nqpad * PL * kp * 8));
  CHECK(ix->w_pcnt.ensure((size_t)nqpad * PL * 4));
  CHECK(ix->w_merged.ensure(merge_workspace_keys(nqpad, PL, kp) * 8));
  CHECK(ix->w_mcnt.ensure((size_t)nqpad * ((PL + merge_groups(kp) - 1) / merge_groups(kp)) * 4 * 2));
  CHECK(ix->w_unc.ensure((size_t)nqpad * 4));
  CHECK(ix->w_cnt.ensure(16));
  CHECK(ix->w_tauest.ensure((size_t)nqpad * 4));
  CHECK(ix->w_sk.ensure((size_t)nqpad * 8));
  // (the per-query state -- q^ padding, tau_g, tau_est, the uncertified counter -- is reset
  // by prep_queries_kernel over the padded batch.  Padded query columns
  // (q^ = 0, every score 0) get the bound ord32(+inf): with bound 0 they passed the epilogue's
  // tile test on every tile and sent their waves down the exact path (r01g).)

  const double gamma_u = accum_gamma(ix->ld);
  const double rho = ix->rho_host;
  // UNIT score kernels (raw dot product as the coarse score) for L2-normalised corpora; the
  // certificate bound grows by (1+eps)(1+u)(unit_dev + u)
  const bool wide = ver == 3 && c3.rt == 256 && c3.qt == 256;   // v4
  const bool unit = (wide || qs || qw || qw1) && ix->unit_dev_host <= kUnitDevMax;
  const double unit_dev = unit ? ix->unit_dev_host : -1.0;
  ix->stats.unit_kernel = unit ? 1 : 0;
  if (ix->stats.score_kernel == 0)
    ix->stats.score_kernel = ver == 1 ? 1 : qw1 ? 7 : qw ? 6 : qs ? 5 : wide ? 4 : 3;

  const unsigned gq = (unsigned)((nqpad + 3) / 4);
  // (a seeded pass right after the sample call on the same queries: q^, eps and the per-query
  // state are what that call's prep left -- its pre-pass writes only the unit maxima)
  const bool prepped = ix->gs_umax && ix->gs_prep_q == d_q && ix->gs_prep_nq == nq && ix->gs_prep_gen == ix->gen;
  ix->gs_prep_q = nullptr;
  if (prepped) {
  } else if (tm_f16)
    hipLaunchKernelGGL((prep_queries_kernel<_Float16>), dim3(gq), dim3(256), 0, st, d_q, nq, nqpad,
                       ix->dim, ix->ld, ix->w_qhat.as<_Float16>(), ix->w_qnorm.as<double>(),
                       ix->w_eps.as<double>(), rho, gamma_u, unit_dev, ix->w_taug.as<uint32_t>(),
                       ix->w_tauest.as<uint32_t>(), ix->w_cnt.as<int>());
  else
    hipLaunchKernelGGL((prep_queries_kernel<__bf16>), dim3(gq), dim3(256), 0, st, d_q, nq, nqpad,
                       ix->dim, ix->ld, ix->w_qhat.as<__bf16>(), ix->w_qnorm.as<double>(),
                       ix->w_eps.as<double>(), rho, gamma_u, unit_dev, ix->w_taug.as<uint32_t>(),
                       ix->w_tauest.as<uint32_t>(), ix->w_cnt.as<int>());
  HIPC(hipGetLastError());

  if (ix->timing) HIPC(hipEventRecord(ix->ev0, st));
  if (ver == 3) {
    // Sampling pre-pass (every kSampleStride-th row tile): the k'-th best coarse key of the
    // sample is <= the global k'-th best coarse key, so it seeds the per-query global bound
    // tau_g exactly; the dense pass then appends only rows that can still be in the top-k'.
    const TestHooks& th = hooks();
    const int min_tiles = th.prepass_min_tiles ? th.prepass_min_tiles : kPrepassMinTilesPerWg;
    if (ix->gs_umax) {
      // global seed: the j-th largest of every shard's unit maxima ([U][nq], gathered by the
      // caller), j from the whole corpus' sampled fraction; the seed always counts as tau_est
      // (the rescore reports the bound of the rows it excluded, the merge certifies)
      const double lam = (double)k * ix->gs_frac;
      int j = th.seed_rank ? th.seed_rank : (int)std::ceil(lam + 5.0 * std::sqrt(lam) + 3.0);
      j = std::min(kp, std::max(1, j));
      const int U = ix->gs_units;
      const dim3 gw((unsigned)((nq + 3) / 4));
      const float* um = ix->gs_umax;
      uint32_t* tg = ix->w_taug.as<uint32_t>();
      uint32_t* te = ix->w_tauest.as<uint32_t>();
      if (U <= 512) hipLaunchKernelGGL(seed_select_kernel<8>, gw, dim3(256), 0, st, um, U, nq, nq, j, tg, te);
      else if (U <= 1024) hipLaunchKernelGGL(seed_select_kernel<16>, gw, dim3(256), 0, st, um, U, nq, nq, j, tg, te);
      else if (U <= 2048) hipLaunchKernelGGL(seed_select_kernel<32>, gw, dim3(256), 0, st, um, U, nq, nq, j, tg, te);
      else if (U <= 4096) hipLaunchKernelGGL(seed_select_kernel<64>, gw, dim3(256), 0, st, um, U, nq, nq, j, tg, te);
      else {
        // (more gathered units than 64 per lane: the block sort over all U, M = next_pow2(U) <=
        // 16384 keys of LDS -- ADVICE r5: seed_select_kernel<64> reads only the first 4096)
        const int M = next_pow2(U);
        static const bool big_lds = hipFuncSetAttribute((const void*)seed_from_maxima_kernel,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                                        160 * 1024) == hipSuccess;
        if (!big_lds && (size_t)M * 8 > 64 * 1024) return set_err(HCR_EHIP, "seed_from_maxima_kernel LDS attribute");
        hipLaunchKernelGGL(seed_from_maxima_kernel, dim3((unsigned)nq), dim3(256), (size_t)M * 8, st, um, U, nq, j,
                           M, tg, te);
      }
      HIPC(hipGetLastError());
    } else if (!th.no_prepass && ntiles >= (int64_t)P * min_tiles) {
      // Seed rank j.  j = k' is rigorous (k' real rows at or above the seed); a smaller j
      // estimates the global k'-th best much more tightly (the sample holds lambda = k' x
      // sampled fraction of the global top-k' on average, Poisson): j = lambda + 5 sqrt(lambda)
      // + 3 leaves fewer than k' rows above the seed with probability ~1e-6 per query, and the
      // certificate then counts the seed as the bound of the excluded rows, so such a query is
      // re-run (widened, rigorous seed, exact fallback) instead of answered wrong.
      // Two pre-pass forms: MAXONLY (default for the 256 x 256 kernel: the largest score of
      // every sampled 128-row unit per query, no candidate lists, stride 64) and the top-k'
      // form (every sampled row a candidate, merged; stride 512; the other tile shapes).
      const bool maxonly = !th.prepass_topk && (wide || qs || qw || qw1);
      int stride = th.sample_stride > 0 ? th.sample_stride
                   : ix->opt_stride > 0 ? ix->opt_stride
                                        : (maxonly ? maxonly_stride((ix->n + 255) / 256)
                                                   : kSampleStrideDefault);
      constexpr int kMaxUnits = 4096;
      // MAXONLY runs on the 256 x 256 kernel: nqpad / 256 query blocks, 256-row tiles (the
      // dense pass's tiles may be 128 rows: QS with two query blocks per wave)
      const int tr_pre = maxonly ? 256 : tr;
      const int64_t ntiles_pre = maxonly ? (ix->n + 255) / 256 : ntiles;
      if (maxonly) stride = std::max<int>(stride, (int)((2 * ntiles_pre + kMaxUnits - 1) / kMaxUnits));
      const int nqb_pre = maxonly ? nqpad / 256 : nqb;
      V3Launch a{nqb_pre, 0, (int)((ntiles_pre + stride - 1) / stride), stride, kp, unit};
      a.P = std::max(1, std::min(a.nvt, (wg_target + nqb_pre - 1) / nqb_pre));
      a.P = std::min(a.P, P);                  // partials / merge buffers are sized for P
      // r05: lambda counts the sample's expected share of the global top-k, not top-k': the
      // seed only has to leave >= k rows above it for the short-list certificate (B = tau_est,
      // DESIGN.md §4), and a lower j halves the dense pass's appends where k' >> k (configs[1]:
      // k = 10, k' = 64, stride 16: j 17 -> 8).
      int j = kp;
      if (!rigorous_seed && !th.rigorous_seed) {
        const int kseed = k;
        const double lam = (double)kseed * ((double)a.nvt * tr_pre) / (double)ix->n;
        j = th.seed_rank ? th.seed_rank : (int)std::ceil(lam + 5.0 * std::sqrt(lam) + 3.0);
        j = std::min(kp, std::max(1, j));
      }
      if (maxonly) {
        const int U = 2 * a.nvt;
        CHECK(ix->w_umax.ensure((size_t)U * nqpad * 4));
        // the sampled tiles on QW when the dense pass is QW with several query blocks (its
        // MAXONLY form, score_qw.h; r03: v4's form is LDS-fill-bound), on v4 otherwise -- with one
        // query block the sample is a few tiles per workgroup and QW's 256-query fragment
        // prologue dominates them (r05pp, interleaved: configs[1] score 0.2150 -> 0.2125 ms; B =
        // 256 at 10M x 768 a tie); HCR_OPT_PREPASS 1 / 2 force v4 / QW (under QS: QW's form when
        // HCR_OPT_PREPASS = 2 on a UNIT corpus without a row mask)
        const bool qw_pre = qw ? (ix->opt_prepass == 2 || (ix->opt_prepass == 0 && nqb_pre > 1))
                               : (qs && ix->opt_prepass == 2 && unit && !ix->has_mask && qw_supported(ix->ld));
        if (qw_pre) {
          QsArgs q{ix->rows.p, ix->ld, ix->n, ix->inv32.as<const float>(), nullptr, ix->w_qhat.p, nqb_pre,
                   a.P, a.nvt * (256 / qw_sample_rows(ix->ld)), a.tstride, ix->w_buf.as<uint64_t>(),
                   ix->w_taug.as<uint32_t>(), ix->w_part.as<uint64_t>(), ix->w_pcnt.as<int>(), kp, 256,
                   true, 0};
          q.umax = ix->w_umax.as<float>();
          CHECK(launch_qw(ix->dtype, q, st));
        } else if (ix->dtype == HCR_F16) CHECK(launch_v4_maxonly<_Float16>(ix, a, st));
        else CHECK(launch_v4_maxonly<__bf16>(ix, a, st));
        if (ix->gs_sample_only) {               // the shard's sample for a global seed: done
          ix->gs_sample_units = U;
          ix->gs_sample_nqpad = nqpad;
          ix->gs_sample_rows = (int64_t)a.nvt * tr_pre;
          ix->gs_prep_q = d_q;
          ix->gs_prep_nq = nq;
          ix->gs_prep_gen = ix->gen;
          if (ix->timing) {                     // (the pre-pass counts in the score phase)
            HIPC(hipEventRecord(ix->ev1, st));
            HIPC(hipEventSynchronize(ix->ev1));
            float ms = 0.f;
            HIPC(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
            ix->stats.score_kernel_ms += ms;
            ix->stats.score_launches += 1;
          }
          return HCR_OK;
        }
        uint32_t* te = j < kp ? ix->w_tauest.as<uint32_t>() : nullptr;
        const dim3 gw((unsigned)((nq + 3) / 4));
        const float* um = ix->w_umax.as<const float>();
        uint32_t* tg = ix->w_taug.as<uint32_t>();
        if (U <= 128) hipLaunchKernelGGL(seed_select_kernel<2>, gw, dim3(256), 0, st, um, U, nqpad, nq, j, tg, te);
        else if (U <= 256) hipLaunchKernelGGL(seed_select_kernel<4>, gw, dim3(256), 0, st, um, U, nqpad, nq, j, tg, te);
        else if (U <= 512) hipLaunchKernelGGL(seed_select_kernel<8>, gw, dim3(256), 0, st, um, U, nqpad, nq, j, tg, te);
        else if (U <= 1024) hipLaunchKernelGGL(seed_select_kernel<16>, gw, dim3(256), 0, st, um, U, nqpad, nq, j, tg, te);
        else {                                   // (the block sort for the largest samples)
          const int M = next_pow2(U);
          hipLaunchKernelGGL(seed_from_maxima_kernel, dim3((unsigned)nq), dim3(256), (size_t)M * 8, st,
                             um, U, nqpad, j, M, tg, te);
        }
        HIPC(hipGetLastError());
      } else {
        if (ix->dtype == HCR_F16) CHECK((dispatch_v3<_Float16>(ix, c3, a, cap, st)));
        else CHECK((dispatch_v3<__bf16>(ix, c3, a, cap, st)));
        const uint64_t* sample_best = nullptr;
        CHECK(merge_lists(ix, nq, nqpad, a.P, kp, st, &sample_best));
        hipLaunchKernelGGL(seed_tau_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st,
                           sample_best, nq, kp, ix->w_taug.as<uint32_t>(), j,
                           j < kp ? ix->w_tauest.as<uint32_t>() : nullptr);
        HIPC(hipGetLastError());
      }
    }
    if (ix->gs_sample_only) return HCR_OK;      // (no MAXONLY sample on this route: 0 units)
    const V3Launch a{nqb, P, (int)ntiles, 1, kp, unit};
    if (ix->dtype == HCR_F16) CHECK((dispatch_v3<_Float16>(ix, c3, a, cap, st)));
    else CHECK((dispatch_v3<__bf16>(ix, c3, a, cap, st)));
  } else if (ix->gs_sample_only) {
    return HCR_OK;
  } else if (ix->dtype == HCR_F16) CHECK((dispatch_score<_Float16, _Float16>(ix, nqb, P, ntiles, kp, cap, st)));
  else if (ix->dtype == HCR_BF16) CHECK((dispatch_score<__bf16, __bf16>(ix, nqb, P, ntiles, kp, cap, st)));
  else CHECK((dispatch_score<float, __bf16>(ix, nqb, P, ntiles, kp, cap, st)));
  if (ix->timing) HIPC(hipEventRecord(ix->ev1, st));

  const int* lcnt = nullptr;
  int lp = 0;
  CHECK(merge_lists(ix, nq, nqpad, PL, kp, st, &merged_ptr, &lcnt, &lp));
  // test hook (hcr_index_test_hook, per handle): a top-scored key naming
  // row n + 7 planted into query 0's first list, as a defective score kernel could leave it
  if (ix->test_plant_bad_key) {
    hipLaunchKernelGGL(plant_key_kernel, dim3(1), dim3(64), 0, st, const_cast<uint64_t*>(merged_ptr),
                       const_cast<int*>(lcnt), (uint32_t)ix->n + 7u);
    HIPC(hipGetLastError());
  }
  CHECK(flags_prepare(ix));            // (the finish / rescore launch's last block stores the flags)
  // fused for small batches (configs[1], B = 256: 0.372 vs 0.376 ms per search); above
  // 512 queries the separate launches (W = 8 rank shape, B = 1024: 1.973-1.985 vs
  // 1.985-1.998 ms: the fused block's merge LDS cuts the rescore's residency; r03f A/B)
  if (!hooks().no_finish && nq <= kFinishMaxQueries && finish_lds(lp, kp, ix->dim) <= kFinishDynLds) {
    // the last merge level and K4 in one launch
    if (ix->dtype == HCR_F16) CHECK(launch_finish<_Float16>(ix, merged_ptr, lcnt, lp, d_q, nq, kp, k, mode, thr, d_out_s, d_out_i, st));
    else if (ix->dtype == HCR_BF16) CHECK(launch_finish<__bf16>(ix, merged_ptr, lcnt, lp, d_q, nq, kp, k, mode, thr, d_out_s, d_out_i, st));
    else CHECK(launch_finish<float>(ix, merged_ptr, lcnt, lp, d_q, nq, kp, k, mode, thr, d_out_s, d_out_i, st));
  } else {
    // (lp lists remain: merge them to the single sorted list, then K4)
    uint64_t* final_dst = ix->w_merged.as<uint64_t>();
    const int G = merge_groups(kp);
    if (lp > 1 || merged_ptr != final_dst) {
      hipLaunchKernelGGL(merge_lists_kernel, dim3(nq, 1), dim3(256), (size_t)next_pow2(std::min(G, lp) * kp) * 8,
                         st, merged_ptr, lcnt, lp, G, kp, final_dst, (int*)nullptr);
      HIPC(hipGetLastError());
    }
    merged_ptr = final_dst;
    if (ix->dtype == HCR_F16) launch_rescore<_Float16>(ix, merged_ptr, d_q, nq, kp, k, mode, thr, d_out_s, d_out_i, st);
    else if (ix->dtype == HCR_BF16) launch_rescore<__bf16>(ix, merged_ptr, d_q, nq, kp, k, mode, thr, d_out_s, d_out_i, st);
    else launch_rescore<float>(ix, merged_ptr, d_q, nq, kp, k, mode, thr, d_out_s, d_out_i, st);
    HIPC(hipGetLastError());
  }

  int cnt2[2] = {0, 0};     // [0] uncertified queries, [1] candidate keys outside the index
  CHECK(read_pass_flags(ix, st, cnt2));
  if (cnt2[1] != 0)
    return set_err(HCR_EINTERNAL, "internal: a candidate key names a row outside the index (%lld rows); "
                   "the search was abandoned", (long long)ix->n);
  const int cnt = cnt2[0];
  *n_unc = cnt;
  if (ix->stats.partitions == 0) {
    ix->stats.partitions = P;
    ix->stats.workgroups = nwg;
  }
  if (ix->timing) {
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    ix->stats.score_kernel_ms += ms;
    ix->stats.score_launches += 1;
  }
  if (cnt > 0 && unc_list) {
    std::vector<int> flags(nq);
    HIPC(hipMemcpy(flags.data(), ix->w_unc.p, (size_t)nq * 4, hipMemcpyDeviceToHost));
    unc_list->clear();
    for (int i = 0; i < nq; ++i)
      if (flags[i]) unc_list->push_back(i);
  }
  return HCR_OK;
}

// ---- exact fallback (K6 + K7, topk_kernels.h) ----
static constexpr int kFallbackCap = 8192;     // buffer slots per query (LDS sort of 2 x 64 KiB)
static constexpr int kFallbackGroup = kFbGroup;  // queries per row scan (K6's LDS histograms)
static constexpr int kFallbackMaxRounds = 64; // each round strictly raises the threshold key
static constexpr int kMaxFastK = 256;         // k' = 2k <= 512: larger k go straight to K6/K7
static constexpr int kMaxK = 2048;            // kFallbackCap > k: every K7 round makes progress

// Exact top-k of the chunk-local queries `idx` of the m x dim device queries `qc` by one fp64
// scan of every row (a K6/K7 round per threshold); results go to rows idx[i] of os / oi.
// sk[i]: the starting threshold (K4's s_k of the candidates; 0 = every row).
// Deep path (k > kMaxK, r06: K7b + the bitonic segment sort of deep_sort.hip): `cap` > K7's
// 8192 LDS slots; the select step finds the exact k-th admitted key by a radix select and only
// the k answers are sorted.
int hcr_seg_sort_desc_pairs(uint64_t* hi, uint64_t* lo, int nseg, int P, hipStream_t st);   // deep_sort.hip
int hcr_launch_select_big(int nq, int k, int cap, int P, const unsigned int* cnt, const uint64_t* buf_hi,
                          const uint64_t* buf_lo, uint64_t* th_hi, uint64_t* th_lo, int* active, int* n_again,
                          double* h_lo, double* h_hi, const unsigned int* h_cnt, const unsigned long long* h_min,
                          int* est, uint64_t* sort_hi, uint64_t* sort_lo, hipStream_t st);
int hcr_launch_deep_emit(int nq, const uint64_t* sh, const uint64_t* sl, int P, int k, int mode, double thr,
                         int64_t id_offset, const int64_t* idmap, const int* out_idx, double* out_s, int64_t* out_i,
                         hipStream_t st);
int hcr_merge_sorted(const double* d_scores, const int64_t* d_ids, int g, int64_t nq, int k, double* d_out_scores,
                     int64_t* d_out_ids, hipStream_t st);
static constexpr size_t kDeepBudget = (size_t)2 << 30;   // admission + sort buffers of a deep group

// Round 0's starting thresholds from K6h's coarse histograms, on the device (r06: no readback
// and host pass between K6h and the first K6m round).  One wave per query without a starting
// threshold: from the top bin down, the first bin where the count reaches need_rows gives T =
// (lower edge) - 1e-5 - eps_q (every row counted there has exact >= T); no such
// bin leaves the query at "every row".  Lane l holds bins 8 l .. 8 l + 7.
__global__ void __launch_bounds__(64)
hist_seed_kernel(const unsigned int* __restrict__ hist, const double* __restrict__ eps, int ng,
                 unsigned long long need_rows, int est_flag, uint64_t* __restrict__ thh,
                 double* __restrict__ hlo, int* __restrict__ est) {
  const int q = blockIdx.x, lane = threadIdx.x;
  if (q >= ng || thh[q] != 0ull || eps[q] < 0.0) return;      // (eps < 0: zero query)
  static_assert(kFbHistBins == 8 * 64, "8 bins per lane");
  const unsigned int* h = hist + (size_t)q * kFbHistBins + lane * 8;
  unsigned long long mine = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) mine += h[i];
  // inclusive suffix sums over the lanes (lane l: bins >= 8 l)
  unsigned long long suf = mine;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long o = __shfl_down(suf, off);
    if (lane + off < 64) suf += o;
  }
  const uint64_t hit = __builtin_amdgcn_ballot_w64(suf >= need_rows);
  if (!hit) return;
  const int L = 63 - __builtin_clzll(hit);                    // the highest lane reaching it
  if (lane != L) return;
  unsigned long long acc = suf - mine;                        // bins above this lane's
  const double bw = 2.0 * kFbHistRange / kFbHistBins;
  for (int i = 7; i >= 0; --i) {
    acc += h[i];
    if (acc >= need_rows) {
      const int b = lane * 8 + i;
      // the host's (-R + b bw) - 1e-5 - eps, operation for operation (no contraction)
      const double T = __dsub_rn(__dsub_rn(__dadd_rn(-(double)kFbHistRange, __dmul_rn((double)b, bw)), 1e-5), eps[q]);
      thh[q] = ord64(T);
      hlo[q] = T;
      est[q] = est_flag;
      return;
    }
  }
}

// A fallback group's per-query state in one launch, a block per query (r06: six host-to-device
// copies, a memset and the query gather before, ~45 µs of the deep path's time line): from `up`
// ([ng] starting thresholds, then [ng] chunk-local query indices) or, up = nullptr, thresholds 0
// for queries idx0 + i; thl 0, active, no estimate, the first round's histogram range [the
// threshold's score (below -1 without one), just above 1], the query's fp32 row gathered into
// fq, and (ch != nullptr) its K6h histogram zeroed.
__global__ void __launch_bounds__(256)
fb_group_init_kernel(int ng, const uint64_t* __restrict__ up, int idx0, const float* __restrict__ qc, int dim,
                     int* __restrict__ idx, uint64_t* __restrict__ thh, uint64_t* __restrict__ thl,
                     int* __restrict__ act, int* __restrict__ est, double* __restrict__ hlo,
                     double* __restrict__ hhi, float* __restrict__ fq, unsigned int* __restrict__ ch) {
  const int i = blockIdx.x;
  if (i >= ng) return;
  const uint64_t t = up ? up[i] : 0ull;
  const int qi = up ? (int)up[ng + i] : idx0 + i;
  if (threadIdx.x == 0) {
    idx[i] = qi;
    thh[i] = t;
    thl[i] = 0ull;
    act[i] = 1;
    est[i] = 0;
    hlo[i] = t == 0ull ? -1.0 - 1e-6 : unord64(t);
    hhi[i] = 1.0 + 1e-6;
  }
  for (int j = threadIdx.x; j < dim; j += blockDim.x) fq[(int64_t)i * dim + j] = qc[(int64_t)qi * dim + j];
  if (ch)
    for (int j = threadIdx.x; j < kFbHistBins; j += blockDim.x) ch[(size_t)i * kFbHistBins + j] = 0u;
}

// A fallback round's counters in one launch (four memsets before, ~5 µs of time line each):
// admissions, the re-run count, the histograms, K6c's pair counts.
__global__ void fb_round_init_kernel(int ng, unsigned int* __restrict__ cnt, int* __restrict__ again,
                                     unsigned int* __restrict__ hcnt, unsigned long long* __restrict__ hmin, int nh,
                                     unsigned long long* __restrict__ pcnt, int npc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nh) {
    hcnt[i] = 0u;
    hmin[i] = ~0ull;
  }
  if (i < ng) cnt[i] = 0u;
  if (i == 0) *again = 0;
  if (pcnt && i < npc) pcnt[i] = 0ull;
}

static int exact_fallback(hcr_index* ix, const float* qc, const std::vector<int>& idx,
                          const std::vector<uint64_t>& sk, int k, int mode, double thr, double* os,
                          int64_t* oi, hipStream_t st, int64_t cap64 = kFallbackCap) {
  const bool big = cap64 > kFallbackCap;
  const int cap = (int)cap64;
  const size_t sel_lds = (size_t)2 * kFallbackCap * 8;
  if (!big)
    HIPC(hipFuncSetAttribute((const void*)exact_select_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)sel_lds));
  // the deep path's sort buffers: P = a power of two >= the most answers a query can have
  int P = 2;
  while (big && P < std::min<int64_t>(k, std::max<int64_t>(ix->n, 1))) P <<= 1;
  // the MFMA prefilter (K6m, and K6h for queries without a starting threshold) for 16-bit rows
  // at ld = 384 / 768 / 1024; K6 (an fp64 dot per row and query) otherwise
  const int ksteps = ix->ld / 32;
  const bool mf = ix->dtype != HCR_F32 && (ksteps == 12 || ksteps == 24 || ksteps == 32) &&
                  !hooks().no_mfma_filter;
  if (mf) CHECK(refresh_norm_stats(ix));
  // MFMA-prefiltered scans take up to kFbGroupsPerScan query groups at once (one pass over the
  // rows for all of them); the fp64 scan (K6) one group
  int super = mf ? kFallbackGroup * kFbGroupsPerScan : kFallbackGroup;
  // K6c's compacted pair list per query group (kFbGroup x cap slots: a group that admits more
  // coarse pairs is rescanned by the inline K6m)
  const bool two_launch = mf && !hooks().k6_inline;
  const int64_t pcap = hooks().k6_pcap > 0 ? hooks().k6_pcap : (int64_t)kFallbackGroup * cap64;
  if (big) {             // (the deep path's buffers per query: cap admitted + P sorted pairs + pairs)
    const int64_t per_q = (cap64 + P) * 16 + (two_launch ? cap64 * 8 : 0);
    const int64_t fit = std::max<int64_t>(1, (int64_t)(kDeepBudget / (size_t)per_q));
    super = (int)std::min<int64_t>(super, fit >= kFallbackGroup ? fit / kFallbackGroup * kFallbackGroup : fit);
  }
  // (MFMA scans: 512 row chunks per query group -- 2 x 512 blocks at the bench's 64 queries, two
  // rounds of blocks at their LDS: r06ac, deep k = 5000 1.32 -> 1.24 ms against 2048 chunks)
  const int64_t mchunks = round_up(std::max<int64_t>(1, std::min<int64_t>((ix->n + 31) / 32,
                                                                          hooks().k6_chunks ? hooks().k6_chunks : 512)), 8);
#define MFIL(TS, KS, MODE, QB)                                                                    \
  hipLaunchKernelGGL((exact_filter_mfma_kernel<TS, KS, MODE, QB>), dim3(grid), dim3(256), 0, st,       \
                     ix->f_qhat.as<const TS>(), ix->f_eps.as<const double>(), ix->f_q.as<const float>(), \
                     ng, ix->dim, ix->f_qn.as<const double>(), ix->rows.as<const TS>(), ix->ld, ix->n, \
                     ix->inv32.as<const float>(), ix->norm64.as<const double>(),                 \
                     ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,                \
                     ix->f_thh.as<const uint64_t>(), ix->f_thl.as<const uint64_t>(),            \
                     ix->f_act.as<const int>(), cap, ix->f_cnt.as<unsigned int>(),               \
                     ix->f_bufh.as<uint64_t>(), ix->f_bufl.as<uint64_t>(),                       \
                     ix->f_hlo.as<const double>(), ix->f_hhi.as<const double>(),                \
                     ix->f_hcnt.as<unsigned int>(), ix->f_hmin.as<unsigned long long>(),        \
                     ix->f_ch.as<unsigned int>(), ngr, hstride, pairs, pcnt, pcap)
#define MFIL_KS(TS, MODE, QB)                                                                     \
  do {                                                                                            \
    if (ksteps == 12) MFIL(TS, 12, MODE, QB); else if (ksteps == 24) MFIL(TS, 24, MODE, QB);     \
    else MFIL(TS, 32, MODE, QB);                                                                  \
  } while (0)
  // (the scan-only modes with both query halves per wave, QB = 2; HCRAG_K6_QB1: one, A/B)
#define MFIL_MODE(TS)                                                                             \
  do {                                                                                            \
    const bool qb1 = hooks().k6_qb1;                                                              \
    if (kmode == kK6Hist) { if (qb1) MFIL_KS(TS, kK6Hist, 1); else MFIL_KS(TS, kK6Hist, 2); }    \
    else if (kmode == kK6Compact) { if (qb1) MFIL_KS(TS, kK6Compact, 1); else MFIL_KS(TS, kK6Compact, 2); } \
    else if (kmode == kK6Rescore) MFIL_KS(TS, kK6Rescore, 1); else MFIL_KS(TS, kK6Inline, 1);    \
  } while (0)
  // kmode: kK6Hist / kK6Inline (pairs = nullptr: every group) / the two-launch form (K6c, K6r,
  // then the inline K6m for the groups whose pair list overflowed)
  auto launch_mfil = [&](int ng, int kmode, int hstride, uint64_t* pairs, unsigned long long* pcnt) {
    const int ngr = (ng + kFallbackGroup - 1) / kFallbackGroup;
    // (K6r: ~2048 blocks over the groups -- 8 waves per CU at its LDS, a few rounds)
    const int rb = hooks().k6r_blocks ? hooks().k6r_blocks : 512;
    const unsigned grid = (unsigned)(kmode == kK6Rescore ? ngr * rb : mchunks * ngr);
    if (ix->dtype == HCR_F16) MFIL_MODE(_Float16);
    else MFIL_MODE(__bf16);
  };
  for (size_t g0 = 0; g0 < idx.size(); g0 += super) {
    const int ng = (int)std::min<size_t>(super, idx.size() - g0);
    const int ngpad = (int)round_up(ng, kFallbackGroup);
    CHECK(ix->f_idx.ensure((size_t)ng * 4));
    CHECK(ix->f_q.ensure((size_t)ng * ix->dim * 4));
    CHECK(ix->f_qn.ensure((size_t)ng * 8));
    CHECK(ix->f_thh.ensure((size_t)ng * 8));
    CHECK(ix->f_thl.ensure((size_t)ng * 8));
    CHECK(ix->f_act.ensure((size_t)ng * 4));
    CHECK(ix->f_est.ensure((size_t)ng * 4));
    CHECK(ix->f_cnt.ensure((size_t)ng * 4));
    CHECK(ix->f_bufh.ensure((size_t)ng * cap * 8));
    CHECK(ix->f_bufl.ensure((size_t)ng * cap * 8));
    if (big) {
      CHECK(ix->f_sorth.ensure((size_t)ng * P * 8));
      CHECK(ix->f_sortl.ensure((size_t)ng * P * 8));
    }
    CHECK(ix->f_again.ensure(16));
    if (two_launch) {
      CHECK(ix->f_pcnt.ensure((size_t)kFbGroupsPerScan * 8 + 64));
      CHECK(ix->f_pairs.ensure((size_t)((ng + kFallbackGroup - 1) / kFallbackGroup) * (size_t)pcap * 8));
    }
    CHECK(ix->f_hlo.ensure((size_t)ng * 8));
    CHECK(ix->f_hhi.ensure((size_t)ng * 8));
    CHECK(ix->f_hcnt.ensure((size_t)ng * (kFbBins + 1) * 4));
    CHECK(ix->f_hmin.ensure((size_t)ng * (kFbBins + 1) * 8));
    const std::vector<uint64_t> thh(sk.begin() + g0, sk.begin() + g0 + ng);
    // the group's state on the device: queries g0 .. g0 + ng - 1 without starting thresholds (the
    // deep path, k > 256) need no upload; otherwise one copy of [thresholds | query indices]
    bool plain = true;
    for (int i = 0; i < ng && plain; ++i) plain = thh[i] == 0ull && idx[g0 + i] == (int)g0 + i;
    const uint64_t* up = nullptr;
    std::vector<uint64_t> upl;
    if (!plain) {
      CHECK(ix->f_tmp.ensure((size_t)round_up(ng, kFallbackGroup) * 24 + 64));   // (the prep's size below)
      upl.resize((size_t)ng * 2);
      for (int i = 0; i < ng; ++i) {
        upl[i] = thh[i];
        upl[ng + i] = (uint64_t)idx[g0 + i];
      }
      HIPC(hipMemcpyAsync(ix->f_tmp.p, upl.data(), (size_t)ng * 16, hipMemcpyHostToDevice, st));
      up = ix->f_tmp.as<const uint64_t>();
    }
    // round 0 (K6h) for the queries without a starting threshold (MFMA prefilter only)
    bool need0 = false;
    for (int i = 0; i < ng; ++i) need0 |= thh[i] == 0ull;
    need0 = need0 && mf;
    if (need0) CHECK(ix->f_ch.ensure((size_t)ngpad * kFbHistBins * 4));
    hipLaunchKernelGGL(fb_group_init_kernel, dim3((unsigned)ng), dim3(256), 0, st, ng, up, (int)g0, qc, ix->dim,
                       ix->f_idx.as<int>(), ix->f_thh.as<uint64_t>(), ix->f_thl.as<uint64_t>(), ix->f_act.as<int>(),
                       ix->f_est.as<int>(), ix->f_hlo.as<double>(), ix->f_hhi.as<double>(), ix->f_q.as<float>(),
                       need0 ? ix->f_ch.as<unsigned int>() : nullptr);
    HIPC(hipGetLastError());
    // (the MFMA route's prep writes the fp64 query norms, the same sum as query_norms_kernel's)
    if (!mf) {
      hipLaunchKernelGGL(query_norms_kernel, dim3((ng + 3) / 4), dim3(256), 0, st,
                         ix->f_q.as<const float>(), ng, ix->dim, ix->f_qn.as<double>());
      HIPC(hipGetLastError());
    }
    if (mf) {
      // the groups' unit MFMA-dtype queries and eps_q for the non-UNIT coarse score c =
      // fl(q^.e . inv32); padded to whole groups with zero queries
      CHECK(ix->f_qhat.ensure((size_t)ngpad * ix->ld * 2));
      CHECK(ix->f_eps.ensure((size_t)ngpad * 8));
      CHECK(ix->f_tmp.ensure((size_t)ngpad * 24 + 64));
      char* tmp = ix->f_tmp.as<char>();
#define PREP(TM)                                                                                   \
  hipLaunchKernelGGL((prep_queries_kernel<TM>), dim3((ngpad + 3) / 4), dim3(256), 0, st,           \
                     ix->f_q.as<const float>(), ng, ngpad, ix->dim, ix->ld, ix->f_qhat.as<TM>(),    \
                     ix->f_qn.as<double>(), ix->f_eps.as<double>(), ix->rho_host,                     \
                     accum_gamma(ix->ld), -1.0, reinterpret_cast<uint32_t*>(tmp + (size_t)ngpad * 8), \
                     reinterpret_cast<uint32_t*>(tmp + (size_t)ngpad * 12),                          \
                     reinterpret_cast<int*>(tmp + (size_t)ngpad * 16))
      if (ix->dtype == HCR_F16) PREP(_Float16); else PREP(__bf16);
#undef PREP
      HIPC(hipGetLastError());
      if (need0) {
        // round 0 (K6h): coarse histograms -> a starting threshold T_q <= the true k-th best
        // (zeroed by fb_group_init_kernel)
        // on a corpus of >= 12 k rows per sampled stride (10M rows, k <= 52k: 16), a sample
        // of runs of 4 16-row tiles, one in hstride: an estimated threshold (see K6h)
        int hstride = 1;
        // (the next stride must leave >= 12 k sampled rows; r06ah, deep k = 5000 on 1M x 384,
        // alternating processes: 100 -- the r05 rule -- 0.675 ms, 25 0.64-0.68, 12 0.63 (a 1/16
        // sample); at 10M rows the stride is 16 either way.  HCRAG_K6H_RATIO overrides, A/B)
        const int64_t ratio = hooks().k6h_ratio ? hooks().k6h_ratio : 12;
        while (hstride < 16 && ix->n / (2 * hstride) >= ratio * k) hstride *= 2;
        const int64_t ntile16 = (ix->n + 15) / 16, run = 4 * (int64_t)hstride;
        const int64_t stiles = ntile16 / run * 4 + std::min<int64_t>(4, ntile16 % run);
        const double frac = std::min(1.0, (double)(stiles * 16) / (double)ix->n);
        const double fk = frac * k;
        const uint64_t need_rows = hstride == 1 ? (uint64_t)k
                                                : (uint64_t)std::ceil(fk + 5.0 * std::sqrt(fk) + 3.0);
        launch_mfil(ng, kK6Hist, hstride, nullptr, nullptr);
        HIPC(hipGetLastError());
        hipLaunchKernelGGL(hist_seed_kernel, dim3((unsigned)ng), dim3(64), 0, st, ix->f_ch.as<const unsigned int>(),
                           ix->f_eps.as<const double>(), ng, (unsigned long long)need_rows, hstride > 1 ? 1 : 0,
                           ix->f_thh.as<uint64_t>(), ix->f_hlo.as<double>(), ix->f_est.as<int>());
        HIPC(hipGetLastError());
        ix->stats.fallback_rounds += 1;
      }
    }
    // (one histogram flush per block: 2048 blocks x 4 waves, ~1.2k rows per wave at 10M rows)
    const unsigned fgrid = (unsigned)std::min<int64_t>((ix->n + 3) / 4, 2048);
    int again = 1, rounds = 0;
    while (again > 0) {
      if (++rounds > kFallbackMaxRounds)
        return set_err(HCR_EHIP, "internal: exact fallback did not converge in %d rounds", kFallbackMaxRounds);
      const int ngr = (ng + kFallbackGroup - 1) / kFallbackGroup;
      const int nh = ng * (kFbBins + 1);
      hipLaunchKernelGGL(fb_round_init_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, ng,
                         ix->f_cnt.as<unsigned int>(), ix->f_again.as<int>(), ix->f_hcnt.as<unsigned int>(),
                         ix->f_hmin.as<unsigned long long>(), nh,
                         two_launch ? ix->f_pcnt.as<unsigned long long>() : nullptr, ngr);
      HIPC(hipGetLastError());
#define FIL(TS)                                                                                  \
  hipLaunchKernelGGL((exact_filter_kernel<TS>), dim3(fgrid), dim3(256), 0, st,                  \
                     ix->f_q.as<const float>(), ng, ix->dim, ix->f_qn.as<const double>(),       \
                     ix->rows.as<const TS>(), ix->ld, ix->n, ix->norm64.as<const double>(),     \
                     ix->has_mask ? ix->maskbits.as<const uint32_t>() : nullptr,                \
                     ix->f_thh.as<const uint64_t>(), ix->f_thl.as<const uint64_t>(),            \
                     ix->f_act.as<const int>(), cap, ix->f_cnt.as<unsigned int>(),               \
                     ix->f_bufh.as<uint64_t>(), ix->f_bufl.as<uint64_t>(),                       \
                     ix->f_hlo.as<const double>(), ix->f_hhi.as<const double>(),                \
                     ix->f_hcnt.as<unsigned int>(), ix->f_hmin.as<unsigned long long>())
      if (two_launch) {
        uint64_t* pr = ix->f_pairs.as<uint64_t>();
        unsigned long long* pc = ix->f_pcnt.as<unsigned long long>();
        launch_mfil(ng, kK6Compact, 1, pr, pc);
        launch_mfil(ng, kK6Rescore, 1, pr, pc);
        launch_mfil(ng, kK6Inline, 1, pr, pc);
      } else if (mf) {
        launch_mfil(ng, kK6Inline, 1, nullptr, nullptr);
      }
      else if (ix->dtype == HCR_F16) FIL(_Float16); else if (ix->dtype == HCR_BF16) FIL(__bf16); else FIL(float);
#undef FIL
      if (big)
        CHECK(hcr_launch_select_big(ng, k, cap, P, ix->f_cnt.as<const unsigned int>(), ix->f_bufh.as<const uint64_t>(),
                                    ix->f_bufl.as<const uint64_t>(), ix->f_thh.as<uint64_t>(), ix->f_thl.as<uint64_t>(),
                                    ix->f_act.as<int>(), ix->f_again.as<int>(), ix->f_hlo.as<double>(),
                                    ix->f_hhi.as<double>(), ix->f_hcnt.as<const unsigned int>(),
                                    ix->f_hmin.as<const unsigned long long>(), ix->f_est.as<int>(),
                                    ix->f_sorth.as<uint64_t>(), ix->f_sortl.as<uint64_t>(), st));
      else
        hipLaunchKernelGGL(exact_select_kernel, dim3(ng), dim3(256), sel_lds, st, k, cap,
                           ix->f_cnt.as<const unsigned int>(), ix->f_bufh.as<const uint64_t>(),
                           ix->f_bufl.as<const uint64_t>(), ix->f_thh.as<uint64_t>(),
                           ix->f_thl.as<uint64_t>(), ix->f_act.as<int>(), ix->f_again.as<int>(), mode,
                           thr, ix->id_offset, ix->has_idmap ? ix->idmap.as<const int64_t>() : nullptr,
                           ix->f_idx.as<const int>(), os, oi, ix->f_hlo.as<double>(),
                           ix->f_hhi.as<double>(), ix->f_hcnt.as<const unsigned int>(),
                           ix->f_hmin.as<const unsigned long long>(), ix->f_est.as<int>());
      HIPC(hipGetLastError());
      if (big) {
        // the sort of the k answers and the outputs, enqueued before the round's re-run count is
        // read (r06: the read-back, sync and launch had the sort wait ~40 µs for the host): a query
        // that finished in this or an earlier round holds its k keys in its sort segment (K7b
        // writes a segment only in the round its query finishes); a query still active gets its
        // segment sorted and emitted again after the round that finishes it, which is the last
        // write of its outputs.  Usually the first K6m round finishes every query.
        CHECK(hcr_seg_sort_desc_pairs(ix->f_sorth.as<uint64_t>(), ix->f_sortl.as<uint64_t>(), ng, P, st));
        CHECK(hcr_launch_deep_emit(ng, ix->f_sorth.as<const uint64_t>(), ix->f_sortl.as<const uint64_t>(), P, k,
                                   mode, thr, ix->id_offset, ix->has_idmap ? ix->idmap.as<const int64_t>() : nullptr,
                                   ix->f_idx.as<const int>(), os, oi, st));
      }
      // (K7 / the deep emit write the outputs before this sync: they are final when the search
      // call returns, hcrag.h)
      HIPC(hipMemcpyAsync(&again, ix->f_again.p, 4, hipMemcpyDeviceToHost, st));
      HIPC(hipStreamSynchronize(st));
    }
    ix->stats.fallback_rounds += rounds;
  }
#undef MFIL_MODE
#undef MFIL_KS
#undef MFIL
  return HCR_OK;
}

// ---- deep top-k: k > kMaxK (the fallback's LDS select holds 8192 slots) ----
// The exact fallback with admission buffers of cap = a power of two >= 4k slots per query (K6h's
// threshold admits ~k rows plus one histogram bin's worth; an overflow tightens it), the k-th
// best admitted key by a radix select, and a bitonic sort of the k answers (deep_sort.hip).  For
// the reference's argsort(...)[::-1][:top_k] at any top_k (experiments/main.py:844,889).
static int deep_topk(hcr_index* ix, const float* qc, int m, int k, int mode, double thr, double* os,
                     int64_t* oi, hipStream_t st) {
  if (ix->n > INT32_MAX) return set_err(HCR_EINVAL, "k > %d needs an index of < 2^31 rows", kMaxK);
  int64_t cap = 16384;
  while (cap < 4 * (int64_t)k && cap < ((int64_t)1 << 30)) cap <<= 1;
  // (no more slots than rows: an index of n <= cap rows never overflows)
  int64_t capn = 2;
  while (capn < ix->n) capn <<= 1;
  cap = std::max<int64_t>(std::min(cap, capn), kFallbackCap * 2);
  std::vector<int> all(m);
  for (int i = 0; i < m; ++i) all[i] = i;
  return exact_fallback(ix, qc, all, std::vector<uint64_t>(m, 0ull), k, mode, thr, os, oi, st, cap);
}

// Full search of nq device queries: certified top-k (K1-K4), certificate widening, and the
// exact fallback for whatever is still uncertified -- every returned list is the exact top-k.
static int search_device_impl(hcr_index* ix, const float* d_q, int64_t nq, int k, int mode,
                              double thr, double* d_out_s, int64_t* d_out_i, hipStream_t st) {
  ix->stats = hcr_search_stats{};
  if (nq == 0) return HCR_OK;
  if (ix->n == 0) {
    const int64_t tot = nq * (int64_t)k;
    hipLaunchKernelGGL(fill_empty, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, d_out_s,
                       d_out_i, tot);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    return HCR_OK;
  }
  const int kp0 = choose_kprime(std::min(k, kMaxFastK));
  ix->stats.kprime = k > kMaxFastK ? 0 : kp0;
  for (int64_t q0 = 0; q0 < nq; q0 += kQueryChunk) {
    const int m = (int)std::min<int64_t>(kQueryChunk, nq - q0);
    const float* qc = d_q + q0 * ix->dim;
    double* os = d_out_s + q0 * k;
    int64_t* oi = d_out_i + q0 * k;
    if (k > kMaxK) {                // deeper than the fallback's select: the sorted full scan
      CHECK(deep_topk(ix, qc, m, k, mode, thr, os, oi, st));
      ix->stats.fallback_queries += m;
      continue;
    }
    if (k > kMaxFastK) {            // no MFMA candidate path this deep: exact scan
      std::vector<int> all(m);
      for (int i = 0; i < m; ++i) all[i] = i;
      CHECK(exact_fallback(ix, qc, all, std::vector<uint64_t>(m, 0ull), k, mode, thr, os, oi, st));
      ix->stats.fallback_queries += m;
      continue;
    }
    int n_unc = 0;
    std::vector<int> unc;
    CHECK(search_pass(ix, qc, m, k, mode, thr, os, oi, kp0, st, &n_unc, &unc));
    std::vector<uint64_t> sk_chunk;     // K4's s_k per chunk query (filled for uncertified ones)
    auto read_sk = [&](int cnt, const std::vector<int>& local, const std::vector<int>* map) -> int {
      std::vector<uint64_t> skv((size_t)cnt);
      HIPC(hipMemcpy(skv.data(), ix->w_sk.p, (size_t)cnt * 8, hipMemcpyDeviceToHost));
      if (sk_chunk.empty()) sk_chunk.assign((size_t)m, 0ull);
      for (int j : local) sk_chunk[(size_t)(map ? (*map)[j] : j)] = skv[(size_t)j];
      return HCR_OK;
    };
    if (n_unc > 0) CHECK(read_sk(m, unc, nullptr));
    int kp = kp0;
    while (n_unc > 0 && kp < kMaxKprime) {
      kp = std::min(kMaxKprime, kp * 4);
      ix->stats.widened_queries += n_unc;
      const int nu = (int)unc.size();
      DevBuf idx, qsub, ssub, isub;
      CHECK(idx.ensure((size_t)nu * 4));
      CHECK(qsub.ensure((size_t)nu * ix->dim * 4));
      CHECK(ssub.ensure((size_t)nu * k * 8));
      CHECK(isub.ensure((size_t)nu * k * 8));
      HIPC(hipMemcpyAsync(idx.p, unc.data(), (size_t)nu * 4, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(gather_rows_f32, dim3(nu), dim3(256), 0, st, qc, idx.as<const int>(), nu,
                         ix->dim, qsub.as<float>());
      HIPC(hipGetLastError());
      std::vector<int> unc2;
      int n2 = 0;
      int rc = search_pass(ix, qsub.as<const float>(), nu, k, mode, thr, ssub.as<double>(),
                           isub.as<int64_t>(), kp, st, &n2, &unc2, /*rigorous_seed=*/true);
      if (rc == HCR_OK) {
        hipLaunchKernelGGL(scatter_topk, dim3(nu), dim3(64), 0, st, ssub.as<const double>(),
                           isub.as<const int64_t>(), idx.as<const int>(), nu, k, os, oi);
        hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = set_err(HCR_EHIP, "scatter: %s", hipGetErrorString(e));
      }
      if (rc == HCR_OK && n2 > 0) rc = read_sk(nu, unc2, &unc);
      // map the still-uncertified subset back to chunk-local query indices
      std::vector<int> mapped;
      for (int j : unc2) mapped.push_back(unc[j]);
      idx.release(); qsub.release(); ssub.release(); isub.release();
      if (rc != HCR_OK) return rc;
      unc.swap(mapped);
      n_unc = n2;
    }
    if (n_unc > 0) {
      // still uncertified at k' = 512 (clusters of near-ties wider than the candidate set, or
      // an over-shot estimated seed): one exact fp64 scan per query group settles them
      std::vector<uint64_t> sk((size_t)n_unc);
      for (int j = 0; j < n_unc; ++j) sk[(size_t)j] = sk_chunk[(size_t)unc[j]];
      CHECK(exact_fallback(ix, qc, unc, sk, k, mode, thr, os, oi, st));
      ix->stats.fallback_queries += n_unc;
    }
  }
  return HCR_OK;
}

extern "C" int hcr_search_device(hcr_index* ix, const float* d_queries, int64_t nq, int k,
                                 int score_mode, double threshold, double* d_out_scores,
                                 int64_t* d_out_ids, void* stream) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (nq < 0) return set_err(HCR_EINVAL, "negative query count");
  if (k <= 0) return set_err(HCR_EINVAL, "k must be >= 1, got %d", k);
  if (score_mode != HCR_SCORE_COSINE && score_mode != HCR_SCORE_UNIT)
    return set_err(HCR_EINVAL, "unknown score_mode %d", score_mode);
  if (nq > 0 && (!d_queries || !d_out_scores || !d_out_ids)) return set_err(HCR_EINVAL, "NULL buffer");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  // NULL = the legacy default stream (as every *_device entry point): the caller's work on
  // it (e.g. torch's default stream producing the input) is ordered before ours
  hipStream_t st = (hipStream_t)stream;
  if (st != ix->stream) HIPC(hipStreamSynchronize(ix->stream));
  return search_device_impl(ix, d_queries, nq, k, score_mode, threshold, d_out_scores, d_out_ids, st);
}

// Global seed across shards.  Step 1 on every shard: the sampling pre-pass only,
// its unit maxima copied to d_umax as [units][nq] floats (units = 0 when this shard's route has
// no MAXONLY sample: the caller then searches every shard the plain way).
extern "C" int hcr_search_sample_device(hcr_index* ix, const float* d_queries, int64_t nq, int k,
                                        float* d_umax, int64_t umax_cap, int* units,
                                        int64_t* sampled_rows, void* stream) {
  if (!ix || !units || !sampled_rows) return set_err(HCR_EINVAL, "NULL argument");
  if (nq <= 0 || nq > kQueryChunk) return set_err(HCR_EINVAL, "nq %lld not in [1, %d]", (long long)nq, kQueryChunk);
  if (k <= 0 || k > kMaxFastK) return set_err(HCR_EINVAL, "global seed: k %d not in [1, %d]", k, kMaxFastK);
  if (!d_queries || !d_umax) return set_err(HCR_EINVAL, "NULL buffer");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  hipStream_t st = (hipStream_t)stream;
  if (st != ix->stream) HIPC(hipStreamSynchronize(ix->stream));
  *units = 0;
  *sampled_rows = 0;
  if (ix->n == 0) return HCR_OK;
  ix->stats = hcr_search_stats{};
  ix->gs_sample_only = true;
  ix->gs_sample_units = 0;
  ix->gs_sample_rows = 0;
  int n_unc = 0;
  const int rc = search_pass(ix, d_queries, (int)nq, k, HCR_SCORE_COSINE, -INFINITY, nullptr, nullptr,
                             choose_kprime(k), st, &n_unc, nullptr);
  ix->gs_sample_only = false;
  CHECK(rc);
  const int U = ix->gs_sample_units;
  if (U == 0) return HCR_OK;
  if ((int64_t)U * nq > umax_cap)
    return set_err(HCR_EINVAL, "umax buffer holds %lld floats, the sample needs %d x %lld", (long long)umax_cap, U,
                   (long long)nq);
  // [U][nqpad] -> [U][nq]
  const int64_t nqpad = ix->gs_sample_nqpad;
  HIPC(hipMemcpy2DAsync(d_umax, (size_t)nq * 4, ix->w_umax.p, (size_t)nqpad * 4, (size_t)nq * 4, (size_t)U,
                        hipMemcpyDeviceToDevice, st));
  *units = U;
  *sampled_rows = ix->gs_sample_rows;
  return HCR_OK;
}

// Step 2 on every shard: the dense pass seeded from all shards' maxima (d_umax_all [units][nq],
// sampled_fraction = the shards' sampled rows / their rows), exact fp64 scores of the shard's
// candidates: its top k (fewer when fewer rows pass the seed: score -inf, id -1) and per query
// the bound every other row of the shard stays at or below (d_out_bound, exact cosine; -inf =
// none left out).  The merged list is exact where its k-th score exceeds every shard's bound.
extern "C" int hcr_search_seeded_device(hcr_index* ix, const float* d_queries, int64_t nq, int k,
                                        const float* d_umax_all, int units, double sampled_fraction,
                                        double* d_out_scores, int64_t* d_out_ids, double* d_out_bound,
                                        void* stream) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (nq <= 0 || nq > kQueryChunk) return set_err(HCR_EINVAL, "nq %lld not in [1, %d]", (long long)nq, kQueryChunk);
  if (k <= 0 || k > kMaxFastK) return set_err(HCR_EINVAL, "global seed: k %d not in [1, %d]", k, kMaxFastK);
  if (units <= 0 || units > 4 * 4096) return set_err(HCR_EINVAL, "units %d not in [1, 16384]", units);
  if (!(sampled_fraction > 0.0 && sampled_fraction <= 1.0))
    return set_err(HCR_EINVAL, "sampled_fraction %g not in (0, 1]", sampled_fraction);
  if (!d_queries || !d_umax_all || !d_out_scores || !d_out_ids || !d_out_bound)
    return set_err(HCR_EINVAL, "NULL buffer");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  hipStream_t st = (hipStream_t)stream;
  if (st != ix->stream) HIPC(hipStreamSynchronize(ix->stream));
  // (stats not reset: they accumulate over the sample + seeded pair of one search)
  if (ix->n == 0) {
    const int64_t tot = nq * (int64_t)k;
    hipLaunchKernelGGL(fill_empty, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, d_out_scores,
                       d_out_ids, tot);
    hipLaunchKernelGGL(fill_f64, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, d_out_bound, nq,
                       -INFINITY);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(st));
    return HCR_OK;
  }
  const int kp = choose_kprime(k);
  ix->stats.kprime = kp;
  ix->gs_umax = d_umax_all;
  ix->gs_units = units;
  ix->gs_frac = sampled_fraction;
  ix->gs_bound = d_out_bound;
  int n_unc = 0;
  const int rc = search_pass(ix, d_queries, (int)nq, k, HCR_SCORE_COSINE, -INFINITY, d_out_scores, d_out_ids,
                             kp, st, &n_unc, nullptr);
  ix->gs_umax = nullptr;
  ix->gs_units = 0;
  ix->gs_frac = 0.0;
  ix->gs_bound = nullptr;
  return rc;
}

extern "C" int hcr_search(hcr_index* ix, const float* queries, int64_t nq, int k, int score_mode,
                          double threshold, double* out_scores, int64_t* out_ids) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (nq < 0) return set_err(HCR_EINVAL, "negative query count");
  if (k <= 0) return set_err(HCR_EINVAL, "k must be >= 1, got %d", k);
  if (score_mode != HCR_SCORE_COSINE && score_mode != HCR_SCORE_UNIT)
    return set_err(HCR_EINVAL, "unknown score_mode %d", score_mode);
  if (nq == 0) return HCR_OK;
  if (!queries || !out_scores || !out_ids) return set_err(HCR_EINVAL, "NULL buffer");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  for (int64_t q0 = 0; q0 < nq; q0 += kQueryChunk) {
    const int64_t m = std::min<int64_t>(kQueryChunk, nq - q0);
    CHECK(ix->w_qin.ensure((size_t)m * ix->dim * 4));
    CHECK(ix->w_outs.ensure((size_t)m * k * 8));
    CHECK(ix->w_outi.ensure((size_t)m * k * 8));
    HIPC(hipMemcpyAsync(ix->w_qin.p, queries + q0 * ix->dim, (size_t)m * ix->dim * 4,
                        hipMemcpyHostToDevice, ix->stream));
    CHECK(search_device_impl(ix, ix->w_qin.as<const float>(), m, k, score_mode, threshold,
                             ix->w_outs.as<double>(), ix->w_outi.as<int64_t>(), ix->stream));
    HIPC(hipMemcpy(out_scores + q0 * k, ix->w_outs.p, (size_t)m * k * 8, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(out_ids + q0 * k, ix->w_outi.p, (size_t)m * k * 8, hipMemcpyDeviceToHost));
  }
  return HCR_OK;
}

extern "C" int hcr_score_all(hcr_index* ix, const float* queries, int64_t nq, int score_mode,
                             double* out_scores) {
  if (!ix) return set_err(HCR_EINVAL, "index is NULL");
  if (nq < 0) return set_err(HCR_EINVAL, "negative query count");
  if (score_mode != HCR_SCORE_COSINE && score_mode != HCR_SCORE_UNIT)
    return set_err(HCR_EINVAL, "unknown score_mode %d", score_mode);
  if (nq == 0 || ix->n == 0) return HCR_OK;
  if (!queries || !out_scores) return set_err(HCR_EINVAL, "NULL buffer");
  HIPC(hipSetDevice(ix->device));
  CHECK(wait_ingest(ix));
  const int64_t qc = 1024;
  for (int64_t q0 = 0; q0 < nq; q0 += qc) {
    const int m = (int)std::min<int64_t>(qc, nq - q0);
    CHECK(ix->w_qin.ensure((size_t)m * ix->dim * 4));
    CHECK(ix->w_qnorm.ensure((size_t)m * 8));
    CHECK(ix->w_outs.ensure((size_t)m * ix->n * 8));
    HIPC(hipMemcpyAsync(ix->w_qin.p, queries + q0 * ix->dim, (size_t)m * ix->dim * 4,
                        hipMemcpyHostToDevice, ix->stream));
    hipLaunchKernelGGL(query_norms_kernel, dim3((m + 3) / 4), dim3(256), 0, ix->stream,
                       ix->w_qin.as<const float>(), m, ix->dim, ix->w_qnorm.as<double>());
    dim3 grid((unsigned)((ix->n + 3) / 4), (unsigned)m);
#define EXA(TS)                                                                              \
  hipLaunchKernelGGL((exact_all_kernel<TS>), grid, dim3(256), 0, ix->stream,                 \
                     ix->w_qin.as<const float>(), ix->dim, ix->w_qnorm.as<const double>(),   \
                     ix->rows.as<const TS>(), ix->ld, ix->n, ix->norm64.as<const double>(), \
                     score_mode, ix->w_outs.as<double>())
    if (ix->dtype == HCR_F16) EXA(_Float16); else if (ix->dtype == HCR_BF16) EXA(__bf16); else EXA(float);
#undef EXA
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(out_scores + q0 * ix->n, ix->w_outs.p, (size_t)m * ix->n * 8,
                        hipMemcpyDeviceToHost, ix->stream));
    HIPC(hipStreamSynchronize(ix->stream));
  }
  return HCR_OK;
}

// ---- shard merges deeper than K5's 8192 LDS keys (g x k per query): hcr_merge_sorted,
// deep_sort.hip (one bitonic sort of (score, ~id) keys per query, the first k) ----

extern "C" int hcr_merge_topk_device(const double* d_scores, const int64_t* d_ids, int g,
                                     int64_t nq, int k, double* d_out_scores, int64_t* d_out_ids,
                                     void* stream) {
  if (g <= 0 || k <= 0 || nq < 0) return set_err(HCR_EINVAL, "bad merge shape g=%d k=%d", g, k);
  if (nq == 0) return HCR_OK;
  if (!d_scores || !d_ids || !d_out_scores || !d_out_ids) return set_err(HCR_EINVAL, "NULL buffer");
  if ((int64_t)g * k > 8192)
    return hcr_merge_sorted(d_scores, d_ids, g, nq, k, d_out_scores, d_out_ids, (hipStream_t)stream);
  const int M = next_pow2(g * k);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(merge_shards_kernel, dim3((unsigned)nq), dim3(256), (size_t)M * 16, st,
                     d_scores, d_ids, g, nq, k, M, d_out_scores, d_out_ids);
  HIPC(hipGetLastError());
  return HCR_OK;
}
