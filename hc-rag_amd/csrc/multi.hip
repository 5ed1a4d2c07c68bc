// multi.hip — single-process, multi-device node-embedding index (SURVEY.md §8(b) "one process
// drives all g devices", §8(e) row sharding + exchange of per-shard top-k).
//
// The reference's callers are single-process Python (experiments/main.py:738-905
// EmbeddingRAGSystem, query_interface.py:166-221 the LlamaIndex retrievers): this object lets
// them use every GPU of a node without torchrun.  Rows are sharded in contiguous blocks over
// the listed devices (a device may be listed more than once: several shards on one GPU), each
// shard is an ordinary hcr_index with its own stream, searched from its own host thread; the
// shards' exact top-k lists are gathered on the first device -- RCCL point-to-point sends to
// it (ncclCommInitAll over the distinct devices, one communicator per device; only the merging
// device receives) or, when devices repeat, RCCL cannot be loaded or its communicators cannot be
// created, peer copies -- and merged there by K5 (merge_shards_kernel).
//
// RCCL is bound at run time (dlopen of librccl.so.1): a process that already holds PyTorch's
// RCCL (same SONAME) shares that one instead of loading a second copy.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hcrag.h"
#include "host_common.h"

namespace {

// ---- RCCL entry points (run-time bound) ----
struct Rccl {
  bool tried = false, ok = false;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return r;
  r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
  r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  r.ok = r.comm_init_all && r.comm_destroy && r.send && r.recv && r.group_start && r.group_end &&
         r.error_string;
  return r;
}

#define NCCLC(expr)                                                                       \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return hcr_set_errorf(HCR_ERCCL, "%s: %s", #expr, rccl().error_string(r_));          \
  } while (0)

constexpr int kMergeMaxKeys = 8192;   // merge_shards_kernel sorts g*k keys in LDS

}  // namespace

struct hcr_multi_shard {
  int dev = 0;
  hcr_index* ix = nullptr;
  hipStream_t st = nullptr;
  DevBuf q, s, i;                     // queries and this shard's [nq][k] exact lists
  std::vector<int64_t> gids;          // global id of each local row (host copy, for masks)
};

struct hcr_multi_index {
  int g = 0, dim = 0, dtype = 0;
  int64_t n = 0;
  std::vector<hcr_multi_shard> sh;
  bool distinct = false;              // every shard on its own device
  bool rccl_init = false;
  int exchange = 0;                   // 1: RCCL gather to shard 0, 0: peer / device copies
  DevBuf gs, gi;                      // on shard 0's device: the merge's second ping-pong pair
  std::vector<ncclComm_t> comms;
  DevBuf cs, ci, ms, mi;              // on shard 0's device: gathered lists, merged lists
  hcr_search_stats stats{};
  bool broken = false;                // a failed add could not be rolled back (shard sizes and
                                      // id maps disagree): every later call refuses
};
static int refuse_broken(const hcr_multi_index* m) {
  return hcr_set_error(HCR_EINTERNAL, "multi-device index unusable: an earlier failed hcr_multi_add "
                                      "could not be rolled back");
}

extern "C" int hcr_multi_create(int n_dev, const int* dev_ids, int dim, int dtype,
                                int64_t capacity_rows, hcr_multi_index** out) {
  if (!out || !dev_ids) return hcr_set_error(HCR_EINVAL, "NULL argument");
  *out = nullptr;
  if (n_dev <= 0 || n_dev > 64) return hcr_set_errorf(HCR_EINVAL, "n_dev must be in [1, 64], got %d", n_dev);
  hcr_multi_index* m = new hcr_multi_index();
  m->g = n_dev;
  m->dim = dim;
  m->dtype = dtype;
  m->sh.resize(n_dev);
  std::vector<int> seen;
  for (int j = 0; j < n_dev; ++j) {
    hcr_multi_shard& s = m->sh[j];
    s.dev = dev_ids[j];
    const int64_t cap = capacity_rows > 0 ? (capacity_rows + n_dev - 1) / n_dev : 0;
    int rc = hcr_index_create(s.dev, dim, dtype, cap, &s.ix);
    if (rc == HCR_OK && hipSetDevice(s.dev) != hipSuccess) rc = hcr_set_error(HCR_EHIP, "hipSetDevice");
    if (rc == HCR_OK && hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking) != hipSuccess)
      rc = hcr_set_error(HCR_EHIP, "hipStreamCreate");
    if (rc != HCR_OK) {
      hcr_multi_destroy(m);
      return rc;
    }
    if (std::find(seen.begin(), seen.end(), s.dev) == seen.end()) seen.push_back(s.dev);
  }
  m->distinct = (int)seen.size() == n_dev;
  *out = m;
  return HCR_OK;
}

extern "C" int hcr_multi_destroy(hcr_multi_index* m) {
  if (!m) return HCR_OK;
  for (ncclComm_t c : m->comms)
    if (c) (void)rccl().comm_destroy(c);
  for (auto& s : m->sh) {
    (void)hipSetDevice(s.dev);
    if (s.st) (void)hipStreamSynchronize(s.st);
    s.q.release(); s.s.release(); s.i.release();
    if (s.st) (void)hipStreamDestroy(s.st);
    if (s.ix) hcr_index_destroy(s.ix);
  }
  if (!m->sh.empty()) {
    (void)hipSetDevice(m->sh[0].dev);
    m->cs.release(); m->ci.release(); m->ms.release(); m->mi.release(); m->gs.release(); m->gi.release();
  }
  delete m;
  return HCR_OK;
}

extern "C" int64_t hcr_multi_size(const hcr_multi_index* m) { return m ? m->n : -1; }
extern "C" int hcr_multi_num_shards(const hcr_multi_index* m) { return m ? m->g : -1; }
extern "C" int64_t hcr_multi_shard_size(const hcr_multi_index* m, int j) {
  return (m && j >= 0 && j < m->g) ? hcr_index_size(m->sh[j].ix) : -1;
}
extern "C" int hcr_multi_exchange_kind(const hcr_multi_index* m) { return m ? m->exchange : -1; }

// n rows -> g contiguous blocks, block j appended to shard j with global ids m->n + offset.
// All or nothing: when shard j's add fails, shards 0..j-1 drop the blocks they just took
// (hcr_index_truncate_internal), so a failed call leaves the index as it was.
extern "C" int hcr_multi_add(hcr_multi_index* m, const void* rows, int64_t n, int rows_dtype,
                             int normalize) {
  if (!m) return hcr_set_error(HCR_EINVAL, "index is NULL");
  if (m->broken) return refuse_broken(m);
  if (n < 0) return hcr_set_error(HCR_EINVAL, "negative row count");
  if (n == 0) return HCR_OK;
  if (!rows) return hcr_set_error(HCR_EINVAL, "rows is NULL");
  if (rows_dtype != HCR_F16 && rows_dtype != HCR_BF16 && rows_dtype != HCR_F32)
    return hcr_set_errorf(HCR_EINVAL, "unknown rows dtype %d", rows_dtype);
  const size_t rb = (size_t)m->dim * (rows_dtype == HCR_F32 ? 4 : 2);
  std::vector<int64_t> old_rows(m->g);
  std::vector<size_t> old_gids(m->g);
  for (int j = 0; j < m->g; ++j) {
    old_rows[j] = hcr_index_size(m->sh[j].ix);
    old_gids[j] = m->sh[j].gids.size();
  }
  for (int j = 0; j < m->g; ++j) {
    const int64_t r0 = n * j / m->g, r1 = n * (j + 1) / m->g;
    if (r1 == r0) continue;
    hcr_multi_shard& s = m->sh[j];
    const size_t old = s.gids.size();
    s.gids.resize(old + (size_t)(r1 - r0));
    for (int64_t r = r0; r < r1; ++r) s.gids[old + (size_t)(r - r0)] = m->n + r;
    // (test hook HCRAG_FAIL_MULTI_ADD=j: shard j's add fails after its rows went in, as an
    // allocation failure part-way through would, in every add after the index's first --
    // tests/test_exact_gpu.py)
    static const int fail_shard = [] {
      const char* e = getenv("HCRAG_FAIL_MULTI_ADD");
      return e ? atoi(e) : -1;
    }();
    int rc = hcr_index_add_ids(s.ix, (const char*)rows + (size_t)r0 * rb, r1 - r0, rows_dtype,
                               normalize, s.gids.data() + old);
    if (rc == HCR_OK && j == fail_shard && m->n > 0) rc = hcr_set_error(HCR_EHIP, "injected failure (HCRAG_FAIL_MULTI_ADD)");
    if (rc != HCR_OK) {
      const std::string msg = hcr_last_error();
      std::string undo_err;
      for (int i = 0; i <= j; ++i) {
        hcr_multi_shard& t = m->sh[i];
        if (hcr_index_size(t.ix) > old_rows[i] &&
            hcr_index_truncate_internal(t.ix, old_rows[i]) != HCR_OK && undo_err.empty())
          undo_err = hcr_last_error();
        // (a shard whose truncation failed keeps ids for every row it holds: no search maps a
        // local row past the end of its id map)
        t.gids.resize(std::max<size_t>(old_gids[i], (size_t)hcr_index_size(t.ix)));
      }
      if (!undo_err.empty()) {
        m->broken = true;
        return hcr_set_errorf(HCR_EINTERNAL, "%s; the rollback failed too (%s): the multi-device index "
                              "is unusable", msg.c_str(), undo_err.c_str());
      }
      return hcr_set_errorf(rc, "%s (hcr_multi_add rolled back: no row of the call was added)", msg.c_str());
    }
  }
  m->n += n;
  return HCR_OK;
}

extern "C" int hcr_multi_set_rowmask(hcr_multi_index* m, const uint8_t* mask, int64_t n) {
  if (!m) return hcr_set_error(HCR_EINVAL, "index is NULL");
  if (m->broken) return refuse_broken(m);
  if (mask && n != m->n) return hcr_set_errorf(HCR_EINVAL, "mask length %lld != index size %lld",
                                               (long long)n, (long long)m->n);
  std::vector<uint8_t> sub;
  for (auto& s : m->sh) {
    if (!mask) {
      CHECK(hcr_index_set_rowmask(s.ix, nullptr, 0));
      continue;
    }
    sub.resize(s.gids.size());
    for (size_t r = 0; r < s.gids.size(); ++r) sub[r] = mask[s.gids[r]];
    CHECK(hcr_index_set_rowmask(s.ix, sub.data(), (int64_t)sub.size()));
  }
  return HCR_OK;
}

static int init_rccl(hcr_multi_index* m) {
  m->rccl_init = true;
  m->exchange = 0;
  if (!m->distinct || !rccl().ok) return HCR_OK;     // peer copies
  std::vector<int> devs(m->g);
  for (int j = 0; j < m->g; ++j) devs[j] = m->sh[j].dev;
  m->comms.assign(m->g, nullptr);
  // a node whose RCCL cannot build communicators still searches, on peer copies
  if (rccl().comm_init_all(m->comms.data(), m->g, devs.data()) != ncclSuccess) {
    m->comms.clear();
    return HCR_OK;
  }
  m->exchange = 1;
  return HCR_OK;
}

extern "C" int hcr_multi_search(hcr_multi_index* m, const float* queries, int64_t nq, int k,
                                int score_mode, double threshold, double* out_scores,
                                int64_t* out_ids) {
  if (!m) return hcr_set_error(HCR_EINVAL, "index is NULL");
  if (m->broken) return refuse_broken(m);
  if (nq < 0) return hcr_set_error(HCR_EINVAL, "negative query count");
  if (k <= 0) return hcr_set_errorf(HCR_EINVAL, "k must be >= 1, got %d", k);
  if (nq == 0) return HCR_OK;
  if (!queries || !out_scores || !out_ids) return hcr_set_error(HCR_EINVAL, "NULL buffer");
  if (!m->rccl_init) CHECK(init_rccl(m));
  const int g = m->g;
  const size_t lst = (size_t)nq * k;          // elements of one shard's lists
  // 1) every shard: queries in, exact top-k of its rows (own thread, own stream)
  std::vector<int> rcs(g, HCR_OK);
  std::vector<std::string> errs(g);
  auto run = [&](int j) {
    hcr_multi_shard& s = m->sh[j];
    auto body = [&]() -> int {
      HIPC(hipSetDevice(s.dev));
      CHECK(s.q.ensure((size_t)nq * m->dim * 4));
      CHECK(s.s.ensure(lst * 8));
      CHECK(s.i.ensure(lst * 8));
      HIPC(hipMemcpyAsync(s.q.p, queries, (size_t)nq * m->dim * 4, hipMemcpyHostToDevice, s.st));
      return hcr_search_device(s.ix, s.q.as<const float>(), nq, k, score_mode, threshold,
                               s.s.as<double>(), s.i.as<int64_t>(), s.st);
    };
    rcs[j] = body();
    if (rcs[j] != HCR_OK) errs[j] = hcr_last_error();
  };
  std::vector<std::thread> th;
  for (int j = 1; j < g; ++j) th.emplace_back(run, j);
  run(0);
  for (auto& t : th) t.join();
  for (int j = 0; j < g; ++j)
    if (rcs[j] != HCR_OK) return hcr_set_errorf(rcs[j], "shard %d: %s", j, errs[j].c_str());
  m->stats = hcr_search_stats{};
  for (int j = 0; j < g; ++j) {
    hcr_search_stats st{};
    CHECK(hcr_index_last_stats(m->sh[j].ix, &st));
    m->stats.kprime = std::max(m->stats.kprime, st.kprime);
    m->stats.widened_queries += st.widened_queries;
    m->stats.uncertified_queries += st.uncertified_queries;
    m->stats.fallback_queries += st.fallback_queries;
    m->stats.fallback_rounds += st.fallback_rounds;
    m->stats.partitions += st.partitions;
    m->stats.workgroups += st.workgroups;
    m->stats.score_kernel = std::max(m->stats.score_kernel, st.score_kernel);
  }
  // 2) exchange: every shard's lists to shard 0's device as [g][nq][k] in m->cs / m->ci
  hcr_multi_shard& s0 = m->sh[0];
  HIPC(hipSetDevice(s0.dev));
  CHECK(m->cs.ensure(lst * g * 8));
  CHECK(m->ci.ensure(lst * g * 8));
  double* S = m->cs.as<double>();
  int64_t* I = m->ci.as<int64_t>();
  HIPC(hipMemcpyAsync(S, s0.s.p, lst * 8, hipMemcpyDeviceToDevice, s0.st));
  HIPC(hipMemcpyAsync(I, s0.i.p, lst * 8, hipMemcpyDeviceToDevice, s0.st));
  if (m->exchange == 1) {
    // a gather, not an all-gather: only the merging device receives (g - 1 lists of
    // nq x k x 16 bytes over its xGMI links)
    NCCLC(rccl().group_start());
    for (int j = 1; j < g; ++j) {
      hcr_multi_shard& s = m->sh[j];
      NCCLC(rccl().send(s.s.p, lst, ncclFloat64, 0, m->comms[j], s.st));
      NCCLC(rccl().send(s.i.p, lst, ncclInt64, 0, m->comms[j], s.st));
      NCCLC(rccl().recv(S + (size_t)j * lst, lst, ncclFloat64, j, m->comms[0], s0.st));
      NCCLC(rccl().recv(I + (size_t)j * lst, lst, ncclInt64, j, m->comms[0], s0.st));
    }
    NCCLC(rccl().group_end());
    for (int j = 1; j < g; ++j) {
      HIPC(hipSetDevice(m->sh[j].dev));
      HIPC(hipStreamSynchronize(m->sh[j].st));
    }
    HIPC(hipSetDevice(s0.dev));
  } else {
    for (int j = 1; j < g; ++j) {
      const hcr_multi_shard& s = m->sh[j];
      HIPC(hipMemcpyPeerAsync(S + (size_t)j * lst, s0.dev, s.s.p, s.dev, lst * 8, s0.st));
      HIPC(hipMemcpyPeerAsync(I + (size_t)j * lst, s0.dev, s.i.p, s.dev, lst * 8, s0.st));
    }
  }
  // 3) K5 merge on shard 0's device, in rounds of at most kMergeMaxKeys / k lists
  CHECK(m->ms.ensure(lst * g * 8));
  CHECK(m->mi.ensure(lst * g * 8));
  int lists = g;
  const double* src_s = S;
  const int64_t* src_i = I;
  // (k > kMergeMaxKeys / 2: one call over every list, merged by sorting -- hcr_merge_topk_device)
  const int G = kMergeMaxKeys / k >= 2 ? kMergeMaxKeys / k : g;
  bool into_m = true;
  CHECK(m->gs.ensure(lst * g * 8));             // cs / ci hold the gathered lists
  CHECK(m->gi.ensure(lst * g * 8));
  double* bs[2] = {m->ms.as<double>(), m->gs.as<double>()};
  int64_t* bi[2] = {m->mi.as<int64_t>(), m->gi.as<int64_t>()};
  while (lists > 1) {
    const int groups = (lists + G - 1) / G;
    double* ds = bs[into_m ? 0 : 1];
    int64_t* di = bi[into_m ? 0 : 1];
    for (int c = 0; c < groups; ++c) {
      const int l0 = c * G, nl = std::min(G, lists - l0);
      CHECK(hcr_merge_topk_device(src_s + (size_t)l0 * lst, src_i + (size_t)l0 * lst, nl, nq, k,
                                  ds + (size_t)c * lst, di + (size_t)c * lst, s0.st));
    }
    src_s = ds;
    src_i = di;
    into_m = !into_m;
    lists = groups;
  }
  HIPC(hipMemcpyAsync(out_scores, src_s, lst * 8, hipMemcpyDeviceToHost, s0.st));
  HIPC(hipMemcpyAsync(out_ids, src_i, lst * 8, hipMemcpyDeviceToHost, s0.st));
  HIPC(hipStreamSynchronize(s0.st));
  return HCR_OK;
}

extern "C" int hcr_multi_last_stats(const hcr_multi_index* m, hcr_search_stats* out) {
  if (!m || !out) return hcr_set_error(HCR_EINVAL, "NULL argument");
  *out = m->stats;
  return HCR_OK;
}
