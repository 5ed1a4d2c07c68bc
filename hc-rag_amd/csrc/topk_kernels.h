// topk_kernels.h — HIP kernels of the brute-force cosine top-k path.
//
// Pipeline for one query batch (all kernels on one stream):
//   K0 ingest_kernel         rows -> storage dtype (+ optional fp64 L2 normalisation),
//                            per-row fp64 norm, fp32 inverse norm, quantisation bound rho.
//   K1 prep_queries_kernel   fp32 queries -> fp64 norm, MFMA-dtype unit query q^, and the
//                            rigorous per-query bound eps_q >= |coarse - exact|.
//   K2 score_topk_kernel     fused MFMA GEMM (corpus tile x query block) + per-query top-k'
//                            epilogue: never materialises the B x N score matrix.
//   K3 merge_lists_kernel    per query, the partitions' surviving keys -> global top-k' keys.
//   K4 rescore_kernel        fp64 exact cosine of the k' candidates, (score desc, id asc)
//                            sort, certificate  c_k' + eps_q < s_k, top-k + mode + threshold.
//   K5 merge_shards_kernel   g row-shards' exact top-k lists -> global top-k (multi-GPU).
#pragma once
#include "device_common.h"
#include "tile_common.h"
#include "ring_common.h"

namespace hcr {

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }

// Global id of a shard-local row: the index's id map when rows were added with explicit ids
// (hcr_index_add_ids), else id_offset + row.
__device__ __forceinline__ int64_t row_id(int64_t id_offset, const int64_t* __restrict__ idmap,
                                          uint32_t row) {
  return idmap ? idmap[row] : id_offset + (int64_t)row;
}

// -------------------------------------------------------------------------------------
// K0: ingest. One wave per row.
// -------------------------------------------------------------------------------------
template <typename TIN, typename TS>
__global__ void __launch_bounds__(256)
ingest_kernel(const TIN* __restrict__ in, int64_t n, int dim, int ld, int normalize,
              TS* __restrict__ out_rows, double* __restrict__ norm64, float* __restrict__ inv32,
              unsigned int* __restrict__ rho_bits) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const TIN* src = in + row * dim;
  double scale = 1.0;
  if (normalize) {
    double ss = 0.0;
    for (int d = lane; d < dim; d += 64) { const double x = (double)to_f32(src[d]); ss += x * x; }
    ss = wave_sum_f64(ss);
    const double nr = sqrt(ss);
    scale = (nr < 10.0 * 2.220446049250313e-16) ? 1.0 : 1.0 / nr;
    // 16-bit storage: the ROUNDED row's norm misses 1 by the rounding (bf16: up to ~2e-3 over
    // 10M rows), which widens the UNIT kernels' certificate.  Of the 17 scales
    // scale * (1 + t 2^-12), |t| <= 8, keep the one whose rounded row's norm is closest to 1
    // (bf16: max deviation ~2e-3 -> ~6e-4): every stored row is still the input direction,
    // rounded once.
    if constexpr (sizeof(TS) == 2) {
      if (scale != 1.0 || nr == 1.0) {
        double best = 1e30, best_scale = scale;
        for (int t = 0; t <= 16; ++t) {
          const double sc = scale * (1.0 + (double)((t + 1) / 2 * ((t & 1) ? 1 : -1)) * 2.44140625e-4);
          double s2 = 0.0;
          for (int d = lane; d < dim; d += 64) {
            const double xd = (double)(float)(TS)(float)((double)to_f32(src[d]) * sc);
            s2 += xd * xd;
          }
          s2 = wave_sum_f64(s2);
          const double dev = fabs(sqrt(s2) - 1.0);
          if (dev < best) { best = dev; best_scale = sc; }
          if (best <= 6.103515625e-05) break;          // 2^-14: good enough
        }
        scale = best_scale;
      }
    }
  }
  double ss2 = 0.0, q2 = 0.0;
  TS* dst = out_rows + row * (int64_t)ld;
  for (int d = lane; d < ld; d += 64) {
    const double x = d < dim ? (double)to_f32(src[d]) * scale : 0.0;
    const TS v = (TS)(float)x;
    dst[d] = v;
    const double xd = (double)(float)v;
    ss2 += xd * xd;
    if constexpr (sizeof(TS) == 2 && __is_same(TS, _Float16)) {
      // f16 subnormals may be flushed by the MFMA: account for them in rho.
      if (xd != 0.0 && fabs(xd) < 6.103515625e-05) q2 += xd * xd;
    } else if constexpr (sizeof(TS) == 4) {
      // f32 rows enter the MFMA as bf16: per-row relative quantisation error.
      const double bq = (double)(float)(__bf16)(float)v;
      q2 += (bq - xd) * (bq - xd);
    }
  }
  ss2 = wave_sum_f64(ss2);
  q2 = wave_sum_f64(q2);
  if (lane == 0) {
    double nr = sqrt(ss2);
    if (nr < 10.0 * 2.220446049250313e-16) nr = 1.0;
    norm64[row] = nr;
    inv32[row] = (float)(1.0 / nr);
    if (q2 > 0.0) {
      const float rho = (float)(sqrt(q2) / nr) * 1.0001f;
      atomicMax(rho_bits, __float_as_uint(rho));
    }
  }
}

// -------------------------------------------------------------------------------------
// K1: query preparation. One wave per query.
//   q_n = q / ||q||_2 (fp64, sklearn zero rule), q^ = TM(q_n) with f16 subnormals -> 0,
//   eps = ||q^ - q_n|| + rho*||q^|| + gamma_u*||q^||*(1+rho)   
//         [+ the UNIT-kernel term when unit_dev >= 0]
//   eps < 0 marks a zero query (all scores exactly 0).
// It also resets the pass's per-query state over the padded batch (one launch instead of a
// memset each): tau_g (0; ord32(+inf) for the padding columns, whose scores are all 0 and
// must never pass an epilogue test), tau_est (0 = no estimated bound) and the pass's
// uncertified counter.
// -------------------------------------------------------------------------------------
template <typename TM>
__global__ void __launch_bounds__(256)
prep_queries_kernel(const float* __restrict__ q32, int nq, int nqpad, int dim, int ld,
                    TM* __restrict__ qhat, double* __restrict__ qnorm, double* __restrict__ eps,
                    double rho, double gamma_u, double unit_dev, uint32_t* __restrict__ tau_g,
                    uint32_t* __restrict__ tau_est, int* __restrict__ ucnt) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nqpad) return;
  if (lane == 0) {
    tau_g[q] = q < nq ? 0u : 0xFF800000u;
    tau_est[q] = 0u;
    if (q == 0) { ucnt[0] = 0; ucnt[1] = 0; ucnt[2] = 0; ucnt[3] = 0; }
  }
  if (q >= nq) {
    for (int d = lane; d < ld; d += 64) qhat[(int64_t)q * ld + d] = (TM)0.0f;
    return;
  }
  const float* src = q32 + (int64_t)q * dim;
  double ss = 0.0;
  for (int d = lane; d < dim; d += 64) { const double x = (double)src[d]; ss += x * x; }
  ss = wave_sum_f64(ss);
  double nr = sqrt(ss);
  const bool zero = !(nr > 0.0);
  if (nr < 10.0 * 2.220446049250313e-16) nr = 1.0;
  double d2 = 0.0, h2 = 0.0;
  TM* dst = qhat + (int64_t)q * ld;
  for (int d = lane; d < ld; d += 64) {
    const double x = d < dim ? (double)src[d] / nr : 0.0;
    TM h = (TM)(float)x;
    if constexpr (__is_same(TM, _Float16)) {
      if (fabs(x) < 6.103515625e-05) h = (TM)0.0f;
    }
    dst[d] = h;
    const double hd = (double)(float)h;
    d2 += (hd - x) * (hd - x);
    h2 += hd * hd;
  }
  d2 = wave_sum_f64(d2);
  h2 = wave_sum_f64(h2);
  if (lane == 0) {
    qnorm[q] = nr;
    const double delta = sqrt(d2), nh = sqrt(h2);
    double e = delta * (1.0 + 1e-9) + rho * nh + gamma_u * nh * (1.0 + rho) + 1e-12;
    // UNIT kernels (unit_dev >= 0): coarse = q^.e instead of fl(q^.e * inv32); the difference
    // is <= (1 + e)(1 + 2^-24)(max_r |1/inv32_r - 1| + 2^-24)
    if (unit_dev >= 0.0) e += (1.0 + e) * (1.0 + 0x1p-24) * (unit_dev + 0x1p-24) + 1e-15;
    eps[q] = zero ? -1.0 : e;
  }
}

// Wave-cooperative compaction of one query's candidate buffer to its best `kp` keys.
// Writes the sorted survivors back to `qbuf` (or to `out` when non-null, zero padded to kp),
// updates the LDS count / local threshold and raises the global threshold.
template <int CAP>
__device__ __forceinline__ void compact_query_inl(uint64_t* __restrict__ qbuf, int* cnt_q,
                                                  uint64_t* tau_key_q, uint32_t* tau_g_q, int kp,
                                                  int lane, uint64_t* __restrict__ out) {
  constexpr int E = CAP / 64;
  const int c = *cnt_q;
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int idx = lane * E + e;
    v[e] = idx < c ? qbuf[idx] : 0ull;
  }
  wave_sort_desc<E>(v, lane);
  const int nk = c < kp ? c : kp;
  if (out) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int idx = lane * E + e;
      if (idx < kp) out[idx] = v[e];      // zeros beyond nk
    }
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int idx = lane * E + e;
      if (idx < nk) qbuf[idx] = v[e];
    }
  }
  uint64_t kth = 0;
  if (nk == kp) {
    const int want = kp - 1, src_lane = want / E, src_e = want % E;
    uint64_t sel = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) sel = (e == src_e) ? v[e] : sel;
    kth = shfl_u64(sel, src_lane);
  }
  if (lane == 0) {
    *cnt_q = nk;
    *tau_key_q = kth;
    if (kth) atomicMax(tau_g_q, (uint32_t)(kth >> 32));
  }
}

// Final lists of a wave's queries ql = ql0, ql0 + qstep, .. < qend (candidate buffers
// wbuf[ql][CAP], LDS counts cnt[ql]): the keys whose coarse score reaches the query's CURRENT
// global bound tau_g go to its list (q, p) of the partials, unsorted (the merge sorts), their
// number to pcnt[q*P + p].  A key below tau_g is outside the global top-k' (tau_g is a
// rigorous k'-th coarse score of some workgroup's list, whose k' keys all pass here, or the
// estimated seed, which the certificate already treats as the bound of the rows it excludes:
// DESIGN.md §4), so dropping it changes no merged list's top-k'.  Most partitions keep a
// handful of keys, so the wave sort runs only when more than kp survive, and the merge reads
// only what was kept.  The next query's keys are loaded while the current one is written (one
// memory latency per query otherwise: the tail of every score kernel).
template <int CAP>
__device__ __forceinline__ void final_lists(uint64_t* __restrict__ wbuf, int* cnt, uint64_t* tau_key,
                                            uint32_t* tau_g, int qbase, int ql0, int qstep,
                                            int qend, int kp, int lane, uint64_t* __restrict__ partials,
                                            int* __restrict__ pcnt, int P, int p) {
  constexpr int E = CAP / 64;
  uint64_t v[E];
  int c = 0;
  uint32_t tg = 0;
  auto load = [&](int ql) __attribute__((always_inline)) {
    c = cnt[ql];
    tg = __hip_atomic_load(tau_g + qbase + ql, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int idx = e * 64 + lane;
      v[e] = idx < c ? wbuf[(size_t)ql * CAP + idx] : 0ull;
    }
  };
  if (ql0 < qend) load(ql0);
  for (int ql = ql0; ql < qend; ql += qstep) {
    bool keep[E];
    uint64_t w[E];
    int n = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      w[e] = v[e];
      keep[e] = w[e] != 0ull && (uint32_t)(w[e] >> 32) >= tg;
      n += __popcll(__ballot(keep[e]));
    }
    const int qg = qbase + ql;
    uint64_t* out = partials + ((size_t)qg * P + p) * kp;
    if (lane == 0) pcnt[(size_t)qg * P + p] = n < kp ? n : kp;
    if (n > kp) {             // more than k' survive: the wave sort, its best k' written
      compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql], tau_g + qg, kp, lane, out);
      if (ql + qstep < qend) load(ql + qstep);
      continue;
    }
    if (ql + qstep < qend) load(ql + qstep);      // in flight under this query's stores
    int base = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint64_t m = __ballot(keep[e]);
      const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (keep[e]) out[base + below] = w[e];
      base += __popcll(m);
    }
  }
}

// Final lists of a wave's queries ql0 + i qstep, i < nqw <= 64 (QW, QW1, QS: consecutive, one
// workgroup of 8 waves per CU), same output as final_lists.  (v3 / v4 / K2 keep final_lists: this
// call's registers -- 248 VGPRs at CAP = 1024 -- would cut their occupancy.)  final_lists walks the queries one after another, one
// dependent global load per query (the global bound, the buffer): ~18 us at the end of every
// configs[1] launch and ~25 us at the W = 8 rank shape (r05p stamps), 9 % of the former's dense
// pass.  Here lane l < nqw reads query l's count and bound at once, the candidates of all queries
// whose buffer holds <= kp keys are laid end to end (a wave prefix sum of the counts) and read
// 4 x 64 at a time -- one memory latency per 256 candidates, not per query -- and each kept key
// takes its slot in its query's list from the ballot.  A query with more than kp candidates (a
// full buffer: rare) goes through final_lists' wave sort.  (Not inlined: inlined, the score
// kernels' register allocation around their main loops changed and spilled.)
__device__ __forceinline__ uint64_t fl_mask_lt(int x) { return x >= 64 ? ~0ull : x <= 0 ? 0ull : (1ull << x) - 1ull; }

template <int CAP>
__device__ __attribute__((noinline)) void final_lists_wave(uint64_t* __restrict__ wbuf, int* cnt, uint64_t* tau_key,
                                                 uint32_t* tau_g, int qbase, int ql0, int qstep, int nqw, int kp,
                                                 int lane, uint64_t* __restrict__ partials,
                                                 int* __restrict__ pcnt, int P, int p) {
  const bool qlive = lane < nqw;
  const int my_ql = ql0 + lane * qstep;
  const int my_c = qlive ? cnt[my_ql] : 0;
  const uint32_t my_tg =
      qlive ? __hip_atomic_load(tau_g + qbase + my_ql, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  const bool big = my_c > kp;
  const int fc = big ? 0 : my_c;                   // candidates this query puts in the gather
  int incl = fc;                                    // inclusive prefix sum of fc over the lanes
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  const int excl = incl - fc;
  const int T = __shfl(incl, 63, 64);
  int nk = 0;                                       // keys kept so far (lane l: query l)
  constexpr int R = 4;
  for (int base = 0; base < T; base += 64 * R) {
    int qv[R];
    uint64_t kv[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int idx = base + u * 64 + lane;
      // the query of candidate idx: the last lane with excl <= idx (a query with fc = 0 shares
      // its excl with the next one, so the last such lane owns idx < T)
      int lo = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const int cand = lo + step;
        const int e = __shfl(excl, cand < 64 ? cand : 63, 64);
        if (cand < nqw && e <= idx) lo = cand;
      }
      qv[u] = lo;
      const int off = idx - __shfl(excl, lo, 64);
      kv[u] = idx < T ? wbuf[(size_t)(ql0 + lo * qstep) * CAP + off] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int b0 = base + u * 64;
      if (b0 >= T) break;
      const int q = qv[u];
      const uint64_t key = kv[u];
      const bool keep = key != 0ull && (uint32_t)(key >> 32) >= (uint32_t)__shfl((int)my_tg, q, 64);
      const uint64_t m = __ballot(keep);
      // this chunk's lanes of query q are [excl_q - b0, ...): the kept ones below this lane
      const int s_q = __shfl(excl, q, 64) - b0;
      const int pos = __shfl(nk, q, 64) + __popcll(m & fl_mask_lt(lane) & ~fl_mask_lt(s_q));
      if (keep) partials[((size_t)(qbase + ql0 + q * qstep) * P + p) * kp + pos] = key;
      // every query lane: its kept keys of this chunk
      nk += __popcll(m & fl_mask_lt(excl + fc - b0) & ~fl_mask_lt(excl - b0));
    }
  }
  if (qlive && !big) pcnt[(size_t)(qbase + my_ql) * P + p] = nk;
  // queries whose buffer holds more than kp keys: final_lists' path, one at a time
  uint64_t bigm = __ballot(big);
  while (bigm) {
    const int l = __builtin_ctzll(bigm);
    bigm &= bigm - 1;
    final_lists<CAP>(wbuf, cnt, tau_key, tau_g, qbase, ql0 + l * qstep, 1, ql0 + l * qstep + 1, kp, lane, partials, pcnt, P, p);
  }
}

template <int CAP>
__device__ __attribute__((noinline)) void compact_query(uint64_t* __restrict__ qbuf, int* cnt_q,
                                                      uint64_t* tau_key_q, uint32_t* tau_g_q,
                                                      int kp, int lane,
                                                      uint64_t* __restrict__ out) {
  compact_query_inl<CAP>(qbuf, cnt_q, tau_key_q, tau_g_q, kp, lane, out);
}

// -------------------------------------------------------------------------------------
// K2: fused score + top-k' kernel.
//   grid  = nqb query blocks x P row partitions (XCD-aware: the nqb blocks sharing one
//           partition's corpus tiles are dispatched consecutively on one XCD so each corpus
//           tile is fetched from HBM once and re-read from that XCD's L2).
//   block = 256 threads = 4 waves in 2 (rows) x 2 (queries); wave tile 64 rows x 64 queries
//           = 4 x 4 MFMA 16x16x32 accumulators.  C = E_tile . Q_block^T, so each lane holds
//           4 consecutive rows of ONE query per accumulator (query = lane & 15).
//   Each workgroup walks its partition's row tiles in ascending order, keeps a private
//   per-query candidate buffer (global, L2/MALL resident, CAP keys per query) and a local
//   threshold = its k'-th best key; a global per-query threshold (atomicMax of every
//   workgroup's local k'-th score, a valid lower bound of the global k'-th score) prunes.
// -------------------------------------------------------------------------------------
template <typename TS, typename TM, int CAP>
__global__ void __launch_bounds__(NT, 2)
score_topk_kernel(const TS* __restrict__ rows, int ld, int64_t n_rows, int ksteps,
                  const float* __restrict__ inv_norm, const uint32_t* __restrict__ mask,
                  const TM* __restrict__ qhat, int nqb, int P, int ntiles,
                  uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                  uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp) {
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  __shared__ __attribute__((aligned(16))) char lds[LDS_STAGES + BQ * 8 + BQ * 4 + 16];
  uint64_t* tau_key = reinterpret_cast<uint64_t*>(lds + LDS_STAGES);
  int* cnt = reinterpret_cast<int*>(lds + LDS_STAGES + BQ * 8);
  int* flag = reinterpret_cast<int*>(lds + LDS_STAGES + BQ * 12);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int qb = g % nqb, p = g / nqb;
  const int t0 = (int)((int64_t)p * ntiles / P);
  const int t1 = (int)((int64_t)(p + 1) * ntiles / P);
  const int qbase = qb * BQ;
  uint64_t* wbuf = buf + (size_t)b * BQ * CAP;

  for (int i = tid; i < BQ; i += NT) { tau_key[i] = 0ull; cnt[i] = 0; }
  if (tid == 0) *flag = 0;

  if (t0 >= t1) {              // an empty partition: empty lists
    for (int i = tid; i < BQ; i += NT) pcnt[(size_t)(qbase + i) * P + p] = 0;
    return;
  }

  const TM* qblk = qhat + (size_t)qbase * ld;
  TileLoader<TS> la;
  TileLoader<TM> lb;

  // fragment read offsets (bytes inside a tile image)
  const int lr = lane & 15;
  const int c0 = (lane >> 4) ^ (lane & 7);       // chunk slot for kk = 0
  const int offA0 = (wr * 64 + lr) * 128 + (c0 << 4);
  const int offA1 = (wr * 64 + lr) * 128 + ((c0 ^ 4) << 4);
  const int offB0 = (wc * 64 + lr) * 128 + (c0 << 4);
  const int offB1 = (wc * 64 + lr) * 128 + ((c0 ^ 4) << 4);

  floatx4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  // prologue: stage 0
  la.load(rows, (int64_t)t0 * BR, n_rows, ld, 0, tid);
  lb.load(qblk, 0, (int64_t)BQ, ld, 0, tid);
  la.store(lds, tid);
  lb.store(lds + BR * 128, tid);
  __syncthreads();

  const int nsteps = (t1 - t0) * ksteps;
  int tile = t0, ks = 0;
  float4 invv[4];
  uint4 mw = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  uint32_t tg[4];

  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = (s + 1) < nsteps;
    int ntile = tile, nks = ks + 1;
    if (nks == ksteps) { nks = 0; ++ntile; }
    const bool last_k = (ks == ksteps - 1);
    if (last_k) {
      const int64_t row0 = (int64_t)tile * BR;
#pragma unroll
      for (int m = 0; m < 4; ++m)
        invv[m] = *reinterpret_cast<const float4*>(inv_norm + row0 + wr * 64 + m * 16 + (lane >> 4) * 4);
      if (mask) mw = *reinterpret_cast<const uint4*>(mask + (row0 >> 5));
#pragma unroll
      for (int n = 0; n < 4; ++n)
        tg[n] = __hip_atomic_load(tau_g + qbase + wc * 64 + n * 16 + lr, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    if (more) {
      la.load(rows, (int64_t)ntile * BR, n_rows, ld, nks * BK, tid);
      lb.load(qblk, 0, (int64_t)BQ, ld, nks * BK, tid);
    }
    {
      const char* sa = lds + cur * STAGE_BYTES;
      const char* sb = sa + BR * 128;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int oa = kk ? offA1 : offA0;
        const int ob = kk ? offB1 : offB0;
        V a[4], bq[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = *reinterpret_cast<const V*>(sa + oa + m * 16 * 128);
#pragma unroll
        for (int n = 0; n < 4; ++n) bq[n] = *reinterpret_cast<const V*>(sb + ob + n * 16 * 128);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[m][n] = Op::run(a[m], bq[n], acc[m][n]);
      }
    }
    if (more) {
      char* st = lds + (cur ^ 1) * STAGE_BYTES;
      la.store(st, tid);
      lb.store(st + BR * 128, tid);
    }
    __syncthreads();

    if (last_k) {
      // ------------------------------- epilogue --------------------------------------
      const int64_t row0 = (int64_t)tile * BR;
      float thr[4];
      uint64_t tk[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int ql = wc * 64 + n * 16 + lr;
        tk[n] = tau_key[ql];
        const float ls = tk[n] ? key_score(tk[n]) : -INFINITY;
        thr[n] = fmaxf(ls, unord32(tg[n]));
      }
      float iv[4][4];
      const uint32_t mwa[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int rl = wr * 64 + m * 16 + (lane >> 4) * 4;   // row inside tile
        const float ivm[4] = {invv[m].x, invv[m].y, invv[m].z, invv[m].w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = rl + r;
          const bool ok = (row0 + rr < n_rows) && ((mwa[rr >> 5] >> (rr & 31)) & 1u);
          iv[m][r] = ok ? ivm[r] : __builtin_nanf("");
        }
      }
      bool hit[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        float mx = -INFINITY;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[m][n][r] * iv[m][r]);
        hit[n] = mx >= thr[n];
      }
      if (__any(hit[0] | hit[1] | hit[2] | hit[3])) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          if (hit[n]) {
            const int ql = wc * 64 + n * 16 + lr;
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float sc = acc[m][n][r] * iv[m][r];
                if (sc >= thr[n]) {
                  const uint32_t lrow = (uint32_t)(row0 + wr * 64 + m * 16 + (lane >> 4) * 4 + r);
                  const uint64_t key = make_key(sc, lrow);
                  if (key > tk[n]) {
                    const int pos = atomicAdd(&cnt[ql], 1);
                    wbuf[(size_t)ql * CAP + pos] = key;
                    if (pos + 1 > CAP - BR) *flag = 1;
                  }
                }
              }
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      __syncthreads();
      if (*flag) {
        for (int ql = wave; ql < BQ; ql += 4) {
          if (cnt[ql] > CAP - BR)
            compact_query<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                               tau_g + qbase + ql, kp, lane, nullptr);
        }
        __syncthreads();
        if (tid == 0) *flag = 0;
      }
    }
    tile = ntile;
    ks = nks;
  }

  // final: every query's surviving keys (at most k') appended to its region of the partials
  final_lists<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wave, 4, BQ, kp, lane, partials, pcnt, P, p);
}

// Radix selection by a block of 256 threads over the keys a[0..c), c > kp: moves to the front
// of a every key whose high word (its coarse score, ord32) is >= that of the kp-th largest key
// and returns their count (kp, more only with tied scores).  Four passes of 8-bit digits of
// the high word: LDS histogram, then one wave finds the digit holding the kp-th key.
__device__ inline int block_select_top_u64(uint64_t* a, int c, int kp, int* hist, int* misc) {
  const int t = threadIdx.x;
  uint32_t prefix = 0, pmask = 0;
  int need = kp;                                   // keys still to take at or below the prefix
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[t] = 0;
    __syncthreads();
    for (int e = t; e < c; e += 256) {
      const uint32_t h = (uint32_t)(a[e] >> 32);
      if ((h & pmask) == prefix) atomicAdd(&hist[(h >> shift) & 255], 1);
    }
    __syncthreads();
    if (t < 64) {
      int v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = hist[4 * t + j];
      const int s = v[0] + v[1] + v[2] + v[3];
      int incl = s;                                // sum over lanes >= t (their bins are higher)
      for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_down(incl, o);
        if (t + o < 64) incl += x;
      }
      int above = incl - s;
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        if (above < need && above + v[j] >= need) { misc[0] = 4 * t + j; misc[1] = above; }
        above += v[j];
      }
    }
    __syncthreads();
    need -= misc[1];
    prefix |= (uint32_t)misc[0] << shift;
    pmask |= 255u << shift;
    __syncthreads();
  }
  if (t == 0) misc[2] = 0;
  __syncthreads();
  for (int e0 = 0; e0 < c; e0 += 256) {            // in-place compaction, chunk by chunk
    const int e = e0 + t;
    const uint64_t v = e < c ? a[e] : 0ull;
    const bool keep = e < c && (uint32_t)(v >> 32) >= prefix;
    __syncthreads();                               // the chunk is read before any write
    if (keep) a[atomicAdd(&misc[2], 1)] = v;       // < e0 + 256: never an unread key
    __syncthreads();
  }
  return misc[2];
}

// -------------------------------------------------------------------------------------
// K3: merge the partition survivors of one query into its global top-k' (sorted desc).
// -------------------------------------------------------------------------------------
// lists: [q][P][kp] slots, list (q, p) holding cnt[q*P + p] keys (a score kernel's final_list
// or a previous level).  One block gathers lists [p0, p0 + np) (np <= blockDim) of query q into
// LDS -- a block scan of their counts places them -- selects and sorts them: on return
// sm_keys[0, m) is sorted descending (m a power of two >= kp, zero padded) and the count of
// real keys kept (min(count, kp) are the top of the merge) is returned.
__device__ __forceinline__ int merge_block_lds(const uint64_t* __restrict__ lists, const int* __restrict__ cnt,
                                               int P, int p0, int np, int kp, int q, uint64_t* sm_keys,
                                               int* s_off, int* s_hist, int* s_misc) {
  const int t = threadIdx.x;
  const int c_t = t < np ? min(cnt[(size_t)q * P + p0 + t], kp) : 0;
  // inclusive scan of the counts: a shuffle scan per wave, then the waves' totals (two block
  // barriers; the block-wide Hillis-Steele scan took sixteen)
  const int lane = t & 63, wv = t >> 6;
  int x = c_t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_misc[wv] = x;                     // (s_misc: 4 ints, 4 waves)
  if (t == 0) s_off[0] = 0;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wv; ++w) base += s_misc[w];
  s_off[t + 1] = base + x;
  __syncthreads();
  const int c = s_off[256];
  // flat gather: key e of the concatenation comes from the list l with s_off[l] <= e <
  // s_off[l + 1] (binary search in LDS), so all loads are independent (a wave per list
  // serialised one memory latency per list: r02m, 68 us at P = 256)
  const uint64_t* src = lists + ((size_t)q * P + p0) * kp;
  for (int e = t; e < c; e += blockDim.x) {
    int lo = 0, hi = np;                                // s_off[lo] <= e < s_off[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_off[mid] <= e) lo = mid; else hi = mid;
    }
    sm_keys[e] = src[(size_t)lo * kp + (e - s_off[lo])];
  }
  __syncthreads();
  // a loose seed leaves several k' keys per query (r02n: ~650 at 1M x 384, k' = 64): select
  // the top k' by score first, then sort only those
  const int cs = c > 2 * kp ? block_select_top_u64(sm_keys, c, kp, s_hist, s_misc) : c;
  int m = 1;
  while (m < cs || m < kp) m <<= 1;                   // <= G * kp (host sizes the LDS)
  for (int i = cs + t; i < m; i += blockDim.x) sm_keys[i] = 0ull;
  __syncthreads();
  block_sort_desc_u64_fast(sm_keys, m);
  return cs;
}

#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
// Block (q, grp) merges lists [grp*G, grp*G + G): with pout == 1 (the last level) it writes the
// sorted top-kp, zero padded, to out[q*kp ..]; otherwise the top min(count, kp) to list
// (q, grp) of the next level, [q][pout][kp] with counts cnt_out.
__global__ void __launch_bounds__(256)
merge_lists_kernel(const uint64_t* __restrict__ lists, const int* __restrict__ cnt, int P, int G,
                   int kp, uint64_t* __restrict__ out, int* __restrict__ cnt_out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm_keys[];
  __shared__ int s_off[257], s_hist[256], s_misc[4];
  const int q = blockIdx.x, grp = blockIdx.y, pout = gridDim.y;
  const int p0 = grp * G;
  const int t = threadIdx.x;
  const int cs = merge_block_lds(lists, cnt, P, p0, min(G, P - p0), kp, q, sm_keys, s_off, s_hist, s_misc);
  if (pout == 1) {
    uint64_t* dst = out + (size_t)q * kp;
    for (int i = t; i < kp; i += blockDim.x) dst[i] = sm_keys[i];
    return;
  }
  const int take = min(cs, kp);
  uint64_t* dst = out + ((size_t)q * pout + grp) * kp;
  for (int i = t; i < take; i += blockDim.x) dst[i] = sm_keys[i];
  if (t == 0) cnt_out[(size_t)q * pout + grp] = take;
}
#endif

// Eight stored elements of a row (one 16-byte load; two for fp32) as floats.
template <typename TS>
__device__ __forceinline__ void load8_f32(const TS* __restrict__ p, float (&x)[8]) {
  if constexpr (__is_same(TS, float)) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = (float)__builtin_bit_cast(TS, (unsigned short)(w[i] & 0xFFFFu));
      x[2 * i + 1] = (float)__builtin_bit_cast(TS, (unsigned short)(w[i] >> 16));
    }
  }
}

// The exact-score summation order shared by K4 and K6 (their scores are bit-identical, which
// the fallback's threshold keys rely on): lane l accumulates dims [8l, 8l + 8), then
// [8l + 512, ...), in order, in fp64; then the wave sum.  Rows are padded to ld >= dim, a
// multiple of 64, so the 8-element loads stay inside the row.
template <typename TQ>
__device__ __forceinline__ void acc8_f64(double& acc, const TQ* __restrict__ q, int d0, int dim,
                                         const float (&x)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (d0 + j < dim) acc += (double)q[d0 + j] * (double)x[j];
}

// -------------------------------------------------------------------------------------
// K4: exact fp64 rescoring + certificate + final top-k.
// -------------------------------------------------------------------------------------
#ifdef HCR_FINISH_STAMPS
// diagnostic build (Makefile stamps_fin): per block (query), s_memrealtime at the phase
// boundaries of finish_kernel / rescore_kernel: [q][8] (tools/finish_stamps.py)
__device__ unsigned long long hcr_fin_stamps[4096 * 8];
#define HCR_FIN_STAMP(i)                                                                       \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                                  \
      hcr_fin_stamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#else
#define HCR_FIN_STAMP(i) do {} while (0)
#endif
// The body of K4 for one query (block): `keys` (LDS) holds its merged top-kp coarse keys,
// sorted descending and zero padded, `qd` (LDS) the fp32 query widened to fp64; hi / lo / nrm
// are kp-slot LDS arrays.  Writes the query's top-k, its certificate flag and s_k.
template <typename TS, int RU = 8>
__device__ __forceinline__ void rescore_block(uint64_t* keys, const double* qd, uint64_t* hi,
                                              uint64_t* lo, double* nrm, int* s_nvalid, int q, int kp,
                                              int dim, const double* __restrict__ qnorm,
                                              const double* __restrict__ eps, const TS* __restrict__ rows,
                                              int ld, int64_t n_rows, const double* __restrict__ norm64, int k, int mode,
                                              double thr, int64_t id_offset, double* __restrict__ out_s,
                                              int64_t* __restrict__ out_i, int* __restrict__ unc_flags,
                                              int* __restrict__ unc_count, const uint32_t* __restrict__ tau_est,
                                              uint64_t* __restrict__ sk_out, const int64_t* __restrict__ idmap,
                                              double* __restrict__ bound_out, int* hflag, int hseq) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // Every row this block dereferences (norm64, rows, idmap) comes from a candidate key.  A key
  // whose row lies outside the index can only come from a defect upstream (a score-kernel or
  // compaction bug): it is dropped here -- an empty slot -- and flagged in unc_count[1], which
  // hcr_search turns into HCR_EINTERNAL, instead of faulting the device on the gather.
  for (int c = threadIdx.x; c < kp; c += blockDim.x) {   // row norms gathered up front
    uint64_t key = keys[c];
    if (key && (int64_t)key_row(key) >= n_rows) {
      keys[c] = key = 0ull;
      atomicOr(unc_count + 1, 1);
    }
    nrm[c] = key ? norm64[key_row(key)] : 1.0;
  }
  if (threadIdx.x == 0) *s_nvalid = 0;
  __syncthreads();
  HCR_FIN_STAMP(2);
  const double qn = qnorm[q];
  // RU candidates per wave at a time, their 16-byte row loads in flight together; per
  // candidate the summation order is acc8_f64's (K6's).  rescore_kernel: RU = 8 (r03): ~100
  // VGPRs, so 4 blocks per CU are resident and a 1024-query batch is one round of blocks (RU =
  // 16: 183 VGPRs, 2 blocks per CU, two rounds of the block's dependent key -> row -> sort chain).
  // finish_kernel (<= 512 queries, at most 2 blocks per CU anyway): RU = 16, k' = 64 in one round
  // of row gathers instead of two (r05r stamps: the fp64 dots were 13.4 of its 25 us at
  // configs[1], two dependent HBM gathers)
  for (int c0 = wave * RU; c0 < kp; c0 += 4 * RU) {
    uint64_t kk[RU];
    const TS* e[RU];
    double acc[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      kk[u] = c0 + u < kp ? keys[c0 + u] : 0ull;
      e[u] = rows + (int64_t)(kk[u] ? key_row(kk[u]) : 0u) * ld;
      acc[u] = 0.0;
    }
    for (int d0 = lane * 8; d0 < dim; d0 += 512) {
      float x[RU][8];
#pragma unroll
      for (int u = 0; u < RU; ++u) load8_f32(e[u] + d0, x[u]);
#pragma unroll
      for (int u = 0; u < RU; ++u) acc8_f64(acc[u], qd, d0, dim, x[u]);
    }
    // the RU wave sums side by side (wave_sum_f64's pairing and order, level by level: the same
    // bits; one after another, each shuffle waited for the last -- r05r stamps: 13 of the finish
    // kernel's 25 us at configs[1]), then lane u < RU finishes candidate c0 + u
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
      for (int u = 0; u < RU; ++u)
        acc[u] += __longlong_as_double((long long)shfl_xor_u64((uint64_t)__double_as_longlong(acc[u]), m));
    double a = 0.0;
    uint64_t ku = 0ull;
#pragma unroll
    for (int u = 0; u < RU; ++u)
      if (lane == u) { a = acc[u]; ku = kk[u]; }
    const int c = c0 + lane;
    const bool mine = lane < RU && c < kp;
    if (mine) {
      if (ku == 0ull) {
        hi[c] = 0ull; lo[c] = 0ull;
      } else {
        hi[c] = ord64(a / (qn * nrm[c]));
        lo[c] = (uint64_t)(0xFFFFFFFFu - key_row(ku));
      }
    }
    const int nv = __popcll(__ballot(mine && ku != 0ull));
    if (lane == 0 && nv) atomicAdd(s_nvalid, nv);
  }
  __syncthreads();
  HCR_FIN_STAMP(3);
  block_sort_desc_pair_fast(hi, lo, kp);
  HCR_FIN_STAMP(4);
  const int nvalid = *s_nvalid;
  if (threadIdx.x == 0) {
    // Every row outside the candidates has coarse score <= B: the k'-th candidate's coarse
    // score when the list is full, and (estimated seed, tau_est != 0) the seed itself, below
    // which no row was ever appended.  Without a seed a short list holds every row.
    bool cert = true;
    const double e = eps[q];
    const uint32_t te = tau_est ? tau_est[q] : 0u;
    double bnd = -INFINITY;                          // every excluded row's exact score is <= bnd
    if (e >= 0.0 && (nvalid >= kp || te != 0u)) {   // e < 0: zero query, exact scores all 0
      const double b = nvalid >= kp ? (double)key_score(keys[kp - 1]) : (double)unord32(te);
      cert = nvalid >= k && b + e < unord64(hi[k - 1]);
      bnd = b + e;
    }
    if (bound_out) {
      // global seed (hcr_search_seeded_device): this shard may hold fewer than k rows above
      // the seed; it returns what it has and the bound, and the certificate moves to the merge
      // of the shards' lists (the merged k-th best must beat every shard's bound)
      bound_out[q] = bnd;
      cert = true;
    }
    unc_flags[q] = cert ? 0 : 1;
    if (!cert) atomicAdd(unc_count, 1);
    // s_k of the candidates (a lower bound on the true k-th best exact score): the starting
    // threshold of the exact fallback for queries that stay uncertified
    if (sk_out) sk_out[q] = nvalid >= k ? hi[k - 1] : 0ull;
  }
  for (int t = threadIdx.x; t < k; t += blockDim.x) {
    double s = -INFINITY;
    int64_t id = -1;
    if (t < nvalid) {
      double v = unord64(hi[t]);
      if (mode == 1) v = (v + 1.0) / 2.0;
      if (v >= thr) { s = v; id = row_id(id_offset, idmap, 0xFFFFFFFFu - (uint32_t)lo[t]); }
    }
    out_s[(size_t)q * k + t] = s;
    out_i[(size_t)q * k + t] = id;
  }
  HCR_FIN_STAMP(5);
  // the pass's flags to the host (HCR_OPT_FLAG_READ 3 / 4, r06): the last block to finish -- a
  // ticket in unc_count[2], reset by prep_queries_kernel -- stores unc_count[0..1] into the
  // pinned host words, then the sequence number the host polls (system scope, vector stores)
  if (hflag) {
    __syncthreads();                                 // (this block's flag atomics are done)
    if (threadIdx.x == 0) {
      __threadfence();
      if (atomicAdd(unc_count + 2, 1) == (int)gridDim.x - 1) {
        __threadfence();
        const int c0 = __hip_atomic_load(unc_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int c1 = __hip_atomic_load(unc_count + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hflag + 1, c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(hflag + 2, c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(hflag, hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

#define HCR_RESCORE_PARAMS                                                                          \
  const float *__restrict__ q32, int dim, const double *__restrict__ qnorm,                       \
      const double *__restrict__ eps, const TS *__restrict__ rows, int ld, int64_t n_rows,          \
      const double *__restrict__ norm64, int k, int mode, double thr, int64_t id_offset,            \
      double *__restrict__ out_s, int64_t *__restrict__ out_i, int *__restrict__ unc_flags,         \
      int *__restrict__ unc_count, const uint32_t *__restrict__ tau_est,                            \
      uint64_t *__restrict__ sk_out, const int64_t *__restrict__ idmap, double *__restrict__ bound_out, \
      int *hflag, int hseq
#define HCR_RESCORE_ARGS                                                                            \
  q, kp, dim, qnorm, eps, rows, ld, n_rows, norm64, k, mode, thr, id_offset, out_s, out_i, unc_flags,      \
      unc_count, tau_est, sk_out, idmap, bound_out, hflag, hseq

// K4 on a merged list ([q][kp] keys in global memory, merge_lists' last level).
// LDS: dim x 8 (query) + kp x 32 + 16.
template <typename TS>
__global__ void __launch_bounds__(256)
rescore_kernel(const uint64_t* __restrict__ merged, int kp, HCR_RESCORE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) char sm_raw[];
  double* qd = reinterpret_cast<double*>(sm_raw);
  uint64_t* hi = reinterpret_cast<uint64_t*>(sm_raw + (size_t)dim * 8);
  uint64_t* lo = hi + kp;
  uint64_t* keys = lo + kp;
  double* nrm = reinterpret_cast<double*>(keys + kp);
  int* s_nvalid = reinterpret_cast<int*>(nrm + kp);
  const int q = blockIdx.x;
  const float* src = q32 + (int64_t)q * dim;
  for (int d = threadIdx.x; d < dim; d += blockDim.x) qd[d] = (double)src[d];
  for (int c = threadIdx.x; c < kp; c += blockDim.x) keys[c] = merged[(size_t)q * kp + c];
  __syncthreads();
  rescore_block<TS>(keys, qd, hi, lo, nrm, s_nvalid, HCR_RESCORE_ARGS);
}

// K3 (last merge level) + K4 fused: one block per query merges its P (<= 256) partition lists
// in LDS and rescores the top kp from there -- no merged list in global memory, one launch and
// one dependent global round trip fewer per search (fuse merge + rescore).
// LDS: M x 8 (the merge, M >= next_pow2(P x kp) as merge_lists sizes it) + dim x 8 + kp x 24 + 16.
template <typename TS>
__global__ void __launch_bounds__(256)
finish_kernel(const uint64_t* __restrict__ lists, const int* __restrict__ cnt, int P, int M, int kp,
              HCR_RESCORE_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) char sm_raw[];
  __shared__ int s_off[257], s_hist[256], s_misc[4];
  uint64_t* sm_keys = reinterpret_cast<uint64_t*>(sm_raw);
  double* qd = reinterpret_cast<double*>(sm_keys + M);
  uint64_t* hi = reinterpret_cast<uint64_t*>(qd + dim);
  uint64_t* lo = hi + kp;
  double* nrm = reinterpret_cast<double*>(lo + kp);
  int* s_nvalid = reinterpret_cast<int*>(nrm + kp);
  const int q = blockIdx.x;
  HCR_FIN_STAMP(0);
  const float* src = q32 + (int64_t)q * dim;
  for (int d = threadIdx.x; d < dim; d += blockDim.x) qd[d] = (double)src[d];   // (under the merge)
  merge_block_lds(lists, cnt, P, 0, P, kp, q, sm_keys, s_off, s_hist, s_misc);
  HCR_FIN_STAMP(1);
  rescore_block<TS, 16>(sm_keys, qd, hi, lo, nrm, s_nvalid, HCR_RESCORE_ARGS);
}

// -------------------------------------------------------------------------------------
// K6/K7: exact fallback (queries the certificate could not settle at k' = 512, and k > 256).
//   K6 scans every row once for a group of <= kFbGroup queries: fp64 cosine in the same
//   summation order as K4 (so the scores are bit-identical), and appends each row whose key
//   (score desc, row asc) is >= the query's threshold key to a per-query buffer of `cap` slots.
//   Beside it, every admitted row lands in a per-query histogram: kFbBins bins linear in the
//   score over [h_lo, h_hi) plus one bin for scores >= h_hi, each with its row count and the
//   smallest score key it holds (LDS per block, flushed by atomics).
//   K7 sorts a query's buffer in LDS.  If it did not overflow it holds every row at or above
//   the threshold, which is <= the true k-th best key, so its top-k IS the exact top-k.  If it
//   overflowed, the next threshold is the larger of
//     (a) the smallest key among the top bins that together hold >= k rows: at least k rows
//         score at or above it, whatever order the scan admitted them in, and the next round's
//         histogram spans only the bin where the k-th best lies (a 1/kFbBins zoom per round);
//     (b) the k-th best key of the slots it kept (strictly above the old threshold because
//         cap > k and keys are unique: progress even through runs of identical scores),
//   both <= the true k-th best key; the host re-runs K6 for those queries.  Starting
//   threshold: K4's s_k (the k-th best exact score among the candidates), or the lowest key.
// -------------------------------------------------------------------------------------
constexpr int kFbGroup = 32;     // queries per K6 scan (the LDS histograms)
constexpr int kFbBins = 128;     // linear score bins per query (+ 1 for scores >= h_hi)

template <typename TS>
__global__ void __launch_bounds__(256)
exact_filter_kernel(const float* __restrict__ q32, int nq, int dim,
                    const double* __restrict__ qnorm, const TS* __restrict__ rows, int ld,
                    int64_t n, const double* __restrict__ norm64,
                    const uint32_t* __restrict__ maskbits, const uint64_t* __restrict__ th_hi,
                    const uint64_t* __restrict__ th_lo, const int* __restrict__ active, int cap,
                    unsigned int* __restrict__ cnt, uint64_t* __restrict__ buf_hi,
                    uint64_t* __restrict__ buf_lo, const double* __restrict__ h_lo,
                    const double* __restrict__ h_hi, unsigned int* __restrict__ h_cnt,
                    unsigned long long* __restrict__ h_min) {
  __shared__ unsigned int s_cnt[kFbGroup][kFbBins + 1];
  __shared__ unsigned long long s_min[kFbGroup][kFbBins + 1];
  for (int i = threadIdx.x; i < kFbGroup * (kFbBins + 1); i += blockDim.x) {
    (&s_cnt[0][0])[i] = 0u;
    (&s_min[0][0])[i] = ~0ull;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool hoist = dim <= 1024;          // the row's first two 512-wide pieces in registers
  for (int64_t row = w0; row < n; row += nw) {
    if (maskbits && !((maskbits[row >> 5] >> (row & 31)) & 1u)) continue;
    const TS* e = rows + row * ld;
    const double nr = norm64[row];
    float xr[2][8];
    if (hoist) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int d0 = lane * 8 + 512 * c;
        if (d0 < dim) load8_f32(e + d0, xr[c]);
        else
#pragma unroll
          for (int j = 0; j < 8; ++j) xr[c][j] = 0.f;
      }
    }
    for (int q = 0; q < nq; ++q) {
      if (!active[q]) continue;
      const float* qs = q32 + (int64_t)q * dim;
      double acc = 0.0;
      if (hoist) {
        acc8_f64(acc, qs, lane * 8, dim, xr[0]);
        acc8_f64(acc, qs, lane * 8 + 512, dim, xr[1]);
      } else {
        for (int d0 = lane * 8; d0 < dim; d0 += 512) {
          float x[8];
          load8_f32(e + d0, x);
          acc8_f64(acc, qs, d0, dim, x);
        }
      }
      acc = wave_sum_f64(acc);
      if (lane == 0) {
        const double sc = acc / (qnorm[q] * nr);
        const uint64_t h = ord64(sc);
        const uint64_t l = (uint64_t)(0xFFFFFFFFu - (uint32_t)row);
        if (h > th_hi[q] || (h == th_hi[q] && l >= th_lo[q])) {
          const unsigned int p = atomicAdd(&cnt[q], 1u);
          if (p < (unsigned int)cap) {
            buf_hi[(size_t)q * cap + p] = h;
            buf_lo[(size_t)q * cap + p] = l;
          }
          const double lo = h_lo[q], hi = h_hi[q];
          int b = kFbBins;
          if (sc < hi) {
            const double t = (sc - lo) * ((double)kFbBins / (hi - lo));
            b = t < 0.0 ? 0 : t >= (double)(kFbBins - 1) ? kFbBins - 1 : (int)t;
          }
          atomicAdd(&s_cnt[q][b], 1u);
          atomicMin(&s_min[q][b], (unsigned long long)h);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nq * (kFbBins + 1); i += blockDim.x) {
    const unsigned int c = (&s_cnt[0][0])[i];
    if (c) {
      atomicAdd(&h_cnt[i], c);
      atomicMin(&h_min[i], (&s_min[0][0])[i]);
    }
  }
}

// -------------------------------------------------------------------------------------
// K6m / K6h: the exact fallback's row scan with an MFMA prefilter (16-bit storage, ld = 32 KS).
//   A group of <= kFbGroup queries is held as MFMA B fragments (q^ = the unit MFMA-dtype
//   queries of prep_queries_kernel, 16 per wave: waves 0 / 2 queries 0-15, 1 / 3 queries
//   16-31), rows stream straight from HBM as A fragments, 16-row tiles; the coarse score is
//   c = fl(q^.e . inv32) with |c - exact| <= eps_q (the non-UNIT bound).
//   One launch scans the rows once for up to kFbGroupsPerScan groups (blocks of a row chunk's
//   groups adjacent on one XCD: the other groups read the rows from L2).
//   K6m (HIST = false): a (row, query) pair whose c reaches T_q - eps_q -- T_q the score of the
//   query's threshold key -- gets the fp64 cosine in K6's summation order (a wave per pair:
//   bit-identical scores), then K6's key test, append and histogram; every row whose exact key
//   is at or above the threshold passes the prefilter, so K7 sees what K6 would have admitted.
//   K6h (HIST = true, round 0 when a query has no starting threshold, k > 256): a histogram of
//   c per query over [-kFbHistRange, kFbHistRange) in kFbHistBins bins, from which the host
//   takes T_q = (lower edge of the bin where k rows are reached from the top) - eps_q: at least
//   k rows have c >= edge, hence exact >= T_q, so T_q <= the true k-th best.  On a large
//   corpus the histogram covers a sample (hstride > 1: one run of 4 tiles in 4 hstride) and
//   the edge is where the sample reaches f k + 5 sqrt(f k) + 3 rows (f the sampled fraction):
//   an ESTIMATED threshold -- if the filter round then admits fewer than k rows, the select
//   (K7) drops it to "every row" and the round repeats, so the result stays exact.
// -------------------------------------------------------------------------------------
constexpr int kFbHistBins = 512;
constexpr int kFbGroupsPerScan = 4;  // query groups of kFbGroup per MFMA-prefiltered scan
constexpr float kFbHistRange = 1.0625f;
// K6m: admitted pairs rescored together, and the per-wave queue slots (a batch's leftover + one
// tile).  (8 at a time at ld = 384 measured the same as 4, r06r: 891.7 vs 900 µs per scan.)
constexpr int kPairBatch = 4;
constexpr int kPairQueue = kPairBatch - 1 + 4 * 64 + 1;
// K6m: admitted keys staged per block in LDS (r06: the returning global atomic per admitted pair
// was one of two dependent round trips in every rescore batch); one atomic per query and block
// at the end reserves their slots; past kStage the pairs append to global memory directly
constexpr int kStage = 384;
// K6 modes (r06): the inline scan (K6m: every admitted pair rescored by the scanning wave), the
// coarse histogram (K6h), and the two-launch form of K6m -- K6c compacts the coarse-admitted
// (row, query) pairs of every query group into a global list per group, K6r rescores that list
// with every wave of the chip (no scan beside it: the rescoring's row gathers no longer stall the
// stream), the group's admissions, staging and histograms exactly as K6m's.  A group whose list
// overflowed its pcap slots is skipped by K6r and scanned by the inline K6m instead (launched
// after it, only that group's blocks do any work).
enum { kK6Inline = 0, kK6Hist = 1, kK6Compact = 2, kK6Rescore = 3 };

__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename TS, int KS, int MODE, int QB = 1>
__global__ void __launch_bounds__(256)
exact_filter_mfma_kernel(const TS* __restrict__ qhat, const double* __restrict__ eps,
                         const float* __restrict__ q32, int nq, int dim,
                         const double* __restrict__ qnorm, const TS* __restrict__ rows, int ld,
                         int64_t n, const float* __restrict__ inv32,
                         const double* __restrict__ norm64, const uint32_t* __restrict__ maskbits,
                         const uint64_t* __restrict__ th_hi, const uint64_t* __restrict__ th_lo,
                         const int* __restrict__ active, int cap, unsigned int* __restrict__ cnt,
                         uint64_t* __restrict__ buf_hi, uint64_t* __restrict__ buf_lo,
                         const double* __restrict__ h_lo, const double* __restrict__ h_hi,
                         unsigned int* __restrict__ h_cnt, unsigned long long* __restrict__ h_min,
                         unsigned int* __restrict__ c_hist, int ngroups, int hstride,
                         uint64_t* __restrict__ pairs, unsigned long long* __restrict__ pcnt, int64_t pcap) {
  constexpr bool HIST = MODE == kK6Hist, COMPACT = MODE == kK6Compact, RESC = MODE == kK6Rescore;
  // QB = 2 (the scan-only modes K6h / K6c, r06): every wave holds both 16-query halves of the
  // group and multiplies each tile's A fragments with both -- a tile is loaded by one wave instead
  // of two, and the block's 4 waves take 4 different tiles
  static_assert(QB == 1 || HIST || COMPACT, "QB = 2: the scan-only modes");
  using Op = MfmaOp<TS>;
  using V = typename Op::V;
  constexpr size_t HB = (size_t)kFbGroup * kFbHistBins * 4;
  constexpr size_t FB = (size_t)kFbGroup * (kFbBins + 1) * 12;
  constexpr size_t FBQ0 = FB + (RESC ? 0 : (size_t)4 * kPairQueue * 8);   // + the pair queues
  // (K6r: a block rescores ~500 pairs at the bench's deep k -- a larger stage, still 2 blocks per CU)
  constexpr int STG = RESC ? 960 : kStage;
  constexpr size_t FBQ = FBQ0 + (size_t)STG * (8 + 4 + 2 + 2);     // + the staged keys
  static_assert(FB % 8 == 0, "pair queue alignment");
  static_assert(FBQ <= 65536, "K6m LDS");
  // (K6c with only its pair queues in LDS, 32 KiB: 4 blocks per CU instead of 2, measured the same
  // -- 224 vs 227 µs, r06ag -- and not kept: the scan is not bound by its occupancy)
  __shared__ __attribute__((aligned(16))) char sm[RESC ? FBQ : (HB > FBQ ? HB : FBQ)];
  __shared__ double s_tc[kFbGroup], s_qn[kFbGroup], s_hlo[kFbGroup], s_hhi[kFbGroup];
  __shared__ uint64_t s_thh[kFbGroup], s_thl[kFbGroup];
  __shared__ unsigned int s_nst, s_qcnt[kFbGroup], s_qbase[kFbGroup];
  unsigned int* s_hist = reinterpret_cast<unsigned int*>(sm);                        // HIST
  unsigned int (*s_cnt)[kFbBins + 1] = reinterpret_cast<unsigned int (*)[kFbBins + 1]>(sm);
  unsigned long long (*s_min)[kFbBins + 1] =
      reinterpret_cast<unsigned long long (*)[kFbBins + 1]>(sm + (size_t)kFbGroup * (kFbBins + 1) * 4);
  // block -> (query group, row chunk): the ngroups groups of one row chunk are consecutive
  // blocks of one XCD (round-robin dispatch), so each row tile comes from HBM once per scan and
  // from that XCD's L2 for the other groups (the grid is a multiple of 8 x ngroups)
  // (K6r: block b rescores pairs of group b % ngroups; no row chunks)
  const int xcd = blockIdx.x & 7, rr = blockIdx.x >> 3;
  const int grp = RESC ? (int)(blockIdx.x % ngroups) : rr % ngroups;
  const int chunk = RESC ? (int)(blockIdx.x / ngroups) : (rr / ngroups) * 8 + xcd;
  const int nchunks = gridDim.x / ngroups;
  const int qg0 = grp * kFbGroup, nqg = min(kFbGroup, nq - qg0);
  // the two-launch form: K6r takes a group whose list fits, the inline K6m one that overflowed
  if (RESC && (pcnt[grp] == 0ull || pcnt[grp] > (unsigned long long)pcap)) return;
  if (MODE == kK6Inline && pcnt && pcnt[grp] <= (unsigned long long)pcap) return;
  if constexpr (HIST) {
    for (int i = threadIdx.x; i < kFbGroup * kFbHistBins; i += blockDim.x) s_hist[i] = 0u;
  } else {
    for (int i = threadIdx.x; !COMPACT && i < kFbGroup * (kFbBins + 1); i += blockDim.x) {
      (&s_cnt[0][0])[i] = 0u;
      (&s_min[0][0])[i] = ~0ull;
    }
    if (threadIdx.x < kFbGroup) {
      const int q = threadIdx.x;
      // the prefilter bound: pairs below it cannot reach the threshold key's score
      s_tc[q] = (q < nqg && active[qg0 + q]) ? unord64(th_hi[qg0 + q]) - eps[qg0 + q] : INFINITY;
      s_qcnt[q] = 0u;
      if (q == 0) s_nst = 0u;
      if (q < nqg) {              // (the admission test's per-query values, read per pair)
        s_qn[q] = qnorm[qg0 + q];
        s_thh[q] = th_hi[qg0 + q];
        s_thl[q] = th_lo[qg0 + q];
        s_hlo[q] = h_lo[qg0 + q];
        s_hhi[q] = h_hi[qg0 + q];
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qb = wave & 1;
  const int ql = qb * 16 + (lane & 15);              // the lane's query (accumulator column)
  // query fragments: lane l holds q^[qb*16 + (l & 15)][32 ks + 8 (l >> 4) .. + 8) (QB = 2: both
  // halves, qlb[b] = b*16 + (l & 15))
  V qf[QB][KS];
  int qlb[QB];
  bool qokb[QB];
  double tcqb[QB];
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    qlb[b] = QB == 1 ? ql : b * 16 + (lane & 15);
    if constexpr (!RESC) {
      const TS* src = qhat + (size_t)(qg0 + qlb[b]) * ld + (lane >> 4) * 8;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) qf[b][ks] = *reinterpret_cast<const V*>(src + ks * 32);
    }
    qokb[b] = qlb[b] < nqg && active[qg0 + qlb[b]];
    tcqb[b] = HIST ? 0.0 : s_tc[qlb[b]];
  }
  // K6m's admitted (row, query) pairs: a queue per wave in the LDS above the histograms (at
  // most kPairBatch - 1 left over + 4 x 64 per tile); entry = row << 8 | group-local query
  uint64_t* pq = reinterpret_cast<uint64_t*>(sm + FB) + wave * kPairQueue;
  int qn = 0;
  // K6c: a queue per wave over the whole LDS array (no histograms, no staging in this mode),
  // flushed to the group's global list -- one returning atomic per flush -- when a tile could
  // overflow it
  constexpr int PQC = (int)((HB > FBQ ? HB : FBQ) / 8 / 4);
  static_assert(PQC >= 2 * 4 * 64, "K6c queue");
  uint64_t* pqc = reinterpret_cast<uint64_t*>(sm) + wave * PQC;
  uint64_t* pg = pairs ? pairs + (size_t)grp * (size_t)pcap : nullptr;
  auto flush_pairs = [&]() __attribute__((always_inline)) {
    lds_wave_sync();
    unsigned long long base = 0ull;
    if (lane == 0) base = atomicAdd(&pcnt[grp], (unsigned long long)qn);
    base = __shfl(base, 0);
    for (int i = lane; i < qn; i += 64)
      if (base + (unsigned long long)i < (unsigned long long)pcap) pg[base + i] = pqc[i];
    qn = 0;
    lds_wave_sync();
  };
  uint64_t* st_h = reinterpret_cast<uint64_t*>(sm + FBQ0);            // key hi
  uint32_t* st_row = reinterpret_cast<uint32_t*>(st_h + STG);      // row (key lo = ~row)
  uint16_t* st_q = reinterpret_cast<uint16_t*>(st_row + STG);      // group-local query
  uint16_t* st_rank = st_q + STG;                                  // slot within its query
  // the exact fp64 cosine of np (<= kPairBatch) queued pairs at once: every lane's 8-wide
  // pieces of all the pairs' rows are loaded together (one memory round trip instead of one per
  // pair), each pair in K6's summation order (so bit-identical to K4 / K6); lane p then runs
  // pair p's key test, append and histogram
  constexpr int PB = RESC ? 8 : kPairBatch;      // (K6r: 8 pairs per wave at a time)
  auto rescore_batch = [&](const uint64_t* e, int np) __attribute__((always_inline)) {
    int64_t prow[PB];
    int pqs[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const uint64_t v = e[p < np ? p : 0];
      prow[p] = (int64_t)(v >> 8);
      pqs[p] = (int)(v & 255u);
    }
    int64_t my_row = prow[0];
    int my_q = pqs[0];
#pragma unroll
    for (int p = 1; p < PB; ++p)
      if (lane == p) { my_row = prow[p]; my_q = pqs[p]; }
    const double nr = lane < np ? norm64[my_row] : 1.0;
    double ex[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) ex[p] = 0.0;
    // (r06: the query's 8 floats as two 16-byte loads when the rows of q32 are 16-byte aligned;
    // the same values, so acc8_f64's order and bits)
    const bool qvec = (dim & 7) == 0;
    for (int d0 = lane * 8; d0 < dim; d0 += 512) {
      float x[PB][8];
#pragma unroll
      for (int p = 0; p < PB; ++p) load8_f32(rows + prow[p] * ld + d0, x[p]);
#pragma unroll
      for (int p = 0; p < PB; ++p) {
        const float* qp = q32 + (int64_t)(qg0 + pqs[p]) * dim;
        if (qvec) {
          float qv[8];
          const float4 u = reinterpret_cast<const float4*>(qp + d0)[0], w = reinterpret_cast<const float4*>(qp + d0)[1];
          qv[0] = u.x; qv[1] = u.y; qv[2] = u.z; qv[3] = u.w; qv[4] = w.x; qv[5] = w.y; qv[6] = w.z; qv[7] = w.w;
#pragma unroll
          for (int j = 0; j < 8; ++j) ex[p] += (double)qv[j] * (double)x[p][j];
        } else {
          acc8_f64(ex[p], qp, d0, dim, x[p]);
        }
      }
    }
    // the PB wave sums side by side, level by level (wave_sum_f64's pairing and order: the same
    // bits; one after another each shuffle waited for the last)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
      for (int p = 0; p < PB; ++p)
        ex[p] += __longlong_as_double((long long)shfl_xor_u64((uint64_t)__double_as_longlong(ex[p]), m));
    double my_ex = 0.0;
#pragma unroll
    for (int p = 0; p < PB; ++p)
      if (lane == p) my_ex = ex[p];
    if (lane < np) {
      const int q = qg0 + my_q;
      const double sc = my_ex / (s_qn[my_q] * nr);
      const uint64_t h = ord64(sc);
      const uint64_t l = (uint64_t)(0xFFFFFFFFu - (uint32_t)my_row);
      if (h > s_thh[my_q] || (h == s_thh[my_q] && l >= s_thl[my_q])) {
        const unsigned int e = atomicAdd(&s_nst, 1u);
        if (e < (unsigned int)STG) {
          st_h[e] = h;
          st_row[e] = (uint32_t)my_row;
          st_q[e] = (uint16_t)my_q;
        } else {                                     // (stage full: straight to the buffer)
          const unsigned int pos = atomicAdd(&cnt[q], 1u);
          if (pos < (unsigned int)cap) {
            buf_hi[(size_t)q * cap + pos] = h;
            buf_lo[(size_t)q * cap + pos] = l;
          }
        }
        const double lo = s_hlo[my_q], hi = s_hhi[my_q];
        int b = kFbBins;
        if (sc < hi) {
          const double tt = (sc - lo) * ((double)kFbBins / (hi - lo));
          b = tt < 0.0 ? 0 : tt >= (double)(kFbBins - 1) ? kFbBins - 1 : (int)tt;
        }
        atomicAdd(&s_cnt[my_q][b], 1u);
        atomicMin(&s_min[my_q][b], (unsigned long long)h);
      }
    }
  };
  if constexpr (RESC) {
    // K6r: the group's compacted pairs, PB per wave at a time, grid-strided
    const int64_t npt = (int64_t)pcnt[grp];
    for (int64_t p0 = ((int64_t)chunk * 4 + wave) * PB; p0 < npt; p0 += (int64_t)nchunks * 4 * PB)
      rescore_batch(pg + p0, (int)min((int64_t)PB, npt - p0));
  }
  const int64_t ntile = RESC ? 0 : (n + 15) / 16;
  const int64_t stride = (int64_t)nchunks * (QB == 2 ? 4 : 2);
  // (HIST: runs of 4 tiles out of every 4 hstride -- a sample of the rows when hstride > 1)
  auto tile_of = [&](int64_t tv) -> int64_t {
    return HIST ? (tv >> 2) * (4 * (int64_t)hstride) + (tv & 3) : tv;
  };
  // A fragments straight from the rows (the slack rows past n are readable; masked below), in
  // NB batches of CH k-steps; the next tile's first batch is issued before this tile's epilogue
  // (after its inv32 / mask loads: vmcnt counts in order), so one tile's load latency hides
  // behind the previous tile's epilogue (r05: 3 dependent batches per tile, no overlap, ran the
  // scan at ~3 TB/s)
  // (KS = 24 in one batch: 262 registers, KS = 32 in 16-deep batches: 264 -- one wave per SIMD)
  constexpr int CH = KS <= 12 ? KS : KS == 24 ? 12 : 8, NB = (KS + CH - 1) / CH;
  auto frag_ptr = [&](int64_t t) { return rows + (t * 16 + (lane & 15)) * ld + (lane >> 4) * 8; };
  V a[CH];
  auto load_batch = [&](const TS* ra, int b) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CH; ++j)
      if (b * CH + j < KS) a[j] = *reinterpret_cast<const V*>(ra + (b * CH + j) * 32);
  };
  int64_t tv = QB == 2 ? (int64_t)chunk * 4 + wave : (int64_t)chunk * 2 + (wave >> 1);
  if (!RESC && tile_of(tv) < ntile) load_batch(frag_ptr(tile_of(tv)), 0);
  for (;; tv += stride) {
    const int64_t t = tile_of(tv);
    if (t >= ntile) break;
    const int64_t r0 = t * 16;
    const int64_t tn = tile_of(tv + stride);
    floatx4 accb[QB];
#pragma unroll
    for (int qbi = 0; qbi < QB; ++qbi) accb[qbi] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int64_t rb = r0 + (lane >> 4) * 4;         // the lane's 4 rows: rb .. rb + 3
    float iv[4];
    bool rowok[4];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int qbi = 0; qbi < QB; ++qbi)
          if (b * CH + j < KS) accb[qbi] = Op::run(a[j], qf[qbi][b * CH + j], accb[qbi]);
      if (b + 1 < NB) {
        load_batch(frag_ptr(t), b + 1);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = rb + r;
          rowok[r] = row < n && (!maskbits || ((maskbits[row >> 5] >> (row & 31)) & 1u));
          iv[r] = row < n ? inv32[row] : 0.f;
        }
        if (tn < ntile) load_batch(frag_ptr(tn), 0);
      }
    }
    const floatx4 acc = accb[0];
    bool rok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rok[r] = rowok[r] && qokb[0];
    const double tcq = tcqb[0];
    if constexpr (HIST) {
#pragma unroll
      for (int qbi = 0; qbi < QB; ++qbi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!(rowok[r] && qokb[qbi])) continue;
          const float c = accb[qbi][r] * iv[r];
          int b = (int)floorf((c + kFbHistRange) * ((float)kFbHistBins / (2.f * kFbHistRange)));
          b = b < 0 ? 0 : b >= kFbHistBins ? kFbHistBins - 1 : b;
          atomicAdd(&s_hist[qlb[qbi] * kFbHistBins + b], 1u);
        }
    } else if constexpr (COMPACT) {
      // admitted pairs go to the wave's queue, flushed to the group's list
#pragma unroll
      for (int qbi = 0; qbi < QB; ++qbi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool adm = rowok[r] && qokb[qbi] && (double)(accb[qbi][r] * iv[r]) >= tcqb[qbi];
          const uint64_t m = __builtin_amdgcn_ballot_w64(adm);
          if (adm) {
            const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            pqc[qn + below] = ((uint64_t)(rb + r) << 8) | (uint64_t)qlb[qbi];
          }
          qn += __builtin_popcountll(m);
        }
      qn = __builtin_amdgcn_readfirstlane(qn);
      if (qn > PQC - 4 * 64 * QB) flush_pairs();
    } else {
      // admitted pairs go to the wave's queue; full batches of kPairBatch are rescored at once
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool adm = rok[r] && (double)(acc[r] * iv[r]) >= tcq;
        const uint64_t m = __builtin_amdgcn_ballot_w64(adm);
        if (adm) {
          const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          pq[qn + below] = ((uint64_t)(rb + r) << 8) | (uint64_t)ql;
        }
        qn += __builtin_popcountll(m);
      }
      qn = __builtin_amdgcn_readfirstlane(qn);
      if (qn >= kPairBatch) {
        lds_wave_sync();
        while (qn >= kPairBatch) {
          qn -= kPairBatch;
          rescore_batch(pq + qn, kPairBatch);
        }
        lds_wave_sync();
      }
    }
  }
  if constexpr (COMPACT) {
    if (qn > 0) flush_pairs();
    return;
  }
  if constexpr (MODE == kK6Inline) {
    if (qn > 0) {
      lds_wave_sync();
      rescore_batch(pq, qn);
    }
  }
  __syncthreads();
  if constexpr (HIST) {
    for (int i = threadIdx.x; i < nqg * kFbHistBins; i += blockDim.x) {
      const unsigned int c = s_hist[i];
      if (c) atomicAdd(&c_hist[(size_t)qg0 * kFbHistBins + i], c);
    }
  } else {
    // the staged keys: ranks within their query (LDS), one slot reservation per query, stores
    const int nst = (int)min(s_nst, (unsigned int)STG);
    for (int e = threadIdx.x; e < nst; e += blockDim.x) st_rank[e] = (uint16_t)atomicAdd(&s_qcnt[st_q[e]], 1u);
    __syncthreads();
    if (threadIdx.x < nqg && s_qcnt[threadIdx.x])
      s_qbase[threadIdx.x] = atomicAdd(&cnt[qg0 + threadIdx.x], s_qcnt[threadIdx.x]);
    __syncthreads();
    for (int e = threadIdx.x; e < nst; e += blockDim.x) {
      const int ql_ = st_q[e];
      const unsigned int pos = s_qbase[ql_] + st_rank[e];
      if (pos < (unsigned int)cap) {
        const size_t o = (size_t)(qg0 + ql_) * cap + pos;
        buf_hi[o] = st_h[e];
        buf_lo[o] = (uint64_t)(0xFFFFFFFFu - st_row[e]);
      }
    }
    for (int i = threadIdx.x; i < nqg * (kFbBins + 1); i += blockDim.x) {
      const unsigned int c = (&s_cnt[0][0])[i];
      if (c) {
        atomicAdd(&h_cnt[(size_t)qg0 * (kFbBins + 1) + i], c);
        atomicMin(&h_min[(size_t)qg0 * (kFbBins + 1) + i], (&s_min[0][0])[i]);
      }
    }
  }
}

#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void __launch_bounds__(256)
exact_select_kernel(int k, int cap, const unsigned int* __restrict__ cnt,
                    const uint64_t* __restrict__ buf_hi, const uint64_t* __restrict__ buf_lo,
                    uint64_t* __restrict__ th_hi, uint64_t* __restrict__ th_lo,
                    int* __restrict__ active, int* __restrict__ n_again, int mode, double thr,
                    int64_t id_offset, const int64_t* __restrict__ idmap,
                    const int* __restrict__ out_idx, double* __restrict__ out_s,
                    int64_t* __restrict__ out_i, double* __restrict__ h_lo,
                    double* __restrict__ h_hi, const unsigned int* __restrict__ h_cnt,
                    const unsigned long long* __restrict__ h_min, int* __restrict__ est) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm_sel[];
  const int q = blockIdx.x;
  if (!active[q]) return;
  const unsigned int c = cnt[q];
  if (est && est[q]) {
    // an estimated starting threshold (K6h over a sample) that admitted fewer than k rows lies
    // above the k-th best: the next round admits every row (rare: ~1e-8 per query)
    if (c < (unsigned int)k) {
      if (threadIdx.x == 0) {
        th_hi[q] = 0ull;
        th_lo[q] = 0ull;
        h_lo[q] = -1.0 - 1e-6;
        h_hi[q] = 1.0 + 1e-6;
        est[q] = 0;
        atomicAdd(n_again, 1);
      }
      return;
    }
    __syncthreads();
    if (threadIdx.x == 0) est[q] = 0;       // (>= k rows at or above it: a valid bound from here)
  }
  const int nload = (int)min(c, (unsigned int)cap);
  int m = 1;
  while (m < nload || m < k) m <<= 1;                  // <= cap (power of two, cap > k)
  uint64_t* hi = sm_sel;
  uint64_t* lo = sm_sel + m;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    const bool v = i < nload;
    hi[i] = v ? buf_hi[(size_t)q * cap + i] : 0ull;
    lo[i] = v ? buf_lo[(size_t)q * cap + i] : 0ull;
  }
  __syncthreads();
  block_sort_desc_pair_fast(hi, lo, m);
  if (c > (unsigned int)cap) {
    if (threadIdx.x == 0) {
      // (a) the histogram: top bins down to the one where k rows are reached (the admitted
      // rows number c > cap > k, so that bin exists)
      const unsigned int* hc = h_cnt + (size_t)q * (kFbBins + 1);
      const unsigned long long* hm = h_min + (size_t)q * (kFbBins + 1);
      unsigned int acc = 0u;
      unsigned long long mn = ~0ull;
      int b = kFbBins;
      for (; b >= 0; --b) {
        acc += hc[b];
        if (hc[b] && hm[b] < mn) mn = hm[b];
        if (acc >= (unsigned int)k) break;
      }
      uint64_t nh = mn, nl = 0ull;
      // (b) the k-th best of the kept slots
      if (hi[k - 1] > nh || (hi[k - 1] == nh && lo[k - 1] > nl)) { nh = hi[k - 1]; nl = lo[k - 1]; }
      const double olo = h_lo[q], ohi = h_hi[q];
      const double nlo = unord64(nh);
      // the k-th best lies in bin b (the bins above it hold < k rows): zoom there
      double nhi = b >= kFbBins ? 2.0 : olo + (double)(b + 1) * ((ohi - olo) / (double)kFbBins);
      if (!(nhi > nlo)) nhi = nextafter(nlo, INFINITY);
      th_hi[q] = nh;
      th_lo[q] = nl;
      h_lo[q] = nlo;
      h_hi[q] = nhi;
      atomicAdd(n_again, 1);
    }
    return;
  }
  const int o = out_idx[q];
  for (int t = threadIdx.x; t < k; t += blockDim.x) {
    double s = -INFINITY;
    int64_t id = -1;
    if (t < nload) {
      double v = unord64(hi[t]);
      if (mode == 1) v = (v + 1.0) / 2.0;
      if (v >= thr) { s = v; id = row_id(id_offset, idmap, 0xFFFFFFFFu - (uint32_t)lo[t]); }
    }
    out_s[(size_t)o * k + t] = s;
    out_i[(size_t)o * k + t] = id;
  }
  __syncthreads();
  if (threadIdx.x == 0) active[q] = 0;
}
#endif

// -------------------------------------------------------------------------------------
// exact fp64 scores of every (query, row) pair (small indexes; isRelevant a1 semantics)
// -------------------------------------------------------------------------------------
template <typename TS>
__global__ void __launch_bounds__(256)
exact_all_kernel(const float* __restrict__ q32, int dim, const double* __restrict__ qnorm,
                 const TS* __restrict__ rows, int ld, int64_t n,
                 const double* __restrict__ norm64, int mode, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int q = blockIdx.y;
  if (row >= n) return;
  const float* qs = q32 + (int64_t)q * dim;
  const TS* e = rows + row * ld;
  double acc = 0.0;
  for (int d0 = lane * 8; d0 < dim; d0 += 512) {     // K4's order: the same scores bit for bit
    float x[8];
    load8_f32(e + d0, x);
    acc8_f64(acc, qs, d0, dim, x);
  }
  acc = wave_sum_f64(acc);
  if (lane == 0) {
    double s = acc / (qnorm[q] * norm64[row]);
    if (mode == 1) s = (s + 1.0) / 2.0;
    out[(int64_t)q * n + row] = s;
  }
}


// -------------------------------------------------------------------------------------
// K5: merge g shards' top-k lists ([g][nq][k], exact fp64 scores, -1 = empty).
// -------------------------------------------------------------------------------------
#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void __launch_bounds__(256)
merge_shards_kernel(const double* __restrict__ s, const int64_t* __restrict__ ids, int g,
                    int64_t nq, int k, int M, double* __restrict__ out_s,
                    int64_t* __restrict__ out_i) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm_pair[];
  uint64_t* hi = sm_pair;
  uint64_t* lo = sm_pair + M;
  const int64_t q = blockIdx.x;
  const int tot = g * k;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    uint64_t h = 0ull, l = 0ull;
    if (i < tot) {
      const int j = i / k, c = i - j * k;
      const size_t off = ((size_t)j * nq + q) * k + c;
      const int64_t id = ids[off];
      if (id >= 0) { h = ord64(s[off]); l = ~(uint64_t)id; }
    }
    hi[i] = h;
    lo[i] = l;
  }
  __syncthreads();
  block_sort_desc_pair_fast(hi, lo, M);
  for (int t = threadIdx.x; t < k; t += blockDim.x) {
    const bool ok = hi[t] != 0ull;
    out_s[q * k + t] = ok ? unord64(hi[t]) : -INFINITY;
    out_i[q * k + t] = ok ? (int64_t)(~lo[t]) : -1;
  }
}
#endif

// gather / scatter helpers for certificate widening
#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void gather_rows_f32(const float* __restrict__ src, const int* __restrict__ idx, int n,
                                int dim, float* __restrict__ dst) {
  const int i = blockIdx.x;
  if (i >= n) return;
  const float* s = src + (int64_t)idx[i] * dim;
  float* d = dst + (int64_t)i * dim;
  for (int j = threadIdx.x; j < dim; j += blockDim.x) d[j] = s[j];
}
#endif
#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void scatter_topk(const double* __restrict__ s, const int64_t* __restrict__ ids,
                             const int* __restrict__ idx, int n, int k, double* __restrict__ out_s,
                             int64_t* __restrict__ out_i) {
  const int i = blockIdx.x;
  if (i >= n) return;
  for (int j = threadIdx.x; j < k; j += blockDim.x) {
    out_s[(int64_t)idx[i] * k + j] = s[(int64_t)i * k + j];
    out_i[(int64_t)idx[i] * k + j] = ids[(int64_t)i * k + j];
  }
}
#endif
#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void iota_ids_kernel(int64_t* __restrict__ ids, int64_t n, int64_t first) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ids[i] = first + i;
}
#endif
#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void fill_empty(double* __restrict__ s, int64_t* __restrict__ ids, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { s[i] = -INFINITY; ids[i] = -1; }
}
#endif
#ifndef HCR_TOPK_TEMPLATES_ONLY   // defined once (hcrag_index.hip): one registration per kernel
__global__ void query_norms_kernel(const float* __restrict__ q32, int nq, int dim,
                                   double* __restrict__ qnorm) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nq) return;
  double ss = 0.0;
  for (int d = lane; d < dim; d += 64) { const double x = (double)q32[(int64_t)q * dim + d]; ss += x * x; }
  ss = wave_sum_f64(ss);
  if (lane == 0) { double nr = sqrt(ss); qnorm[q] = nr < 10.0 * 2.220446049250313e-16 ? 1.0 : nr; }
}
#endif

}  // namespace hcr
