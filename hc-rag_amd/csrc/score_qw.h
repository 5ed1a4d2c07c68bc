// score_qw.h — K2 "QW": query-stationary fused score + top-k' for LARGE batches (> 256
// queries, the MFMA-bound regime of configs[2]: 10M x 768, B = 1024).
//
// Why a third kernel.  v4 (score_v4.h) fills a 256-row and a 256-query tile into LDS for every
// 32-deep stage: 32 KiB of LDS-DMA per 4.2 MFLOP, i.e. 32 B/clk/CU at the MFMA peak, against
// a measured LDS-DMA fill ceiling of ~12-16 B/clk/CU (7.6 TB/s chip-wide) -- the
// main loop is fill-bound at ~40 % of the MFMA peak.  QS (score_qs.h) keeps the queries in
// VGPRs but only 128 per workgroup at D = 768 (16 per wave), so rows are still filled once per
// 128 queries.  QW holds 256 queries x the whole K in the workgroup's registers -- 32 queries
// per wave, 2 x KS fragments each (192 VGPRs at D = 768: three quarters of the CU's register
// file are query operands) -- and streams only rows: 16 B/clk/CU at the MFMA peak, half of v4.
//
//  * a stage is a whole row tile over the full K: SR rows x ld (SR = 32 at D = 768, 64 at
//    D = 384: 48 KiB), a 3-deep ring (two stages in flight), one barrier per stage;
//  * the stage's LDS image is the v3 one (1 KiB pieces of 16 rows x 32 k, XOR-swizzled chunks):
//    piece (rb, ks) at (rb x KS + ks) KiB; each wave DMAs 6 of the 48 pieces plus its 32 global
//    bounds (a 4-byte-per-lane LDS-DMA: 7 vmcnt-counted ops per wave per stage), issued right
//    after the stage barrier;
//  * per stage a wave runs RB x KS x 2 MFMAs (96 at D = 768: 1536 cycles) on 4 independent
//    accumulator chains (row-block pair x query-block pair), fragment reads two groups ahead;
//  * the epilogue is per stage (the accumulators of SR rows x 32 queries: 16 VGPRs), a max +
//    compare against max(local k'-th key, global bound); appends, compactions and the final
//    lists are the wave's alone (its queries), as in QS.
//
// UNIT corpora only (raw dot product = coarse score) and no row mask: other
// batches run on v4.  Rows of the last tile past n_rows are excluded in its epilogue.
// Grid: nqb query blocks x P row partitions (XCD-aware as v3/v4), one workgroup per CU (LDS).
#pragma once
#include <utility>

#include "score_v3.h"

namespace hcr {

#ifdef HCR_QW_STAMPS
// Diagnostic build only (Makefile target `stamps_qw`, tools/qw_stamps.py): per wave of the dense
// launch, s_memtime cycles summed over the stages: [0] vmcnt wait + barrier, [1] DMA issue +
// bound reads, [2] the MFMA groups (issue), [3] the epilogue, [4] stages.  Never in the product.
__device__ unsigned long long hcr_qw_stamps[4096 * 8 * 8];
#define HCR_QW_STAMP(t)                                                                \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");         \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#endif

constexpr int QW_QT = 256;      // queries per workgroup (8 waves x 32; kQwQueries on the host)
constexpr int QW_NST = 3;       // ring stages

// rows per stage for KS 32-deep k-steps: 48 KiB stages (RB = SR / 16 row blocks, even)
constexpr int qw_sr(int ks) { return ks == 24 ? 32 : ks == 12 ? 64 : 0; }

template <int KS, int SR_ = qw_sr(KS), int NST_ = QW_NST>
struct QwLayout {
  static constexpr int SR = SR_, RB = SR / 16, NST = NST_;
  static constexpr int PIECES = RB * KS;                  // 1 KiB pieces per stage
  static constexpr int PPW = PIECES / 8;                  // ... per wave
  static constexpr int STAGE = PIECES * 1024;
  static constexpr int TGS = NST * STAGE;                 // [NST][8 waves][64 lanes] u32 bounds
  static constexpr int TAU = TGS + NST * 8 * 256;         // u64 tau_key[QT]
  static constexpr int CNT = TAU + QW_QT * 8;             // int cnt[QT]
  static constexpr int TOTAL = CNT + QW_QT * 4;
  static_assert(SR > 0 && SR % 16 == 0 && PIECES % 8 == 0, "QW stage shape");
  static_assert(TOTAL <= 160 * 1024, "LDS budget");
};

// the 2 fragments of a group: pieces p and p + OFF2 KiB (row blocks 2i, 2i+1 at one k-step:
// OFF2 = KS; or one row block at k-steps 2i, 2i+1: OFF2 = 1), issued with no wait
// (qw_frag_wait<N> waits and re-defines them)
template <int OFF2, typename V>
__device__ __forceinline__ void qw_issue_frags(uint32_t sbase, uint32_t voff, V (&av)[2]) {
  uint32_t a;
  asm volatile(
      "v_add_u32 %2, %3, %4\n\t"
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %2 offset:%5"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(a)
      : "s"(sbase), "v"(voff), "n"(OFF2 * 1024)
      : "memory");
}
template <int N, typename V>
__device__ __forceinline__ void qw_frag_wait(V (&av)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(av[0]), "+v"(av[1]) : "n"(N) : "memory");
}

// Epilogue helpers of the query-stationary kernels (the per-stage test "does any of a query's
// scores reach its threshold"), without fmaxf's sNaN canonicalisation (a v_max per operand) and
// the float <-> ordered-key round trips: v_max3_f32 over the raw accumulators (a quiet NaN, the
// mark of rows past the corpus, never wins a maximum unless every operand is one), and the
// threshold kept as an ordered key: max(high word of the local k'-th key, the global bound).
// The caller has covered the MFMA -> VALU wait states of the accumulators (asm operands).
__device__ __forceinline__ float qw_max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float qw_max4(const floatx4& v) { return qw_max3(qw_max3(v[0], v[1], v[2]), v[3], v[3]); }
__device__ __forceinline__ uint32_t qw_ord32(float f) {
  const uint32_t u = __float_as_uint(f);
  return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
}

// MAXONLY: the sampling pre-pass on QW (DESIGN.md §4 "Estimated seed"): ntiles counts virtual
// stages of the sampled 256-row tiles (tile vt * tstride, 256 / SR stages each), partitions are
// whole 128-row units, and per unit and query the largest coarse score goes to
// umax[unit][nqb * QT] -- no candidate lists (v4's MAXONLY form is LDS-fill-bound).
// SPREAD: when a stage's LDS-DMA ops are issued.  false: every wave its PPW pieces + its bounds
// right after the stage barrier; true: one op every GSTEP MFMA groups over the first 3/4 of the
// wave's groups (r05, DESIGN.md §5.2: 8 % fewer cycles per stage; the default with one query
// block -- with several, the query blocks of a row partition drift apart and each row stage
// is fetched from HBM once per block).  r05 also measured, and removed: waves 0-3 issuing every
// op (at the barrier or spread), a per-partition arrival counter keeping the query blocks in
// step, and LDS ready / done counters in place of the stage barrier (profiles/r05/).
// STG (r05, 64-row stages at D = 384 only -- its accumulators fit twice): waves 4-7 run each
// stage's epilogue one stage late, right after the next stage barrier, so that the epilogue of
// one wave of a SIMD overlaps the MFMAs of the other (MI355X_MICROARCH.md 'Two waves per SIMD'
// item 9): waves 0-3 -- first in issue priority -- otherwise finish their MFMAs early, run their
// epilogue, and wait ~2.4k cycles per stage at the barrier for waves 4-7, whose epilogue then
// runs with the MFMA pipe idle.
template <typename TM, int CAP, int KS, int SR_ = qw_sr(KS), int NST_ = QW_NST, bool MAXONLY = false,
          bool SPREAD = false, int STG = 0>
__global__ void __launch_bounds__(V3_NT, 1)
score_topk_qw_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows,
                     const TM* __restrict__ qhat, int nqb, int P, int ntiles,
                     uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                     uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp,
                     int tstride = 1, float* __restrict__ umax = nullptr) {
  using L = QwLayout<KS, SR_, NST_>;
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int SR = L::SR, RB = L::RB, PPW = L::PPW, QT = QW_QT, NST = L::NST, D = NST - 1;
  constexpr int OPS = PPW + 1;                       // vmcnt-counted ops per wave per stage
  // fragment groups per stage: (row-block pair, k-step) for the row-block pairs, then (the odd
  // last row block, k-step pair) when RB is odd
  constexpr int NGP = (RB / 2) * KS, NG = NGP + (RB % 2) * (KS / 2);
  constexpr int GSTEP = (NG * 3 / 4) / OPS > 0 ? (NG * 3 / 4) / OPS : 1;   // SPREAD: groups per op
  static_assert(CAP >= 128 && CAP % 64 == 0, "candidate buffer");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  uint64_t* tau_key = reinterpret_cast<uint64_t*>(lds + L::TAU);
  int* cnt = reinterpret_cast<int*>(lds + L::CNT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef HCR_QW_STAMPS
  const uint64_t st_e0 = __builtin_amdgcn_s_memrealtime();   // kernel entry (100 MHz ticks)
#endif

  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  // (wave-uniform values kept in SGPRs: derived in VGPRs by the integer divisions, they were
  // spilled, and a reload after the stage barrier sat in the ring's vmcnt stream)
  const int qb = __builtin_amdgcn_readfirstlane(g % nqb), p = __builtin_amdgcn_readfirstlane(g / nqb);
  constexpr int SPT8 = 256 / SR;                      // stages per sampled 256-row tile
  constexpr int SPU = 128 / SR;                       // stages per 128-row unit (MAXONLY)
  const int t0 = MAXONLY ? (int)((int64_t)p * (ntiles / SPU) / P) * SPU : (int)((int64_t)p * ntiles / P);
  const int t1 = MAXONLY ? (int)((int64_t)(p + 1) * (ntiles / SPU) / P) * SPU : (int)((int64_t)(p + 1) * ntiles / P);
  // a virtual stage's row stage (MAXONLY: of sampled tile vs / SPT8)
  auto real_stage = [&](int vs) __attribute__((always_inline)) {
    return MAXONLY ? (int64_t)(vs / SPT8) * tstride * SPT8 + vs % SPT8 : (int64_t)vs;
  };
  const int qbase = qb * QT;
  uint64_t* wbuf = buf + (size_t)b * QT * CAP;
  const int wq0 = wave * 32;                          // this wave's first query (block-local)
  const int qlane = wq0 + (lane & 15);                // + 16 n: the query of accumulator block n

  if (lane < 32) { tau_key[wq0 + lane] = 0ull; cnt[wq0 + lane] = 0; }
  if (t0 >= t1) {
    if (!MAXONLY && lane < 32) pcnt[(size_t)(qbase + wq0 + lane) * P + p] = 0;
    return;
  }

  // query fragments: lane l holds q^[qlane + 16 n][ks*32 + 8*(l >> 4) .. +8)
  V qf[2][KS];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const TM* src = qhat + (size_t)(qbase + qlane + 16 * n) * ld + (lane >> 4) * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[n][ks] = *reinterpret_cast<const V*>(src + ks * 32);
  }

  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int ldb = ld * 2;
  const int voff = drow * ldb + dchunk * 16;
  const char* rows_b = reinterpret_cast<const char*>(rows);

  const int nsteps = t1 - t0;
  // Stage i (tile t0 + i) goes to ring slot i % NST: this wave's PPW row pieces (piece j =
  // wave + 8 u: row block j / KS, k-step j % KS) and its 32 global bounds -- OPS ops.  Stages
  // past the partition's end are issued too, through zero-record descriptors (the loads return
  // nothing and their LDS writes land in the slot of stage i - NST, already consumed), so every
  // stage costs every wave exactly OPS vmcnt-counted ops and the loop has no tail cases.
  struct StageDesc { __amdgpu_buffer_rsrc_t a, t; int slot; };
  auto stage_desc = [&](int i) __attribute__((always_inline)) {
    const bool live = i < nsteps;
    StageDesc d;
    d.slot = __builtin_amdgcn_readfirstlane(i % NST);
    const int64_t tile = real_stage(__builtin_amdgcn_readfirstlane(t0 + (live ? i : 0)));
    d.a = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(rows_b + (size_t)tile * SR * ldb), (short)0,
                                            live ? SR * ldb : 0, 0x00020000);
    d.t = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(tau_g + qbase), (short)0, live ? QT * 4 : 0,
                                            0x00020000);
    return d;
  };
  auto issue_op = [&](const StageDesc& d, int u) __attribute__((always_inline)) {
    if (u < PPW) {
      const int j = wave + 8 * u;
      // the piece's source offset re-derived per stage from an opaque copy of the row pitch:
      // hoisted, the PPW offsets hold PPW SGPRs across the loop (48-row stages: SGPR spills)
      int ldbs = ldb;
      asm volatile("" : "+s"(ldbs));
      dma16(d.a, lds + d.slot * L::STAGE + j * 1024, voff, (j / KS) * 16 * ldbs + (j % KS) * (V3_BK * 2));
    } else {
      // the lane offset re-derived here (opaque to the compiler: hoisted, it was spilled and
      // its reload waited for the ring)
      int tv;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\t"
                   "v_and_b32 %0, 31, %0\n\tv_lshlrev_b32 %0, 2, %0" : "=v"(tv));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          d.t, (__attribute__((address_space(3))) void*)(lds + L::TGS + (d.slot * 8 + wave) * 256),
          4, tv, wq0 * 4, 0, 0);
    }
  };
  for (int i = 0; i < D; ++i) {
    const StageDesc d = stage_desc(i);
#pragma unroll
    for (int u = 0; u < OPS; ++u) issue_op(d, u);
  }

  const uint32_t offA = (uint32_t)((lane & 15) * 64 + v3_slot(lane >> 4, lane & 15) * 16);
  const uint32_t lds0 = lds_addr(lds);

  bool need = false;
  uint64_t tkr[2] = {0ull, 0ull};
  float umx[2] = {0.f, 0.f};                         // MAXONLY: the current unit's maxima
  // Candidate counts of the lane's two queries (qle, qle + 16), the same in the query's 4 lanes
  // (l, l ^ 16, l ^ 32, l ^ 48).  A query belongs to one wave, so an append takes its slot from
  // the wave's ballot -- the lanes below it with a key for the same query -- instead of an LDS
  // counter round trip (r05: ~1.5k cycles per append under the fragment reads' LDS load).  The
  // LDS counts are written only for a compaction and the final lists.
  // (packed: query qle in the low half, qle + 16 in the high half -- one VGPR; the D = 768 loop
  // has none to spare)
  uint32_t cqp = 0u;
  // the stage's appends: every score >= thr whose key beats the local k'-th key, per query n
  auto append_stage = [&](const floatx4 (&acc)[RB][2], const bool (&hit)[2], const float (&thr)[2],
                          uint32_t row0u, int lq, int le, int qle) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      if (!__any(hit[n])) continue;
#pragma unroll
      for (int m = 0; m < RB; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sc = acc[m][n][r];
          const bool c = sc >= thr[n];
          if (__builtin_amdgcn_ballot_w64(c)) {
            const uint64_t key = make_key(sc, row0u + (uint32_t)(m * 16 + lq * 4 + r));
            const bool a = c && key > tkr[n];
            const uint64_t ba = __builtin_amdgcn_ballot_w64(a);
            if (ba) {
              // the 4 lanes of this lane's query (l & 15) + 16 j, j = 0..3, as a nibble
              const uint64_t t = ba >> (le & 15);
              const uint32_t nib = (uint32_t)(t & 1u) | (uint32_t)((t >> 15) & 2u) |
                                   (uint32_t)((t >> 30) & 4u) | (uint32_t)((t >> 45) & 8u);
              const uint32_t base = (cqp >> (16 * n)) & 0xFFFFu;
              if (a) wbuf[(size_t)(qle + 16 * n) * CAP + base + __popc(nib & ((1u << lq) - 1u))] = key;
              cqp += (uint32_t)__popc(nib) << (16 * n);
            }
          }
        }
      }
    }
    need = (cqp & 0xFFFFu) > (uint32_t)(CAP - SR) || (cqp >> 16) > (uint32_t)(CAP - SR);
  };
#ifdef HCR_QW_STAMPS
  uint64_t st_t0, st_t1, st_t2, st_t3, st_t4, st_acc[4] = {0, 0, 0, 0};
  const uint64_t st_c0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  if constexpr (STG) {
    static_assert(!MAXONLY, "STG: dense pass only");
    const bool late = wave >= 4;                     // waves 4-7: the epilogue one stage late
    constexpr int FD = RB > 2 ? 2 : 3;
    // the MFMA groups of stage s into acc (and the spread DMA ops of stage s + D)
    auto mfma_stage = [&](floatx4 (&acc)[RB][2], uint32_t st, const StageDesc& nd, uint32_t (&tg)[2])
        __attribute__((always_inline)) {
#pragma unroll
      for (int m = 0; m < RB; ++m) acc[m][0] = acc[m][1] = floatx4{0.f, 0.f, 0.f, 0.f};
      auto gbase = [&](int j) {
        return st + (uint32_t)((j < NGP ? 2 * (j / KS) * KS + j % KS : (RB - 1) * KS + 2 * (j - NGP)) * 1024);
      };
      auto issue = [&](int j, V (&dst)[2]) __attribute__((always_inline)) {
        if (j < NGP) qw_issue_frags<KS, V>(gbase(j), offA, dst);
        else qw_issue_frags<1, V>(gbase(j), offA, dst);
      };
      V av[FD][2];
#pragma unroll
      for (int j = 0; j < FD - 1; ++j) issue(j, av[j]);
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        if constexpr (SPREAD) {
          if (j % GSTEP == 0 && j / GSTEP < OPS) issue_op(nd, j / GSTEP);
        }
        if (j + FD - 1 < NG) {
          issue(j + FD - 1, av[(j + FD - 1) % FD]);
          qw_frag_wait<2 * (FD - 1)>(av[j % FD]);
        } else if (j + 1 < NG) {
          qw_frag_wait<2>(av[j % FD]);
        } else {
          qw_frag_wait<0>(av[j % FD]);
          asm volatile("" : "+v"(tg[0]), "+v"(tg[1]));
        }
        if (j >= NGP) {
          const int i = j - NGP;
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[RB - 1][n] = Op::run(av[j % FD][kk], qf[n][2 * i + kk], acc[RB - 1][n]);
        } else {
          const int m0 = 2 * (j / KS), k0 = j % KS;
#pragma unroll
          for (int mm = 0; mm < 2; ++mm)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[m0 + mm][n] = Op::run(av[j % FD][mm], qf[n][k0], acc[m0 + mm][n]);
        }
      }
    };
    // the per-stage test and appends of stage s (as the loop below)
    auto epilogue = [&](floatx4 (&acc)[RB][2], int s, const uint32_t (&tg)[2]) __attribute__((always_inline)) {
      int le;
      asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
      const int lq = le >> 4;
      const int qle = wq0 + (le & 15);
      const int64_t row0 = real_stage(t0 + s) * SR;
      const uint32_t nr32 = (uint32_t)n_rows;
      if (nr32 < (uint32_t)SR || (uint32_t)row0 > nr32 - (uint32_t)SR) {
#pragma unroll
        for (int m = 0; m < RB; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (row0 + m * 16 + lq * 4 + r >= n_rows) acc[m][0][r] = acc[m][1][r] = __builtin_nanf("");
      }
      bool hit[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        float mx = qw_max4(acc[0][n]);
#pragma unroll
        for (int m = 1; m < RB; ++m) mx = qw_max3(mx, qw_max3(acc[m][n][0], acc[m][n][1], acc[m][n][2]), acc[m][n][3]);
        hit[n] = qw_ord32(mx) >= max((uint32_t)(tkr[n] >> 32), tg[n]);
      }
      if (__any(hit[0] || hit[1])) {
        float thr[2];
        thr[0] = unord32(max((uint32_t)(tkr[0] >> 32), tg[0]));
        thr[1] = unord32(max((uint32_t)(tkr[1] >> 32), tg[1]));
        append_stage(acc, hit, thr, (uint32_t)row0, lq, le, qle);
        if (__any(need)) {
          if (le < 16) { cnt[qle] = (int)(cqp & 0xFFFFu); cnt[qle + 16] = (int)(cqp >> 16); }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
          for (int ql = wq0; ql < wq0 + 32; ++ql) {
            if ((int)v3_lds_u32(cnt + ql) > CAP - SR)
              compact_query<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                                 tau_g + qbase + ql, kp, lane, nullptr);
          }
          need = false;
          tkr[0] = v3_lds_u64(tau_key + qle);
          tkr[1] = v3_lds_u64(tau_key + qle + 16);
          cqp = v3_lds_u32(cnt + qle) | (v3_lds_u32(cnt + qle + 16) << 16);
        }
      }
    };
    // one stage: acc / tg this stage's, pacc / ptg the previous stage's (late waves)
    auto stage = [&](int s, floatx4 (&acc)[RB][2], uint32_t (&tg)[2], floatx4 (&pacc)[RB][2],
                     uint32_t (&ptg)[2]) __attribute__((always_inline)) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS * (D - 1)) : "memory");
      v3_barrier();
      if constexpr (!SPREAD) {
        const StageDesc nd = stage_desc(s + D);
#pragma unroll
        for (int u = 0; u < OPS; ++u) issue_op(nd, u);
      }
      [[maybe_unused]] const StageDesc nd = SPREAD ? stage_desc(s + D) : StageDesc{};
      const int slot = s % NST;
      const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)(slot * L::STAGE)));
      {
        int le0;
        asm volatile("v_mov_b32 %0, %1" : "=v"(le0) : "v"(lane));
        const uint32_t ta = lds_addr(lds + L::TGS + (slot * 8 + wave) * 256 + (le0 & 15) * 4);
        asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %2 offset:64"
                     : "=&v"(tg[0]), "=&v"(tg[1]) : "v"(ta) : "memory");
      }
      if (late && s > 0) epilogue(pacc, s - 1, ptg);
      mfma_stage(acc, st, nd, tg);
      if (!late) epilogue(acc, s, tg);
    };
    // STG 1: two accumulator sets (the late waves' epilogue of stage s - 1 free to interleave with
    // the MFMAs of stage s; 256 VGPRs, 2 spilled); STG 2: one set (228 VGPRs) -- the late waves
    // test stage s - 1 before their MFMAs of stage s overwrite it.  (D = 768 has no room for
    // either: its plain loop already holds 256 VGPRs; built, it went to 704 B of scratch.)
    floatx4 acc0[RB][2], acc1s[RB][2];
    floatx4 (&acc1)[RB][2] = STG == 1 ? acc1s : acc0;
    uint32_t tg0[2] = {0u, 0u}, tg1[2] = {0u, 0u};
    int s = 0;
    for (; s + 1 < nsteps; s += 2) {
      stage(s, acc0, tg0, acc1, tg1);
      stage(s + 1, acc1, tg1, acc0, tg0);
    }
    if (s < nsteps) stage(s, acc0, tg0, acc1, tg1);
    if (late) {                                      // the last stage's epilogue
      if (nsteps % 2) epilogue(acc0, nsteps - 1, tg0);
      else epilogue(acc1, nsteps - 1, tg1);
    }
  } else
  for (int s = 0; s < nsteps; ++s) {
#ifdef HCR_QW_STAMPS
    if constexpr (!MAXONLY) HCR_QW_STAMP(st_t0);
#endif
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS * (D - 1)) : "memory");
    v3_barrier();                  // everyone's pieces of stage s; everyone done with slot s-1
#ifdef HCR_QW_STAMPS
    if constexpr (!MAXONLY) HCR_QW_STAMP(st_t1);
#endif
    // stage s + D into the slot everyone has finished with, all OPS ops at once: spread over the
    // MFMA groups they cost 10 % fewer wave cycles but the 4 query blocks of a row partition
    // drifted apart and FETCH_SIZE grew 2.6x (their shared L2 reuse broken: DESIGN.md §5)
    if constexpr (!SPREAD) {
      const StageDesc nd = stage_desc(s + D);
#pragma unroll
      for (int u = 0; u < OPS; ++u) issue_op(nd, u);
    }
    [[maybe_unused]] const StageDesc nd = SPREAD ? stage_desc(s + D) : StageDesc{};

    const int slot = s % NST;
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)(slot * L::STAGE)));
    // this stage's global bounds of the lane's two queries: read now, waited for with the
    // last fragment group
    uint32_t tg2[2];
    {
      int le0;
      asm volatile("v_mov_b32 %0, %1" : "=v"(le0) : "v"(lane));
      const uint32_t ta = lds_addr(lds + L::TGS + (slot * 8 + wave) * 256 + (le0 & 15) * 4);
      asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %2 offset:64"
                   : "=&v"(tg2[0]), "=&v"(tg2[1]) : "v"(ta) : "memory");
    }
#ifdef HCR_QW_STAMPS
    if constexpr (!MAXONLY) HCR_QW_STAMP(st_t2);
#endif
    floatx4 acc[RB][2];
#pragma unroll
    for (int m = 0; m < RB; ++m) acc[m][0] = acc[m][1] = floatx4{0.f, 0.f, 0.f, 0.f};
    // group j: row blocks (2 (j / KS), +1) at k-step j % KS; FD groups of reads in flight
    constexpr int FD = RB > 2 ? 2 : 3;              // (48-row stages: 8 more accumulator VGPRs)
    auto gbase = [&](int j) {
      return st + (uint32_t)((j < NGP ? 2 * (j / KS) * KS + j % KS : (RB - 1) * KS + 2 * (j - NGP)) * 1024);
    };
    // (the second fragment of a group: the next row block, KS KiB on, or the next k-step)
    auto issue = [&](int j, V (&dst)[2]) __attribute__((always_inline)) {
      if (j < NGP) qw_issue_frags<KS, V>(gbase(j), offA, dst);
      else qw_issue_frags<1, V>(gbase(j), offA, dst);
    };
    V av[FD][2];
#pragma unroll
    for (int j = 0; j < FD - 1; ++j) issue(j, av[j]);
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      if constexpr (SPREAD) {       // op u at group u * GSTEP (folds to constants when unrolled)
        if (j % GSTEP == 0 && j / GSTEP < OPS) issue_op(nd, j / GSTEP);
      }
      if (j + FD - 1 < NG) {
        issue(j + FD - 1, av[(j + FD - 1) % FD]);
        qw_frag_wait<2 * (FD - 1)>(av[j % FD]);
      } else if (j + 1 < NG) {
        qw_frag_wait<2>(av[j % FD]);
      } else {
        qw_frag_wait<0>(av[j % FD]);
        asm volatile("" : "+v"(tg2[0]), "+v"(tg2[1]));   // (read before the fragments: landed)
      }
      if (j >= NGP) {
        const int i = j - NGP;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[RB - 1][n] = Op::run(av[j % FD][kk], qf[n][2 * i + kk], acc[RB - 1][n]);
      } else {
        const int m0 = 2 * (j / KS), k0 = j % KS;
#pragma unroll
        for (int mm = 0; mm < 2; ++mm)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[m0 + mm][n] = Op::run(av[j % FD][mm], qf[n][k0], acc[m0 + mm][n]);
      }
    }

#ifdef HCR_QW_STAMPS
    if constexpr (!MAXONLY) HCR_QW_STAMP(st_t3);
#endif
    // ---- epilogue of tile t0 + s: this wave's 32 queries x SR rows ----
    int le;
    asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
    const int lq = le >> 4;
    const int qle = wq0 + (le & 15);                 // the query of accumulator block 0
    const int64_t row0 = real_stage(t0 + s) * SR;
    // the corpus' last tile: rows past the end never pass (NaN).  A 32-bit scalar test (rows per
    // shard < 2^32): the 64-bit compare is a VALU op on a VGPR copy of n_rows, spilled at SR = 48
    const uint32_t nr32 = (uint32_t)n_rows;
    if (nr32 < (uint32_t)SR || (uint32_t)row0 > nr32 - (uint32_t)SR) {
#pragma unroll
      for (int m = 0; m < RB; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row0 + m * 16 + lq * 4 + r >= n_rows) acc[m][0][r] = acc[m][1][r] = __builtin_nanf("");
    }
    if constexpr (MAXONLY) {
      // per query: the largest of the stage's SR rows (the lane's RB x 4, then over the 4
      // row-group lanes l, l ^ 16, l ^ 32, l ^ 48), folded into the unit's maximum; a quiet NaN
      // (rows past the corpus) never wins a maximum unless every operand is one
      const int vs = t0 + s;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        float mx = qw_max4(acc[0][n]);
#pragma unroll
        for (int m = 1; m < RB; ++m) mx = qw_max3(mx, qw_max3(acc[m][n][0], acc[m][n][1], acc[m][n][2]), acc[m][n][3]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        umx[n] = (vs % SPU == 0) ? mx : fmaxf(umx[n], mx);
      }
      if (vs % SPU == SPU - 1 && lane < 16) {
        const int u = (vs / SPT8) * 2 + (vs % SPT8) / SPU;
        float* dst = umax + (size_t)u * ((size_t)nqb * QT) + qbase + qle;
        dst[0] = umx[0];
        dst[16] = umx[1];
      }
      continue;
    }
    // the stage test as QW1's (r04): v_max3 over the raw accumulators and the threshold as an
    // ordered key, max(high word of the local k'-th key, global bound) -- no fmaxf sNaN
    // canonicalisation, no key -> float round trips (a NaN maximum passes; its scores fail below)
    bool hit[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      float mx = qw_max4(acc[0][n]);
#pragma unroll
      for (int m = 1; m < RB; ++m) mx = qw_max3(mx, qw_max3(acc[m][n][0], acc[m][n][1], acc[m][n][2]), acc[m][n][3]);
      hit[n] = qw_ord32(mx) >= max((uint32_t)(tkr[n] >> 32), tg2[n]);
    }
    if (__any(hit[0] || hit[1])) {
      float thr[2];
      thr[0] = unord32(max((uint32_t)(tkr[0] >> 32), tg2[0]));
      thr[1] = unord32(max((uint32_t)(tkr[1] >> 32), tg2[1]));
      append_stage(acc, hit, thr, (uint32_t)row0, lq, le, qle);
      // a query whose buffer cannot take another tile's appends is compacted to its best k'
      // (rare: drains this wave's stores and, in order, its ring pieces)
      if (__any(need)) {
        if (le < 16) { cnt[qle] = (int)(cqp & 0xFFFFu); cnt[qle + 16] = (int)(cqp >> 16); }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
        for (int ql = wq0; ql < wq0 + 32; ++ql) {
          if ((int)v3_lds_u32(cnt + ql) > CAP - SR)
            compact_query<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                               tau_g + qbase + ql, kp, lane, nullptr);
        }
        need = false;
        tkr[0] = v3_lds_u64(tau_key + qle);
        tkr[1] = v3_lds_u64(tau_key + qle + 16);
        cqp = v3_lds_u32(cnt + qle) | (v3_lds_u32(cnt + qle + 16) << 16);
      }
    }
#ifdef HCR_QW_STAMPS
    if constexpr (!MAXONLY) {
      HCR_QW_STAMP(st_t4);
      st_acc[0] += st_t1 - st_t0;
      st_acc[1] += st_t2 - st_t1;
      st_acc[2] += st_t3 - st_t2;
      st_acc[3] += st_t4 - st_t3;
    }
#endif
  }
#ifdef HCR_QW_STAMPS
  const uint64_t st_c1 = __builtin_amdgcn_s_memtime(), st_r1 = __builtin_amdgcn_s_memrealtime();
#endif

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (MAXONLY) return;
  if (lane < 16) { cnt[wq0 + lane] = (int)(cqp & 0xFFFFu); cnt[wq0 + lane + 16] = (int)(cqp >> 16); }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  final_lists_wave<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wq0, 1, 32, kp, lane, partials, pcnt, P, p);
#ifdef HCR_QW_STAMPS
  if (lane == 0 && b < 4096) {
    // o[4]: stages | prologue ticks << 24 | final-lists ticks << 44; o[7]: entry (absolute)
    const uint64_t st_r2 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = hcr_qw_stamps + ((size_t)b * 8 + wave) * 8;
    o[0] = st_acc[0]; o[1] = st_acc[1]; o[2] = st_acc[2]; o[3] = st_acc[3];
    o[4] = (uint64_t)nsteps | ((st_r0 - st_e0) << 24) | ((st_r2 - st_r1) << 44);
    o[5] = st_c1 - st_c0;                                  // shader cycles over the loop ...
    o[6] = st_r1 - st_r0;                                  // ... and 100 MHz ticks: the clock
    o[7] = st_e0;
  }
#endif
}

}  // namespace hcr
