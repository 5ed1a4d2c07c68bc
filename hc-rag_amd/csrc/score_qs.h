// score_qs.h — K2 "query-stationary" (QS): the fused score + top-k' kernel for the batches
// between the streaming regime (B <= 16, 256 x 16 tiles) and the MFMA-bound regime (B > 256,
// v4's 256 x 256 tiles): 17..256 queries, where the corpus stream -- N x D x 2 bytes, once --
// is the roofline (1M x 384 at B = 256 is HBM-bound, 10M x 768 at B <= 64 too).
//
// v3/v4 bring a query tile into LDS with every row tile, so the LDS-DMA fill per flop doubles
// (256 rows + 256 queries per stage) and the fill -- ~7.5 TB/s for the whole chip, near the HBM
// rate -- becomes the bound at half the HBM roofline.  Here the queries are
// loaded ONCE into VGPRs as MFMA B fragments (16 queries x the whole K: K/8 VGPRs), and only
// the corpus rows stream through the LDS-DMA ring:
//
//  * workgroup = 8 waves; wave w owns NQ blocks of 16 queries (QT = 128 NQ queries per
//    workgroup) and computes all RT rows of every tile for them (RT/16 row blocks x NQ of
//    16x16x32 MFMAs per 32-deep half stage): NQ = 1 on 256-row tiles, or NQ = 2 on 128-row
//    tiles (KS <= 12), where every row is filled into LDS once per 256 queries;
//  * the row tile is streamed in stages of RT x 64 k (32 or 16 KiB of 1 KiB LDS-DMA pieces),
//    an NST-deep ring (4 x 32 or 8 x 16 KiB), each wave waits for its own pieces then one
//    barrier per stage (as v3);
//  * the k-step loop over a tile is fully unrolled (KS = ld / 32 is a template parameter) so
//    the query fragments stay in registers;
//  * the epilogue needs no block synchronisation: a query belongs to one wave, so its
//    candidate appends, compactions and final list are that wave's alone (compact_query_inl);
//    its common case (no row of the tile beats any of the wave's bounds) is a max over the
//    accumulators -- raw for UNIT, scaled by 4 LDS quads of inverse norms otherwise.
//
// Grid: nqb query blocks x P row partitions (XCD-aware as v3).  Same outputs as v3: every
// query's surviving coarse keys of its partition appended to partials[q] (final_list), tau_g
// raised.
#pragma once
#include <utility>

#include "score_v3.h"

namespace hcr {

#ifdef HCR_QS_STAMPS
// Diagnostic build only (Makefile target `stamps`, tools/qs_stamps.py): per wave, the s_memtime
// cycles spent waiting for a stage (vmcnt + barrier), issuing a stage (DMA + fragment reads +
// MFMAs), in the tile epilogue, and the tile count.  Never compiled into the product library.
__device__ unsigned long long hcr_qs_stamps[4096 * 8 * 8];
#define HCR_QS_STAMP(t)                                                                \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");          \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#endif

// 4 row-block fragments (1 KiB apart) at LDS address sbase + voff, issued with no wait;
// qs_frag_wait<N> then waits until at most N LDS reads are outstanding (they complete in
// order) and re-defines the fragments so no use of them is scheduled above the wait.  Inline
// asm: a compiler-visible LDS read after the ring's LDS-DMA gets a vmcnt(0) (ring drained).
// The stage base is a wave-uniform SGPR operand so that one VGPR (the lane's offset) serves
// every stage: per-stage address VGPRs were spilled (r02: 249 VGPRs, a scratch reload and a
// ring drain per tile).
template <typename V>
__device__ __forceinline__ void qs_issue_frags4(uint32_t sbase, uint32_t voff, V (&av)[4]) {
  uint32_t a;
  asm volatile(
      "v_add_u32 %4, %5, %6\n\t"
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:1024\n\t"
      "ds_read_b128 %2, %4 offset:2048\n\t"
      "ds_read_b128 %3, %4 offset:3072"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(a)
      : "s"(sbase), "v"(voff)
      : "memory");
}
template <int N, typename V>
__device__ __forceinline__ void qs_frag_wait(V (&av)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]) : "n"(N) : "memory");
}

// four of a lane's inverse-norm quads (row blocks m0 .. m0+3: 64 B apart), one wait
__device__ __forceinline__ void qs_read_inv4(uint32_t a, float4 (&v)[4]) {
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:64\n\t"
      "ds_read_b128 %2, %4 offset:128\n\t"
      "ds_read_b128 %3, %4 offset:192\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(a)
      : "memory");
}

// the 8 row-mask words of a tile (32 B), one wait
__device__ __forceinline__ void qs_read_u32x8(uint32_t a, uint32_t (&w)[8]) {
  uint4 x, y;
  asm volatile(
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %2 offset:16\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x), "=&v"(y)
      : "v"(a)
      : "memory");
  w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
  w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
}

constexpr int QS_NW = 8;         // waves per workgroup (two per SIMD)

template <int NST, int KS, int RT_, int NQ, int HS = 2>
struct QsLayout {
  static constexpr int NW = QS_NW;
  static constexpr int RT = RT_, QT = 16 * NQ * NW;
  static constexpr int SPT = KS / HS;                      // stages per tile (32 HS-deep stages)
  static constexpr int STAGE = RT * 64 * HS;               // RT rows x 32 HS k: HS 32-deep halves
  // tile slots of inverse norms / bounds / mask words: a tile's slot must outlive the NST-1
  // stages of look-ahead, (NIS - 1) * SPT > NST - 1
  static constexpr int NIS = (NST - 1) / SPT + 2;
  static constexpr int INV = NST * STAGE;                  // NIS x RT floats
  static constexpr int INV_SLOT = RT * 4;
  static constexpr int TG = INV + NIS * INV_SLOT;          // NIS x QT u32 global bounds
  static constexpr int TG_SLOT = QT * 4;
  static constexpr int MSK = TG + NIS * TG_SLOT;           // NIS x 32 B of row-mask words
  static constexpr int TAU = MSK + NIS * 64;               // u64 tau_key[QT]
  static constexpr int CNT = TAU + QT * 8;                 // int cnt[QT]
  static constexpr int LS = 8;                             // staged append slots per query
  static constexpr int SLOTS = CNT + QT * 4;               // u64 slots[QT][LS] (staged appends)
  static constexpr int TOTAL = SLOTS + QT * LS * 8;
  static_assert(KS % HS == 0, "whole stages per tile");
  static_assert(TOTAL <= 160 * 1024, "LDS budget");
};

// UNIT: the coarse score is the raw dot product (L2-normalised corpora, as score_v4.h UNIT;
// the host widens the certificate by the corpus' norm deviation).
// NQ x 16 queries per wave on RT-row tiles: (1, 256) -- 128 queries per workgroup, any
// KS <= 24 -- or (2, 128) -- 256 queries per workgroup for KS <= 12 (2 x KS x 4 VGPRs of query
// fragments): every row is filled into LDS once per 256 queries instead of once per 128.
//
// HS: 32-deep k-steps per stage (2: 64-deep stages; 4 at configs[1]'s KS = 12: 3 barriers per
// tile instead of 6, each amortising the skew between the SIMD's two waves and the
// fragment-read start-up over more MFMAs).  (r03 also built a 4-wave two-workgroups-per-CU form,
// QS4, and 192-deep stages; neither measured faster -- profiles/r03/qs_forms/ -- removed in r04.)
template <typename TM, int CAP, int KS, bool UNIT, int NQ = 1, int RT_ = 256,
          int NST = (RT_ == 256 ? 4 : 8), int HS = 2>
__global__ void __launch_bounds__(QS_NW * 64, 1)
score_topk_qs_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows,
                     const float* __restrict__ inv_norm, const uint32_t* __restrict__ mask,
                     const TM* __restrict__ qhat, int nqb, int P, int ntiles, int tstride,
                     uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                     uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp) {
  using L = QsLayout<NST, KS, RT_, NQ, HS>;
  constexpr int NW = QS_NW;
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int RT = L::RT, QT = L::QT, MT = RT / 16, D = NST - 1, SPT = L::SPT;
  constexpr int PPH = RT / 16;            // 1 KiB LDS-DMA pieces per 32-deep half of a stage
  constexpr int PPW = HS * PPH / NW;      // ... per wave per stage
  static_assert((HS * PPH) % NW == 0, "stage pieces per wave");
  constexpr int NG = MT / 4 * HS;         // groups of 4 row blocks per stage (HS halves)
  static_assert(CAP >= 2 * RT, "candidate buffer must hold a tile's appends after a compaction");
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  uint64_t* tau_key = reinterpret_cast<uint64_t*>(lds + L::TAU);
  int* cnt = reinterpret_cast<int*>(lds + L::CNT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int qb = g % nqb, p = g / nqb;
  const int t0 = (int)((int64_t)p * ntiles / P);
  const int t1 = (int)((int64_t)(p + 1) * ntiles / P);
  const int qbase = qb * QT;
  uint64_t* wbuf = buf + (size_t)b * QT * CAP;
  const int wq0 = wave * 16 * NQ;                 // this wave's first query (block-local)
  // the query of this lane's accumulators in query block n: wq0 + 16 n + (lane & 15)
  const int qlane = wq0 + (lane & 15);

  // each wave initialises and owns its queries' state (no block barrier needed for it)
  if (lane < 16 * NQ) { tau_key[wq0 + lane] = 0ull; cnt[wq0 + lane] = 0; }

  if (t0 >= t1) {              // an empty partition: empty lists
    if (lane < 16 * NQ) pcnt[(size_t)(qbase + wq0 + lane) * P + p] = 0;
    return;
  }

  // query fragments: lane l holds q^[wq0 + 16 n + (l & 15)][ks*32 + 8*(l >> 4) .. +8)
  V qf[NQ][KS];
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    const TM* src = qhat + (size_t)(qbase + qlane + 16 * n) * ld + (lane >> 4) * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[n][ks] = *reinterpret_cast<const V*>(src + ks * 32);
  }

  // DMA: a stage is RT rows x 64 k as two 32-deep halves of the v3 image (PPH 1 KiB pieces of
  // 16 rows x 64 B each); wave w issues pieces w, w+8, ... (PPW of them)
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int ldb = ld * 2;
  const int voff = drow * ldb + dchunk * 16;
  const char* rows_b = reinterpret_cast<const char*>(rows);
  const __amdgpu_buffer_rsrc_t inv_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(inv_norm), (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t tg_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(tau_g + qbase), (short)0, QT * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t msk_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(mask), (short)0, 0x7FFFFFFF, 0x00020000);
  // tile-start pieces: inverse norms (not read by the UNIT kernel), bounds, mask words -- by
  // the last three waves
  const bool extra = (!UNIT && wave == NW - 1) || wave == NW - 2 || (wave == NW - 3 && mask);

  const int nsteps = (t1 - t0) * SPT;
  // Issue virtual tile vt's stage SP2 into ring slot `slot`.  Every wave issues its PPW row
  // pieces; at a tile's first stage waves NW-1 / NW-2 / NW-3 also issue the tile's inverse norms, query
  // bounds and mask words (SP2 is a compile-time constant, so is that choice).  The per-lane
  // offsets are re-derived from `lane` here rather than kept live across the loop.
  auto issue_stage = [&](auto sp2_c, int vt_, int slot_) __attribute__((always_inline)) {
    constexpr int SP2 = decltype(sp2_c)::value;
    const int vt = __builtin_amdgcn_readfirstlane(vt_);
    const int slot = __builtin_amdgcn_readfirstlane(slot_);
    const int tile = vt * tstride;
    char* sa = lds + slot * L::STAGE;
    const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        uniform_ptr(rows_b + (size_t)tile * RT * ldb), (short)0, RT * ldb, 0x00020000);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int j = wave + NW * i;           // piece: half j / PPH, rows (j % PPH) * 16 ..
      dma16(a_rsrc, sa + j * 1024, voff, (j % PPH) * 16 * ldb + (HS * SP2 + j / PPH) * (V3_BK * 2));
    }
    if constexpr (SP2 == 0) {
      const int is = vt % L::NIS;
      int l16;
      asm volatile("v_lshlrev_b32 %0, 4, %1" : "=v"(l16) : "v"(lane));
      if (!UNIT && wave == NW - 1 && lane < RT / 4)   // RT inverse norms
        dma16(inv_rsrc, lds + L::INV + is * L::INV_SLOT, l16, tile * (RT * 4));
      if (wave == NW - 2 && lane < QT / 4)
        dma16(tg_rsrc, lds + L::TG + is * L::TG_SLOT, l16, 0);
      if (wave == NW - 3 && mask && lane < RT / 32)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            msk_rsrc, (__attribute__((address_space(3))) void*)(lds + L::MSK + is * 64),
            4, l16 >> 2, tile * (RT / 8), 0, 0);
    }
  };
  // prologue: the first D stages (global stage i = tile t0 + i / SPT, stage i % SPT)
  [&]<int... I>(std::integer_sequence<int, I...>) {
    ((I < nsteps ? issue_stage(std::integral_constant<int, I % SPT>{}, t0 + I / SPT, I % NST)
                 : void()), ...);
  }(std::make_integer_sequence<int, D>{});

  const uint32_t offA = (uint32_t)((lane & 15) * 64 + v3_slot(lane >> 4, lane & 15) * 16);
  const uint32_t lds0 = lds_addr(lds);

  floatx4 acc[MT][NQ];
#ifdef HCR_QS_STAMPS
  unsigned long long st_wait = 0, st_comp = 0, st_epi = 0, st_fast = 0, st_slow_n = 0, st_t0, st_t1, st_t2;
  // the in-kernel clock: s_memtime (shader clock) over s_memrealtime (100 MHz) across the loop
  unsigned long long st_c0, st_r0, st_c1, st_r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_c0), "=s"(st_r0)::"memory");
#endif
  bool need = false;                           // some query's buffer must be compacted
  // the lane's query's local k'-th key (only this wave changes it: kept in registers) and its
  // global bound, re-read every 4th tile: the LDS is the busiest unit of this kernel (every
  // wave reads every row fragment), an epilogue read waits behind the fragment reads, and a
  // stale bound is a lower one (more appends, same lists)
  uint64_t tkr[NQ];
  uint32_t tgr[NQ];
  // the lane's query's append count (r04: in registers -- the same in the query's 4 lanes --
  // instead of an LDS atomic with return per append; cnt[] in LDS is written back before a
  // compaction and at the end) and the count at its last flush: candidates at positions
  // [flushed, flushed + LS) wait in the query's LDS slots (see flush_slots)
  int cntr[NQ], flushed[NQ];
#pragma unroll
  for (int n = 0; n < NQ; ++n) { tkr[n] = 0; tgr[n] = 0; cntr[n] = 0; flushed[n] = 0; }
  // Staged appends to their global positions, 64 per store instruction: lane l copies slots
  // (l >> 4) + 4 i of its query.  Why staged (r04): the ring's waits count this wave's vector
  // memory operations in issue order, so every store instruction an epilogue issues (one per
  // append step with a hit) pushes the next D - 1 stage waits past pieces of later stages --
  // per-append global stores cost ~1k cycles of stage wait per tile at configs[1] (r03 diag).
  // A flush issues NQ x LS / 4 store instructions, when a query's slots are half full.
  auto flush_slots = [&](int lane4) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      const int ql = qlane + 16 * n;
      const int staged = min(cntr[n] - flushed[n], L::LS);
#pragma unroll
      for (int i = 0; i < L::LS / 4; ++i) {
        const int j = lane4 + 4 * i;
        if (j < staged)
          wbuf[(size_t)ql * CAP + flushed[n] + j] = v3_lds_u64(lds + L::SLOTS + (ql * L::LS + j) * 8);
      }
      flushed[n] = cntr[n];
    }
  };
  int s = 0;                                   // global stage index
  for (int vt = t0; vt < t1; ++vt) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto step = [&](auto sp_c) __attribute__((always_inline)) {
      constexpr int SP = decltype(sp_c)::value;
      // stage s landed: this wave's pieces of it.  In steady state the D-1 later stages stay
      // in flight: PPW pieces each, +1 on waves 5-7 for a tile-start stage among them (a
      // compile-time count: tile starts are the stages with SP + j == 0 mod SPT); the
      // stream's last stages wait for everything (nothing left to overlap).
      constexpr int STARTS = [] {
        int c = 0;
        for (int j = 1; j < D; ++j) c += ((SP + j) % SPT == 0) ? 1 : 0;
        return c;
      }();
#ifdef HCR_QS_STAMPS
      HCR_QS_STAMP(st_t0);
#endif
      if (s + D - 1 < nsteps) {
        if (extra && STARTS) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW * (D - 1) + STARTS) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW * (D - 1)) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      v3_barrier();                      // everyone's pieces; everyone done with stage s-1's slot
#ifdef HCR_QS_STAMPS
      HCR_QS_STAMP(st_t1);
      st_wait += st_t1 - st_t0;
#endif
      if (s + D < nsteps)
        issue_stage(std::integral_constant<int, (SP + D) % SPT>{}, vt + (SP + D) / SPT, (s + D) % NST);
      const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane(
          (int)(lds0 + (uint32_t)((s % NST) * L::STAGE)));
      // NG groups of 4 row blocks (HS halves x MT/4), group j+1's reads in flight under group
      // j's MFMAs
      constexpr int GPH = MT / 4;
      V av[2][4];
      qs_issue_frags4<V>(st, offA, av[0]);
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const int h = j / GPH, g4 = j % GPH;
        if (j < NG - 1) {
          qs_issue_frags4<V>(st + (uint32_t)(((j + 1) / GPH) * (RT * 64) + ((j + 1) % GPH) * 4096),
                             offA, av[(j + 1) & 1]);
          qs_frag_wait<4>(av[j & 1]);
        } else {
          qs_frag_wait<0>(av[j & 1]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int n = 0; n < NQ; ++n)
            acc[g4 * 4 + i][n] = Op::run(av[j & 1][i], qf[n][HS * SP + h], acc[g4 * 4 + i][n]);
      }
#ifdef HCR_QS_STAMPS
      HCR_QS_STAMP(st_t2);
      st_comp += st_t2 - st_t1;
#endif
      ++s;
    };
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (step(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, SPT>{});

    // ---- epilogue of tile vt (this wave's 16 queries only; no block synchronisation) ----
#ifdef HCR_QS_STAMPS
    HCR_QS_STAMP(st_t0);
#endif
    // the lane id through an opaque move: per-row constants derived from it are otherwise
    // hoisted out of the tile loop as 64 loop-invariant VGPRs (and spilled)
    int le;
    asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
    const int lq = le >> 4;
    const int64_t row0 = (int64_t)vt * tstride * RT;
    // rows of the tile inside the corpus (row ids fit 32 bits: the coarse keys carry them so)
    const int nlive = (int)__builtin_amdgcn_readfirstlane(
        (int)(n_rows - row0 < (int64_t)RT ? n_rows - row0 : (int64_t)RT));
    const uint32_t row0u = (uint32_t)row0;
    const int is = vt % L::NIS;
    const char* invl = lds + L::INV + is * L::INV_SLOT + lq * 16;
    const char* mskl = lds + L::MSK + is * 64;
    if (((vt - t0) & 3) == 0) {   // (from the opaque lane copy: a qlane-based address was spilled)
#pragma unroll
      for (int n = 0; n < NQ; ++n) tgr[n] = v3_lds_u32(lds + L::TG + is * L::TG_SLOT + (wq0 + (le & 15) + 16 * n) * 4);
    }
    float thr[NQ];
#pragma unroll
    for (int n = 0; n < NQ; ++n) thr[n] = fmaxf(tkr[n] ? key_score(tkr[n]) : -INFINITY, unord32(tgr[n]));
    // scores of row block m: the accumulators scaled by the rows' inverse norms (1 for UNIT),
    // NaN for rows past the corpus end or masked out (they never pass a >= test).  The
    // inverse norms come 4 row blocks at a time (qs_read_inv4), the mask words at once.
    const bool live = !mask && nlive == RT;   // every row of the tile counts
    uint32_t mw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) mw[i] = 0xFFFFFFFFu;
    if (mask) qs_read_u32x8(lds_addr(mskl), mw);
    auto checked4 = [&](int m4, float (&iv)[4][4]) __attribute__((always_inline)) {
      float4 v[4];
      if constexpr (UNIT) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = make_float4(1.f, 1.f, 1.f, 1.f);
      } else {
        qs_read_inv4(lds_addr(invl + m4 * 64), v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = (m4 + i) * 16 + lq * 4;
        const float vv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = (rl + r < nlive) && ((mw[(m4 + i) >> 1] >> ((rl + r) & 31)) & 1u);
          iv[i][r] = ok ? vv[r] : __builtin_nanf("");
        }
      }
    };
    // The tile's scores in place (r04): a UNIT corpus's whole tile is its raw accumulators;
    // otherwise they are scaled by the rows' inverse norms (1 for UNIT) and set to NaN for rows
    // past the corpus end or masked out (NaN never passes a >= test).  One epilogue path
    // follows for every tile (r03 kept a checked twin of the whole epilogue: twice the append
    // code, see below).
    if (!(UNIT && live)) {
#pragma unroll
      for (int m4 = 0; m4 < MT; m4 += 4) {
        float iv[4][4];
        checked4(m4, iv);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int n = 0; n < NQ; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m4 + i][n][r] *= iv[i][r];
      }
    }
    // per row block maxima (kept for the slow path's block test), then per query block
    float bmx[MT][NQ], mx[NQ];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n)
        bmx[m][n] = fmaxf(fmaxf(acc[m][n][0], acc[m][n][1]), fmaxf(acc[m][n][2], acc[m][n][3]));
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      mx[n] = bmx[0][n];
#pragma unroll
      for (int m = 1; m < MT; ++m) mx[n] = fmaxf(mx[n], bmx[m][n]);
    }
    bool hit[NQ];
    bool anyhit = false;
#pragma unroll
    for (int n = 0; n < NQ; ++n) { hit[n] = mx[n] >= thr[n]; anyhit |= hit[n]; }
#ifdef HCR_QS_STAMPS
    HCR_QS_STAMP(st_t2);
    st_fast += st_t2 - st_t0;
    st_slow_n += __any(anyhit) ? 1 : 0;
#endif
    if (__any(anyhit)) {
      // a row is appended when its key beats the query's local k'-th key (same scores as the
      // max above: x * 1 == x, and the checked path equals the plain one on live rows).
      // Code size (r04): the slow path had a checked twin for tail / masked / non-UNIT tiles,
      // each with NQ x MT x 4 copies of the append: 62 KB of kernel code at configs[1], 90-100
      // KB at KS = 24, against a 64 KB instruction cache shared by two CUs (every entry into
      // the slow path missed in it: ~2.3k cycles per entry whatever the append did -- r04
      // stamps with the appends staged in LDS: no change).  The scores are now made in place
      // above, and one unrolled path serves every tile.
      // Appends without an LDS round trip (r04): the lanes of one query (lane & 15 equal: its 4
      // row groups lq) take consecutive positions from the ballot of the hits -- a lane's
      // position is the count so far plus the hits of the query's lanes below it (mbcnt) --
      // and every lane adds the query's hit count to its copy of the counter.
      const uint64_t qmask = 0x0001000100010001ull << (le & 15);
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        if (!__any(hit[n])) continue;
        // the row blocks holding a score at or above the threshold (a wave-uniform test per
        // block, unrolled: no append code here), then one rolled loop over those blocks, block
        // m's accumulators picked by a wave-uniform select, with the append body in it once
        uint32_t blocks = 0;
#pragma unroll
        for (int m = 0; m < MT; ++m)
          if (__builtin_amdgcn_ballot_w64(bmx[m][n] >= thr[n])) blocks |= 1u << m;
        const int ql = qlane + 16 * n;
        uint64_t* wq = wbuf + (size_t)ql * CAP;
        char* sq = lds + L::SLOTS + ql * L::LS * 8;
#pragma unroll 1
        while (blocks) {
          const int m = __builtin_ctz(blocks);
          blocks &= blocks - 1;
          floatx4 v = acc[0][n];
#pragma unroll
          for (int mm = 1; mm < MT; ++mm)
            if (m == mm) v = acc[mm][n];
          const uint32_t rowb = row0u + (uint32_t)(m * 16 + lq * 4);
          // this lane's rows of the block at or above the threshold; one of them per lane per
          // pass, lowest first (r04: the typical entry has one hit in the wave, and the body
          // once per row r cost ~2.3k cycles per entry in VALU issue alone)
          const float t = thr[n];
          uint32_t hm = (v[0] >= t ? 1u : 0u) | (v[1] >= t ? 2u : 0u) | (v[2] >= t ? 4u : 0u) |
                        (v[3] >= t ? 8u : 0u);
#pragma unroll 1
          while (__any(hm != 0u)) {
            const bool live = hm != 0u;
            const uint32_t r = (uint32_t)__builtin_ctz(hm | 16u);
            const float sc = r == 0u ? v[0] : r == 1u ? v[1] : r == 2u ? v[2] : v[3];
            hm &= hm - 1u;
            // a row is appended when its key beats the query's local k'-th key (same scores as
            // the max above: x * 1 == x, and the checked path equals the plain one on live rows)
            const uint64_t key = make_key(sc, rowb + r);
            const bool h = live && key > tkr[n];
            const uint64_t bq = __builtin_amdgcn_ballot_w64(h) & qmask;
            if (h) {
              const int pos = cntr[n] + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bq >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bq, 0u));
              const int sp = pos - flushed[n];
              if (sp < L::LS) v3_lds_store_u64(sq + sp * 8, key);
              else wq[pos] = key;            // (the slots are full: rare)
            }
            cntr[n] += __builtin_popcountll(bq);
          }
        }
        need |= cntr[n] > CAP - RT;
      }
      bool half = false;
#pragma unroll
      for (int n = 0; n < NQ; ++n) half |= cntr[n] - flushed[n] >= L::LS / 2;
      if (__any(half) && !__any(need)) flush_slots(lq);
      // a query whose buffer cannot take another tile's appends is compacted to its best k'
      // (rare: drain this wave's stores -- and, in order, its ring pieces -- only then)
      if (__any(need)) {
        flush_slots(lq);
#pragma unroll
        for (int n = 0; n < NQ; ++n)
          if (le < 16) v3_lds_store_u32(&cnt[qlane + 16 * n], (uint32_t)cntr[n]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
        for (int ql = wq0; ql < wq0 + 16 * NQ; ++ql) {
          if ((int)v3_lds_u32(cnt + ql) > CAP - RT)
            compact_query<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                               tau_g + qbase + ql, kp, lane, nullptr);
        }
        need = false;
#pragma unroll
        for (int n = 0; n < NQ; ++n) {
          tkr[n] = v3_lds_u64(tau_key + qlane + 16 * n);
          cntr[n] = flushed[n] = (int)v3_lds_u32(cnt + qlane + 16 * n);
        }
      }
    }
#ifdef HCR_QS_STAMPS
    HCR_QS_STAMP(st_t1);
    st_epi += st_t1 - st_t0;
#endif
  }
#ifdef HCR_QS_STAMPS
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_c1), "=s"(st_r1)::"memory");
  if (lane == 0 && b < 4096) {
    unsigned long long* o = hcr_qs_stamps + ((size_t)b * 8 + wave) * 8;
    o[0] = st_wait; o[1] = st_comp; o[2] = st_epi; o[3] = (unsigned long long)(t1 - t0);
    o[6] = st_c1 - st_c0; o[7] = st_r1 - st_r0;
    o[4] = st_fast; o[5] = st_slow_n;
  }
#endif

  // final: every query's surviving keys (at most k') appended to its region of the partials
  flush_slots(lane >> 4);
#pragma unroll
  for (int n = 0; n < NQ; ++n)
    if (lane < 16) v3_lds_store_u32(&cnt[qlane + 16 * n], (uint32_t)cntr[n]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  final_lists_wave<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wq0, 1, 16 * NQ, kp, lane, partials, pcnt, P, p);
}

}  // namespace hcr
