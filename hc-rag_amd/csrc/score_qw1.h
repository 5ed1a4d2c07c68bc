// score_qw1.h — K2 "QW1": the wide query-stationary score + top-k' kernel at ONE wave per
// SIMD, for large batches at D = 1024 (MFMA-bound: configs[4], bge-large 100M x 1024 bf16).
//
// Why.  QW (score_qw.h) runs two waves per SIMD with 32 queries x the whole K each in 256
// registers, which caps K at 768.  QW1 gives each wave a whole SIMD -- 512 registers -- and 3
// query blocks of 16 at D = 1024: each A (row) fragment read from LDS feeds 6 MFMAs and the CU
// reads 4 x the stage per stage.
//
//  * query fragments: QB x KS x 4 = 384 registers, the first 64 fragments in
//    AGPRs (an MFMA takes its A/B operands from either half of the unified file), the rest in
//    VGPRs; loaded once by inline asm with "=a" / "=v" outputs so the compiler never copies them;
//  * a stage is SR = 16 rows x the whole K (32 KiB) in a 4-deep LDS-DMA ring, the v3 piece image (1 KiB pieces of 16
//    rows x 32 k, XOR-swizzled 16-byte chunks); each wave DMAs PIECES / 4 pieces + its 64 global
//    bounds (a 4-byte-per-lane DMA) per stage;
//  * fragment reads: one VGPR base per stage, every group's reads through the ds_read offset
//    field (no per-group address arithmetic), FD groups in flight;
//  * the DMA issue of stage s + NST - 1 is spread over the MFMA groups (with no partner wave on
//    the SIMD, an issue slot between MFMAs is the only place to hide it);
//  * the epilogue is QW's: per stage, the max of each query's SR scores against max(local k'-th
//    key, global bound), appends into the wave's own candidate buffers, compaction when full,
//    final lists at the end (topk_kernels.h).
//
// UNIT corpora only (raw dot product = coarse score), no row mask.
#pragma once
#include <utility>

#include "score_qw.h"

namespace hcr {

constexpr int QW1_NW = 4;       // waves per workgroup: one per SIMD

#ifdef HCR_QW1_STAMPS
// Diagnostic build only (Makefile target `stamps_qw1`, tools/qw1_stamps.py): per wave, s_memtime
// cycles summed over the stages: [0] vmcnt wait + barrier, [1] DMA issue + bounds / first
// fragment reads, [2] the MFMA groups, [3] the epilogue, [4] stages.  Never in the product.
__device__ unsigned long long hcr_qw1_stamps[4096 * 8 * 8];
#define HCR_QW1_STAMP(t)                                                               \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");         \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#endif

// f(std::integral_constant<int, I>{}) for I = 0 .. N-1: compile-time indices (asm immediates)
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
  }(std::make_integer_sequence<int, N>{});
}

// D = 1024 (configs[4], bge-large): 3 query blocks of 16 per wave, 16-row stages (32 KiB) in a
// 4-deep ring.  (r03 also built D = 384 / 768 shapes, an 8-wave form and a software-pipelined
// QW1P; none measured faster than QS / QW on those shapes -- profiles/r03/ab_c1_*, ab_c2_* --
// and they were removed in r04.)
template <int KS> struct Qw1Shape;
template <> struct Qw1Shape<32> { static constexpr int QB = 3, SR = 16, NST = 4; };

template <int KS, int QB = Qw1Shape<KS>::QB, int SR_ = Qw1Shape<KS>::SR, int NST_ = Qw1Shape<KS>::NST>
struct Qw1Layout {
  static constexpr int SR = SR_, RB = SR / 16, NST = NST_;
  static constexpr int QPW = 16 * QB, QT = QW1_NW * QPW;    // queries per wave / workgroup
  static constexpr int PIECES = RB * KS;                    // 1 KiB pieces per stage
  static constexpr int PPW = PIECES / QW1_NW;               // ... per wave
  static constexpr int STAGE = PIECES * 1024;
  static constexpr int TGS = NST * STAGE;                   // [NST][NW waves][64 lanes] u32 bounds
  static constexpr int TAU = TGS + NST * QW1_NW * 256;      // u64 tau_key[QT]
  static constexpr int CNT = TAU + QT * 8;                  // int cnt[QT]
  static constexpr int TOTAL = CNT + QT * 4;
  static constexpr int NF = QB * KS;                        // query fragments per wave
  // ... of them in AGPRs: 64 (256 registers) at one wave per SIMD
  static constexpr int FA = NF < 64 ? NF : 64;
  static constexpr int FV = NF - FA;                        // ... in VGPRs
  static_assert(SR > 0 && (RB == 1 || RB % 2 == 0) && PIECES % QW1_NW == 0, "QW1 stage shape");
  static_assert(QPW <= 64, "one 4-byte bound per lane");
  static_assert(STAGE <= 65536, "group offsets in the 16-bit ds_read offset field");
  static_assert(TOTAL <= 160 * 1024, "LDS budget");
};

template <typename TM> struct Qw1Mfma;
template <> struct Qw1Mfma<_Float16> {
  template <bool BA>
  static __device__ __forceinline__ void run(floatx4& acc, const half8& a, const half8& b) {
    if constexpr (BA) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  }
  template <bool BA>
  static __device__ __forceinline__ void first(floatx4& acc, const half8& a, const half8& b) {
    if constexpr (BA) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
  }
};
template <> struct Qw1Mfma<__bf16> {
  template <bool BA>
  static __device__ __forceinline__ void run(floatx4& acc, const bf16x8& a, const bf16x8& b) {
    if constexpr (BA) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
    else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  }
  template <bool BA>
  static __device__ __forceinline__ void first(floatx4& acc, const bf16x8& a, const bf16x8& b) {
    if constexpr (BA) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
    else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
  }
};

// the two A fragments of a group at vbase + OFF and vbase + OFF + OFF2 (byte offsets in the
// ds_read immediate), issued with no wait
template <int OFF, int OFF2, typename V>
__device__ __forceinline__ void qw1_issue_frags(uint32_t vbase, V (&av)[2]) {
  asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4"
               : "=&v"(av[0]), "=&v"(av[1])
               : "v"(vbase), "n"(OFF), "n"(OFF + OFF2)
               : "memory");
}

template <typename TM, int CAP, int KS>
__global__ void __launch_bounds__(QW1_NW * 64, 1)
score_topk_qw1_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows,
                      const TM* __restrict__ qhat, int nqb, int P, int ntiles,
                      uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                      uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp) {
  using L = Qw1Layout<KS>;
  using V = typename MfmaOp<TM>::V;
  using M = Qw1Mfma<TM>;
  constexpr int NW = QW1_NW;
  constexpr int SR = L::SR, RB = L::RB, PPW = L::PPW, QT = L::QT, QPW = L::QPW, NST = L::NST;
  constexpr int QB = QPW / 16, D = NST - 1, FA = L::FA, FV = L::FV;
  constexpr int OPS = PPW + 1;                        // vmcnt-counted ops per wave per stage
  // fragment groups per stage (of the wave's RB row blocks): (row-block pair, k-step), or
  // (row block, k-step pair) if RB = 1
  constexpr int NG = RB == 1 ? KS / 2 : (RB / 2) * KS;
  constexpr int OFF2 = (RB == 1 ? 1 : KS) * 1024;
  constexpr int FD = 3;                               // fragment groups in flight
  static_assert(CAP >= 128 && CAP % 64 == 0, "candidate buffer");
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
  const int wq0 = wave * QPW;                         // this wave's first query (block-local)

  if (lane < QPW) { tau_key[wq0 + lane] = 0ull; cnt[wq0 + lane] = 0; }
  if (t0 >= t1) {
    if (lane < QPW) pcnt[(size_t)(qbase + wq0 + lane) * P + p] = 0;
    return;
  }

  // query fragments: fragment f = n KS + ks, lane l holds q^[wq0 + 16 n + (l & 15)][ks 32 +
  // 8 (l >> 4) .. +8); f < FA in AGPRs, the rest in VGPRs (asm loads: never copied)
  V qa[FA];
  V qv[FV > 0 ? FV : 1];
  {
    const TM* src0 = qhat + (size_t)(qbase + wq0 + (lane & 15)) * ld + (lane >> 4) * 8;
#pragma unroll
    for (int f = 0; f < L::NF; ++f) {
      const TM* src = src0 + (size_t)(f / KS) * 16 * ld + (f % KS) * 32;
      if (f < FA) asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(qa[f]) : "v"(src) : "memory");
      else asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qv[f - FA]) : "v"(src) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int f = 0; f < FA; ++f) asm volatile("" : "+a"(qa[f]));
#pragma unroll
    for (int f = 0; f < FV; ++f) asm volatile("" : "+v"(qv[f]));
  }

  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int ldb = ld * 2;
  const int voff = drow * ldb + dchunk * 16;
  const char* rows_b = reinterpret_cast<const char*>(rows);

  const int nsteps = t1 - t0;
  // Stage i (tile t0 + i) goes to ring slot i % NST: this wave's PPW row pieces (piece j =
  // wave + NW u: row block j / KS, k-step j % KS) and its global bounds -- OPS ops.  Stages past
  // the partition's end are issued through zero-record descriptors (nothing is read; their LDS
  // writes land in a slot already consumed), so the loop has no tail cases.
  struct StageDesc { __amdgpu_buffer_rsrc_t a, t; int slot; };
  auto stage_desc = [&](int i) __attribute__((always_inline)) {
    const bool live = i < nsteps;
    StageDesc d;
    d.slot = __builtin_amdgcn_readfirstlane(i % NST);
    const int tile = __builtin_amdgcn_readfirstlane(t0 + (live ? i : 0));
    d.a = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(rows_b + (size_t)tile * SR * ldb), (short)0,
                                            live ? SR * ldb : 0, 0x00020000);
    d.t = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(tau_g + qbase), (short)0, live ? QT * 4 : 0,
                                            0x00020000);
    return d;
  };
  auto issue_op = [&](const StageDesc& d, int u) __attribute__((always_inline)) {
    if (u < PPW) {
      const int j = wave + NW * u;
      dma16(d.a, lds + d.slot * L::STAGE + j * 1024, voff, (j / KS) * 16 * ldb + (j % KS) * (V3_BK * 2));
    } else {
      int tv;   // the lane's byte offset, opaque (a hoisted copy would be spilled)
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\t"
                   "v_lshlrev_b32 %0, 2, %0" : "=v"(tv));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          d.t, (__attribute__((address_space(3))) void*)(lds + L::TGS + (d.slot * NW + wave) * 256),
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
  // candidate counts of the lane's QB queries, the same in a query's 4 lanes (a query belongs to
  // one wave: appends take their slots from the wave's ballot); LDS cnt[] is written for a
  // compaction and the final lists
  int cq[QB];
#pragma unroll
  for (int n = 0; n < QB; ++n) cq[n] = 0;
  uint64_t tkr[QB];
#pragma unroll
  for (int n = 0; n < QB; ++n) tkr[n] = 0ull;
#ifdef HCR_QW1_STAMPS
  uint64_t st_t0, st_t1, st_t2, st_t3, st_t4, st_acc[4] = {0, 0, 0, 0};
#endif
  for (int s = 0; s < nsteps; ++s) {
#ifdef HCR_QW1_STAMPS
    HCR_QW1_STAMP(st_t0);
#endif
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS * (D - 1)) : "memory");
    v3_barrier();                  // everyone's pieces of stage s; everyone done with slot s-1
#ifdef HCR_QW1_STAMPS
    HCR_QW1_STAMP(st_t1);
#endif
    const StageDesc nd = stage_desc(s + D);   // issued spread over the MFMA groups below

    const int slot = s % NST;
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)(slot * L::STAGE)));
    uint32_t vbase;
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(vbase) : "s"(st), "v"(offA));
    // this stage's global bounds of the lane's QB queries: read now, waited for with the last
    // fragment group
    uint32_t tg[QB];
    {
      int le0;
      asm volatile("v_mov_b32 %0, %1" : "=v"(le0) : "v"(lane));
      const uint32_t ta = lds_addr(lds + L::TGS + (slot * NW + wave) * 256 + (le0 & 15) * 4);
      static_for<QB>([&](auto nc) {
        constexpr int N = decltype(nc)::value;
        uint32_t& t = tg[N];       // (named outside the asm: operands alone do not capture)
        const uint32_t a = ta;
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=&v"(t) : "v"(a), "n"(N * 64) : "memory");
      });
    }
#ifdef HCR_QW1_STAMPS
    HCR_QW1_STAMP(st_t2);
#endif
    floatx4 acc[RB][QB];
    V av[FD][2];
    // group J: row blocks (2 (J / KS), +1) at k-step J % KS (RB >= 2), or row block 0 at
    // k-steps 2 J, 2 J + 1 (RB = 1); its two A fragments at these stage offsets
    auto goff = [](int j) constexpr { return (RB == 1 ? 2 * j : 2 * (j / KS) * KS + j % KS) * 1024; };
    auto mma = [&](auto fc, auto firstc, floatx4& c, const V& a) __attribute__((always_inline)) {
      constexpr int F = decltype(fc)::value;
      if constexpr (decltype(firstc)::value) {
        if constexpr (F < FA) M::template first<true>(c, a, qa[F]);
        else M::template first<false>(c, a, qv[F - FA]);
      } else {
        if constexpr (F < FA) M::template run<true>(c, a, qa[F]);
        else M::template run<false>(c, a, qv[F - FA]);
      }
    };
    static_for<FD - 1>([&](auto jc) {
      constexpr int J = decltype(jc)::value;
      if constexpr (J < NG) qw1_issue_frags<goff(J), OFF2, V>(vbase, av[J]);
    });
    static_for<NG>([&](auto jc) {
      constexpr int J = decltype(jc)::value;
      if constexpr (J + FD - 1 < NG) {
        qw1_issue_frags<goff(J + FD - 1), OFF2, V>(vbase, av[(J + FD - 1) % FD]);
        qw_frag_wait<2 * (FD - 1)>(av[J % FD]);
      } else if constexpr (J + 1 < NG) {
        qw_frag_wait<2>(av[J % FD]);
      } else {
        qw_frag_wait<0>(av[J % FD]);
#pragma unroll
        for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(tg[n]));   // (read before: landed)
      }
      // the next stage's DMA issue spread over the MFMA groups: with no partner wave on the
      // SIMD, an issue slot between MFMAs is the only place to hide it
      static_for<OPS>([&](auto uc) {
        constexpr int U = decltype(uc)::value;
        if constexpr (U * NG / OPS == J) issue_op(nd, U);
      });
      if constexpr (RB == 1) {
        static_for<2>([&](auto kc) {
          constexpr int KK = decltype(kc)::value;
          static_for<QB>([&](auto nc) {
            constexpr int N = decltype(nc)::value;
            mma(std::integral_constant<int, N * KS + 2 * J + KK>{},
                std::integral_constant<bool, J == 0 && KK == 0>{}, acc[0][N], av[J % FD][KK]);
          });
        });
      } else {
        constexpr int M0 = 2 * (J / KS), K0 = J % KS;
        static_for<2>([&](auto mc) {
          constexpr int MM = decltype(mc)::value;
          static_for<QB>([&](auto nc) {
            constexpr int N = decltype(nc)::value;
            mma(std::integral_constant<int, N * KS + K0>{}, std::integral_constant<bool, K0 == 0>{},
                acc[M0 + MM][N], av[J % FD][MM]);
          });
        });
      }
    });
#ifdef HCR_QW1_STAMPS
    HCR_QW1_STAMP(st_t3);
#endif
    // MFMA results -> VALU readers: the XDL write-back wait states the compiler does not see
    // (the MFMAs are asm), with every accumulator named so nothing reads one earlier
#pragma unroll
    for (int m = 0; m < RB; ++m)
#pragma unroll
      for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(acc[m][n]));
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
    for (int m = 0; m < RB; ++m)
#pragma unroll
      for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(acc[m][n]));

    // ---- epilogue of tile t0 + s: this wave's QPW queries x SR rows ----
    int le;
    asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
    const int lq = le >> 4;
    const int qle = wq0 + (le & 15);                 // the query of accumulator block 0
    const int64_t row0 = (int64_t)(t0 + s) * SR;    // the tile's first row
    if (row0 + RB * 16 > n_rows) { // the corpus' last tile: rows past the end never pass (NaN)
#pragma unroll
      for (int m = 0; m < RB; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row0 + m * 16 + lq * 4 + r >= n_rows)
#pragma unroll
            for (int n = 0; n < QB; ++n) acc[m][n][r] = __builtin_nanf("");
    }
    bool hit[QB];
    bool any_hit = false;
#pragma unroll
    for (int n = 0; n < QB; ++n) {
      float mx = qw_max4(acc[0][n]);
#pragma unroll
      for (int m = 1; m < RB; ++m) mx = qw_max3(mx, qw_max3(acc[m][n][0], acc[m][n][1], acc[m][n][2]), acc[m][n][3]);
      const uint32_t tk = max((uint32_t)(tkr[n] >> 32), tg[n]);
      hit[n] = qw_ord32(mx) >= tk;       // (a NaN maximum passes here; its scores fail below)
      any_hit |= hit[n];
    }
    if (__any(any_hit)) {
      float thr[QB];
#pragma unroll
      for (int n = 0; n < QB; ++n) thr[n] = unord32(max((uint32_t)(tkr[n] >> 32), tg[n]));
      const uint32_t row0u = (uint32_t)row0;
#pragma unroll
      for (int n = 0; n < QB; ++n) {
        if (!__any(hit[n])) continue;
#pragma unroll
        for (int m = 0; m < RB; ++m) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sc = acc[m][n][r];
            const bool c = sc >= thr[n];
            if (__builtin_amdgcn_ballot_w64(c)) {
              // the slot from the wave's ballot (QW's r05 form: no LDS counter round trip)
              const uint64_t key = make_key(sc, row0u + (uint32_t)(m * 16 + lq * 4 + r));
              const bool a = c && key > tkr[n];
              const uint64_t ba = __builtin_amdgcn_ballot_w64(a);
              if (ba) {
                const uint64_t t = ba >> (le & 15);
                const uint32_t nib = (uint32_t)(t & 1u) | (uint32_t)((t >> 15) & 2u) |
                                     (uint32_t)((t >> 30) & 4u) | (uint32_t)((t >> 45) & 8u);
                if (a) wbuf[(size_t)(qle + 16 * n) * CAP + cq[n] + __popc(nib & ((1u << lq) - 1u))] = key;
                cq[n] += __popc(nib);
              }
            }
          }
        }
        need |= cq[n] > CAP - SR;
      }
      // a query whose buffer cannot take another tile's appends is compacted to its best k'
      // (rare: drains this wave's stores and, in order, its ring pieces)
      if (__any(need)) {
#pragma unroll
        for (int n = 0; n < QB; ++n)
          if (le < 16) cnt[qle + 16 * n] = cq[n];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
        for (int ql = wq0; ql < wq0 + QPW; ++ql) {
          if ((int)v3_lds_u32(cnt + ql) > CAP - SR)
            compact_query<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                               tau_g + qbase + ql, kp, lane, nullptr);
        }
        need = false;
#pragma unroll
        for (int n = 0; n < QB; ++n) {
          tkr[n] = v3_lds_u64(tau_key + qle + 16 * n);
          cq[n] = (int)v3_lds_u32(cnt + qle + 16 * n);
        }
      }
    }
#ifdef HCR_QW1_STAMPS
    HCR_QW1_STAMP(st_t4);
    st_acc[0] += st_t1 - st_t0;
    st_acc[1] += st_t2 - st_t1;
    st_acc[2] += st_t3 - st_t2;
    st_acc[3] += st_t4 - st_t3;
#endif
  }
#ifdef HCR_QW1_STAMPS
  if (lane == 0 && b < 4096) {
    unsigned long long* o = hcr_qw1_stamps + ((size_t)b * 8 + wave) * 8;
    o[0] = st_acc[0]; o[1] = st_acc[1]; o[2] = st_acc[2]; o[3] = st_acc[3]; o[4] = nsteps;
  }
#endif

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int n = 0; n < QB; ++n)
    if (lane < 16) cnt[wq0 + lane + 16 * n] = cq[n];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  final_lists_wave<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wq0, 1, QPW, kp, lane, partials, pcnt, P, p);
}

}  // namespace hcr
