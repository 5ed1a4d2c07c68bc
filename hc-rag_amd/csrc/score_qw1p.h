// score_qw1p.h — QW1P: the one-wave-per-SIMD query-stationary kernel (score_qw1.h) with its
// stage loop software-pipelined, for MFMA-bound large batches.
//
// At one wave per SIMD nothing hides what the wave does between its MFMAs: in QW1 the stamps
// build (tools/qw1_stamps.py) splits a stage into the barrier wait, the DMA issue + the first
// fragment reads after the barrier, the MFMA groups and the epilogue, all serial.  QW1P
//  * double-buffers the accumulators (stages alternate between two sets, the loop is unrolled
//    by two) and spreads the epilogue of stage s - 1 over the first MFMA groups of stage s:
//    group j < QB computes query block j's maximum, group E the thresholds and the (rare)
//    append branch, each piece pinned between two groups' MFMAs by opaque asm operands;
//  * moves the stage barrier from the top of stage s to just before its last FD - 1 groups:
//    after it the wave issues the next stage's DMA and the next stage's first fragment reads,
//    whose LDS latency then hides behind stage s's last groups.  The barrier still guarantees
//    what the ring needs: every wave's pieces of stage s + 1 have landed (each wave's counted
//    vmcnt before it) and every wave is done reading stage s - 1, whose slot the DMA of stage
//    s + NST - 1 now refills;
//  * keeps QW1's data layout, query fragments (AGPRs + VGPRs), candidate buffers, epilogue
//    arithmetic and final lists, so its results are the same keys.
// Stage s + 1's data is needed at stage s's barrier, so the ring keeps NST - 2 stages in
// flight: 16-row stages in a 6-deep ring at D = 768 (4 stages of prefetch).
#pragma once
#include "score_qw1.h"

namespace hcr {

template <typename TM, int CAP, int KS, int SR_, int NST_, int FD>
__global__ void __launch_bounds__(QW1_NW * 64, 1)
score_topk_qw1p_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows,
                       const TM* __restrict__ qhat, int nqb, int P, int ntiles,
                       uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                       uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp) {
  using L = Qw1Layout<KS, QW1_NW, Qw1Shape<KS>::QB, SR_, NST_>;
  using V = typename MfmaOp<TM>::V;
  using M = Qw1Mfma<TM>;
  constexpr int SR = L::SR, RB = L::RB, PPW = L::PPW, QT = L::QT, QPW = L::QPW, NST = L::NST;
  constexpr int QB = QPW / 16, D = NST - 1, FA = L::FA, FV = L::FV;
  constexpr int OPS = PPW + 1;                        // vmcnt-counted ops per wave per stage
  constexpr int NG = RB == 1 ? KS / 2 : (RB / 2) * KS;
  constexpr int OFF2 = (RB == 1 ? 1 : KS) * 1024;
  constexpr int JB = NG - (FD - 1);                   // the group the barrier precedes
  constexpr int JE = QB > FD - 1 ? QB : FD - 1;       // the group of the thresholds + appends
  static_assert(D >= 2, "stage s + 1 must be in flight at stage s's barrier");
  static_assert(JE < JB, "the previous stage's epilogue fits before the barrier");
  // group J reads into av[J % FD], the next stage's group j into av[(NG + j) % FD]: the same
  // buffer only when FD divides NG (D = 1024: NG = 16, FD = 4)
  static_assert(NG % FD == 0, "fragment buffers must line up across stages");
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
  const int wq0 = wave * QPW;

  if (lane < QPW) { tau_key[wq0 + lane] = 0ull; cnt[wq0 + lane] = 0; }
  if (t0 >= t1) {
    if (lane < QPW) pcnt[(size_t)(qbase + wq0 + lane) * P + p] = 0;
    return;
  }

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
  auto issue_stage = [&](int i) __attribute__((always_inline)) {
    const StageDesc d = stage_desc(i);
#pragma unroll
    for (int u = 0; u < OPS; ++u) {
      if (u < PPW) {
        const int j = wave + QW1_NW * u;
        dma16(d.a, lds + d.slot * L::STAGE + j * 1024, voff, (j / KS) * 16 * ldb + (j % KS) * (V3_BK * 2));
      } else {
        int tv;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\t"
                     "v_lshlrev_b32 %0, 2, %0" : "=v"(tv));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            d.t, (__attribute__((address_space(3))) void*)(lds + L::TGS + (d.slot * QW1_NW + wave) * 256),
            4, tv, wq0 * 4, 0, 0);
      }
    }
  };

  const uint32_t offA = (uint32_t)((lane & 15) * 64 + v3_slot(lane >> 4, lane & 15) * 16);
  const uint32_t lds0 = lds_addr(lds);
  auto stage_vbase = [&](int i) __attribute__((always_inline)) {
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)((i % NST) * L::STAGE)));
    uint32_t v;
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(v) : "s"(st), "v"(offA));
    return v;
  };
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

  // ---- prologue: stages 0 .. D-1 in flight, stage 0 landed, its first FD-1 groups read ----
  for (int i = 0; i < D; ++i) issue_stage(i);
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS * (D - 1)) : "memory");
  v3_barrier();
  V av[FD][2];
  uint32_t vcur = stage_vbase(0);
  static_for<FD - 1>([&](auto jc) {
    constexpr int J = decltype(jc)::value;
    qw1_issue_frags<goff(J), OFF2, V>(vcur, av[J]);
  });

  bool need = false;
  uint64_t tkr[QB];
#pragma unroll
  for (int n = 0; n < QB; ++n) tkr[n] = 0ull;
  floatx4 accA[RB][QB], accB[RB][QB];
#pragma unroll
  for (int m = 0; m < RB; ++m)
#pragma unroll
    for (int n = 0; n < QB; ++n) accA[m][n] = accB[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  int le;
  asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
  const int lq = le >> 4;
  const int qle = wq0 + (le & 15);

  // The epilogue of a finished stage's accumulators (rows row0 .. row0 + SR): NaN for rows past
  // the corpus, max per query block against max(local k'-th key, global bound), appends.
  auto tail_mask = [&](floatx4 (&acc)[RB][QB], int64_t row0) __attribute__((always_inline)) {
    if (row0 + SR > n_rows) {
#pragma unroll
      for (int m = 0; m < RB; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row0 + m * 16 + lq * 4 + r >= n_rows)
#pragma unroll
            for (int n = 0; n < QB; ++n) acc[m][n][r] = __builtin_nanf("");
    }
  };
  auto block_max = [&](const floatx4 (&acc)[RB][QB], int n) __attribute__((always_inline)) {
    float mx = qw_max4(acc[0][n]);
#pragma unroll
    for (int m = 1; m < RB; ++m) mx = qw_max3(mx, qw_max3(acc[m][n][0], acc[m][n][1], acc[m][n][2]), acc[m][n][3]);
    return mx;
  };
  auto appends = [&](const floatx4 (&acc)[RB][QB], const float (&mx)[QB], const uint32_t (&tg)[QB],
                     int64_t row0) __attribute__((always_inline)) {
    bool hit[QB];
    bool any_hit = false;
#pragma unroll
    for (int n = 0; n < QB; ++n) {
      hit[n] = qw_ord32(mx[n]) >= max((uint32_t)(tkr[n] >> 32), tg[n]);   // (NaN: fails below)
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
              if (c) {
                const uint64_t key = make_key(sc, row0u + (uint32_t)(m * 16 + lq * 4 + r));
                if (key > tkr[n]) {
                  const int ql = qle + 16 * n;
                  const int pos = v3_lds_add_rtn(&cnt[ql], 1);
                  wbuf[(size_t)ql * CAP + pos] = key;
                  need |= pos + 1 > CAP - SR;
                }
              }
            }
          }
        }
      }
      if (__any(need)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll 1
        for (int ql = wq0; ql < wq0 + QPW; ++ql) {
          if ((int)v3_lds_u32(cnt + ql) > CAP - SR)    // (inline: a call spills the pipeline's registers)
            compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                                   tau_g + qbase + ql, kp, lane, nullptr);
        }
        need = false;
#pragma unroll
        for (int n = 0; n < QB; ++n) tkr[n] = v3_lds_u64(tau_key + qle + 16 * n);
      }
    }
  };
  auto read_bounds = [&](int i, uint32_t (&tg)[QB]) __attribute__((always_inline)) {
    int le0;
    asm volatile("v_mov_b32 %0, %1" : "=v"(le0) : "v"(lane));
    const uint32_t ta = lds_addr(lds + L::TGS + ((i % NST) * QW1_NW + wave) * 256 + (le0 & 15) * 4);
    static_for<QB>([&](auto nc) {
      constexpr int N = decltype(nc)::value;
      uint32_t& t = tg[N];
      const uint32_t a = ta;
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=&v"(t) : "v"(a), "n"(N * 64) : "memory");
    });
  };

  // ---- one stage: MFMAs of stage s into `acc`, the epilogue of stage s - 1 (`accp`) in its
  // first groups, the barrier and the next stage's DMA + first reads before its last groups ----
  auto stage = [&](floatx4 (&acc)[RB][QB], floatx4 (&accp)[RB][QB], int s) __attribute__((always_inline)) {
    const bool has_prev = s > 0;
    const int64_t row0p = (int64_t)(t0 + s - 1) * SR;
    uint32_t tgp[QB];
    read_bounds(s + NST - 1, tgp);          // the bounds of stage s - 1 (slot (s - 1) % NST)
    float mx[QB];
    uint32_t vnext = 0;
    // the MFMA results of stage s - 1 -> VALU readers: XDL write-back wait states
#pragma unroll
    for (int m = 0; m < RB; ++m)
#pragma unroll
      for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(accp[m][n]));
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
    for (int m = 0; m < RB; ++m)
#pragma unroll
      for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(accp[m][n]));
    if (has_prev) tail_mask(accp, row0p);
    static_for<NG>([&](auto jc) {
      constexpr int J = decltype(jc)::value;
      if constexpr (J == JB) {
        // stage s + 1 landed (everyone's), everyone done with stage s - 1's slot
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS * (D - 2)) : "memory");
        v3_barrier();
        issue_stage(s + D);
        vnext = stage_vbase(s + 1);
      }
      constexpr int JN = J + FD - 1;
      if constexpr (JN < NG) qw1_issue_frags<goff(JN), OFF2, V>(vcur, av[JN % FD]);
      else qw1_issue_frags<goff(JN - NG), OFF2, V>(vnext, av[JN % FD]);   // (= av[(JN - NG) % FD])
      // LDS reads complete in order: the bounds (issued before group FD-1's fragments) are
      // younger than groups 0 .. FD-2
      if constexpr (J < FD - 1) qw_frag_wait<2 * (FD - 1) + QB>(av[J % FD]);
      else qw_frag_wait<2 * (FD - 1)>(av[J % FD]);
      if constexpr (J == FD - 1) {
#pragma unroll
        for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(tgp[n]));   // landed
      }
      // epilogue piece of stage s - 1
      if constexpr (J < QB) {
#pragma unroll
        for (int m = 0; m < RB; ++m) asm volatile("" : "+v"(accp[m][J]));
        mx[J] = block_max(accp, J);
        asm volatile("" : "+v"(mx[J]));
      }
      if constexpr (J == JE) {
        if (has_prev) appends(accp, mx, tgp, row0p);
      }
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
    vcur = vnext;
  };

  int s = 0;
  for (; s + 1 < nsteps; s += 2) {
    stage(accA, accB, s);
    stage(accB, accA, s + 1);
  }
  // the last stage's epilogue, after its MFMAs (no next stage to hide it in)
  auto drain = [&](floatx4 (&acc)[RB][QB], int sl) __attribute__((always_inline)) {
    // the last stage read its (nonexistent) successor's first groups: an inline-asm read the
    // compiler sees no use of frees its VGPRs while the LDS return is pending, so wait for them
    // with the registers still held (the drain's first registers were overwritten without it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int f = 0; f < FD; ++f) asm volatile("" : "+v"(av[f][0]), "+v"(av[f][1]));
#pragma unroll
    for (int m = 0; m < RB; ++m)
#pragma unroll
      for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(acc[m][n]));
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
    for (int m = 0; m < RB; ++m)
#pragma unroll
      for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(acc[m][n]));
    const int64_t row0 = (int64_t)(t0 + sl) * SR;
    uint32_t tg[QB];
    read_bounds(sl, tg);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int n = 0; n < QB; ++n) asm volatile("" : "+v"(tg[n]));
    tail_mask(acc, row0);
    float mx[QB];
#pragma unroll
    for (int n = 0; n < QB; ++n) mx[n] = block_max(acc, n);
    appends(acc, mx, tg, row0);
  };
  if (s < nsteps) {                 // odd count: stage nsteps - 1 on set A, stage nsteps - 2's
    stage(accA, accB, s);           // epilogue inside it; then stage nsteps - 1's
    drain(accA, s);
  } else {
    drain(accB, nsteps - 1);
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  final_lists<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wq0, 1, wq0 + QPW, kp, lane, partials, pcnt, P, p);
}

}  // namespace hcr
