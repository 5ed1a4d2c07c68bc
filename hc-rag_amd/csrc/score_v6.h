// score_v6.h — K2 v6: v4 with the two halves of the workgroup staggered by half a step.
//
// v4's 8 waves run in lockstep: after every stage barrier all of them read their fragments
// (12 x ds_read_b128 each, 96 KiB per CU) and only then issue MFMAs, so the LDS read burst
// and the matrix pipes alternate instead of overlapping (r01d stamps: 35 % of the wave cycles
// between the barrier and the last fragment).  v6 keeps v4's ring, tiles, pieces and epilogue
// but splits the roles of the two waves that share a SIMD (waves w and w + 4):
//   group A (waves 0-3): [epilogue] read fragments of step i, MFMAs of step i   | barrier
//   group B (waves 4-7): MFMAs of step i-1 (fragments read before the barrier),
//                        [epilogue], read fragments of step i                   | barrier
// so in every interval one wave of each SIMD reads while its partner multiplies, and the two
// tile epilogues of a SIMD fall beside the partner's MFMAs.  B's fragments live across the
// barrier (no extra registers: it reads them after its MFMAs).  Ring protocol (NST = D + 1):
// A issues stage i + D during MFMA(i) into the slot of stage i - 1, which both groups have
// read before barrier i; B issues the same stage i + D during its MFMA(i - 1) (B's interval 0
// issues stage D alone), so both wait for stage i + 1 with D - 1 later stages in flight.
// MI355X_MICROARCH.md, "Two waves per SIMD", item 9 (stagger by wave number >= 4).
//
// Same contract as score_topk_v3_kernel (score_v3.h).  Built from the r01 measurements of v3
// at 10M x 768, B = 1024 (tests/debug/v3_ablate.hip, profiles/r01/): an L2-resident corpus
// ran no faster (not HBM-bound); per wave-step 38 % of the cycles went to ISSUING the LDS-DMA
// pieces (all 8 waves push their pieces right after the barrier, so the CU's fill path
// serialises them and no MFMA overlaps), and the per-tile epilogue cost ~8 ms even with a
// perfect bound (16 dependent LDS round trips per tile, each behind the DMA traffic).  v4:
//
//  * 256 x 256 tiles, K = 32 per stage: 16 row pieces + 16 query pieces = exactly 4 per wave,
//    with a fixed kind per slot (no branches in the issue);
//  * the 4 pieces of stage s + NST - 1 are interleaved between the MFMA groups of stage s
//    (sched_group_barrier), tail stages go through a zero-record descriptor into a slot that
//    is already consumed, so the step is one basic block;
//  * issue coordinates advance incrementally (no per-step division);
//  * per-tile inverse norms / global bounds / mask words are read in ONE asm block with one
//    wait; the candidate-buffer bookkeeping (tau_key / cnt / flag) lives in __shared__ arrays
//    separate from the DMA ring, so the compiler can see that it does not alias the DMA.
#pragma once
#include <type_traits>

#include "score_v4.h"

namespace hcr {



// UNIT: the coarse score is the raw dot product q^.e (L2-normalised corpora; the host widens
// eps_q by the rows' deviation from unit norm).  The epilogue of a tile with
// neither masked nor out-of-range rows is then a max + compare on the accumulators.
template <typename TM, int CAP, int NST, bool UNIT = false>
__global__ void __launch_bounds__(V3_NT, 2)
score_topk_v6_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows, int ksteps,
                     const float* __restrict__ inv_norm, const uint32_t* __restrict__ mask,
                     const TM* __restrict__ qhat, int nqb, int P, int ntiles, int tstride,
                     uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                     uint64_t* __restrict__ partials, int kp) {
  using L = V4Layout<NST>;
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int RT = V4_RT, QT = V4_QT, WN = 4;
  constexpr int MT = 8, NQ = 4;          // 16x16 MFMA blocks per wave: 128 rows x 64 queries
  constexpr int NA = RT / 16;            // row pieces per stage (16); query pieces too
  constexpr int D = NST - 1;
  __shared__ __attribute__((aligned(16))) char ring[L::TOTAL];
  __shared__ uint64_t tau_key[QT];
  __shared__ int cnt[QT];
  __shared__ int flag[2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int qb = g % nqb, p = g / nqb;
  const int t0 = (int)((int64_t)p * ntiles / P);
  const int t1 = (int)((int64_t)(p + 1) * ntiles / P);
  const int qbase = qb * QT;
  uint64_t* wbuf = buf + (size_t)b * QT * CAP;

  for (int i = tid; i < QT; i += V3_NT) { tau_key[i] = 0ull; cnt[i] = 0; }
  if (tid == 0) { flag[0] = 0; flag[1] = 0; }

  if (t0 >= t1) {
    for (int i = tid; i < QT * kp; i += V3_NT) {
      const int ql = i / kp, j = i - ql * kp;
      partials[((size_t)(qbase + ql) * P + p) * kp + j] = 0ull;
    }
    return;
  }

  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int ldb = ld * 2;
  const int voff = drow * ldb + dchunk * 16;
  const char* rows_b = reinterpret_cast<const char*>(rows);
  const char* q_b = reinterpret_cast<const char*>(qhat) + (size_t)qbase * ldb;
  const __amdgpu_buffer_rsrc_t inv_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(inv_norm), (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t tg_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(tau_g + qbase), (short)0, QT * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t msk_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(mask), (short)0, 0x7FFFFFFF, 0x00020000);

  const int nsteps = (t1 - t0) * ksteps;
  // issue cursor: the next stage to issue (global step index, virtual tile, k-step, ring slot)
  int is_s = 0, is_vt = t0, is_ks = 0, is_slot = 0;

  // the tile-slot pieces of a stage that starts a tile (once per tile; uniform branch)
  auto issue_tile_slot = [&](int vt) {
    const int tile = vt * tstride;
    const int slot = vt % L::NIS;
    if (wave == 7) dma16(inv_rsrc, ring + L::INV + slot * 1024, lane * 16, tile * (RT * 4));
    if (wave == 5) dma16(tg_rsrc, ring + L::TG + slot * 1024, lane * 16, 0);
    if (wave == 6 && mask) {
      if (lane < RT / 32)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            msk_rsrc, (__attribute__((address_space(3))) void*)(ring + L::MSK + slot * 64), 4,
            lane * 4, tile * (RT / 8), 0, 0);
    }
  };
  // descriptors of the stage at the cursor (zero records past the end: the loads are dropped
  // and their LDS writes land in a slot that is no longer read)
  struct Desc { __amdgpu_buffer_rsrc_t a, q; int kofs; char* sa; };
  auto cursor_desc = [&]() {
    const bool live = is_s < nsteps;
    const int tile = __builtin_amdgcn_readfirstlane(is_vt * tstride);
    Desc d;
    d.a = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(rows_b + (size_t)tile * RT * ldb), (short)0,
                                            live ? RT * ldb : 0, 0x00020000);
    d.q = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(q_b), (short)0, live ? QT * ldb : 0,
                                            0x00020000);
    d.kofs = __builtin_amdgcn_readfirstlane(is_ks * (V3_BK * 2));
    d.sa = ring + __builtin_amdgcn_readfirstlane(is_slot) * L::STAGE;
    return d;
  };
  // piece i (0..3) of this wave: i < 2 -> row group wave + 8i, else query group wave + 8(i-2)
  auto issue_piece = [&](const Desc& d, int i) {
    if (i < 2) {
      const int j = wave + 8 * i;
      dma16(d.a, d.sa + j * 1024, voff, j * 16 * ldb + d.kofs);
    } else {
      const int j = wave + 8 * (i - 2);
      dma16(d.q, d.sa + L::A_BYTES + j * 1024, voff, j * 16 * ldb + d.kofs);
    }
  };
  auto advance_cursor = [&]() {
    ++is_s;
    is_slot = (is_slot + 1 == NST) ? 0 : is_slot + 1;
    if (++is_ks == ksteps) { is_ks = 0; ++is_vt; }
  };

  // prologue: D stages
  for (int i = 0; i < D; ++i) {
    if (is_s < nsteps && is_ks == 0) issue_tile_slot(is_vt);
    const Desc d = cursor_desc();
#pragma unroll
    for (int k = 0; k < 4; ++k) issue_piece(d, k);
    advance_cursor();
  }

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = v3_slot(fc, fr);
  const int offA = (wm * 128 + fr) * 64 + fslot * 16;
  const int offB = L::A_BYTES + (wn * 64 + fr) * 64 + fslot * 16;

  // group B issues one stage more up front (it issues stage i + D one interval late, during
  // MFMA(i - 1)); then stage 0 landed (this wave's pieces), then everyone's
  if (wm == 1) {
    if (is_s < nsteps && is_ks == 0) issue_tile_slot(is_vt);
    const Desc d = cursor_desc();
#pragma unroll
    for (int k = 0; k < 4; ++k) issue_piece(d, k);
    advance_cursor();
    v3_wait_vmcnt(D * 4);
  } else {
    v3_wait_vmcnt((D - 1) * 4);
  }
  v3_barrier();

  // Compaction of the queries whose buffers passed the flag level during the previous interval
  // (flag of that interval's parity); both groups call it at the top of every interval, so
  // the two __syncthreads inside pair up.  Returns true if it ran (callers reload their k'-th).
  auto compaction_check = [&](int i) __attribute__((always_inline)) {
    int* f = flag + ((i + 1) & 1);           // = parity of interval i - 1
    if (i == 0 || !*f) return false;
    __syncthreads();                         // every wave's candidate stores are visible
    for (int ql = wave; ql < QT; ql += V3_NT / 64)
      if (cnt[ql] > CAP - RT)
        compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                               tau_g + qbase + ql, kp, lane, nullptr);
    __syncthreads();
    if (tid == 0) *f = 0;
    return true;
  };

  // Tile epilogue (v4's): scores of tile ep_vt against the bounds, candidates appended.
  auto epilogue = [&](auto& acc, uint64_t (&tkr)[NQ], int ep_vt, int* cur_flag)
      __attribute__((always_inline)) {
#ifdef HCR_V3_NO_EPI
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        if (acc[m][n][0] == 12345.f) cnt[0] = 1;
        acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    return;
#endif
    int le;
    asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
    const int lr = le & 15, lq = le >> 4;
    const int64_t row0 = (int64_t)ep_vt * tstride * RT;
    const int slot = ep_vt % L::NIS;
    V4TileVals tv;
    v4_read_tile_vals(lds_addr(ring + L::INV + slot * 1024 + (wm * 128 + lq * 4) * 4),
                      lds_addr(ring + L::TG + slot * 1024 + (wn * 64 + lr) * 4),
                      lds_addr(ring + L::MSK + slot * 64 + wm * 16), tv);
    const uint32_t mw[4] = {tv.mw.x, tv.mw.y, tv.mw.z, tv.mw.w};
    float thr[NQ];
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      const float ls = tkr[n] ? key_score(tkr[n]) : -INFINITY;
      thr[n] = fmaxf(ls, unord32(tv.tg[n]));
    }
    auto epi = [&](auto plain_c) __attribute__((always_inline)) {
      constexpr bool PLAIN = decltype(plain_c)::value;
      float iv[MT][4];
      if constexpr (!PLAIN) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const float vv[4] = {tv.iv[m].x, tv.iv[m].y, tv.iv[m].z, tv.iv[m].w};
          const int rl = wm * 128 + m * 16 + lq * 4;
          const uint32_t word = mask ? mw[m >> 1] : 0xFFFFFFFFu;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool ok = (row0 + rl + r < n_rows) && ((word >> ((rl + r) & 31)) & 1u);
            iv[m][r] = ok ? (UNIT ? 1.f : vv[r]) : __builtin_nanf("");
          }
        }
      }
      auto score = [&](int m, int n, int r) __attribute__((always_inline)) {
        if constexpr (PLAIN) return acc[m][n][r];
        else return acc[m][n][r] * iv[m][r];
      };
      bool any = false;
      bool hit[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        float mx = -INFINITY;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, score(m, n, r));
        hit[n] = mx >= thr[n];
        any |= hit[n];
      }
      if (__any(any)) {
#pragma unroll
        for (int n = 0; n < NQ; ++n) {
          if (hit[n]) {
            const int ql = wn * 64 + n * 16 + lr;
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float sc = score(m, n, r);
                if (sc >= thr[n]) {
                  const uint32_t rowl = (uint32_t)(row0 + wm * 128 + m * 16 + lq * 4 + r);
                  const uint64_t key = make_key(sc, rowl);
                  if (key > tkr[n]) {
                    const int pos = v3_lds_add_rtn(&cnt[ql], 1);
                    wbuf[(size_t)ql * CAP + pos] = key;
                    if (pos + 1 > CAP - RT) v3_lds_store_u32(cur_flag, 1u);
                  }
                }
              }
          }
        }
      }
    };
    if (UNIT && !mask && row0 + RT <= n_rows) epi(std::true_type{});
    else epi(std::false_type{});
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  };

  // MFMAs of one stage with this wave's 4 DMA pieces of the stage at the cursor between them
  auto mma_step = [&](auto& acc, const V (&av)[MT], const V (&bq)[NQ])
      __attribute__((always_inline)) {
    if (is_ks == 0 && is_s < nsteps) issue_tile_slot(is_vt);
    const Desc d = cursor_desc();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int m = 2 * i; m < 2 * i + 2; ++m)
#pragma unroll
        for (int n = 0; n < NQ; ++n) acc[m][n] = Op::run(av[m], bq[n], acc[m][n]);
      issue_piece(d, i);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NQ, 0);  // 8 MFMAs
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);       // 1 DMA piece
    }
    advance_cursor();
  };

  auto run = [&](auto group_b) __attribute__((always_inline)) {
    constexpr bool GB = decltype(group_b)::value;
    floatx4 acc[MT][NQ];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
    uint64_t tkr[NQ];
#pragma unroll
    for (int n = 0; n < NQ; ++n) tkr[n] = 0ull;
    V av[MT], bq[NQ];                    // group B: fragments carried across the barrier
    int rslot = 0;                       // ring slot of the next stage to read
    int mks = 0, mvt = t0;               // k-step / tile of the next MFMA step
    for (int i = 0; i <= nsteps; ++i) {
      if (compaction_check(i)) {
#pragma unroll
        for (int n = 0; n < NQ; ++n) tkr[n] = tau_key[wn * 64 + n * 16 + (lane & 15)];
      }
      int* cur_flag = flag + (i & 1);
      if constexpr (!GB) {
        // A: epilogue of the tile finished by MFMA(i - 1), then read + MFMA of stage i
        if (i > 0 && mks == 0) epilogue(acc, tkr, mvt - 1, cur_flag);
        if (i == nsteps) break;
        {
          const char* st = ring + rslot * L::STAGE;
          v4_read_frags<V>(lds_addr(st + offA), lds_addr(st + offB), av, bq);
        }
        mma_step(acc, av, bq);
        if (++mks == ksteps) { mks = 0; ++mvt; }
        rslot = (rslot + 1 == NST) ? 0 : rslot + 1;
        v3_wait_vmcnt((D - 1) * 4);
      } else {
        // B: MFMA of stage i - 1 (fragments read last interval) with the pieces of stage
        // i + D (as A: B's prologue issued stage D too), its epilogue, read stage i
        if (i > 0) {
          mma_step(acc, av, bq);
          if (++mks == ksteps) {
            mks = 0;
            ++mvt;
            epilogue(acc, tkr, mvt - 1, cur_flag);
          }
        }
        if (i == nsteps) break;
        {
          const char* st = ring + rslot * L::STAGE;
          v4_read_frags<V>(lds_addr(st + offA), lds_addr(st + offB), av, bq);
        }
        rslot = (rslot + 1 == NST) ? 0 : rslot + 1;
        v3_wait_vmcnt((D - 1) * 4);
      }
      v3_barrier();
    }
  };
  if (wm == 0) run(std::false_type{});
  else run(std::true_type{});

  __syncthreads();
  for (int ql = wave; ql < QT; ql += V3_NT / 64) {
    compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql], tau_g + qbase + ql, kp,
                           lane, partials + ((size_t)(qbase + ql) * P + p) * kp);
  }
}

}  // namespace hcr
