// score_v4.h — K2 v4: the large-batch (MFMA-bound) fused score + top-k' kernel.
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

#include "score_v3.h"

namespace hcr {

constexpr int V4_RT = 256, V4_QT = 256;


template <int NST>
struct V4Layout {
  static constexpr int A_BYTES = V4_RT * 64, B_BYTES = V4_QT * 64;
  static constexpr int STAGE = A_BYTES + B_BYTES;          // 32 KiB
  static constexpr int NIS = 3;                             // tile slots (host: 2*ksteps > NST-1)
  static constexpr int INV = NST * STAGE;                   // NIS x 256 floats
  static constexpr int TG = INV + NIS * 1024;               // NIS x 256 u32 global bounds
  static constexpr int MSK = TG + NIS * 1024;               // NIS x 8 row-mask words (64 B)
  static constexpr int TOTAL = MSK + NIS * 64;
  static_assert(TOTAL + V4_QT * 12 + 16 <= 160 * 1024, "LDS budget");
};

// one wait for the tile-slot reads of an epilogue: 8 x 4 inverse norms, 4 global bounds,
// 4 row-mask words (a b128 of the wave's row half)
struct V4TileVals {
  float4 iv[8];
  uint32_t tg[4];
  uint4 mw;
};
__device__ __forceinline__ void v4_read_tile_vals(uint32_t inv_a, uint32_t tg_a, uint32_t msk_a,
                                                  V4TileVals& o) {
  asm volatile(
      "ds_read_b128 %0, %13\n\t"
      "ds_read_b128 %1, %13 offset:64\n\t"
      "ds_read_b128 %2, %13 offset:128\n\t"
      "ds_read_b128 %3, %13 offset:192\n\t"
      "ds_read_b128 %4, %13 offset:256\n\t"
      "ds_read_b128 %5, %13 offset:320\n\t"
      "ds_read_b128 %6, %13 offset:384\n\t"
      "ds_read_b128 %7, %13 offset:448\n\t"
      "ds_read_b32 %8, %14\n\t"
      "ds_read_b32 %9, %14 offset:64\n\t"
      "ds_read_b32 %10, %14 offset:128\n\t"
      "ds_read_b32 %11, %14 offset:192\n\t"
      "ds_read_b128 %12, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(o.iv[0]), "=&v"(o.iv[1]), "=&v"(o.iv[2]), "=&v"(o.iv[3]), "=&v"(o.iv[4]),
        "=&v"(o.iv[5]), "=&v"(o.iv[6]), "=&v"(o.iv[7]), "=&v"(o.tg[0]), "=&v"(o.tg[1]),
        "=&v"(o.tg[2]), "=&v"(o.tg[3]), "=&v"(o.mw)
      : "v"(inv_a), "v"(tg_a), "v"(msk_a)
      : "memory");
}

// UNIT: the coarse score is the raw dot product q^.e (L2-normalised corpora; the host widens
// eps_q by the rows' deviation from unit norm).  The epilogue of a tile with
// neither masked nor out-of-range rows is then a max + compare on the accumulators.
// MAXONLY: the sampling pre-pass form.  No candidates: for every 128-row half tile ("unit")
// and query the largest coarse score goes to ((float*)buf)[(vt * 2 + wm) * nqpad + q]
// (nqpad = nqb * 256); partials / tau_g are not touched.  The seed kernel then takes the j-th
// largest unit maximum per query: j distinct rows at or above it.
template <typename TM, int CAP, int NST, bool UNIT = false, bool MAXONLY = false>
__global__ void __launch_bounds__(V3_NT, 2)
score_topk_v4_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows, int ksteps,
                     const float* __restrict__ inv_norm, const uint32_t* __restrict__ mask,
                     const TM* __restrict__ qhat, int nqb, int P, int ntiles, int tstride,
                     uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                     uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp) {
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

  if (t0 >= t1) {              // an empty partition: empty lists
    if constexpr (!MAXONLY)
      for (int i = tid; i < QT; i += V3_NT) pcnt[(size_t)(qbase + i) * P + p] = 0;
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

  floatx4 acc[MT][NQ];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  uint64_t tkr[NQ];                      // this lane's queries' local k'-th keys (LDS copy)
#pragma unroll
  for (int n = 0; n < NQ; ++n) tkr[n] = 0ull;

  int rslot = 0;                         // ring slot of the stage being consumed
  int ks = 0, vt = t0;
  int ep_vt = -1;                        // virtual tile whose epilogue is pending
  for (int s = 0; s <= nsteps; ++s) {
    // 1) epilogue of the tile finished by step s-1
    if (ep_vt >= 0) {
      int* prev_flag = flag + ((ep_vt + 1) & 1);
      if (*prev_flag) {                  // set >= 1 barrier ago; uniform across the block
        __syncthreads();                 // other waves' candidate stores (global) are visible
        for (int ql = wave; ql < QT; ql += V3_NT / 64) {
          if (cnt[ql] > CAP - RT)
            compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                                   tau_g + qbase + ql, kp, lane, nullptr);
        }
        __syncthreads();
        if (tid == 0) *prev_flag = 0;
#pragma unroll
        for (int n = 0; n < NQ; ++n) tkr[n] = tau_key[wn * 64 + n * 16 + (lane & 15)];
      }
      int* cur_flag = flag + (ep_vt & 1);
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
      // PLAIN (UNIT, no row mask, tile inside the corpus): scores are the accumulators
      auto epi = [&](auto plain_c) __attribute__((always_inline)) {
        constexpr bool PLAIN = decltype(plain_c)::value;
        // inverse norm of this lane's rows (NaN past the end / masked out; 1 in UNIT mode)
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
          if constexpr (MAXONLY) {
            // lanes lq = 0..3 hold the same 16 queries over different rows
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            if (lq == 0)
              reinterpret_cast<float*>(buf)[((size_t)ep_vt * 2 + wm) * ((size_t)nqb * QT) + qbase +
                                            wn * 64 + n * 16 + lr] = mx;
          }
          hit[n] = mx >= thr[n];
          any |= hit[n];
        }
        if constexpr (MAXONLY) any = false;
        if (__any(any)) {
          // wave-uniform tests per query block and per 4-row block, lanes predicated inside
          // (per-lane branches over every element cost ~3x as much: r02 stamps of the QS
          // kernel's identical path)
#pragma unroll
          for (int n = 0; n < NQ; ++n) {
            if (!__any(hit[n])) continue;
            const int ql = wn * 64 + n * 16 + lr;
#pragma unroll
            for (int m = 0; m < MT; ++m) {
              const bool cg = fmaxf(fmaxf(score(m, n, 0), score(m, n, 1)),
                                    fmaxf(score(m, n, 2), score(m, n, 3))) >= thr[n];
              if (__builtin_amdgcn_ballot_w64(cg)) {
                if (cg) {
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
          }
        }
      };
      if (UNIT && !mask && row0 + RT <= n_rows) epi(std::true_type{});
      else epi(std::false_type{});
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      ep_vt = -1;
    }
    if (s == nsteps) break;

    // 2) stage s landed (this wave's pieces; D-1 later stages stay in flight), then everyone's
    v3_wait_vmcnt((D - 1) * 4);
    v3_barrier();

    // 3) tile-slot pieces for the stage being issued (once per tile), then the MFMAs of stage s
    //    with the 4 pieces of stage s + D between them
    if (is_ks == 0 && is_s < nsteps) issue_tile_slot(is_vt);
    const Desc d = cursor_desc();
    {
      const char* st = ring + rslot * L::STAGE;
      V bq[NQ], av[MT];
      v4_read_frags<V>(lds_addr(st + offA), lds_addr(st + offB), av, bq);
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
    }
    advance_cursor();
    rslot = (rslot + 1 == NST) ? 0 : rslot + 1;
    if (ks == ksteps - 1) ep_vt = vt;
    if (++ks == ksteps) { ks = 0; ++vt; }
  }

  if constexpr (MAXONLY) return;
  __syncthreads();
  final_lists<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wave, V3_NT / 64, QT, kp, lane, partials, pcnt, P, p);
}

}  // namespace hcr
