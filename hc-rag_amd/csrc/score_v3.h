// score_v3.h — K2 v3: fused score + top-k' with a deep LDS-DMA ring.
//
// Same contract as score_topk_kernel (topk_kernels.h): every workgroup scores a row
// partition against one query block, keeps each query's best k' coarse keys in its
// candidate buffer and appends them to partials[q] (final_list).  What changes is the memory
// pipeline, after the r01 profile of v2 (profiles/r01/pmc_summary.txt: 28 % MFMA busy, waves
// parked 50 % of their cycles in s_waitcnt / barrier, i.e. latency-bound on a 2-deep ring):
//
//  * a stage is K = 32 (one 16x16x32 MFMA k-step) instead of 64, and NST stages are in the
//    ring, NST-1 of them in flight while one is consumed: 4x the bytes in flight of v2 at the
//    large shape (120 KiB vs 60 KiB of requests outstanding per CU).
//  * each wave waits only for ITS OWN DMA pieces of the stage it is about to consume
//    (s_waitcnt vmcnt(N), N = its pieces of the later stages), then one barrier per stage.
//  * LDS image of a stage: [row][4 x 16 B]; chunk slot = chunk ^ f((row >> 2) & 3) with
//    f = {0, 2, 3, 1}: for the ds_read_b128 lane groups of CDNA4 ({0-3,12-15,20-27},
//    {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}) the 16 lanes of a group hit
//    16 distinct 16-byte bank quads (checked in tests/test_lds_swizzle.py).
//  * tile shapes are template parameters: RT rows x QT queries per workgroup, WM x WN waves
//    (8 waves), so one kernel serves the MFMA-bound large batch (224 x 256) and the HBM-bound
//    small batch (256 x 64 / 256 x 16).
#pragma once
#include "topk_kernels.h"

namespace hcr {

constexpr int V3_NIS = 3;   // tile slots of inverse norms / mask words / global bounds; the
                            // host requires (V3_NIS - 1) * ksteps > NST - 1


template <int RT, int QT, int NST>
struct V3Layout {
  static constexpr int A_BYTES = RT * 64, B_BYTES = QT * 64;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int NIS = V3_NIS;
  static constexpr int INV = NST * STAGE;                 // NIS x RT floats
  static constexpr int INV_SLOT = ((RT * 4 + 1023) / 1024) * 1024;
  static constexpr int TG = INV + NIS * INV_SLOT;         // NIS x QT u32 global bounds
  static constexpr int TG_SLOT = ((QT * 4 + 1023) / 1024) * 1024;
  static constexpr int MSK = TG + NIS * TG_SLOT;          // NIS x 64 B of row-mask words
  static constexpr int TAU = MSK + NIS * 64;              // u64 tau_key[QT]
  static constexpr int CNT = TAU + QT * 8;                // int cnt[QT]
  static constexpr int FLAG = CNT + QT * 4;               // int flag[2]
  static constexpr int TOTAL = FLAG + 16;
  static_assert(TOTAL <= 160 * 1024, "LDS budget");
  static_assert(RT % 32 == 0 && QT % 16 == 0 && RT <= 256 && QT <= 256, "tile shape");
};

template <typename TM, int CAP, int RT, int QT, int WM, int WN, int NST>
__global__ void __launch_bounds__(V3_NT, 2)
score_topk_v3_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows, int ksteps,
                     const float* __restrict__ inv_norm, const uint32_t* __restrict__ mask,
                     const TM* __restrict__ qhat, int nqb, int P, int ntiles, int tstride,
                     uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                     uint64_t* __restrict__ partials, int* __restrict__ pcnt, int kp) {
  // ntiles counts VIRTUAL tiles v; virtual tile v is row tile v * tstride (tstride > 1: the
  // sampling pre-pass over every tstride-th tile).  Ring slots and flag parity follow v.
  static_assert(WM * WN == V3_NT / 64, "8 waves");
  using L = V3Layout<RT, QT, NST>;
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int MT = RT / WM / 16;       // 16-row MFMA blocks per wave
  constexpr int NQ = QT / WN / 16;       // 16-query MFMA blocks per wave
  static_assert(MT * WM * 16 == RT && NQ * WN * 16 == QT, "wave tiling");
  constexpr int NA = RT / 16, NB = QT / 16, NP = NA + NB;   // 1 KiB DMA pieces per stage
  constexpr int D = NST - 1;             // stages in flight
  __shared__ __attribute__((aligned(16))) char lds[L::TOTAL];
  uint64_t* tau_key = reinterpret_cast<uint64_t*>(lds + L::TAU);
  int* cnt = reinterpret_cast<int*>(lds + L::CNT);
  int* flag = reinterpret_cast<int*>(lds + L::FLAG);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int my_pieces = (NP - wave + 7) / 8;               // DMA pieces this wave issues per stage

  // XCD-aware bijective remap: the query blocks sharing a partition run on one XCD
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
    for (int i = tid; i < QT; i += V3_NT) pcnt[(size_t)(qbase + i) * P + p] = 0;
    return;
  }

  // DMA lane roles: a 1 KiB piece covers 16 rows x 4 chunks; lane -> (row, slot) of the LDS
  // image, source chunk = slot ^ f(row)
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int ldb = ld * 2;
  const int voff = drow * ldb + dchunk * 16;
  const char* rows_b = reinterpret_cast<const char*>(rows);
  const __amdgpu_buffer_rsrc_t q_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(qhat) + (size_t)qbase * ldb), (short)0, QT * ldb,
      0x00020000);
  const __amdgpu_buffer_rsrc_t inv_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(inv_norm), (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t tg_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(tau_g + qbase), (short)0, QT * 4, 0x00020000);   // reads past QT give 0
  const __amdgpu_buffer_rsrc_t msk_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(mask), (short)0, 0x7FFFFFFF, 0x00020000);

  // issue the DMA pieces of global stage s (tile t0 + s / ksteps, k-step s % ksteps)
  auto issue_stage = [&](int s_) {
    const int s = __builtin_amdgcn_readfirstlane(s_);
    const int vt = t0 + s / ksteps, ks = s - (s / ksteps) * ksteps;
    const int tile = vt * tstride;
    char* sa = lds + (s % NST) * L::STAGE;
    const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        uniform_ptr(rows_b + (size_t)tile * RT * ldb), (short)0, RT * ldb, 0x00020000);
    const int kofs = ks * (V3_BK * 2);
#pragma unroll
    for (int i = 0; i < (NP + 7) / 8; ++i) {
      const int j = wave + 8 * i;                              // piece index (uniform)
      if (j < NA) dma16(a_rsrc, sa + j * 1024, voff, j * 16 * ldb + kofs);
      else if (j < NP) dma16(q_rsrc, sa + L::A_BYTES + (j - NA) * 1024, voff, (j - NA) * 16 * ldb + kofs);
    }
    if (ks == 0 && wave == 7)   // this tile's inverse norms (RT floats, 1 KiB piece)
      dma16(inv_rsrc, lds + L::INV + (vt % L::NIS) * L::INV_SLOT, lane * 16, tile * (RT * 4));
    if (ks == 0 && wave == 5)   // the block's global per-query bounds for this tile's epilogue
      dma16(tg_rsrc, lds + L::TG + (vt % L::NIS) * L::TG_SLOT, lane * 16, 0);
    if (ks == 0 && wave == 6 && mask) {
      if (lane < RT / 32)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            msk_rsrc, (__attribute__((address_space(3))) void*)(lds + L::MSK + (vt % L::NIS) * 64),
            4, lane * 4, tile * (RT / 8), 0, 0);
    }
  };

  // fragment read offsets inside a stage (rows of 64 B)
  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = v3_slot(fc, fr);
  const int offA = (wm * (RT / WM) + fr) * 64 + fslot * 16;
  const int offB = L::A_BYTES + (wn * (QT / WN) + fr) * 64 + fslot * 16;

  floatx4 acc[MT][NQ];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (t1 - t0) * ksteps;

  for (int i = 0; i < D; ++i)
    if (i < nsteps) issue_stage(i);

  int tile = t0, ks = 0;
  int ep_tile = -1;                      // tile whose epilogue is pending
  for (int s = 0; s <= nsteps; ++s) {
    // 1) epilogue of the tile finished by step s-1 (accumulators complete)
    if (ep_tile >= 0) {
      int* prev_flag = flag + ((ep_tile + 1) & 1);
      if (v3_lds_u32(prev_flag)) {       // set >= 1 barrier ago; uniform across the block
        __syncthreads();                 // other waves' candidate stores (global) are visible
        for (int ql = wave; ql < QT; ql += V3_NT / 64) {
          if (cnt[ql] > CAP - RT)
            compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql],
                                   tau_g + qbase + ql, kp, lane, nullptr);
        }
        __syncthreads();
        if (tid == 0) *prev_flag = 0;
      }
      int* cur_flag = flag + (ep_tile & 1);
      int le;
      asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
      const int lr = le & 15, lq = le >> 4;
      const int64_t row0 = (int64_t)ep_tile * tstride * RT;
      const char* invl = lds + L::INV + (ep_tile % L::NIS) * L::INV_SLOT;
      const char* mskl = lds + L::MSK + (ep_tile % L::NIS) * 64;
      const char* tgl = lds + L::TG + (ep_tile % L::NIS) * L::TG_SLOT;
      float thr[NQ];
      uint64_t tk[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        const int ql = wn * (QT / WN) + n * 16 + lr;
        tk[n] = v3_lds_u64(tau_key + ql);
        const float ls = tk[n] ? key_score(tk[n]) : -INFINITY;
        thr[n] = fmaxf(ls, unord32(v3_lds_u32(tgl + ql * 4)));
      }
      auto inv4 = [&](int m, float (&iv)[4]) {
        const int rl = wm * (RT / WM) + m * 16 + lq * 4;        // row inside the tile
        const float4 v = lds_read_f4_now(invl + rl * 4);
        uint32_t mword = 0xFFFFFFFFu;
        if (mask) mword = lds_read_u32_now(mskl + (rl >> 5) * 4);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = (row0 + rl + r < n_rows) && ((mword >> ((rl + r) & 31)) & 1u);
          iv[r] = ok ? vv[r] : __builtin_nanf("");
        }
      };
      float mx[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) mx[n] = -INFINITY;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float iv[4];
        inv4(m, iv);
#pragma unroll
        for (int n = 0; n < NQ; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx[n] = fmaxf(mx[n], acc[m][n][r] * iv[r]);
      }
      bool hit[NQ];
      bool any = false;
#pragma unroll
      for (int n = 0; n < NQ; ++n) { hit[n] = mx[n] >= thr[n]; any |= hit[n]; }
      if (__any(any)) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          float iv[4];
          inv4(m, iv);
#pragma unroll
          for (int n = 0; n < NQ; ++n) {
            if (hit[n]) {
              const int ql = wn * (QT / WN) + n * 16 + lr;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float sc = acc[m][n][r] * iv[r];
                if (sc >= thr[n]) {
                  const uint32_t rowl = (uint32_t)(row0 + wm * (RT / WM) + m * 16 + lq * 4 + r);
                  const uint64_t key = make_key(sc, rowl);
                  if (key > tk[n]) {
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
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      ep_tile = -1;
    }
    if (s == nsteps) break;

    // 2) stage s landed: this wave's pieces (later stages may stay in flight), then everyone's
    {
      const int later = min(D - 1, nsteps - 1 - s);
      v3_wait_vmcnt(later * my_pieces);
    }
    v3_barrier();                        // also: every wave is done reading stage s-1's slot
    if (s + D < nsteps) issue_stage(s + D);

    // 3) MFMAs of stage s
    const bool last_k = (ks == ksteps - 1);
    {
      // all fragment reads of the stage first, then the MFMAs (the scheduler is told so; the
      // waitcnt pass then gives each MFMA group the smallest lgkmcnt it needs)
      const char* st = lds + (s % NST) * L::STAGE;
      V bq[NQ], av[MT];
#pragma unroll
      for (int n = 0; n < NQ; ++n) bq[n] = *reinterpret_cast<const V*>(st + offB + n * 16 * 64);
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = *reinterpret_cast<const V*>(st + offA + m * 16 * 64);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NQ; ++n) {
          acc[m][n] = Op::run(av[m], bq[n], acc[m][n]);
        }
      __builtin_amdgcn_sched_group_barrier(0x100, NQ + MT, 0);   // DS reads
      __builtin_amdgcn_sched_group_barrier(0x008, MT * NQ, 0);   // MFMAs
    }
    if (last_k) ep_tile = tile;
    if (++ks == ksteps) { ks = 0; ++tile; }
  }

  // final: every query's surviving keys (at most k') appended to its region of the partials.
  // All waves' appends first.
  __syncthreads();
  final_lists<CAP>(wbuf, cnt, tau_key, tau_g, qbase, wave, V3_NT / 64, QT, kp, lane, partials, pcnt, P, p);
}

}  // namespace hcr
