// score_v5.h — K2 v5: the large-batch fused score + top-k' kernel with the top-k' epilogue
// folded into the MFMA stream.
//
// Same contract, tiling (256 rows x 256 queries, 8 waves of 128 x 64), LDS-DMA ring and grid
// mapping as score_topk_v4_kernel (score_v4.h).  What changes is WHERE the per-tile epilogue
// runs, after the r01b measurements (profiles/r01b): with every wave of a workgroup reaching a
// tile boundary at the same barrier, v4's epilogue (128 multiplies + 128 maxima + 128
// accumulator zeroings + row-validity masks per wave) ran with the matrix pipe idle: ~13 % of
// the wave cycles even when no row survived, ~20 % of the in-situ kernel time.
//
//  * The epilogue's fast test is 128 compares of the raw accumulators against a per-query
//    threshold (no multiplies, no row masks); only a 16-row block with a surviving lane
//    (wave-uniform branch) takes the exact path (inverse norm, row bound, row mask, key
//    compare, LDS-atomic append).
//  * No zeroing: the first k-step of every tile runs its MFMAs on C = 0.
//  * A first version that folded the epilogue into the next tile's first k-step (nested tile /
//    k-step loops) spilled VGPRs; every scratch reload then drained the LDS-DMA ring
//    (s_waitcnt vmcnt(0)): 45 % slower.  The flat single loop of v4 is kept.
//  * UNIT (host-selected when every stored row has | ||e|| - 1 | <= 2^-10, i.e. L2-normalised
//    corpora such as HuggingFaceEmbedding(normalize=True) output): the coarse score is the raw
//    dot product q^ . e, no inverse-norm multiply; the host widens the certificate bound eps_q
//    by the norm deviation, so the final top-k stays exact.
#pragma once
#include "score_v4.h"

namespace hcr {

// one wait for the 4 global bounds of the lane's queries (64 B apart)
__device__ __forceinline__ void v5_read_tg(uint32_t a, uint32_t (&tg)[4]) {
  asm volatile(
      "ds_read_b32 %0, %4\n\t"
      "ds_read_b32 %1, %4 offset:64\n\t"
      "ds_read_b32 %2, %4 offset:128\n\t"
      "ds_read_b32 %3, %4 offset:192\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(tg[0]), "=&v"(tg[1]), "=&v"(tg[2]), "=&v"(tg[3])
      : "v"(a)
      : "memory");
}
// one wait for the 8 x 4 inverse norms of the lane's rows (blocks of 16 rows, 64 B apart)
__device__ __forceinline__ void v5_read_iv(uint32_t a, float4 (&v)[8]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\t"
      "ds_read_b128 %1, %8 offset:64\n\t"
      "ds_read_b128 %2, %8 offset:128\n\t"
      "ds_read_b128 %3, %8 offset:192\n\t"
      "ds_read_b128 %4, %8 offset:256\n\t"
      "ds_read_b128 %5, %8 offset:320\n\t"
      "ds_read_b128 %6, %8 offset:384\n\t"
      "ds_read_b128 %7, %8 offset:448\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
        "=&v"(v[6]), "=&v"(v[7])
      : "v"(a)
      : "memory");
}

// The last k-step of a tile: its 12 MFMA fragments plus what the tile's epilogue needs from
// LDS (the compaction flag and the 4 global bounds of the lane's queries), one wait -- the
// epilogue then makes no LDS round trip of its own (the LDS is busy with the DMA and the other
// waves' fragment reads: each round trip there costs hundreds of cycles).
template <typename V>
__device__ __forceinline__ void v5_read_frags_epi(uint32_t a, uint32_t b, uint32_t fa, uint32_t ta,
                                                  V (&av)[8], V (&bq)[4], uint32_t& fl,
                                                  uint32_t (&tg)[4]) {
  asm volatile(
      "ds_read_b128 %0, %17\n\t"
      "ds_read_b128 %1, %17 offset:1024\n\t"
      "ds_read_b128 %2, %17 offset:2048\n\t"
      "ds_read_b128 %3, %17 offset:3072\n\t"
      "ds_read_b128 %4, %17 offset:4096\n\t"
      "ds_read_b128 %5, %17 offset:5120\n\t"
      "ds_read_b128 %6, %17 offset:6144\n\t"
      "ds_read_b128 %7, %17 offset:7168\n\t"
      "ds_read_b128 %8, %18\n\t"
      "ds_read_b128 %9, %18 offset:1024\n\t"
      "ds_read_b128 %10, %18 offset:2048\n\t"
      "ds_read_b128 %11, %18 offset:3072\n\t"
      "ds_read_b32 %12, %19\n\t"
      "ds_read_b32 %13, %20\n\t"
      "ds_read_b32 %14, %20 offset:64\n\t"
      "ds_read_b32 %15, %20 offset:128\n\t"
      "ds_read_b32 %16, %20 offset:192\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]),
        "=&v"(av[6]), "=&v"(av[7]), "=&v"(bq[0]), "=&v"(bq[1]), "=&v"(bq[2]), "=&v"(bq[3]),
        "=&v"(fl), "=&v"(tg[0]), "=&v"(tg[1]), "=&v"(tg[2]), "=&v"(tg[3])
      : "v"(a), "v"(b), "v"(fa), "v"(ta)
      : "memory");
}

#ifdef HCR_V5_COUNT
// diagnostic build only: [0] slow-path blocks, [1] appends, [2] epilogues (per wave), [3] compactions
__device__ unsigned long long g_v5_count[4];
#endif

template <typename TM, int CAP, int NST, bool UNIT>
__global__ void __launch_bounds__(V3_NT, 2)
score_topk_v5_kernel(const TM* __restrict__ rows, int ld, int64_t n_rows, int ksteps,
                     const float* __restrict__ inv_norm, const uint32_t* __restrict__ mask,
                     const TM* __restrict__ qhat, int nqb, int P, int ntiles, int tstride,
                     uint64_t* __restrict__ buf, uint32_t* __restrict__ tau_g,
                     uint64_t* __restrict__ partials, int kp) {
  using L = V4Layout<NST>;
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int RT = V4_RT, QT = V4_QT, WN = 4;
  constexpr int MT = 8, NQ = 4;          // 16x16 MFMA blocks per wave: 128 rows x 64 queries
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
  int is_s = 0, is_vt = t0, is_ks = 0, is_slot = 0;   // DMA issue cursor

  auto issue_tile_slot = [&](int vt) {
    const int tile = vt * tstride;
    const int slot = vt % L::NIS;
    if (!UNIT && wave == 7) dma16(inv_rsrc, ring + L::INV + slot * 1024, lane * 16, tile * (RT * 4));
    if (wave == 5) dma16(tg_rsrc, ring + L::TG + slot * 1024, lane * 16, 0);
    if (wave == 6 && mask) {
      if (lane < RT / 32)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            msk_rsrc, (__attribute__((address_space(3))) void*)(ring + L::MSK + slot * 64), 4,
            lane * 4, tile * (RT / 8), 0, 0);
    }
  };
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
#ifdef HCR_V5_NO_ZEROC
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
#endif
  uint64_t tkr[NQ];                      // this lane's queries' local k'-th keys (LDS copy)
#pragma unroll
  for (int n = 0; n < NQ; ++n) tkr[n] = 0ull;

  // per-tile epilogue state (tile `ep`): thresholds of this lane's 4 queries
  float thr[NQ];
  int ep = -1;                           // virtual tile whose epilogue is pending

  // wait for the stage at the consume position, then everyone's pieces of it
  auto stage_wait = [&]() {
    v3_wait_vmcnt((D - 1) * 4);
    v3_barrier();
  };

  // compaction round (a query's buffer could overflow in this epilogue): whole workgroup
  auto maybe_compact = [&](int ept, uint32_t pre_flag) {
    int* prev_flag = flag + ((ept + 1) & 1);
    if (__builtin_amdgcn_readfirstlane(pre_flag)) {   // set >= 1 barrier ago; uniform
      __syncthreads();
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
  };
  auto load_thr = [&](const uint32_t (&tg)[NQ]) {
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      const float ls = tkr[n] ? key_score(tkr[n]) : -INFINITY;
      thr[n] = fmaxf(ls, unord32(tg[n]));
    }
  };
  // exact path of row block m of tile ept: appends the lane's surviving (row, query) keys.
  // Hits are sparse (a handful per tile and wave once the bound is seeded), so the work is
  // gated by wave-uniform skips per query block and per row: a lone hit costs ~16 compares +
  // ballots and one append instead of a walk over all 16 (query, row) values of every lane.
  auto block_exact = [&](int ept, int m) {
#ifdef HCR_V5_COUNT
    if (lane == 0) atomicAdd(&g_v5_count[0], 1ull);
#endif
    int le;
    asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
    const int lr = le & 15, lq = le >> 4;
    const int slot = ept % L::NIS;
    const int rl = wm * 128 + m * 16 + lq * 4;
    float vv[4] = {1.f, 1.f, 1.f, 1.f};
    if constexpr (!UNIT) {
      const float4 v = lds_read_f4_now(ring + L::INV + slot * 1024 + rl * 4);
      vv[0] = v.x; vv[1] = v.y; vv[2] = v.z; vv[3] = v.w;
    }
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      float sc[4];
      bool h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sc[r] = UNIT ? acc[m][n][r] : acc[m][n][r] * vv[r];
        h[r] = sc[r] >= thr[n];
      }
      if (!__any(h[0] || h[1] || h[2] || h[3])) continue;
      const int ql = wn * 64 + n * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!__any(h[r])) continue;
        if (h[r]) {
          const int64_t row = (int64_t)ept * tstride * RT + rl + r;
          bool ok = row < n_rows;
          if (mask) ok = ok && ((lds_read_u32_now(ring + L::MSK + slot * 64 + ((rl + r) >> 5) * 4) >>
                                 ((rl + r) & 31)) & 1u);
          const uint64_t key = make_key(sc[r], (uint32_t)row);
          if (ok && key > tkr[n]) {
#ifdef HCR_V5_COUNT
            atomicAdd(&g_v5_count[1], 1ull);
#endif
            const int pos = v3_lds_add_rtn(&cnt[ql], 1);
            wbuf[(size_t)ql * CAP + pos] = key;
            if (pos + 1 > CAP - RT) v3_lds_store_u32(flag + (ept & 1), 1u);
          }
        }
      }
    }
  };
  // max inverse norm of the tile's rows this lane holds (non-UNIT)
  auto tile_ivmax = [&](int ept) -> float {
    if constexpr (UNIT) return 1.f;
    const int slot = ept % L::NIS;
    float4 v[MT];
    v5_read_iv(lds_addr(ring + L::INV + slot * 1024 + (wm * 128 + (lane >> 4) * 4) * 4), v);
    float x = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m) x = fmaxf(x, fmaxf(fmaxf(v[m].x, v[m].y), fmaxf(v[m].z, v[m].w)));
    return x;
  };
  // The epilogue of tile ept.  Fast test on the raw dot products against t_n: UNIT t_n = thr_n;
  // otherwise t_n = thr_n / iv_max shrunk by 1e-5 (fl(acc * iv) >= thr > 0 implies acc >=
  // thr (1 - u) / iv_max > t_n; acc <= 0 never reaches a positive threshold; thr <= 0 tests
  // everything).  No multiplies, no row-validity masks, no zeroing (the next tile's first
  // k-step runs its MFMAs on C = 0): 128 compares per lane.  Only row blocks with a lane at
  // or above its threshold take the exact path.
  auto epilogue = [&](int ept, uint32_t pre_flag, const uint32_t (&pre_tg)[NQ]) {
#ifdef HCR_V5_COUNT
    if (lane == 0) atomicAdd(&g_v5_count[2], 1ull);
    if (lane == 0 && __builtin_amdgcn_readfirstlane(pre_flag)) atomicAdd(&g_v5_count[3], 1ull);
#endif
    maybe_compact(ept, pre_flag);
    load_thr(pre_tg);
    float t[NQ];
    if constexpr (UNIT) {
#pragma unroll
      for (int n = 0; n < NQ; ++n) t[n] = thr[n];
    } else {
      const float ivmax = tile_ivmax(ept);
#pragma unroll
      for (int n = 0; n < NQ; ++n) t[n] = thr[n] > 0.f ? thr[n] / ivmax * 0.99999f : -INFINITY;
    }
    bool hm[MT];
    bool any = false;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      bool h = false;
#pragma unroll
      for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) h |= acc[m][n][r] >= t[n];
      hm[m] = h;
      any |= h;
    }
    if (__any(any)) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        if (__any(hm[m])) block_exact(ept, m);
    }
#ifdef HCR_V5_NO_ZEROC
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
#endif
  };

  int rslot = 0;                         // ring slot of the stage being consumed
  int ks = 0, vt = t0;
  uint32_t pre_flag = 0, pre_tg[NQ] = {0u, 0u, 0u, 0u};   // read with the tile's last k-step
#ifdef HCR_V3_STAMPS
  uint64_t st_epi = 0, st_wait = 0, st_issue = 0, st_mma = 0, ta, tb;
#endif
  for (int s = 0; s <= nsteps; ++s) {
#ifdef HCR_V3_STAMPS
    V3_STAMP(ta);
#endif
    // 1) epilogue of the tile finished by step s-1 (accumulators complete)
#ifndef HCR_V5_NO_EPI
    if (ep >= 0) {
      epilogue(ep, pre_flag, pre_tg);
      ep = -1;
    }
#else
    if (ep >= 0) {                       // diagnostic: keep the accumulators alive only
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NQ; ++n)
          if (acc[m][n][0] == 12345.f) cnt[0] = 1;
      ep = -1;
    }
#endif
#ifdef HCR_V3_STAMPS
    V3_STAMP(tb); st_epi += tb - ta; ta = tb;
#endif
    if (s == nsteps) break;

    // 2) stage s landed (this wave's pieces; D-1 later stages stay in flight), then everyone's
    v3_wait_vmcnt((D - 1) * 4);
    v3_barrier();
#ifdef HCR_V3_STAMPS
    V3_STAMP(tb); st_wait += tb - ta; ta = tb;
#endif

    // 3) tile-slot pieces for the stage being issued (once per tile), then the MFMAs of stage s
    //    with the 4 pieces of stage s + D between them.  The first k-step of a tile accumulates
    //    onto C = 0 (its pieces go out in a different order, so the compiler cannot hoist the
    //    two branches' identical DMA instructions above the branch and cluster them)
    if (is_ks == 0 && is_s < nsteps) issue_tile_slot(is_vt);
    const Desc d = cursor_desc();
    {
      const char* st = ring + rslot * L::STAGE;
      V bq[NQ], av[MT];
      if (ks == ksteps - 1)
        v5_read_frags_epi<V>(lds_addr(st + offA), lds_addr(st + offB),
                             lds_addr(flag + ((vt + 1) & 1)),
                             lds_addr(ring + L::TG + (vt % L::NIS) * 1024 + (wn * 64 + (lane & 15)) * 4),
                             av, bq, pre_flag, pre_tg);
      else
        v4_read_frags<V>(lds_addr(st + offA), lds_addr(st + offB), av, bq);
#ifdef HCR_V3_STAMPS
      V3_STAMP(tb); st_issue += tb - ta; ta = tb;
#endif
#ifndef HCR_V5_NO_ZEROC
      if (ks == 0) {
#else
      if (false) {
#endif
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int m = 2 * i; m < 2 * i + 2; ++m)
#pragma unroll
            for (int n = 0; n < NQ; ++n)
              acc[m][n] = Op::run(av[m], bq[n], floatx4{0.f, 0.f, 0.f, 0.f});
          issue_piece(d, i ^ 2);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * NQ, 0);  // 8 MFMAs
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);       // 1 DMA piece
        }
      } else {
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
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * NQ, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
      }
    }
#ifdef HCR_V3_STAMPS
    V3_STAMP(tb); st_mma += tb - ta; ta = tb;
#endif
    advance_cursor();
    rslot = (rslot + 1 == NST) ? 0 : rslot + 1;
    if (ks == ksteps - 1) ep = vt;
    if (++ks == ksteps) { ks = 0; ++vt; }
  }
#ifdef HCR_V3_STAMPS
  if (lane == 0 && g_v3_stamps) {
    uint64_t* o = g_v3_stamps + ((size_t)blockIdx.x * 8 + wave) * 4;
    o[0] = st_epi; o[1] = st_wait; o[2] = st_issue; o[3] = st_mma;
  }
#endif

  __syncthreads();
  for (int ql = wave; ql < QT; ql += V3_NT / 64) {
    compact_query_inl<CAP>(wbuf + (size_t)ql * CAP, &cnt[ql], &tau_key[ql], tau_g + qbase + ql, kp,
                           lane, partials + ((size_t)(qbase + ql) * P + p) * kp);
  }
}

}  // namespace hcr
