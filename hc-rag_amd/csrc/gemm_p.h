// gemm_p.h — persistent encoder projection GEMM: one workgroup per CU streams its share of the
// 256 x 256 output tiles through ONE continuous LDS-DMA ring (the score kernel's cursor,
// score_v4.h), so a tile's prologue latency and epilogue stores overlap the next tile's DMA.
//
// r01c profile of the one-tile-per-workgroup gemm_v4 (profiles/r01c): a 256 x 256 x 768 tile
// took ~32.6 us per round against ~21.8 us for the same 24 MFMA stages inside the score
// kernel's stream -- ~10 us per tile of ring fill + epilogue with the matrix pipe idle.
//
// C[token][feature] = X[token][:] . W[feature][:] + bias (+ GELU).  Epilogues have NO global
// loads (a load would need every older in-flight LDS-DMA piece to land first: vmcnt counts in
// issue order): the bias comes through the ring as a per-tile LDS slot, and the residual add
// of the two residual projections moves into the LayerNorm kernel that follows them
// (layernorm4_res_kernel).  Stores are unconditional (out-of-range features / tokens go to a
// trash line), so every wave has the same 32 stores outstanding after an epilogue and the
// next D k-steps wait for vmcnt((D-1)*4 + 32) instead of draining the ring.
#pragma once
#include <type_traits>
#include "encoder_kernels.h"
#include "ring_common.h"

namespace hcr {

constexpr int GP_T = 256;    // features and tokens per tile
constexpr int GP_NIS = 3;    // bias tile slots (a slot outlives NST - 1 stages of look-ahead)

// EPI_BIAS -> out_h (MFMA dtype), EPI_BIAS_GELU -> out_h, EPI_BIAS_RESID -> out_f (fp32,
// projection + bias only; the residual is added by layernorm4_res_kernel)
template <typename TM, int EPI, int NST>
__global__ void __launch_bounds__(V3_NT, 2)
gemm_p_kernel(const TM* __restrict__ W, const TM* __restrict__ X, int K, int N_real, int T_real,
              int n_tiles_feat, int n_tiles, const float* __restrict__ bias,
              TM* __restrict__ out_h, float* __restrict__ out_f, int ldo, float4* __restrict__ trash) {
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int STAGE = 2 * GP_T * 64;   // W rows then X rows, 64 B each (32 KiB)
  constexpr int A_BYTES = GP_T * 64;
  constexpr int MT = 8, NQ = 4, WN = 4, D = NST - 1;
  constexpr int NSTORE = MT * NQ;        // epilogue stores per lane (and per wave)
  static_assert(NST * STAGE + GP_NIS * 1024 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char ring[NST * STAGE + GP_NIS * 1024];
  char* bias_lds = ring + NST * STAGE;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int tb = (int)((int64_t)g * n_tiles / nwg);
  const int te = (int)((int64_t)(g + 1) * n_tiles / nwg);
  if (tb >= te) return;

  const int ldb = K * 2;
  const int ksteps = K / V3_BK;
  const int nsteps = (te - tb) * ksteps;
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int voff = drow * ldb + dchunk * 16;
  const char* Wb = reinterpret_cast<const char*>(W);
  const char* Xb = reinterpret_cast<const char*>(X);
  const __amdgpu_buffer_rsrc_t bias_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(bias), (short)0, 0x7FFFFFFF, 0x00020000);

  // DMA issue cursor: stage is_s = (tile is_t, k-step is_ks) into ring slot is_slot
  int is_s = 0, is_t = tb, is_ks = 0, is_slot = 0;
  struct Desc { __amdgpu_buffer_rsrc_t w, x; int kofs; char* sa; };
  auto cursor_desc = [&]() __attribute__((always_inline)) {
    const bool live = is_s < nsteps;
    const int t = __builtin_amdgcn_readfirstlane(is_t);
    const int ft = t % n_tiles_feat, tt = t / n_tiles_feat;
    Desc d;
    d.w = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(Wb + (size_t)ft * GP_T * ldb), (short)0,
                                            live ? GP_T * ldb : 0, 0x00020000);
    d.x = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(Xb + (size_t)tt * GP_T * ldb), (short)0,
                                            live ? GP_T * ldb : 0, 0x00020000);
    d.kofs = __builtin_amdgcn_readfirstlane(is_ks * (V3_BK * 2));
    d.sa = ring + __builtin_amdgcn_readfirstlane(is_slot) * STAGE;
    return d;
  };
  // fixed piece kinds per slot i: 0 / 3 -> W pieces wave / wave + 8, 1 / 2 -> X pieces
  auto issue_piece = [&](const Desc& d, int i) __attribute__((always_inline)) {
    if (i == 0 || i == 3) {
      const int j = wave + (i == 3 ? 8 : 0);
      dma16(d.w, d.sa + j * 1024, voff, j * 16 * ldb + d.kofs);
    } else {
      const int j = wave + (i == 2 ? 8 : 0);
      dma16(d.x, d.sa + A_BYTES + j * 1024, voff, j * 16 * ldb + d.kofs);
    }
  };
  // the tile's 256 biases into its LDS slot (with the tile's first stage; wave 7)
  auto issue_bias = [&]() __attribute__((always_inline)) {
    if (wave == 7 && is_s < nsteps) {
      const int t = __builtin_amdgcn_readfirstlane(is_t);
      dma16(bias_rsrc, bias_lds + (t % GP_NIS) * 1024, lane * 16, (t % n_tiles_feat) * GP_T * 4);
    }
  };
  auto advance_cursor = [&]() __attribute__((always_inline)) {
    ++is_s;
    is_slot = (is_slot + 1 == NST) ? 0 : is_slot + 1;
    if (++is_ks == ksteps) { is_ks = 0; ++is_t; }
  };

  for (int i = 0; i < D; ++i) {
    if (is_ks == 0) issue_bias();
    const Desc d = cursor_desc();
#pragma unroll
    for (int k = 0; k < 4; ++k) issue_piece(d, k);
    advance_cursor();
  }

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = v3_slot(fc, fr);
  const int offA = (wm * 128 + fr) * 64 + fslot * 16;
  const int offB = A_BYTES + (wn * 64 + fr) * 64 + fslot * 16;
  floatx4 acc[MT][NQ];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  // epilogue of tile t: bias from the LDS slot, GELU, unconditional stores
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int ft = t % n_tiles_feat, tt = t / n_tiles_feat;
    const int fl = wm * 128 + (lane >> 4) * 4;           // + m * 16: feature inside the tile
    const int tok0 = tt * GP_T + wn * 64 + (lane & 15);  // + n * 16
    const char* bl = bias_lds + (t % GP_NIS) * 1024;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 bb = lds_read_f4_now(bl + (fl + m * 16) * 4);
      const int f = ft * GP_T + fl + m * 16;
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        const int tok = tok0 + n * 16;
        const bool ok = f < N_real && tok < T_real;
        float v0 = acc[m][n][0] + bb.x, v1 = acc[m][n][1] + bb.y;
        float v2 = acc[m][n][2] + bb.z, v3 = acc[m][n][3] + bb.w;
        if constexpr (EPI == EPI_BIAS_GELU) {
          v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
        }
        if constexpr (EPI == EPI_BIAS_RESID) {
          float4* dst = ok ? reinterpret_cast<float4*>(out_f + (size_t)tok * ldo + f) : trash + lane;
          *dst = float4{v0, v1, v2, v3};
        } else {
          union { TM h[4]; uint2 u; } pk;
          pk.h[0] = (TM)v0; pk.h[1] = (TM)v1; pk.h[2] = (TM)v2; pk.h[3] = (TM)v3;
          uint2* dst = ok ? reinterpret_cast<uint2*>(out_h + (size_t)tok * ldo + f)
                          : reinterpret_cast<uint2*>(trash + lane);
          *dst = pk.u;
        }
        acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  int rslot = 0, ks = 0, vt = tb;
  int ep = -1;              // tile whose epilogue is pending
  int after_epi = 0;        // k-steps left whose wait must also allow the epilogue's stores
  for (int s = 0; s <= nsteps; ++s) {
    if (ep >= 0) {
      epilogue(ep);
      ep = -1;
      after_epi = D;
    }
    if (s == nsteps) break;
    // stage s landed: younger than it are the pieces of D - 1 later stages (+ the NSTORE
    // stores of an epilogue issued within the last D steps)
    if (after_epi > 0) { v3_wait_vmcnt((D - 1) * 4 + NSTORE); --after_epi; }
    else v3_wait_vmcnt((D - 1) * 4);
    v3_barrier();
    if (is_ks == 0) issue_bias();
    const Desc d = cursor_desc();
    {
      const char* st = ring + rslot * STAGE;
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
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NQ, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
    advance_cursor();
    rslot = (rslot + 1 == NST) ? 0 : rslot + 1;
    if (ks == ksteps - 1) ep = vt;
    if (++ks == ksteps) { ks = 0; ++vt; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // zero-record tail pieces and stores
}

}  // namespace hcr
