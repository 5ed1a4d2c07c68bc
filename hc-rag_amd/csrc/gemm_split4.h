// gemm_split4.h — the reference-precision (split-f16) projection GEMM with ONE wave per SIMD
// (r06).  Same operands, products and epilogues as gemm_split_kernel
// (gemm_v4.h): X' = [Xh | - | Xl 2^11], W' = [Wh 2^11 | Wl 2^11 | Wh], C = oscale (Xl'.Wh +
// Xh.(Wh 2^11) + Xh.Wl') + bias (+ epilogue), 256-feature x 256-token tiles over the whole K,
// 32-deep stages of the 4 distinct tiles (Wh, Wl', Xh, Xl': 64 KiB) through a 2-slot LDS-DMA
// ring.  What changes is the wave layout:
//   * 4 waves (256 threads), one per SIMD, each 128 features x 128 tokens: 8 x 8 16x16x32 blocks,
//     256 accumulator registers (AGPRs) -- per stage 192 MFMAs (3072 cycles) from 32 fragment
//     reads, against gemm_split_kernel's two waves per SIMD of 96 MFMAs from 24 reads each;
//   * no partner wave on the SIMD, so the stage is software-pipelined inside the wave: the
//     first product's fragments (Wh, Xl') are read first and its 64 MFMAs run while Xh and Wl'
//     land; a second barrier after that product frees the stage's slot, and the 16 LDS-DMA
//     pieces of the stage after next are spread over the other two products' 128 MFMAs (one per
//     8): two stages in flight across the whole stage.
// r06 counters (profiles/r06/): gemm_split_kernel sat at 0.50-0.53 MFMA busy with 0.35-0.44 of
// the wave cycles parked at vmcnt / barrier whatever the DMA placement (DM 0-4); the vendor GEMM
// at 256 x 256 x 64 tiles runs 0.88.
#pragma once
#include "gemm_v4.h"

namespace hcr {

// 8 fragments (1 KiB apart) issued, no wait; g4_wait<N> waits until at most N LDS reads are
// outstanding and re-defines the registers so no use is scheduled above the wait
__device__ __forceinline__ void g4_issue8(uint32_t a, half8 (&v)[8]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\t"
      "ds_read_b128 %1, %8 offset:1024\n\t"
      "ds_read_b128 %2, %8 offset:2048\n\t"
      "ds_read_b128 %3, %8 offset:3072\n\t"
      "ds_read_b128 %4, %8 offset:4096\n\t"
      "ds_read_b128 %5, %8 offset:5120\n\t"
      "ds_read_b128 %6, %8 offset:6144\n\t"
      "ds_read_b128 %7, %8 offset:7168"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(a)
      : "memory");
}
template <int N>
__device__ __forceinline__ void g4_wait(half8 (&x)[8], half8 (&y)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%16)"
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                 "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7])
               : "n"(N)
               : "memory");
}

template <int EPI, bool LIBERF = false>
__global__ void __launch_bounds__(256, 1)
gemm_split4_kernel(const _Float16* __restrict__ W, const _Float16* __restrict__ X, int K, int N_real, int T_real,
                   int n_tiles_feat, const float* __restrict__ bias, const float* __restrict__ resid,
                   _Float16* __restrict__ out_h, float* __restrict__ out_f, int ldo, float oscale) {
  using Op = MfmaOp<_Float16>;
  using V = half8;
  constexpr int FT = 256, TT = 256, NST = 2;
  constexpr int REG = 256 * 64;                          // one 256-row x 32-k tile: 16 KiB
  constexpr int WH = 0, WL = REG, XH = 2 * REG, XL = 3 * REG, STAGE = 4 * REG;
  constexpr int PPW = 16;                                // DMA pieces per wave per stage
  __shared__ __attribute__((aligned(16))) char ring[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;               // features wm*128, tokens wn*128
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int ft = g % n_tiles_feat, tt = g / n_tiles_feat;
  const int f0 = ft * FT, t0 = tt * TT;
  const int nsteps = K / V3_BK;

  const int ldb = 3 * K * 2;                             // bytes per split row
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int voff = drow * ldb + dchunk * 16;
  const __amdgpu_buffer_rsrc_t w_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(W) + (size_t)f0 * ldb), (short)0, FT * ldb, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(X) + (size_t)t0 * ldb), (short)0, TT * ldb, 0x00020000);
  const __amdgpu_buffer_rsrc_t w_null = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(W), (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_null = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(X), (short)0, 0, 0x00020000);

  // piece i (0 .. 15) of this wave for stage `is`: region i / 4 (Wh, Wl', Xh, Xl'), 16-row block
  // wave + 4 (i % 4); the segment of the split rows: Wh = 2, Wl' = 1, Xh = 0, Xl' = 2.  Stages
  // past the K range go through zero-record descriptors (every stage is PPW counted ops).
  auto issue_piece = [&](int is, int i) __attribute__((always_inline)) {
    const bool live = is < nsteps;
    const int kofs = __builtin_amdgcn_readfirstlane(is * (V3_BK * 2));
    char* sa = ring + __builtin_amdgcn_readfirstlane(is & 1) * STAGE;
    const int region = i >> 2, jb = wave + 4 * (i & 3);
    const int seg = region == 0 ? 2 : region == 1 ? 1 : region == 2 ? 0 : 2;
    if (region < 2)
      dma16(live ? w_rsrc : w_null, sa + region * REG + jb * 1024, voff, jb * 16 * ldb + seg * 2 * K + kofs);
    else
      dma16(live ? x_rsrc : x_null, sa + region * REG + jb * 1024, voff, jb * 16 * ldb + seg * 2 * K + kofs);
  };
#pragma unroll
  for (int i = 0; i < PPW; ++i) issue_piece(0, i);
#pragma unroll
  for (int i = 0; i < PPW; ++i) issue_piece(1, i);

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = v3_slot(fc, fr);
  const uint32_t offA = (uint32_t)((wm * 128 + fr) * 64 + fslot * 16);
  const uint32_t offB = (uint32_t)((wn * 128 + fr) * 64 + fslot * 16);
  floatx4 acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  const uint32_t l0 = lds_addr(ring);

  for (int s = 0; s < nsteps; ++s) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW) : "memory");   // stage s landed (s + 1 in flight)
    v3_barrier();
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(l0 + (uint32_t)((s & 1) * STAGE)));
    V wh[8], xl[8], xh[8], wl[8];
    // (lgkmcnt counts at most 15: the first product's 16 fragments are waited for in full, the
    // other 16 are issued behind them and land under its MFMAs)
    g4_issue8(st + WH + offA, wh);
    g4_issue8(st + XL + offB, xl);
    g4_wait<0>(wh, xl);
    g4_issue8(st + XH + offB, xh);
    g4_issue8(st + WL + offA, wl);
    // Xl' . Wh
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[m][n] = Op::run(wh[m], xl[n], acc[m][n]);
    g4_wait<0>(xh, wl);
    v3_barrier();                    // every wave holds stage s in registers: its slot is free
#pragma unroll
    for (int m = 0; m < 8; ++m) wh[m] = wh[m] * (_Float16)2048.0f;
    // Xh . (Wh 2^11), then Xh . Wl', with the 16 pieces of stage s + 2 one per 8 MFMAs
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[m][n] = Op::run(wh[m], xh[n], acc[m][n]);
      issue_piece(s + 2, m);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[m][n] = Op::run(wl[m], xh[n], acc[m][n]);
      issue_piece(s + 2, 8 + m);
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                       // every wave done with the ring

  // epilogues: each wave's 128 tokens as two 64-token halves through the shared helpers (two
  // explicit calls: every index into acc must be a compile-time constant, or acc goes to scratch)
  auto epi_half = [&](auto hc) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
    floatx4 a4[8][4];
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) a4[m][n] = acc[m][4 * h + n];
    const int tbase = t0 + wn * 128 + h * 64;
    if constexpr (EPI == EPI_BIAS_GELU_SPLIT)
      ffn1_split_epilogue<LIBERF>(ring + wave * 32768, lane, a4, f0 + wm * 128, tbase, N_real, T_real, bias, out_h,
                                  ldo, oscale);
    else
      staged_epilogue_f32<EPI, 8>(ring + wave * 32768, lane, a4, f0 + wm * 128, tbase, N_real, T_real, bias, resid,
                                  out_f, ldo, oscale);
  };
  epi_half(std::integral_constant<int, 0>{});
  epi_half(std::integral_constant<int, 1>{});
}

}  // namespace hcr
