// gemm_v4.h — encoder projection GEMM on the LDS-DMA ring of the v4 score kernel
// (score_v4.h): C[token][feature] = X[token][:] · W[feature][:] + bias (+ GELU | + residual).
//
// Fast modes (f16 / bf16 operands).  The reference-precision mode's split operands run on
// gemm_split_kernel below; `oscale` undoes the split's 2^11 and the weights' power-of-two scale
// (1 in the fast modes: fma(acc, 1, bias) = acc + bias exactly).
//
// One workgroup = one 256-feature x 256-token output tile over the whole K; 8 waves (2 x 4),
// each 128 features x 64 tokens as 8 x 4 16x16x32 MFMA blocks; K = 32 per stage, NST-stage
// LDS-DMA ring with the 4 DMA pieces of stage s + NST - 1 interleaved between the MFMA groups
// of stage s.  Weights as HF nn.Linear stores them ([out][in], K contiguous), rows padded to a
// multiple of 256 with zeros; activations [Tp][K] with Tp a multiple of 256 (rows past T are
// never written out).  Replaces the register-staged 128 x 128 gemm_nt_kernel on gfx950.
#pragma once
#include <type_traits>
#include "encoder_kernels.h"
#include "ring_common.h"

namespace hcr {

constexpr int G4_T = 256;     // features and tokens per tile

// Output epilogues staged through LDS (the tile's ring, idle after the main loop): from the
// accumulators a lane holds 4 features of one token, so a direct store covers 16 rows x 16 B
// (fp32) or 16 rows x 8 B (16-bit) per instruction; staged, each wave writes its tile's rows as
// 128-B (fp32) or 64-B (16-bit) pieces.  Per chunk of 2 row blocks a wave stages 32 features x
// 64 tokens in its own `vs` (8 KiB; 16-B granules XOR-swizzled by token), then reads back 8
// (fp32) or 16 (16-bit) rows per instruction.  fbase / tbase: the wave's first feature / token.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int EPI, int MT>
__device__ __forceinline__ void staged_epilogue_f32(char* vs, int lane, const floatx4 (&acc)[MT][4],
                                                    int fbase, int tbase, int N_real, int T_real,
                                                    const float* __restrict__ bias,
                                                    const float* __restrict__ resid,
                                                    float* __restrict__ out_f, int ldo, float oscale) {
#pragma unroll
  for (int c = 0; c < MT / 2; ++c) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int m = 2 * c + mi;
      const int fl = mi * 16 + (lane >> 4) * 4;
      const float4 bb = *reinterpret_cast<const float4*>(bias + min(fbase + c * 32 + fl, N_real - 4));
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int tl = n * 16 + (lane & 15);
        const float4 v = {fmaf(acc[m][n][0], oscale, bb.x), fmaf(acc[m][n][1], oscale, bb.y),
                          fmaf(acc[m][n][2], oscale, bb.z), fmaf(acc[m][n][3], oscale, bb.w)};
        *reinterpret_cast<float4*>(vs + tl * 128 + (((fl >> 2) ^ (tl & 7)) << 4)) = v;
      }
    }
    wave_lds_sync();
    const int gr = lane & 7;
    const int fcol = fbase + c * 32 + gr * 4;
    // the 8 rows' residual pieces loaded together (one wait), clamped into the matrix
    float4 rr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = tbase + i * 8 + (lane >> 3);
      rr[i] = float4{0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_BIAS_RESID)
        rr[i] = *reinterpret_cast<const float4*>(resid + (size_t)min(t, T_real - 1) * ldo +
                                                 min(fcol, N_real - 4));
      if constexpr (EPI == EPI_BIAS_RESID_XH) {
        // the residual stream as the LayerNorm left it in the split activations: h + l 2^-11
        // ([T][3 ldo] f16, h at column f, l at 2 ldo + f; |x - h - l 2^-11| <= |x| 2^-23)
        const _Float16* xr = reinterpret_cast<const _Float16*>(resid) + (size_t)min(t, T_real - 1) * 3 * ldo +
                             min(fcol, N_real - 4);
        union { uint2 u; _Float16 e[4]; } h, l;
        h.u = *reinterpret_cast<const uint2*>(xr);
        l.u = *reinterpret_cast<const uint2*>(xr + 2 * ldo);
        constexpr float r = 1.f / kSplitLo;
        rr[i] = float4{fmaf((float)l.e[0], r, (float)h.e[0]), fmaf((float)l.e[1], r, (float)h.e[1]),
                       fmaf((float)l.e[2], r, (float)h.e[2]), fmaf((float)l.e[3], r, (float)h.e[3])};
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int tl = i * 8 + (lane >> 3);
      const int t = tbase + tl;
      float4 v = *reinterpret_cast<const float4*>(vs + tl * 128 + ((gr ^ (tl & 7)) << 4));
      if (t < T_real && fcol < N_real) {
        v.x += rr[i].x; v.y += rr[i].y; v.z += rr[i].z; v.w += rr[i].w;
        *reinterpret_cast<float4*>(out_f + (size_t)t * ldo + fcol) = v;
      }
    }
    wave_lds_sync();
  }
}
template <typename TM, bool GELU, int MT>
__device__ __forceinline__ void staged_epilogue_h(char* vs, int lane, const floatx4 (&acc)[MT][4],
                                                  int fbase, int tbase, int N_real, int T_real,
                                                  const float* __restrict__ bias,
                                                  TM* __restrict__ out_h, int ldo, float oscale) {
#pragma unroll
  for (int c = 0; c < MT / 2; ++c) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int m = 2 * c + mi;
      const int fl = mi * 16 + (lane >> 4) * 4;              // 4 features = half a 16-B granule
      const float4 bb = *reinterpret_cast<const float4*>(bias + min(fbase + c * 32 + fl, N_real - 4));
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int tl = n * 16 + (lane & 15);
        float v[4] = {fmaf(acc[m][n][0], oscale, bb.x), fmaf(acc[m][n][1], oscale, bb.y),
                      fmaf(acc[m][n][2], oscale, bb.z), fmaf(acc[m][n][3], oscale, bb.w)};
        union { TM e[4]; uint2 u; } ph;
#pragma unroll
        for (int r = 0; r < 4; ++r) ph.e[r] = (TM)(GELU ? gelu_erf(v[r]) : v[r]);
        *reinterpret_cast<uint2*>(vs + tl * 64 + (((fl >> 3) ^ (tl & 3)) << 4) + (fl & 7) * 2) = ph.u;
      }
    }
    wave_lds_sync();
    const int gr = lane & 3;
    const int fcol = fbase + c * 32 + gr * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int tl = i * 16 + (lane >> 2);
      const int t = tbase + tl;
      const uint4 v = *reinterpret_cast<const uint4*>(vs + tl * 64 + ((gr ^ (tl & 3)) << 4));
      if (t < T_real && fcol < N_real) *reinterpret_cast<uint4*>(out_h + (size_t)t * ldo + fcol) = v;
    }
    wave_lds_sync();
  }
}

// FT = features per tile: 256 (8 row blocks per wave) or 192 (6), the latter for N = 768 /
// 2304 where 256-wide tiles leave the last round of workgroups half empty (1.5 and 4.5 rounds
// of 256 CUs at T = 32768 tokens).
template <typename TM, int EPI, int NST, int FT>
__global__ void __launch_bounds__(V3_NT, 2)
gemm_v4_kernel(const TM* __restrict__ W, const TM* __restrict__ X, int K, int N_real, int T_real,
               int n_tiles_feat, const float* __restrict__ bias, const float* __restrict__ resid,
               TM* __restrict__ out_h, float* __restrict__ out_f, int ldo, float oscale) {
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  static_assert(FT == 256 || FT == 192, "feature tile");
  constexpr int STAGE = (FT + G4_T) * 64;   // W rows then X rows, 64 B each
  constexpr int A_BYTES = FT * 64;
  constexpr int MT = FT / 32, NQ = 4, WN = 4, D = NST - 1;
  constexpr int NA = FT / 16, NP = NA + G4_T / 16;   // 1 KiB DMA pieces per stage
  __shared__ __attribute__((aligned(16))) char ring[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware: consecutive g share the token tile (X) and run on one XCD
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int ft = g % n_tiles_feat, tt = g / n_tiles_feat;
  const int f0 = ft * FT, t0 = tt * G4_T;

  const int ldb = K * 2;
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int voff = drow * ldb + dchunk * 16;
  const int nsteps = K / V3_BK;
  const __amdgpu_buffer_rsrc_t w_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(W) + (size_t)f0 * ldb), (short)0, FT * ldb, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(X) + (size_t)t0 * ldb), (short)0, G4_T * ldb, 0x00020000);
  // zero-record descriptors for the tail stages (their LDS writes land in a consumed slot)
  const __amdgpu_buffer_rsrc_t w_null = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(W), (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_null = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(X), (short)0, 0, 0x00020000);

  int is_s = 0, is_slot = 0;
  auto issue_piece = [&](int i) __attribute__((always_inline)) {
    const bool live = is_s < nsteps;
    const int kofs = __builtin_amdgcn_readfirstlane(is_s * (V3_BK * 2));
    char* sa = ring + __builtin_amdgcn_readfirstlane(is_slot) * STAGE;
    // piece kinds fixed per slot i (no runtime choice between the W and X descriptors: a
    // divergent-looking select of buffer descriptors is lowered to a stack table + waterfall):
    // i = 0 / 1 -> W pieces wave / wave + 8 (the latter only below NA), i = 2 / 3 -> X pieces
    if (i < 2) {
      const int j = wave + 8 * i;
      if (NA == 16 || j < NA) dma16(live ? w_rsrc : w_null, sa + j * 1024, voff, j * 16 * ldb + kofs);
    } else {
      const int j = wave + 8 * (i - 2);
      dma16(live ? x_rsrc : x_null, sa + A_BYTES + j * 1024, voff, j * 16 * ldb + kofs);
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    ++is_s;
    is_slot = (is_slot + 1 == NST) ? 0 : is_slot + 1;
  };
  for (int i = 0; i < D; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) issue_piece(k);
    advance();
  }

  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = v3_slot(fc, fr);
  const int offA = (wm * (FT / 2) + fr) * 64 + fslot * 16;
  const int offB = A_BYTES + (wn * 64 + fr) * 64 + fslot * 16;
  floatx4 acc[MT][NQ];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int my_pieces = (wave + 8 < NA) ? 4 : 3;   // 4 (3 for waves 4-7 at FT = 192)
  int rslot = 0;
  for (int s = 0; s < nsteps; ++s) {
    // constant immediates only (a runtime count would become a jump table on scratch)
    if (NP == 32 || my_pieces == 4) v3_wait_vmcnt((D - 1) * 4);
    else v3_wait_vmcnt((D - 1) * 3);
    v3_barrier();
    const char* st = ring + rslot * STAGE;
    V bq[NQ], av[MT];
    if constexpr (MT == 8) v4_read_frags<V>(lds_addr(st + offA), lds_addr(st + offB), av, bq);
    else v4_read_frags6<V>(lds_addr(st + offA), lds_addr(st + offB), av, bq);
    // MFMA groups between the 4 DMA pieces: row blocks [i*MT/4, (i+1)*MT/4)
    auto group = [&](auto lo_c, auto hi_c) __attribute__((always_inline)) {
      constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
#pragma unroll
      for (int m = LO; m < HI; ++m)
#pragma unroll
        for (int n = 0; n < NQ; ++n) acc[m][n] = Op::run(av[m], bq[n], acc[m][n]);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, MT / 4>;
    using I2 = std::integral_constant<int, (2 * MT) / 4>;
    using I3 = std::integral_constant<int, (3 * MT) / 4>;
    using I4 = std::integral_constant<int, MT>;
    group(I0{}, I1{});
    issue_piece(0);
    group(I1{}, I2{});
    issue_piece(1);
    group(I2{}, I3{});
    issue_piece(2);
    group(I3{}, I4{});
    issue_piece(3);
    constexpr int G0 = (MT / 4) * NQ, G1 = ((2 * MT) / 4 - MT / 4) * NQ;
    constexpr int G2 = ((3 * MT) / 4 - (2 * MT) / 4) * NQ, G3 = (MT - (3 * MT) / 4) * NQ;
    __builtin_amdgcn_sched_group_barrier(0x008, G0, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, G1, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, G2, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, G3, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    advance();
    rslot = (rslot + 1 == NST) ? 0 : rslot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tail pieces retired before exit

  if constexpr (EPI != EPI_BIAS_GELU_SPLIT) {
    __syncthreads();                                 // every wave done with the ring
    char* vs = ring + wave * 8192;
    if constexpr (EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_F32)
      staged_epilogue_f32<EPI, MT>(vs, lane, acc, f0 + wm * (FT / 2), t0 + wn * 64, N_real, T_real,
                                   bias, resid, out_f, ldo, oscale);
    else
      staged_epilogue_h<TM, EPI == EPI_BIAS_GELU, MT>(vs, lane, acc, f0 + wm * (FT / 2), t0 + wn * 64,
                                                      N_real, T_real, bias, out_h, ldo, oscale);
    return;
  }

  // epilogue: lane holds features f..f+3 of token t for each (m, n) block
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int f = f0 + wm * (FT / 2) + m * 16 + (lane >> 4) * 4;
    if (f >= N_real) continue;           // N_real % 4 == 0 (host-checked)
    const float4 bb = *reinterpret_cast<const float4*>(bias + f);
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      const int t = t0 + wn * 64 + n * 16 + (lane & 15);
      if (t >= T_real) continue;
      float v0 = fmaf(acc[m][n][0], oscale, bb.x), v1 = fmaf(acc[m][n][1], oscale, bb.y);
      float v2 = fmaf(acc[m][n][2], oscale, bb.z), v3 = fmaf(acc[m][n][3], oscale, bb.w);
      if constexpr (EPI == EPI_BIAS_GELU) {
        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
      }
      if constexpr (EPI == EPI_BIAS_GELU_SPLIT) {
        v0 = gelu_exact(v0); v1 = gelu_exact(v1); v2 = gelu_exact(v2); v3 = gelu_exact(v3);
        store_act4<TM, true>(out_h + (size_t)t * 3 * ldo, ldo, f, float4{v0, v1, v2, v3});
      } else if constexpr (EPI == EPI_BIAS_RESID) {
        const float4 rr = *reinterpret_cast<const float4*>(resid + (size_t)t * ldo + f);
        float4 o;
        o.x = v0 + rr.x; o.y = v1 + rr.y; o.z = v2 + rr.z; o.w = v3 + rr.w;
        *reinterpret_cast<float4*>(out_f + (size_t)t * ldo + f) = o;
      } else if constexpr (EPI == EPI_BIAS_F32) {
        *reinterpret_cast<float4*>(out_f + (size_t)t * ldo + f) = float4{v0, v1, v2, v3};
      } else {
        store_act4<TM, false>(out_h + (size_t)t * ldo, ldo, f, float4{v0, v1, v2, v3});
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Reference-precision GEMM without duplicated operand tiles.  The split operands are stored
// X' = [Xh | - | Xl 2^11] and W' = [Wh 2^11 | Wl 2^11 | Wh] (row length 3K); run as one GEMM of
// depth 3K over [Xh | Xh | Xl'] they needed 6 tiles (Xh and Wh twice) for 3 products.  Here a
// 32-deep stage fills the 4 distinct tiles -- Wh (segment 2), Wl 2^11 (segment 1), Xh (segment
// 0), Xl 2^11 (segment 2) -- and runs the 3 products from them: Xl'.Wh, then Xh.(Wh 2^11) with
// the Wh fragments scaled by 2^11 in registers (exact: |Wh| <= 16 after the upload's power-of-
// two scale, so |Wh 2^11| <= 32768 < 65504), then Xh.Wl'.  Every product carries the same 2^11
// as gemm_v4_kernel's, so `oscale` and the epilogues are unchanged.  LDS fill per MFMA flop is
// 2/3 of the concatenated form (64 KiB per 3 x 256 x 256 x 32 products), 2 x 64 KiB ring.
// 256-feature x 256-token tiles, 8 waves as gemm_v4_kernel (same fragment images and epilogue).
__device__ __forceinline__ void g5_read4(uint32_t b, half8 (&bq)[4]) {
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:1024\n\t"
      "ds_read_b128 %2, %4 offset:2048\n\t"
      "ds_read_b128 %3, %4 offset:3072\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(bq[0]), "=&v"(bq[1]), "=&v"(bq[2]), "=&v"(bq[3])
      : "v"(b)
      : "memory");
}
__device__ __forceinline__ void g5_read8(uint32_t a, half8 (&av)[8]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\t"
      "ds_read_b128 %1, %8 offset:1024\n\t"
      "ds_read_b128 %2, %8 offset:2048\n\t"
      "ds_read_b128 %3, %8 offset:3072\n\t"
      "ds_read_b128 %4, %8 offset:4096\n\t"
      "ds_read_b128 %5, %8 offset:5120\n\t"
      "ds_read_b128 %6, %8 offset:6144\n\t"
      "ds_read_b128 %7, %8 offset:7168\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]),
        "=&v"(av[6]), "=&v"(av[7])
      : "v"(a)
      : "memory");
}

// every fragment of a stage (Wh, Wl', Xh, Xl'), one wait: DM = 3 reads the whole stage into
// registers before its second barrier, which frees the slot for the stage after next
template <int MT>
__device__ __forceinline__ void g5_read_stage(uint32_t wh, uint32_t wl, uint32_t xh, uint32_t xl, half8 (&av)[MT],
                                              half8 (&aw)[MT], half8 (&bq)[4], half8 (&bl)[4]) {
  if constexpr (MT == 8) {
    asm volatile(
        "ds_read_b128 %0, %24\n\t"
        "ds_read_b128 %1, %24 offset:1024\n\t"
        "ds_read_b128 %2, %24 offset:2048\n\t"
        "ds_read_b128 %3, %24 offset:3072\n\t"
        "ds_read_b128 %4, %24 offset:4096\n\t"
        "ds_read_b128 %5, %24 offset:5120\n\t"
        "ds_read_b128 %6, %24 offset:6144\n\t"
        "ds_read_b128 %7, %24 offset:7168\n\t"
        "ds_read_b128 %16, %26\n\t"
        "ds_read_b128 %17, %26 offset:1024\n\t"
        "ds_read_b128 %18, %26 offset:2048\n\t"
        "ds_read_b128 %19, %26 offset:3072\n\t"
        "ds_read_b128 %20, %27\n\t"
        "ds_read_b128 %21, %27 offset:1024\n\t"
        "ds_read_b128 %22, %27 offset:2048\n\t"
        "ds_read_b128 %23, %27 offset:3072\n\t"
        "ds_read_b128 %8, %25\n\t"
        "ds_read_b128 %9, %25 offset:1024\n\t"
        "ds_read_b128 %10, %25 offset:2048\n\t"
        "ds_read_b128 %11, %25 offset:3072\n\t"
        "ds_read_b128 %12, %25 offset:4096\n\t"
        "ds_read_b128 %13, %25 offset:5120\n\t"
        "ds_read_b128 %14, %25 offset:6144\n\t"
        "ds_read_b128 %15, %25 offset:7168\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]), "=&v"(av[6]),
          "=&v"(av[7]), "=&v"(aw[0]), "=&v"(aw[1]), "=&v"(aw[2]), "=&v"(aw[3]), "=&v"(aw[4]), "=&v"(aw[5]),
          "=&v"(aw[6]), "=&v"(aw[7]), "=&v"(bq[0]), "=&v"(bq[1]), "=&v"(bq[2]), "=&v"(bq[3]), "=&v"(bl[0]),
          "=&v"(bl[1]), "=&v"(bl[2]), "=&v"(bl[3])
        : "v"(wh), "v"(wl), "v"(xh), "v"(xl)
        : "memory");
  } else {
    static_assert(MT == 6, "row blocks per wave");
    asm volatile(
        "ds_read_b128 %0, %20\n\t"
        "ds_read_b128 %1, %20 offset:1024\n\t"
        "ds_read_b128 %2, %20 offset:2048\n\t"
        "ds_read_b128 %3, %20 offset:3072\n\t"
        "ds_read_b128 %4, %20 offset:4096\n\t"
        "ds_read_b128 %5, %20 offset:5120\n\t"
        "ds_read_b128 %12, %22\n\t"
        "ds_read_b128 %13, %22 offset:1024\n\t"
        "ds_read_b128 %14, %22 offset:2048\n\t"
        "ds_read_b128 %15, %22 offset:3072\n\t"
        "ds_read_b128 %16, %23\n\t"
        "ds_read_b128 %17, %23 offset:1024\n\t"
        "ds_read_b128 %18, %23 offset:2048\n\t"
        "ds_read_b128 %19, %23 offset:3072\n\t"
        "ds_read_b128 %6, %21\n\t"
        "ds_read_b128 %7, %21 offset:1024\n\t"
        "ds_read_b128 %8, %21 offset:2048\n\t"
        "ds_read_b128 %9, %21 offset:3072\n\t"
        "ds_read_b128 %10, %21 offset:4096\n\t"
        "ds_read_b128 %11, %21 offset:5120\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]), "=&v"(aw[0]),
          "=&v"(aw[1]), "=&v"(aw[2]), "=&v"(aw[3]), "=&v"(aw[4]), "=&v"(aw[5]), "=&v"(bq[0]), "=&v"(bq[1]),
          "=&v"(bq[2]), "=&v"(bq[3]), "=&v"(bl[0]), "=&v"(bl[1]), "=&v"(bl[2]), "=&v"(bl[3])
        : "v"(wh), "v"(wl), "v"(xh), "v"(xl)
        : "memory");
  }
}

// FT = 256, or 192 for N = 768 (4 x 128 tiles at T = 32768 fill 2 rounds of 256 CUs exactly;
// 256-feature tiles leave the second of 2 rounds half empty).
__device__ __forceinline__ void g5_read6(uint32_t a, half8 (&av)[6]) {
  asm volatile(
      "ds_read_b128 %0, %6\n\t"
      "ds_read_b128 %1, %6 offset:1024\n\t"
      "ds_read_b128 %2, %6 offset:2048\n\t"
      "ds_read_b128 %3, %6 offset:3072\n\t"
      "ds_read_b128 %4, %6 offset:4096\n\t"
      "ds_read_b128 %5, %6 offset:5120\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5])
      : "v"(a)
      : "memory");
}

// Split of the last round (the reference-precision mode's wave quantization: at bge-base T ~
// 24.6k packed tokens O-proj / FFN2 are 384 192-wide tiles -- a full round of 256 CUs and a
// second of 128 -- and QKV / FFN1 1152: 4 rounds and a half).  The R tiles left after the full
// rounds run as s K-chunks each (s = ncu / R, at most 8), one workgroup per chunk, all in one
// round: chunk c of a tile takes K steps [c n / s, (c + 1) n / s).  The chunks of every tile
// run at the same time, so workgroups that share a token tile's activations read each K chunk
// of them together (one fetch from HBM, the rest from L2) -- what a stream-K split over a
// linear (tile, k) order lost (r04n).  Every chunk stores its fp32 accumulators to the tile's
// slab c (write-through), drains, and draws a ticket; the tile's last arriver sums slabs 0 ..
// s-1 in that order (the result does not depend on the arrival order) and runs the epilogue,
// and resets the counter for the next launch (zeroed once when allocated).  No workgroup waits
// for another: no residency is assumed.
typedef __attribute__((address_space(1))) uint32_t sk_gu32;
typedef uint32_t uint32x4 __attribute__((ext_vector_type(4)));

// slab image: the accumulators in register order, float4 (wave, m, n) per lane -- 1 KiB per
// instruction per wave both ways.  Returns true in the tile's last arriving workgroup, with acc
// = the sum of the tile's s chunks (in chunk order).
template <int MT>
__device__ __forceinline__ bool split_gather(floatx4 (&acc)[MT][4], char* ring, float* slabs, uint32_t* cnt,
                                             int chunk, int s, int tid) {
  constexpr int NQ = 4;
  constexpr int SLAB = MT * NQ * 256 * 8;          // floats per slab (8 waves)
  const int lane = tid & 63, wave = tid >> 6;
  float* mine = slabs + (size_t)chunk * SLAB + (size_t)wave * (MT * NQ * 256);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<char*>(mine)), (short)0, MT * NQ * 1024, 0x00020000);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      const floatx4 v = acc[m][n];
      __builtin_amdgcn_raw_buffer_store_b128(
          uint32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])},
          rs, ((m * NQ + n) * 64 + lane) * 16, 0, 16 /* sc1: write-through */);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();                                   // (and every wave is out of the ring)
  if (tid == 0)
    *reinterpret_cast<uint32_t*>(ring) = __hip_atomic_fetch_add((sk_gu32*)cnt, 1u, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t ticket = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(ring));
  if (ticket != (uint32_t)(s - 1)) return false;
  if (tid == 0) __hip_atomic_store((sk_gu32*)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // every slab byte was stored write-through (sc1) and drained before its ticket, and every load
  // of it below is an sc1 load (past this CU's L1): no agent-scope acquire, only the compiler
  // kept from hoisting the loads above the ticket
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float* base = slabs + (size_t)wave * (MT * NQ * 256) + lane * 4;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  // two slabs' pieces of a row block in flight at a time, added in chunk order
  int c = 0;
#pragma unroll 1
  for (; c + 1 < s; c += 2) {
    const float* src = base + (size_t)c * SLAB;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      floatx4 p0, p1, p2, p3, q0, q1, q2, q3;
      asm volatile(
          "global_load_dwordx4 %0, %8, off sc1\n\t"
          "global_load_dwordx4 %1, %8, off offset:1024 sc1\n\t"
          "global_load_dwordx4 %2, %8, off offset:2048 sc1\n\t"
          "global_load_dwordx4 %3, %8, off offset:3072 sc1\n\t"
          "global_load_dwordx4 %4, %9, off sc1\n\t"
          "global_load_dwordx4 %5, %9, off offset:1024 sc1\n\t"
          "global_load_dwordx4 %6, %9, off offset:2048 sc1\n\t"
          "global_load_dwordx4 %7, %9, off offset:3072 sc1\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3), "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3)
          : "v"(src + m * NQ * 256), "v"(src + SLAB + m * NQ * 256)
          : "memory");
      acc[m][0] += p0; acc[m][1] += p1; acc[m][2] += p2; acc[m][3] += p3;
      acc[m][0] += q0; acc[m][1] += q1; acc[m][2] += q2; acc[m][3] += q3;
    }
  }
  if (c < s) {
    const float* src = base + (size_t)c * SLAB;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      floatx4 p0, p1, p2, p3;
      asm volatile(
          "global_load_dwordx4 %0, %4, off sc1\n\t"
          "global_load_dwordx4 %1, %4, off offset:1024 sc1\n\t"
          "global_load_dwordx4 %2, %4, off offset:2048 sc1\n\t"
          "global_load_dwordx4 %3, %4, off offset:3072 sc1\n\t"
          "s_waitcnt vmcnt(0)"
          : "=&v"(p0), "=&v"(p1), "=&v"(p2), "=&v"(p3)
          : "v"(src + m * NQ * 256)
          : "memory");
      acc[m][0] += p0; acc[m][1] += p1; acc[m][2] += p2; acc[m][3] += p3;
    }
  }
  return true;
}

// FFN1 (reference-precision mode): the split activations (h, l) of a wave's 128 features x 64
// tokens go out through LDS.  Stored straight from the accumulators a lane writes 4 features of
// one token: 32-B pieces of 16 different rows per instruction, half-line writes on ~400 MB per
// launch.  Here the wave stages 64 features x 64 tokens of h and of l (8 KiB each, 16-B granules
// XOR-swizzled by token) in its 16 KiB at `hs`, then writes 128-B row pieces: 8 lanes per token
// row.  fbase / tbase: the wave's first feature / token.
template <bool LIBERF>
__device__ __forceinline__ void ffn1_split_epilogue(char* hs, int lane, const floatx4 (&acc)[8][4], int fbase,
                                                    int tbase, int N_real, int T_real,
                                                    const float* __restrict__ bias, _Float16* __restrict__ out_h,
                                                    int ldo, float oscale) {
  char* ls = hs + 8192;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = hh * 4 + mi;
      const int fl = mi * 16 + (lane >> 4) * 4;               // feature within the 64
      const float4 bb = *reinterpret_cast<const float4*>(bias + fbase + hh * 64 + fl);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int tl = n * 16 + (lane & 15);                  // token within the 64
        float v[4] = {fmaf(acc[m][n][0], oscale, bb.x), fmaf(acc[m][n][1], oscale, bb.y),
                      fmaf(acc[m][n][2], oscale, bb.z), fmaf(acc[m][n][3], oscale, bb.w)};
        union { _Float16 e[4]; uint2 u; } ph, pl;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = LIBERF ? gelu_exact(v[r]) : gelu_erf(v[r]);
          ph.e[r] = (_Float16)v[r];
          pl.e[r] = (_Float16)((v[r] - (float)ph.e[r]) * kSplitLo);
        }
        const int off = tl * 128 + (((fl >> 3) ^ (tl & 7)) << 4) + (fl & 7) * 2;
        *reinterpret_cast<uint2*>(hs + off) = ph.u;
        *reinterpret_cast<uint2*>(ls + off) = pl.u;
      }
    }
    wave_lds_sync();
    // 64 rows x 8 granules: 8 rows per instruction, lane -> (row lane / 8, granule lane % 8)
    const int gr = lane & 7;
    const int fcol = fbase + hh * 64 + gr * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int tl = i * 8 + (lane >> 3);
      const int t = tbase + tl;
      const int off = tl * 128 + ((gr ^ (tl & 7)) << 4);
      const uint4 h4 = *reinterpret_cast<const uint4*>(hs + off);
      const uint4 l4 = *reinterpret_cast<const uint4*>(ls + off);
      if (t < T_real && fcol < N_real) {
        _Float16* row = out_h + (size_t)t * 3 * ldo;
        *reinterpret_cast<uint4*>(row + fcol) = h4;
        *reinterpret_cast<uint4*>(row + 2 * ldo + fcol) = l4;
      }
    }
    wave_lds_sync();
  }
}

// LIBERF: the FFN1 epilogue's GELU with the library erff (~50 instructions) instead of erf_as
// (A&S 7.1.26, |error| <= 1.5e-7 + the rcp / exp2 approximations, ~12 instructions).
// SPLIT = false: one whole tile per workgroup (tile = the workgroup's XCD-remapped index);
// SPLIT = true: workgroup g is chunk g % nsplit of tile tile_base + g / nsplit (see above).
// DM: the stage pipeline.  0: one stage in flight -- a single barrier per stage, the pieces of
// stage s + 1 issued in three groups after the three products of stage s, vmcnt(0) at the next
// stage's top.  4 (the default, r06): two stages in flight -- after the stage barrier every wave
// reads the whole stage into registers (24 fragments), a second barrier frees the slot, and the
// pieces of the stage after next are spread evenly over all 3 MT NQ MFMAs of the stage (one per
// ~12), so the CU's vector-memory path sees an even demand.  r06 A/B (profiles/r06/, bge-base
// f32 encoder, 1024 x 32 ragged): DM 4 -1.2 % against DM 0; the placements tried in between --
// all pieces right after the barrier, all inside the first product, DM 4's structure with them
// inside the first product -- tied with DM 0, and without any stage DMA (a diagnostic with stale
// operands) the encoder ran only 11 % faster: the DMA is not what holds the split GEMM at ~0.5
// MFMA busy; the per-stage fragment reads and barriers of two waves per SIMD in lockstep are.
// A one-wave-per-SIMD form (4 waves of 128 x 128, 256 AGPR accumulators) measured 9 % slower;
// a staggered DM 4 (waves 4-7 deferring each stage's third product past the next barrier, so the
// two waves of a SIMD are not in their read phase together) needs the deferred fragments beside
// DM 4's registers: 832 B/lane of scratch, 36x slower (profiles/r06/r06g); DM 4 with the
// slot-freeing barrier moved into the MFMA phase (after the first or second product, so a wave
// starts its MFMAs as soon as its own fragments land) measured 1.5-2.5 % slower (r06j); a
// one-wave-per-SIMD kernel software-pipelined inside the wave (4 waves of 128 x 128, AGPR
// accumulators through tied inline-asm MFMAs, the next fragments' reads in flight under the
// current product, one barrier per stage) ran 13.84 ms against DM 4's 13.1 (r06k): that wave
// also issues all 16 LDS-DMA pieces of a stage, ~60-185 cycles each (MI355X_MICROARCH.md), with
// no partner wave to hide them; loader waves issuing all the DMA beside compute waves that only
// read and multiply (256 x 128 tiles, a 3-slot ring: bit-identical, 14.5 ms, r06p) fill at ~26
// GB/s per CU -- 6.7 TB/s chip-wide, where DM 4 runs at ~5 TB/s of L2 -> LDS fill with a third
// fewer bytes per flop -- none of these kept.
template <int EPI, int FT = G4_T, bool LIBERF = false, bool SPLIT = false, int DM = 0>
__global__ void __launch_bounds__(V3_NT, 1)
gemm_split_kernel(const _Float16* __restrict__ W, const _Float16* __restrict__ X, int K, int N_real,
                  int T_real, int n_tiles_feat, const float* __restrict__ bias,
                  const float* __restrict__ resid, _Float16* __restrict__ out_h,
                  float* __restrict__ out_f, int ldo, float oscale, int tile_base, int nsplit,
                  float* __restrict__ split_ws, uint32_t* __restrict__ split_cnt) {
  using Op = MfmaOp<_Float16>;
  using V = half8;
  static_assert(FT == 256 || FT == 192, "feature tile");
  constexpr int NST = 2;
  constexpr int REGW = FT * 64, REGX = G4_T * 64;   // one FT- / 256-row x 32-k tile
  constexpr int WH = 0, WL = REGW, XH = 2 * REGW, XL = 2 * REGW + REGX, STAGE = 2 * REGW + 2 * REGX;
  constexpr int MT = FT / 32, NQ = 4, WN = 4;
  constexpr int NPW = FT / 16;                      // pieces per W region (16 or 12)
  constexpr int PPW = (2 * NPW + 32) / 8;           // pieces per wave per stage (8 or 7)
  __shared__ __attribute__((aligned(16))) char ring[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int nsteps = K / V3_BK;
  int tile = g, ks0 = 0, ks1 = nsteps, chunk = 0;
  if constexpr (SPLIT) {
    const int t = g / nsplit;
    chunk = g - t * nsplit;
    tile = tile_base + t;
    ks0 = chunk * nsteps / nsplit;
    ks1 = (chunk + 1) * nsteps / nsplit;
  }
  tile = __builtin_amdgcn_readfirstlane(tile);
  ks0 = __builtin_amdgcn_readfirstlane(ks0);
  ks1 = __builtin_amdgcn_readfirstlane(ks1);
  const int ft = tile % n_tiles_feat, tt = tile / n_tiles_feat;
  const int f0 = ft * FT, t0 = tt * G4_T;

  const int ldb = 3 * K * 2;                   // bytes per split row
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int voff = drow * ldb + dchunk * 16;
  const __amdgpu_buffer_rsrc_t w_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(W) + (size_t)f0 * ldb), (short)0, FT * ldb, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(reinterpret_cast<const char*>(X) + (size_t)t0 * ldb), (short)0, G4_T * ldb, 0x00020000);
  const __amdgpu_buffer_rsrc_t w_null = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(W), (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_null = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(X), (short)0, 0, 0x00020000);

  // piece i (0 .. PPW-1) of this wave for stage `is`.  FT = 256: region i / 2 (Wh, Wl', Xh,
  // Xl'), 16-row block wave + 8 (i % 2).  FT = 192: i = 0 Wh block wave; i = 1 Wh block 8 +
  // wave (waves 0-3) or Wl block wave - 4 (waves 4-7: same W descriptor, a wave-uniform
  // choice of offsets); i = 2 Wl block 4 + wave; i = 3, 4 Xh; i = 5, 6 Xl.  The segment of the
  // split rows: Wh = 2, Wl' = 1, Xh = 0, Xl' = 2.
  auto issue_piece = [&](int is, int i) __attribute__((always_inline)) {
    const bool live = is < ks1;
    const int kofs = __builtin_amdgcn_readfirstlane(is * (V3_BK * 2));
    char* sa = ring + __builtin_amdgcn_readfirstlane(is & 1) * STAGE;
    int region, jb;
    if constexpr (FT == 256) {
      region = i >> 1;
      jb = wave + 8 * (i & 1);
    } else {
      if (i == 0) { region = 0; jb = wave; }
      else if (i == 1) { region = wave < 4 ? 0 : 1; jb = wave < 4 ? 8 + wave : wave - 4; }
      else if (i == 2) { region = 1; jb = 4 + wave; }
      else { region = 2 + (i - 3) / 2; jb = wave + 8 * ((i - 3) & 1); }
    }
    const int seg = region == 0 ? 2 : region == 1 ? 1 : region == 2 ? 0 : 2;
    const int rbase = region == 0 ? WH : region == 1 ? WL : region == 2 ? XH : XL;
    if (region < 2)
      dma16(live ? w_rsrc : w_null, sa + rbase + jb * 1024, voff, jb * 16 * ldb + seg * 2 * K + kofs);
    else
      dma16(live ? x_rsrc : x_null, sa + rbase + jb * 1024, voff, jb * 16 * ldb + seg * 2 * K + kofs);
  };
#pragma unroll
  for (int i = 0; i < PPW; ++i) issue_piece(ks0, i);
  if constexpr (DM >= 4) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) issue_piece(ks0 + 1, i);
  }
  const int fr = lane & 15, fc = lane >> 4;
  const int fslot = v3_slot(fc, fr);
  const int offA = (wm * (FT / 2) + fr) * 64 + fslot * 16;
  const int offB = (wn * 64 + fr) * 64 + fslot * 16;
  floatx4 acc[MT][NQ];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int s = ks0; s < ks1; ++s) {
    if constexpr (DM == 4) {
      // DM 3's two stages in flight with the PPW pieces spread evenly over all 3 x MT x NQ
      // MFMAs of the stage (one per ~12): the CU's vector-memory path sees an even demand
      // instead of a burst per product
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PPW) : "memory");
      v3_barrier();
      const char* st = ring + (s & 1) * STAGE;
      V av[MT], aw[MT], bq[NQ], bl[NQ];
      g5_read_stage<MT>(lds_addr(st + WH + offA), lds_addr(st + WL + offA), lds_addr(st + XH + offB),
                        lds_addr(st + XL + offB), av, aw, bq, bl);
      v3_barrier();
      V as[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) as[m] = av[m] * (_Float16)2048.0f;
      constexpr int NM = 3 * MT * NQ, GAP = NM / PPW;
#pragma unroll
      for (int u = 0; u < NM; ++u) {
        const int prod = u / (MT * NQ), m = (u / NQ) % MT, n = u % NQ;
        if (prod == 0) acc[m][n] = Op::run(av[m], bl[n], acc[m][n]);
        else if (prod == 1) acc[m][n] = Op::run(as[m], bq[n], acc[m][n]);
        else acc[m][n] = Op::run(aw[m], bq[n], acc[m][n]);
        if (u % GAP == GAP - 1 && u / GAP < PPW) issue_piece(s + 2, u / GAP);
      }
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, GAP, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      continue;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    v3_barrier();                 // stage s landed everywhere; everyone done with slot s-1
    const char* st = ring + (s & 1) * STAGE;
    V av[MT], bq[NQ], bl[NQ];
    if constexpr (MT == 8) g5_read8(lds_addr(st + WH + offA), av);
    else g5_read6(lds_addr(st + WH + offA), av);
    g5_read4(lds_addr(st + XL + offB), bl);
    g5_read4(lds_addr(st + XH + offB), bq);
    // Xl' . Wh
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = Op::run(av[m], bl[n], acc[m][n]);
    issue_piece(s + 1, 0);
    issue_piece(s + 1, 1);
    issue_piece(s + 1, 2);
    // Xh . (Wh 2^11): the fragments scaled in registers (exact power of two)
#pragma unroll
    for (int m = 0; m < MT; ++m) av[m] = av[m] * (_Float16)2048.0f;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = Op::run(av[m], bq[n], acc[m][n]);
    issue_piece(s + 1, 3);
    issue_piece(s + 1, 4);
    issue_piece(s + 1, 5);
    // Xh . Wl'
    if constexpr (MT == 8) g5_read8(lds_addr(st + WL + offA), av);
    else g5_read6(lds_addr(st + WL + offA), av);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NQ; ++n) acc[m][n] = Op::run(av[m], bq[n], acc[m][n]);
    issue_piece(s + 1, 6);
    if constexpr (PPW == 8) issue_piece(s + 1, 7);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if constexpr (SPLIT) {
    const int slot = tile - tile_base;
    if (!split_gather<MT>(acc, ring, split_ws + (size_t)slot * nsplit * (MT * NQ * 256 * 8),
                          split_cnt + slot, chunk, nsplit, tid))
      return;
  }

  if constexpr (EPI == EPI_BIAS_GELU_SPLIT) {
    static_assert(FT == 256, "the FFN1 epilogue stages 64-feature halves of a 128-feature wave");
    __syncthreads();                               // every wave done with the ring
    ffn1_split_epilogue<LIBERF>(ring + wave * 16384, lane, acc, f0 + wm * 128, t0 + wn * 64, N_real, T_real,
                                bias, out_h, ldo, oscale);
  } else {
    // fp32 outputs (QKV: bias; O / FFN2: bias + residual) through LDS as well
    static_assert(EPI == EPI_BIAS_F32 || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_RESID_XH, "split GEMM epilogues");
    __syncthreads();                               // every wave done with the ring
    staged_epilogue_f32<EPI, MT>(ring + wave * 8192, lane, acc, f0 + wm * (FT / 2), t0 + wn * 64,
                                 N_real, T_real, bias, resid, out_f, ldo, oscale);
  }
}

}  // namespace hcr
