// gemm_ws.h — weight-stationary encoder projection GEMM ("WS") for the fast modes (f16 / bf16
// operands, fp32 accumulation), K = 384 or 768, 16-bit outputs with bias (+ GELU): the QKV and
// FFN1 projections of a BERT layer, C[token][feature] = X[token][:] . W[feature][:] + bias.
//
// Why.  gemm_v4_kernel fills a 256-feature AND a 256-token tile into LDS for every 32-deep
// stage (32 KiB of LDS-DMA per 4.2 MFLOP): at K = 768 its main loop is fill-bound like the v4
// score kernel was (QKV ~800 TF/s).  WS does for the encoder what QW did for the
// score: the workgroup holds 256 features x the whole K of W in its registers -- 8 waves x 32
// features, 2 x KS MFMA fragments per wave (192 VGPRs at K = 768) -- and streams only tokens:
// a stage is SR tokens x K (48 KiB: SR = 32 at K = 768, 64 at K = 384) through a 3-deep LDS-DMA
// ring, one barrier per stage, the v3 LDS image (1 KiB pieces of 16 tokens x 32 k).
//
//  * W fragments are the MFMA A operand and token fragments the B operand, so a lane's
//    accumulator holds 4 CONSECUTIVE features of one token: one 8-byte store per 16x16 block;
//  * the epilogue of stage s (bias from LDS, GELU, pack to 16 bits) runs after its MFMAs, but
//    its stores are issued in stage s + 1, after that stage's barrier and DMA issue: a store is
//    vmcnt-counted like the ring's LDS-DMA and may retire out of order with loads, so a store
//    issued just before the next stage's counted wait would hold that wait (and every wave's
//    barrier) for its write acknowledgement; issued a stage earlier it has retired by then;
//  * grid: nft feature tiles x P token partitions (XCD-aware: the nft tiles of a partition are
//    consecutive workgroups of one XCD and share its token stream in L2), one workgroup per CU.
// Rows of W are padded to a multiple of 768 (>= nft x 256) with zeros; X has Tp (a multiple of
// 256) rows; outputs past N_real / T_real are not written.
#pragma once
#include "gemm_v4.h"
#include "score_qw.h"

namespace hcr {

constexpr int WS_FT = 256;                        // features per workgroup (8 waves x 32)
constexpr int WS_NST = 3;                         // ring stages
constexpr int ws_sr(int ks) { return ks == 24 ? 32 : ks == 12 ? 64 : 0; }   // tokens per stage

template <typename TM, int EPI, int KS>
__global__ void __launch_bounds__(V3_NT, 1)
gemm_ws_kernel(const TM* __restrict__ W, const TM* __restrict__ X, int K, int N_real, int T_real,
               int nft, int P, int ntiles, const float* __restrict__ bias, TM* __restrict__ out_h,
               int ldo, float oscale) {
  static_assert(EPI == EPI_BIAS || EPI == EPI_BIAS_GELU, "16-bit output epilogues");
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int SR = ws_sr(KS), RB = SR / 16, NST = WS_NST, D = NST - 1;
  constexpr int PIECES = RB * KS, OPS = PIECES / 8, STAGE = PIECES * 1024;
  constexpr int NG = (RB / 2) * KS;               // groups: (token-block pair, k-step)
  constexpr int FD = 3;                           // fragment groups in flight
  constexpr int BIAS = NST * STAGE;               // fp32 bias of the workgroup's 256 features
  static_assert(SR > 0 && RB % 2 == 0 && PIECES % 8 == 0, "WS stage shape");
  static_assert(BIAS + WS_FT * 4 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char lds[BIAS + WS_FT * 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int ft = g % nft, p = g / nft;
  const int t0 = (int)((int64_t)p * ntiles / P);
  const int t1 = (int)((int64_t)(p + 1) * ntiles / P);
  if (t0 >= t1) return;                           // (the whole workgroup, before any barrier)
  const int f0 = ft * WS_FT;
  const int fw = f0 + wave * 32;                  // the wave's first feature

  // bias of the workgroup's features into LDS (read back per stage: no VGPRs held)
  if (tid < WS_FT / 4) {
    const int f = f0 + tid * 4;
    const float4 v = f < N_real ? *reinterpret_cast<const float4*>(bias + f) : float4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<float4*>(lds + BIAS + tid * 16) = v;
  }

  // weight fragments: lane l holds W[fw + 16 n + (l & 15)][32 ks + 8 (l >> 4) .. + 8)
  V wf[2][KS];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const TM* src = W + (size_t)(fw + 16 * n + (lane & 15)) * K + (lane >> 4) * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wf[n][ks] = *reinterpret_cast<const V*>(src + ks * 32);
  }
  // landed before the ring starts, and re-defined here: the compiler otherwise places its
  // first-use waits for these loads inside the stage loop, where their counts would hold the
  // in-flight ring stages
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(wf[n][ks]));

  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ (int)((V3_SWZ >> (((lane >> 4) & 3) * 4)) & 3u);
  const int ldb = K * 2;
  const int voff = drow * ldb + dchunk * 16;
  const char* x_b = reinterpret_cast<const char*>(X);
  const int nsteps = t1 - t0;
  // stage i (token tile t0 + i) into ring slot i % NST: this wave's OPS pieces (piece j = wave
  // + 8 u: token block j / KS, k-step j % KS); stages past the partition through zero-record
  // descriptors (nothing loaded, every stage costs every wave exactly OPS counted ops)
  auto issue_stage = [&](int i) __attribute__((always_inline)) {
    const bool live = i < nsteps;
    const int slot = __builtin_amdgcn_readfirstlane(i % NST);
    const int tile = __builtin_amdgcn_readfirstlane(t0 + (live ? i : 0));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        uniform_ptr(x_b + (size_t)tile * SR * ldb), (short)0, live ? SR * ldb : 0, 0x00020000);
#pragma unroll
    for (int u = 0; u < OPS; ++u) {
      const int j = wave + 8 * u;
      dma16(rs, lds + slot * STAGE + j * 1024, voff, (j / KS) * 16 * ldb + (j % KS) * (V3_BK * 2));
    }
  };
  for (int i = 0; i < D; ++i) issue_stage(i);

  const uint32_t offA = (uint32_t)((lane & 15) * 64 + v3_slot(lane >> 4, lane & 15) * 16);
  const uint32_t lds0 = lds_addr(lds);
  // the previous stage's outputs, packed: block (token block m, feature block n)
  uint2 pend[RB][2];
  auto store_pending = [&](int sp) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < RB; ++m) {
      const int t = (t0 + sp) * SR + m * 16 + (lane & 15);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int f = fw + 16 * n + 4 * (lane >> 4);
        if (t < T_real && f < N_real) *reinterpret_cast<uint2*>(out_h + (size_t)t * ldo + f) = pend[m][n];
      }
    }
  };

  for (int s = 0; s < nsteps; ++s) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS * (D - 1)) : "memory");
    v3_barrier();                  // everyone's pieces of stage s; everyone done with slot s-1
    issue_stage(s + D);
    if (s > 0) store_pending(s - 1);

    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)((s % NST) * STAGE)));
    floatx4 acc[RB][2];
#pragma unroll
    for (int m = 0; m < RB; ++m) acc[m][0] = acc[m][1] = floatx4{0.f, 0.f, 0.f, 0.f};
    // group j: token blocks 2 (j / KS), +1 at k-step j % KS
    auto gbase = [&](int j) { return st + (uint32_t)((2 * (j / KS) * KS + j % KS) * 1024); };
    V av[FD][2];
#pragma unroll
    for (int j = 0; j < FD - 1; ++j) qw_issue_frags<KS, V>(gbase(j), offA, av[j]);
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      if (j + FD - 1 < NG) {
        qw_issue_frags<KS, V>(gbase(j + FD - 1), offA, av[(j + FD - 1) % FD]);
        qw_frag_wait<2 * (FD - 1)>(av[j % FD]);
      } else if (j + 1 < NG) {
        qw_frag_wait<2>(av[j % FD]);
      } else {
        qw_frag_wait<0>(av[j % FD]);
      }
      const int m0 = 2 * (j / KS), k0 = j % KS;
#pragma unroll
      for (int mm = 0; mm < 2; ++mm)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m0 + mm][n] = Op::run(wf[n][k0], av[j % FD][mm], acc[m0 + mm][n]);
    }

    // epilogue of stage s: lane holds features fw + 16 n + 4 (l >> 4) + r of token (l & 15)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      // (asm read: a compiler-visible LDS read after the ring's LDS-DMA makes it drain vmcnt)
      const float4 bb = lds_read_f4_now(lds + BIAS + (wave * 32 + 16 * n + 4 * (lane >> 4)) * 4);
#pragma unroll
      for (int m = 0; m < RB; ++m) {
        float v[4] = {fmaf(acc[m][n][0], oscale, bb.x), fmaf(acc[m][n][1], oscale, bb.y),
                      fmaf(acc[m][n][2], oscale, bb.z), fmaf(acc[m][n][3], oscale, bb.w)};
        union { TM e[4]; uint2 u; } ph;
#pragma unroll
        for (int r = 0; r < 4; ++r) ph.e[r] = (TM)(EPI == EPI_BIAS_GELU ? gelu_erf(v[r]) : v[r]);
        pend[m][n] = ph.u;
      }
    }
  }
  store_pending(nsteps - 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tail pieces retired before exit
}

}  // namespace hcr
