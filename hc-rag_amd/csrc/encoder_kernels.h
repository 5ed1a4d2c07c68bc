// encoder_kernels.h — HIP kernels of the BERT sentence-embedding forward (SURVEY.md §8(a)
// a8-a9: tokenise -> embedding lookup -> encoder -> mean-pool -> L2-normalise).
//
// Replaces the torch-CPU BertModel + Pooling(mean) + Normalize of sentence-transformers
// 4.1.0 / transformers 4.52.4 reached through SentenceTransformer.encode
// (experiments/embedding_generator.py:124,197,337; experiments/main.py:807) and
// HuggingFaceEmbedding (graph_builder.py:146-149).
//
// Layout: tokens T = B*S (padded to 128); residual stream x [T][H] fp32; its MFMA-dtype copy
// xh [T][H]; projection weights W [N][K] exactly as HF nn.Linear stores them (K contiguous),
// rows padded to 128 with zeros.  GEMM: C[feature][token] = W · xhᵀ on MFMA 16x16x32, so each
// lane ends with 4 consecutive features of one token (16-byte bias / residual loads, 8-byte
// f16 stores).
#pragma once
#include "device_common.h"
#include "tile_common.h"   // MfmaOp, TileLoader (same LDS image and fragment reads as K2)

namespace hcr {

// -------------------------------------------------------------------------------------
// Activation stores.  Fast modes (TM = f16 / bf16): the MFMA-dtype copy xh [T][n].
// Reference-precision mode (SPLIT, TM = f16): a 3n-wide row [h | - | l] with h = f16(v) and
// l = f16((v - h) * 2^11), the X operand of the three-term split GEMM (gemm_v4.h
// gemm_split_kernel): against weights stored [Wh * 2^11 | Wl * 2^11 | Wh] it forms
// 2^11 (Xh Wh + Xh Wl + Xl Wh) in one fp32 accumulator -- about 22 bits of operand precision,
// and the 2^11 keeps the low parts out of the f16 subnormal range.  The middle segment (a
// second copy of h for the K-concatenated form of that product) is no longer written: the
// split kernel reads segments 0 and 2 only (r02: 1/3 fewer activation bytes written).
// -------------------------------------------------------------------------------------
constexpr float kSplitLo = 2048.f;          // 2^11: f16 has an 11-bit significand

template <typename TM, bool SPLIT>
__device__ __forceinline__ void store_act4(TM* __restrict__ row, int n, int f, float4 o) {
  union { TM h[4]; uint2 u; } ph;
  ph.h[0] = (TM)o.x; ph.h[1] = (TM)o.y; ph.h[2] = (TM)o.z; ph.h[3] = (TM)o.w;
  *reinterpret_cast<uint2*>(row + f) = ph.u;
  if constexpr (SPLIT) {
    union { TM h[4]; uint2 u; } pl;
    pl.h[0] = (TM)((o.x - (float)ph.h[0]) * kSplitLo);
    pl.h[1] = (TM)((o.y - (float)ph.h[1]) * kSplitLo);
    pl.h[2] = (TM)((o.z - (float)ph.h[2]) * kSplitLo);
    pl.h[3] = (TM)((o.w - (float)ph.h[3]) * kSplitLo);
    *reinterpret_cast<uint2*>(row + 2 * n + f) = pl.u;
  }
}
template <typename TM, bool SPLIT>
__device__ __forceinline__ void store_act1(TM* __restrict__ row, int n, int f, float v) {
  const TM h = (TM)v;
  row[f] = h;
  if constexpr (SPLIT) {
    row[2 * n + f] = (TM)((v - (float)h) * kSplitLo);
  }
}
template <bool SPLIT> __host__ __device__ constexpr int act_width() { return SPLIT ? 3 : 1; }

// -------------------------------------------------------------------------------------
// Embedding gather + LayerNorm (one wave per token).  HF BertEmbeddings: word + position +
// token_type(0), LayerNorm(eps), dropout (identity at inference).
// -------------------------------------------------------------------------------------
// row LayerNorm helper: values come from a functor (re-evaluated per pass; rows are L1-hot)
template <typename TM, bool SPLIT, typename F>
__device__ __forceinline__ void ln_row(F val, int H, const float* __restrict__ g,
                                       const float* __restrict__ b, float eps, int lane,
                                       float* __restrict__ xo, TM* __restrict__ xho) {
  float s = 0.f;
  for (int d = lane; d < H; d += 64) s += val(d);
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  const float mean = s / H;
  float q = 0.f;
  for (int d = lane; d < H; d += 64) { const float dd = val(d) - mean; q += dd * dd; }
  for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m, 64);
  const float rstd = rsqrtf(q / H + eps);
  for (int d = lane; d < H; d += 64) {
    const float y = (val(d) - mean) * rstd * g[d] + b[d];
    xo[d] = y;
    store_act1<TM, SPLIT>(xho, H, d, y);
  }
}

// Vectorised row LayerNorm for H % 4 == 0 and H <= 1024 (every BERT width used here): one
// wave per row, the row held in registers as up to 4 float4 per lane (one HBM pass), float4
// gamma/beta loads, 16-byte fp32 and 8-byte MFMA-dtype stores.  Same arithmetic as ln_row
// (mean, then the centred second moment, rsqrtf(var + eps)).
template <typename TM, bool SPLIT>
__device__ __forceinline__ void ln_row4(float4 (&v)[4], int H, const float* __restrict__ g,
                                        const float* __restrict__ b, float eps, int lane,
                                        float* __restrict__ xo, TM* __restrict__ xho) {
  const int H4 = H >> 2;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < H4) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  const float mean = s / H;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < H4) {
      const float a = v[i].x - mean, c = v[i].y - mean, d = v[i].z - mean, e = v[i].w - mean;
      q += (a * a + c * c) + (d * d + e * e);
    }
  for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m, 64);
  const float rstd = rsqrtf(q / H + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d4 = lane + 64 * i;
    if (d4 >= H4) continue;
    const float4 gg = reinterpret_cast<const float4*>(g)[d4];
    const float4 bb = reinterpret_cast<const float4*>(b)[d4];
    float4 o;
    o.x = (v[i].x - mean) * rstd * gg.x + bb.x;
    o.y = (v[i].y - mean) * rstd * gg.y + bb.y;
    o.z = (v[i].z - mean) * rstd * gg.z + bb.z;
    o.w = (v[i].w - mean) * rstd * gg.w + bb.w;
    if (xo) reinterpret_cast<float4*>(xo)[d4] = o;    // (NULL: the residual stream is read from xh)
    store_act4<TM, SPLIT>(xho, H, 4 * d4, o);
  }
}

template <typename TM, bool SPLIT>
__global__ void __launch_bounds__(256)
layernorm4_kernel(const float* __restrict__ y, int T_real, int H, const float* __restrict__ g,
                  const float* __restrict__ b, float eps, float* __restrict__ x, TM* __restrict__ xh) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T_real) return;
  const float4* yr = reinterpret_cast<const float4*>(y + (size_t)t * H);
  float4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = (lane + 64 * i < (H >> 2)) ? yr[lane + 64 * i] : float4{0.f, 0.f, 0.f, 0.f};
  ln_row4<TM, SPLIT>(v, H, g, b, eps, lane, x ? x + (size_t)t * H : nullptr,
                     xh + (size_t)t * H * act_width<SPLIT>());
}

template <typename TM, bool SPLIT>
__global__ void __launch_bounds__(256)
embed_ln4_kernel(const int32_t* __restrict__ ids, const int32_t* __restrict__ tok_map, int T_real, int S, int H,
                 const float* __restrict__ wemb, const float* __restrict__ pemb,
                 const float* __restrict__ temb, const float* __restrict__ g,
                 const float* __restrict__ b, float eps, float* __restrict__ x, TM* __restrict__ xh) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T_real) return;
  const int o = tok_map ? tok_map[t] : t;        // packed row -> its padded token index
  const float4* w = reinterpret_cast<const float4*>(wemb + (size_t)ids[o] * H);
  const float4* p = reinterpret_cast<const float4*>(pemb + (size_t)(o % S) * H);
  const float4* ty = reinterpret_cast<const float4*>(temb);
  float4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d4 = lane + 64 * i;
    if (d4 < (H >> 2)) {
      // HF BertEmbeddings order: (word + token_type) + position
      const float4 a = w[d4], c = p[d4], e = ty[d4];
      v[i] = float4{(a.x + e.x) + c.x, (a.y + e.y) + c.y, (a.z + e.z) + c.z, (a.w + e.w) + c.w};
    } else {
      v[i] = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  ln_row4<TM, SPLIT>(v, H, g, b, eps, lane, x ? x + (size_t)t * H : nullptr,
                     xh + (size_t)t * H * act_width<SPLIT>());
}

template <typename TM, bool SPLIT>
__global__ void __launch_bounds__(256)
embed_ln_kernel(const int32_t* __restrict__ ids, const int32_t* __restrict__ tok_map, int T_real, int S, int H,
                const float* __restrict__ wemb, const float* __restrict__ pemb,
                const float* __restrict__ temb, const float* __restrict__ g,
                const float* __restrict__ b, float eps, float* __restrict__ x, TM* __restrict__ xh) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T_real) return;
  const int o = tok_map ? tok_map[t] : t;
  const float* w = wemb + (size_t)ids[o] * H;
  const float* p = pemb + (size_t)(o % S) * H;
  ln_row<TM, SPLIT>([&](int d) { return (w[d] + temb[d]) + p[d]; }, H, g, b, eps, lane,
                    x + (size_t)t * H, xh + (size_t)t * H * act_width<SPLIT>());
}

// LayerNorm of y (fp32, already = residual + sublayer output) -> x fp32 and xh MFMA dtype.
template <typename TM, bool SPLIT>
__global__ void __launch_bounds__(256)
layernorm_kernel(const float* __restrict__ y, int T_real, int H, const float* __restrict__ g,
                 const float* __restrict__ b, float eps, float* __restrict__ x, TM* __restrict__ xh) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T_real) return;
  const float* yr = y + (size_t)t * H;
  ln_row<TM, SPLIT>([&](int d) { return yr[d]; }, H, g, b, eps, lane, x + (size_t)t * H,
                    xh + (size_t)t * H * act_width<SPLIT>());
}

// -------------------------------------------------------------------------------------
// GEMM epilogues (gemm_v4.h):  C[token][feature] = oscale * sum_k X[token][k] W[feature][k]
// + bias[feature], then
//   EPI_BIAS            -> MFMA-dtype out_h [T][ldo]                   (fast QKV)
//   EPI_BIAS_GELU       -> GELU, MFMA-dtype out_h [T][ldo]             (fast FFN1)
//   EPI_BIAS_RESID      -> + resid fp32, fp32 out_f [T][ldo]           (O-proj / FFN2)
//   EPI_BIAS_F32        -> fp32 out_f [T][ldo]                         (split QKV)
//   EPI_BIAS_GELU_SPLIT -> exact-erf GELU, split out_h [T][3 ldo]      (split FFN1)
// -------------------------------------------------------------------------------------
//   EPI_BIAS_RESID_XH   -> + resid from the split activations (h + l 2^-11 of [T][3 ldo] f16),
//                          fp32 out_f [T][ldo]   (split O-proj / FFN2 when the LayerNorms do not
//                          write the fp32 residual stream, r06)
enum : int { EPI_BIAS = 0, EPI_BIAS_GELU = 1, EPI_BIAS_RESID = 2, EPI_BIAS_F32 = 3,
             EPI_BIAS_GELU_SPLIT = 4, EPI_BIAS_RESID_XH = 5 };

// GELU(x) = x/2 (1 + erf(x / sqrt 2)) (HF BERT "gelu", exact-erf form).  erf by Abramowitz &
// Stegun 7.1.26 (|error| <= 1.5e-7, far below the fp16/bf16 output rounding) on v_rcp / v_exp:
// ~12 instructions instead of the ~50 of the library erff -- the FFN1 epilogue evaluates 128 of
// them per lane per tile.  The reference-precision mode uses it too: its error (<= ~3e-7
// absolute with the rcp / exp2 approximations, a few fp32 ulps of erf near 1) leaves the
// encoder's max |diff| vs fp32 BertModel at the 1e-6 level (tests/test_encoder_gpu.py, 1e-4
// bar); HCRAG_GELU_LIBERF=1 selects the library erff there.
__device__ __forceinline__ float erf_as(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  const float r = fmaf(-p * t, e, 1.f);
  return copysignf(r, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erf_as(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_exact(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// -------------------------------------------------------------------------------------
// Self-attention for one (sequence, head): softmax(Q Kᵀ / sqrt(dh) + mask) V.
//   qkv [T][3H] (MFMA dtype: q | k | v), key mask from attention_mask (0 -> -inf, HF uses the
//   dtype minimum; both give exactly 0 weight after softmax when any key is valid).
//   One workgroup per (b, head); K and V of the sequence staged in LDS as fp32 (S*dh*8 bytes,
//   S <= 256 at dh = 64); one wave per query row group; fp32 softmax.
// -------------------------------------------------------------------------------------
template <typename TM>
__global__ void __launch_bounds__(256)
attention_kernel(const TM* __restrict__ qkv, const int32_t* __restrict__ mask,
                 const int32_t* __restrict__ seq_off, int S_pad, int H, int heads, TM* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float att_sm[];
  const int dh = H / heads;
  const int bidx = blockIdx.x / heads, h = blockIdx.x % heads;
  // sequence bidx's rows: padded (rows bidx S_pad .., key mask = attention_mask) or packed
  // (seq_off, key mask = the packed rows' own mask bits: pack_tokens_kernel)
  const size_t row0 = seq_off ? (size_t)seq_off[bidx] : (size_t)bidx * S_pad;
  const int S = seq_off ? seq_off[bidx + 1] - seq_off[bidx] : S_pad;
  if (S == 0) return;
  float* Mk = att_sm;                                   // [S] additive key mask
  float* Pw = Mk + S;                                   // [4 waves][S] probabilities
  float* Qs = Pw + 4 * S;                               // [4 waves][dh] current query rows
  TM* Ks = reinterpret_cast<TM*>(Qs + 4 * dh);          // [S][dh]
  TM* Vs = Ks + (size_t)S * dh;                         // [S][dh]
  const int ld3 = 3 * H;
  for (int i = threadIdx.x; i < S * dh; i += blockDim.x) {
    const int j = i / dh, d = i - j * dh;
    const TM* base = qkv + (row0 + j) * ld3 + h * dh + d;
    Ks[i] = base[H];
    Vs[i] = base[2 * H];
  }
  for (int j = threadIdx.x; j < S; j += blockDim.x) Mk[j] = mask[row0 + j] ? 0.f : -INFINITY;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float scale = rsqrtf((float)dh);
  float* pw = Pw + wave * S;
  float* qs = Qs + wave * dh;
  for (int i = wave; i < S; i += 4) {
    const TM* qrow = qkv + (row0 + i) * ld3 + h * dh;
    for (int d = lane; d < dh; d += 64) qs[d] = (float)qrow[d];
    __builtin_amdgcn_wave_barrier();
    float mx = -INFINITY;
    for (int j = lane; j < S; j += 64) {
      float acc = 0.f;
      const TM* kr = Ks + (size_t)j * dh;
      for (int d = 0; d < dh; ++d) acc += qs[d] * (float)kr[d];
      const float sc = acc * scale + Mk[j];
      pw[j] = sc;
      mx = fmaxf(mx, sc);
    }
    for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    float sum = 0.f;
    for (int j = lane; j < S; j += 64) {
      const float e = (mx == -INFINITY) ? 0.f : __expf(pw[j] - mx);
      pw[j] = e;
      sum += e;
    }
    for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m, 64);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    __builtin_amdgcn_wave_barrier();
    for (int d = lane; d < dh; d += 64) {
      float o = 0.f;
      for (int j = 0; j < S; ++j) o += pw[j] * (float)Vs[(size_t)j * dh + d];
      ctx[(row0 + i) * H + h * dh + d] = (TM)(o * inv);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// -------------------------------------------------------------------------------------
// MFMA self-attention for one (sequence, head), head dim DH in {32, 64}, up to 16*KB keys.
//   Sᵀ = K·Qᵀ on 16x16x32 MFMAs (keys on the M axis): each lane ends with one query and 4
//   keys per 16-key block, which after the softmax is exactly the A-operand layout of P·V
//   when the contraction index is permuted as key(g, e) = 32c + 16(e >> 2) + 4g + (e & 3);
//   V is staged transposed (Vt[c][key]) so its B operand is two 8-byte LDS reads.
//   LDS rows are padded (K by 16, Vt by 8 elements): conflict-free fragment reads
//   (tests/test_lds_swizzle.py).  fp32 scores / softmax / accumulation.
// -------------------------------------------------------------------------------------
template <typename TM, int DH, int KB>
__global__ void __launch_bounds__(256)
attention_mfma_kernel(const TM* __restrict__ qkv, const int32_t* __restrict__ mask,
                      const int32_t* __restrict__ seq_off, int S_pad, int H, int heads, TM* __restrict__ ctx) {
  using Op = MfmaOp<TM>;
  using V = typename Op::V;
  constexpr int KS = DH + 16;                 // K row stride (elements)
  extern __shared__ __attribute__((aligned(16))) char att_mfma_sm[];
  const int bidx = blockIdx.x / heads, h = blockIdx.x % heads;
  // sequence bidx's rows: padded (rows bidx S_pad .., key mask = attention_mask) or packed
  // (seq_off, key mask = the packed rows' own mask bits: pack_tokens_kernel)
  const size_t row0 = seq_off ? (size_t)seq_off[bidx] : (size_t)bidx * S_pad;
  const int S = seq_off ? seq_off[bidx + 1] - seq_off[bidx] : S_pad;
  if (S == 0) return;
  const int Sp = (S + 31) & ~31;
  const int VS = Sp + 8;                      // Vt row stride (elements)
  TM* Ks = reinterpret_cast<TM*>(att_mfma_sm);
  TM* Vt = Ks + (size_t)Sp * KS;
  float* Mk = reinterpret_cast<float*>(att_mfma_sm + (((size_t)Sp * KS + (size_t)DH * VS) * sizeof(TM) + 15) / 16 * 16);
  const int ld3 = 3 * H;
  for (int i = threadIdx.x; i < Sp * (DH / 8); i += blockDim.x) {
    const int j = i / (DH / 8), c8 = i - j * (DH / 8);
    uint4 kv = {0u, 0u, 0u, 0u}, vv = {0u, 0u, 0u, 0u};
    if (j < S) {
      const TM* base = qkv + (row0 + j) * ld3 + h * DH + c8 * 8;
      kv = *reinterpret_cast<const uint4*>(base + H);
      vv = *reinterpret_cast<const uint4*>(base + 2 * H);
    }
    *reinterpret_cast<uint4*>(Ks + (size_t)j * KS + c8 * 8) = kv;
    const TM* ve = reinterpret_cast<const TM*>(&vv);
#pragma unroll
    for (int e = 0; e < 8; ++e) Vt[(size_t)(c8 * 8 + e) * VS + j] = ve[e];
  }
  for (int j = threadIdx.x; j < Sp; j += blockDim.x)
    Mk[j] = (j < S && mask[row0 + j]) ? 0.f : -INFINITY;
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int nkb = Sp / 16;
  const float scale = rsqrtf((float)DH);
  for (int qb = wave; qb * 16 < S; qb += blockDim.x / 64) {
    const int qi = qb * 16 + li;
    V qf[DH / 32];
#pragma unroll
    for (int kk = 0; kk < DH / 32; ++kk) {
      if (qi < S) qf[kk] = *reinterpret_cast<const V*>(qkv + (row0 + qi) * ld3 + h * DH + kk * 32 + lg * 8);
      else for (int e = 0; e < 8; ++e) qf[kk][e] = (TM)0.f;
    }
    floatx4 sc[KB];
    float mx = -INFINITY;
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      sc[b] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (b < nkb) {
#pragma unroll
        for (int kk = 0; kk < DH / 32; ++kk) {
          const V kf = *reinterpret_cast<const V*>(Ks + (size_t)(b * 16 + li) * KS + kk * 32 + lg * 8);
          sc[b] = Op::run(kf, qf[kk], sc[b]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = sc[b][r] * scale + Mk[b * 16 + lg * 4 + r];
          sc[b][r] = v;
          mx = fmaxf(mx, v);
        }
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      if (b < nkb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pexp = (mx == -INFINITY) ? 0.f : __expf(sc[b][r] - mx);
          sc[b][r] = pexp;
          sum += pexp;
        }
      }
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    floatx4 o[DH / 16];
#pragma unroll
    for (int cb = 0; cb < DH / 16; ++cb) o[cb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < KB / 2; ++ch) {
      if (2 * ch < nkb) {
        V pa;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pa[e] = (TM)sc[2 * ch][e];
          pa[4 + e] = (TM)sc[2 * ch + 1][e];
        }
#pragma unroll
        for (int cb = 0; cb < DH / 16; ++cb) {
          const TM* vr = Vt + (size_t)(cb * 16 + li) * VS + ch * 32 + lg * 4;
          V vb;
          const uint2 lo = *reinterpret_cast<const uint2*>(vr);
          const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
          uint4 packed = {lo.x, lo.y, hi.x, hi.y};
          vb = *reinterpret_cast<const V*>(&packed);
          o[cb] = Op::run(pa, vb, o[cb]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float invr = __shfl(inv, lg * 4 + r, 64);
      const int row = qb * 16 + lg * 4 + r;
      if (row < S) {
#pragma unroll
        for (int cb = 0; cb < DH / 16; ++cb)
          ctx[(row0 + row) * H + h * DH + cb * 16 + li] = (TM)(o[cb][r] * invr);
      }
    }
  }
}

template <typename TM, int DH>
size_t attention_mfma_lds(int S) {
  const int Sp = (S + 31) & ~31;
  return (((size_t)Sp * (DH + 16) + (size_t)DH * (Sp + 8)) * sizeof(TM) + 15) / 16 * 16 + (size_t)Sp * 4;
}


// -------------------------------------------------------------------------------------
// fp32 self-attention (reference-precision mode): one workgroup (4 waves) per (sequence,
// head).  qkv fp32 [T][3H] (q | k | v); K and V of the sequence staged in LDS when they fit
// (K rows padded to dh + 1 floats: lane-per-key reads are conflict-free), read from L2
// otherwise.  Scores, softmax (library expf) and P.V in fp32 FMA -- the arithmetic of the
// torch CPU reference up to summation order; ctx is written as split rows [T][3H].
// -------------------------------------------------------------------------------------
__host__ __device__ inline size_t attention_f32_lds(int S, int dh, bool kv_lds) {
  return ((size_t)5 * S + 4 * dh + (kv_lds ? (size_t)S * (2 * dh + 1) : 0)) * 4;
}

template <bool KV_LDS>
__global__ void __launch_bounds__(256)
attention_f32_kernel(const float* __restrict__ qkv, const int32_t* __restrict__ mask,
                     const int32_t* __restrict__ seq_off, int S_pad, int H, int heads,
                     _Float16* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float attf_sm[];
  const int dh = H / heads;
  const int bidx = blockIdx.x / heads, h = blockIdx.x % heads;
  // sequence bidx's rows: padded (rows bidx S_pad .., key mask = attention_mask) or packed
  // (seq_off, key mask = the packed rows' own mask bits: pack_tokens_kernel)
  const size_t row0 = seq_off ? (size_t)seq_off[bidx] : (size_t)bidx * S_pad;
  const int S = seq_off ? seq_off[bidx + 1] - seq_off[bidx] : S_pad;
  if (S == 0) return;
  const int ld3 = 3 * H;
  float* Mk = attf_sm;                    // [S] additive key mask
  float* Pw = Mk + S;                     // [4 waves][S]
  float* Qs = Pw + 4 * S;                 // [4 waves][dh]
  float* Ks = Qs + 4 * dh;                // [S][dh + 1]   (KV_LDS)
  float* Vs = Ks + (size_t)S * (dh + 1);  // [S][dh]       (KV_LDS)
  const float* kbase;
  const float* vbase;
  int ks, vs;
  if constexpr (KV_LDS) {
    for (int i = threadIdx.x; i < S * dh; i += blockDim.x) {
      const int j = i / dh, d = i - j * dh;
      const float* base = qkv + (row0 + j) * ld3 + h * dh + d;
      Ks[(size_t)j * (dh + 1) + d] = base[H];
      Vs[i] = base[2 * H];
    }
    kbase = Ks; ks = dh + 1;
    vbase = Vs; vs = dh;
  } else {
    kbase = qkv + row0 * ld3 + H + h * dh; ks = ld3;
    vbase = qkv + row0 * ld3 + 2 * H + h * dh; vs = ld3;
  }
  for (int j = threadIdx.x; j < S; j += blockDim.x) Mk[j] = mask[row0 + j] ? 0.f : -INFINITY;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float sq = sqrtf((float)dh);      // HF: scores / sqrt(head_size)
  float* pw = Pw + wave * S;
  float* qs = Qs + wave * dh;
  const int G = dh >= 64 ? 1 : 64 / dh;   // key groups in the P.V pass (dh = 32: 2 halves)
  for (int i = wave; i < S; i += 4) {
    const float* qrow = qkv + (row0 + i) * ld3 + h * dh;
    for (int d = lane; d < dh; d += 64) qs[d] = qrow[d];
    __builtin_amdgcn_wave_barrier();
    float mx = -INFINITY;
    for (int j = lane; j < S; j += 64) {
      const float* kr = kbase + (size_t)j * ks;
      float acc = 0.f;
      for (int d = 0; d < dh; ++d) acc = fmaf(qs[d], kr[d], acc);
      const float sc = acc / sq + Mk[j];
      pw[j] = sc;
      mx = fmaxf(mx, sc);
    }
    for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    float sum = 0.f;
    for (int j = lane; j < S; j += 64) {
      const float e = (mx == -INFINITY) ? 0.f : expf(pw[j] - mx);
      pw[j] = e;
      sum += e;
    }
    for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m, 64);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    __builtin_amdgcn_wave_barrier();
    _Float16* crow = ctx + (row0 + i) * ld3;
    if (G == 1) {
      for (int d = lane; d < dh; d += 64) {
        float o = 0.f;
        for (int j = 0; j < S; ++j) o = fmaf(pw[j], vbase[(size_t)j * vs + d], o);
        store_act1<_Float16, true>(crow, H, h * dh + d, o * inv);
      }
    } else {
      const int d = lane % dh, grp = lane / dh;
      float o = 0.f;
      for (int j = grp; j < S; j += G) o = fmaf(pw[j], vbase[(size_t)j * vs + d], o);
      for (int m = dh; m < 64; m <<= 1) o += __shfl_xor(o, m, 64);
      if (grp == 0) store_act1<_Float16, true>(crow, H, h * dh + d, o * inv);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Reference-precision attention for short sequences (S <= 64, the query-embedding regime) on
// the f32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation; MICROARCH
// "FP32-input MFMA"): one 64-thread workgroup per (sequence, head).  Q, K and V go from global
// memory straight into the lanes' MFMA operand registers as 16-byte loads, with no LDS staging:
//  * Q.K^T sums over d in any order, so lane (lr, lk) holds the float4 chunks lk + 4u (u < DH/16)
//    of rows t*16 + lr of Q and of K, and k-step 4u + w of the MFMA takes element w of chunk u:
//    the 4 k-values of a step are d = 16u + 4lk + w (lk = 0..3), every d once over the DH/4 steps;
//  * O = P.V: lane (lr, lk) computes columns 4 lr + dt (dt < 4) of a 16-column block set, so its
//    V operand at step j is the float4 V[4j + lk][4 lr .. 4 lr + 3];
// only P goes through LDS (the softmax's C layout -> the A layout of P.V).  S = Q.K^T / sqrt(DH)
// + key mask as NT x NT 16x16 tiles, the row softmax across the 16 lanes of a tile row, O = P.V
// scaled by 1 / row sum.  LDS per workgroup 29 -> 4.4 KiB at bge-base S = 32 (r02: Q, K, V staged
// in LDS, 124 us per layer call, latency-bound at 5 workgroups per CU; r03 with 4-byte operand
// loads from global, 192 us: 16-line gathers; the wave-per-query attention_f32_kernel: 399 us).
__host__ __device__ inline size_t attention_f32_mfma_lds(int nt, int dh) {
  const int s16 = 16 * nt;
  (void)dh;
  return ((size_t)s16 * (s16 + 1) + s16) * 4;
}
template <int DH, int NT>
__global__ void __launch_bounds__(64)
attention_f32_mfma_kernel(const float* __restrict__ qkv, const int32_t* __restrict__ mask,
                          const int32_t* __restrict__ seq_off, int S_pad, int H, int heads,
                          _Float16* __restrict__ ctx) {
  constexpr int S16 = 16 * NT, LP = S16 + 1, CU = DH / 16, JI = S16 / 4;
  static_assert(DH % 16 == 0 && DH / 4 <= 16 * 4, "head size");
  extern __shared__ __attribute__((aligned(16))) float attm_sm[];
  float* Ps = attm_sm;
  float* mk = Ps + S16 * LP;
  const int lane = threadIdx.x, lr = lane & 15, lk = lane >> 4;
  const int bidx = blockIdx.x / heads, h = blockIdx.x % heads;
  // sequence bidx's rows: padded (rows bidx S_pad .., key mask = attention_mask) or packed
  // (seq_off, key mask = the packed rows' own mask bits: pack_tokens_kernel)
  const size_t row0 = seq_off ? (size_t)seq_off[bidx] : (size_t)bidx * S_pad;
  const int S = seq_off ? seq_off[bidx + 1] - seq_off[bidx] : S_pad;
  if (S == 0) return;
  const int ld3 = 3 * H;
  const float* base = qkv + row0 * ld3 + (size_t)h * DH;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // operands (rows >= S are zero: their P entries are 0, and 0 x V must not meet a NaN)
  float4 qa[NT][CU], kb[NT][CU];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int r = t * 16 + lr;
    const float4* p = reinterpret_cast<const float4*>(base + (size_t)(r < S ? r : 0) * ld3) + lk;
#pragma unroll
    for (int u = 0; u < CU; ++u) {            // (row clamped above: the loads stay in bounds)
      qa[t][u] = p[4 * u];
      kb[t][u] = p[H / 4 + 4 * u];
    }
    if (r >= S) {
#pragma unroll
      for (int u = 0; u < CU; ++u) { qa[t][u] = z4; kb[t][u] = z4; }
    }
  }
  // (DH / 16 column groups of 4: lane lr's columns 4 lr + dt only exist for lr < DH / 4)
  constexpr int VL = DH / 4;
  float4 vb[JI];
#pragma unroll
  for (int j = 0; j < JI; ++j) {
    const int r = 4 * j + lk;
    const bool ok = r < S && lr < VL;
    vb[j] = *(reinterpret_cast<const float4*>(base + (size_t)(ok ? r : 0) * ld3 + 2 * H) + (ok ? lr : 0));
    if (!ok) vb[j] = z4;
  }
  for (int j = lane; j < S16; j += 64) mk[j] = (j < S && mask[row0 + j]) ? 0.f : -INFINITY;
  __syncthreads();
  // scores
  floatx4 c[NT][NT];
#pragma unroll
  for (int it = 0; it < NT; ++it)
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) c[it][jt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < CU; ++u)
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int it = 0; it < NT; ++it)
#pragma unroll
        for (int jt = 0; jt < NT; ++jt) {
          const float a = w == 0 ? qa[it][u].x : w == 1 ? qa[it][u].y : w == 2 ? qa[it][u].z : qa[it][u].w;
          const float b = w == 0 ? kb[jt][u].x : w == 1 ? kb[jt][u].y : w == 2 ? kb[jt][u].z : kb[jt][u].w;
          c[it][jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[it][jt], 0, 0, 0);
        }
  // row softmax: row it*16 + 4 lk + r lives in the 16 lanes with this lk (column = jt*16 + lr)
  const float sq = sqrtf((float)DH);      // HF: scores / sqrt(head_size)
  float inv[NT][4];
#pragma unroll
  for (int it = 0; it < NT; ++it)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int jt = 0; jt < NT; ++jt) {
        const float v = c[it][jt][r] / sq + mk[jt * 16 + lr];
        c[it][jt][r] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
      float sum = 0.f;
#pragma unroll
      for (int jt = 0; jt < NT; ++jt) {
        const float e = (mx == -INFINITY) ? 0.f : expf(c[it][jt][r] - mx);
        Ps[(it * 16 + 4 * lk + r) * LP + jt * 16 + lr] = e;
        sum += e;
      }
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) sum += __shfl_xor(sum, m, 64);
      inv[it][r] = sum > 0.f ? 1.f / sum : 0.f;
    }
  __syncthreads();
  // O = P.V: output block dt holds columns 4 lr + dt (lanes lr < DH / 4; DH = 32 leaves lanes
  // 8-15 of each 16 idle in the 16-wide MFMA, their V operand zero).  All four blocks are kept,
  // so a lane stores its 4 consecutive columns of a row as one 8-byte h and one 8-byte l piece
  // (r04: was 2-byte stores per element, 4x the store instructions; same values)
  floatx4 o[4][NT];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
    for (int it = 0; it < NT; ++it) o[dt][it] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < JI; ++j) {
      const float b = dt == 0 ? vb[j].x : dt == 1 ? vb[j].y : dt == 2 ? vb[j].z : vb[j].w;
#pragma unroll
      for (int it = 0; it < NT; ++it)
        o[dt][it] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ps[(it * 16 + lr) * LP + 4 * j + lk], b, o[dt][it], 0, 0, 0);
    }
  }
  if (lr < VL) {
#pragma unroll
    for (int it = 0; it < NT; ++it)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = it * 16 + 4 * lk + r;
        if (i < S)
          store_act4<_Float16, true>(ctx + (row0 + i) * ld3, H, h * DH + 4 * lr,
                                     make_float4(o[0][it][r] * inv[it][r], o[1][it][r] * inv[it][r],
                                                 o[2][it][r] * inv[it][r], o[3][it][r] * inv[it][r]));
      }
  }
}

// -------------------------------------------------------------------------------------
// Token packing ("unpadding"): the tokens whose attention-mask bit is 1 -- plus position 0 of
// every sequence when the pooling reads it (CLS; kept as a query row, a key only if its mask bit
// is 1) -- stored contiguously, sequence after sequence in position order, so the projections,
// FFN, LayerNorms and attention spend nothing on padding.  Row-wise kernels produce the same
// values for a token either way; attention over the packed keys of a sequence is the padded
// attention with its -inf keys left out (exactly 0 weight there).  One block: seq_off[n + 1]
// (exclusive prefix sums of the per-sequence counts), tok_map[t] = b S + p (the padded index of
// packed row t), key_ok[t] = that token's mask bit, total[0] = the packed row count.
// -------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024)
pack_tokens_kernel(const int32_t* __restrict__ mask, int64_t n, int S, int keep0,
                   int32_t* __restrict__ seq_off, int32_t* __restrict__ tok_map,
                   int32_t* __restrict__ key_ok, int32_t* __restrict__ total) {
  __shared__ int32_t sc[1024];
  int carry = 0;
  for (int64_t b0 = 0; b0 < n; b0 += 1024) {
    const int64_t b = b0 + threadIdx.x;
    int c = 0;
    if (b < n)
      for (int p = 0; p < S; ++p) c += (mask[b * S + p] != 0 || (keep0 && p == 0)) ? 1 : 0;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {            // inclusive scan of the block's counts
      const int v = threadIdx.x >= (unsigned)o ? sc[threadIdx.x - o] : 0;
      __syncthreads();
      sc[threadIdx.x] += v;
      __syncthreads();
    }
    if (b < n) {
      int t = carry + sc[threadIdx.x] - c;
      seq_off[b] = t;
      for (int p = 0; p < S; ++p) {
        const int m = mask[b * S + p] != 0;
        if (m || (keep0 && p == 0)) {
          tok_map[t] = (int32_t)(b * S + p);
          key_ok[t] = m;
          ++t;
        }
      }
    }
    carry += sc[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    seq_off[n] = carry;
    total[0] = carry;
  }
}

// -------------------------------------------------------------------------------------
// Pooling + L2 normalise (one block per sequence).
//   mode 0 (sentence-transformers Pooling mean): sum_t h_t m_t / max(sum_t m_t, 1e-9)
//   mode 1 (CLS, bge): h_0
//   normalise: x / max(||x||, 1e-12)  (torch.nn.functional.normalize)
// -------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
pool_normalize_kernel(const float* __restrict__ x, const int32_t* __restrict__ mask,
                      const int32_t* __restrict__ seq_off, int S_pad, int H, int mode, int normalize,
                      float* __restrict__ out) {
  __shared__ float red[256];
  const int bidx = blockIdx.x;
  // (packed rows: mask = the rows' own mask bits; a CLS sequence always holds its row 0)
  const size_t row0 = seq_off ? (size_t)seq_off[bidx] : (size_t)bidx * S_pad;
  const int S = seq_off ? seq_off[bidx + 1] - seq_off[bidx] : S_pad;
  float cnt = 0.f;
  if (mode == 0)
    for (int t = 0; t < S; ++t) cnt += (float)mask[row0 + t];
  const float denom = fmaxf(cnt, 1e-9f);
  float local = 0.f;
  for (int d = threadIdx.x; d < H; d += blockDim.x) {
    float v;
    if (mode == 0) {
      v = 0.f;
      for (int t = 0; t < S; ++t) v += x[(row0 + t) * H + d] * (float)mask[row0 + t];
      v /= denom;
    } else {
      v = x[row0 * H + d];
    }
    out[(size_t)bidx * H + d] = v;
    local += v * v;
  }
  red[threadIdx.x] = local;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (!normalize) return;
  const float nrm = fmaxf(sqrtf(red[0]), 1e-12f);
  for (int d = threadIdx.x; d < H; d += blockDim.x) out[(size_t)bidx * H + d] /= nrm;
}

// Reference-precision weights: W [rows][cols] fp32 (times the power-of-two `scale` that puts
// max |W| near 16) -> [rows_pad][3 cols] f16 = [Wh * 2^11 | Wl * 2^11 | Wh] with Wh = f16(W),
// Wl = W - Wh (see store_act4); rows past `rows` are zero.
__global__ void to_split_weights(const float* __restrict__ src, int64_t rows, int64_t rows_pad,
                                 int cols, float scale, _Float16* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_pad * cols) return;
  const int64_t r = i / cols;
  const int c = (int)(i - r * cols);
  const float w = r < rows ? src[i] * scale : 0.f;
  const _Float16 hi = (_Float16)w;
  _Float16* o = dst + r * 3 * cols;
  o[c] = (_Float16)((float)hi * kSplitLo);
  o[cols + c] = (_Float16)((w - (float)hi) * kSplitLo);
  o[2 * cols + c] = hi;
}

// fp32 -> MFMA dtype conversion with zero padding of rows [rows, rows_pad)
template <typename TM>
__global__ void to_mfma_dtype(const float* __restrict__ src, int64_t rows, int64_t rows_pad,
                              int cols, TM* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_pad * cols) return;
  const int64_t r = i / cols;
  dst[i] = r < rows ? (TM)src[i] : (TM)0.f;
}

}  // namespace hcr
