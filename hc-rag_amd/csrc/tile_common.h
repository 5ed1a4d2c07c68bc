// tile_common.h — MFMA tile constants, MFMA op wrappers and the register-staged tile loader
// shared by the score kernels (topk_kernels.h) and the encoder GEMMs (encoder_kernels.h).
#pragma once
#include "device_common.h"

namespace hcr {

constexpr int BR = 128;       // corpus rows per tile
constexpr int BQ = 128;       // queries per block
constexpr int BK = 64;        // K (embedding dim) per stage
constexpr int NT = 256;       // threads per workgroup (4 waves, 2x2 over rows x queries)
constexpr int STAGE_BYTES = (BR + BQ) * BK * 2;   // 32 KiB: A (rows) 16 KiB + B (queries) 16 KiB
constexpr int LDS_STAGES = 2 * STAGE_BYTES;        // double buffered

template <typename T> struct MfmaOp;
template <> struct MfmaOp<_Float16> {
  using V = half8;
  static __device__ __forceinline__ floatx4 run(V a, V b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct MfmaOp<__bf16> {
  using V = bf16x8;
  static __device__ __forceinline__ floatx4 run(V a, V b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};

// -------------------------------------------------------------------------------------
// K2 helpers: global -> register -> LDS staging of one 128 x 64 tile (16 KiB, MFMA dtype).
// LDS image: [row][8 chunks of 16 B], chunk slot = chunk ^ (row & 7)  (conflict-free for
// the 16x16x32 fragment reads).
// -------------------------------------------------------------------------------------
template <typename TS> struct TileLoader;   // corpus rows in storage dtype TS

// 16-bit storage: 4 x 16 B per thread.
template <typename TS> struct TileLoader {
  uint4 r[4];
  __device__ __forceinline__ void load(const TS* __restrict__ base, int64_t row0, int64_t nrows,
                                       int ld, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      const int row = c >> 3, ch = c & 7;
      int64_t gr = row0 + row;
      gr = gr < nrows ? gr : nrows - 1;
      r[i] = *reinterpret_cast<const uint4*>(base + gr * ld + k0 + ch * 8);
    }
  }
  __device__ __forceinline__ void store(char* lds_tile, int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      const int row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(lds_tile + row * 128 + ((ch ^ (row & 7)) << 4)) = r[i];
    }
  }
};
// f32 storage: 8 x 16 B per thread, converted to bf16 on the way into LDS.
template <> struct TileLoader<float> {
  float4 r[8];
  __device__ __forceinline__ void load(const float* __restrict__ base, int64_t row0,
                                       int64_t nrows, int ld, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      const int row = c >> 3, ch = c & 7;
      int64_t gr = row0 + row;
      gr = gr < nrows ? gr : nrows - 1;
      const float4* p = reinterpret_cast<const float4*>(base + gr * ld + k0 + ch * 8);
      r[2 * i] = p[0];
      r[2 * i + 1] = p[1];
    }
  }
  __device__ __forceinline__ void store(char* lds_tile, int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + NT * i;
      const int row = c >> 3, ch = c & 7;
      bf16x8 v;
      v[0] = (__bf16)r[2 * i].x; v[1] = (__bf16)r[2 * i].y;
      v[2] = (__bf16)r[2 * i].z; v[3] = (__bf16)r[2 * i].w;
      v[4] = (__bf16)r[2 * i + 1].x; v[5] = (__bf16)r[2 * i + 1].y;
      v[6] = (__bf16)r[2 * i + 1].z; v[7] = (__bf16)r[2 * i + 1].w;
      *reinterpret_cast<bf16x8*>(lds_tile + row * 128 + ((ch ^ (row & 7)) << 4)) = v;
    }
  }
};


}  // namespace hcr
