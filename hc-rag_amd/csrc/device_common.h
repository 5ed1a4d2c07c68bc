// device_common.h — small device helpers shared by the HIP kernels of libhcrag_hip.so.
// gfx950 only: wave64, MFMA 16x16x32 f16/bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hcr {

constexpr int kWave = 64;

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// ---- order-preserving integer images of floating-point values (larger = better) -------
__device__ __forceinline__ uint32_t ord32(float f) {
  const uint32_t u = __float_as_uint(f);
  return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}
__device__ __forceinline__ float unord32(uint32_t u) {
  if (u == 0u) return -INFINITY;
  const uint32_t b = (u & 0x80000000u) ? (u ^ 0x80000000u) : ~u;
  return __uint_as_float(b);
}
__device__ __forceinline__ uint64_t ord64(double d) {
  const uint64_t u = (uint64_t)__double_as_longlong(d);
  return u ^ ((u >> 63) ? 0xFFFFFFFFFFFFFFFFull : 0x8000000000000000ull);
}
__device__ __forceinline__ double unord64(uint64_t u) {
  if (u == 0ull) return -INFINITY;
  const uint64_t b = (u & 0x8000000000000000ull) ? (u ^ 0x8000000000000000ull) : ~u;
  return __longlong_as_double((long long)b);
}

// Candidate key: (coarse score desc, shard-local row asc) as one u64, larger = better.
// 0 is the empty slot (every finite score maps to a key > 0).
__device__ __forceinline__ uint64_t make_key(float s, uint32_t row) {
  return ((uint64_t)ord32(s) << 32) | (uint64_t)(0xFFFFFFFFu - row);
}
__device__ __forceinline__ uint32_t key_row(uint64_t key) { return 0xFFFFFFFFu - (uint32_t)key; }
__device__ __forceinline__ float key_score(uint64_t key) { return unord32((uint32_t)(key >> 32)); }

// ---- wave64 shuffles for 64-bit values ------------------------------------------------
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, kWave);
  const int hi = __shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const int lo = __shfl((int)(uint32_t)v, src, kWave);
  const int hi = __shfl((int)(uint32_t)(v >> 32), src, kWave);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t o = shfl_xor_u64((uint64_t)__double_as_longlong(v), m);
    v += __longlong_as_double((long long)o);
  }
  return v;
}

__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t o = shfl_xor_u64((uint64_t)__double_as_longlong(v), m);
    v = fmax(v, __longlong_as_double((long long)o));
  }
  return v;
}

// ---- bitonic sort of 64*E u64 keys held E per lane (index = lane*E + e), descending ----
// Every loop has a template-constant trip count so the network fully unrolls and v[] stays
// in registers (a runtime index would send it to scratch).
template <int E, int LOGSIZE>
__device__ __forceinline__ void bitonic_stage_desc(uint64_t (&v)[E], int lane) {
  constexpr int size = 1 << LOGSIZE;
#pragma unroll
  for (int ld2 = LOGSIZE - 1; ld2 >= 0; --ld2) {
    const int d = 1 << ld2;
    if (d >= E) {
      const int lm = d / E;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        const uint64_t o = shfl_xor_u64(v[e], lm);
        const bool lower = (i & d) == 0;
        const bool desc = (i & size) == 0;
        const uint64_t mx = v[e] > o ? v[e] : o;
        const uint64_t mn = v[e] > o ? o : v[e];
        v[e] = (lower == desc) ? mx : mn;
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((e & d) == 0) {
          const int e2 = e | d;
          const int i = lane * E + e;
          const bool desc = (i & size) == 0;
          const uint64_t a = v[e], b = v[e2];
          const uint64_t mx = a > b ? a : b, mn = a > b ? b : a;
          v[e] = desc ? mx : mn;
          v[e2] = desc ? mn : mx;
        }
      }
    }
  }
}
template <int E, int LOGSIZE, int LOGN>
__device__ __forceinline__ void bitonic_all_desc(uint64_t (&v)[E], int lane) {
  if constexpr (LOGSIZE <= LOGN) {
    bitonic_stage_desc<E, LOGSIZE>(v, lane);
    bitonic_all_desc<E, LOGSIZE + 1, LOGN>(v, lane);
  }
}
template <int E>
__device__ __forceinline__ void wave_sort_desc(uint64_t (&v)[E], int lane) {
  constexpr int LOGE = (E == 1) ? 0 : (E == 2) ? 1 : (E == 4) ? 2 : (E == 8) ? 3 : 4;
  static_assert((1 << LOGE) == E, "E must be a power of two <= 16");
  bitonic_all_desc<E, 1, 6 + LOGE>(v, lane);
}

// ---- (hi, lo) pairs, lexicographic, descending: the same network as wave_sort_desc ----
template <int E, int LOGSIZE>
__device__ __forceinline__ void bitonic_stage_desc_pair(uint64_t (&h)[E], uint64_t (&l)[E], int lane) {
  constexpr int size = 1 << LOGSIZE;
#pragma unroll
  for (int ld2 = LOGSIZE - 1; ld2 >= 0; --ld2) {
    const int d = 1 << ld2;
    if (d >= E) {
      const int lm = d / E;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        const uint64_t oh = shfl_xor_u64(h[e], lm), ol = shfl_xor_u64(l[e], lm);
        const bool lower = (i & d) == 0;
        const bool desc = (i & size) == 0;
        const bool gt = h[e] > oh || (h[e] == oh && l[e] > ol);   // mine is the larger
        const bool take_mine = (lower == desc) ? gt : !gt;
        if (!take_mine) { h[e] = oh; l[e] = ol; }
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((e & d) == 0) {
          const int e2 = e | d;
          const int i = lane * E + e;
          const bool desc = (i & size) == 0;
          const bool gt = h[e] > h[e2] || (h[e] == h[e2] && l[e] > l[e2]);
          if (gt != desc) {
            const uint64_t th = h[e], tl = l[e];
            h[e] = h[e2]; l[e] = l[e2]; h[e2] = th; l[e2] = tl;
          }
        }
      }
    }
  }
}
template <int E, int LOGSIZE, int LOGN>
__device__ __forceinline__ void bitonic_all_desc_pair(uint64_t (&h)[E], uint64_t (&l)[E], int lane) {
  if constexpr (LOGSIZE <= LOGN) {
    bitonic_stage_desc_pair<E, LOGSIZE>(h, l, lane);
    bitonic_all_desc_pair<E, LOGSIZE + 1, LOGN>(h, l, lane);
  }
}

// Wave 0 sorts a[0, 64 E) (LDS) in registers; the caller synchronises before and after.
template <int E>
__device__ __forceinline__ void wave0_sort_lds_u64(uint64_t* a) {
  const int lane = threadIdx.x;
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = a[lane * E + e];
  wave_sort_desc<E>(v, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) a[lane * E + e] = v[e];
}
template <int E>
__device__ __forceinline__ void wave0_sort_lds_pair(uint64_t* hi, uint64_t* lo) {
  constexpr int LOGE = (E == 1) ? 0 : (E == 2) ? 1 : (E == 4) ? 2 : 3;
  static_assert((1 << LOGE) == E, "E must be a power of two <= 8");
  const int lane = threadIdx.x;
  uint64_t h[E], l[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { h[e] = hi[lane * E + e]; l[e] = lo[lane * E + e]; }
  bitonic_all_desc_pair<E, 1, 6 + LOGE>(h, l, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) { hi[lane * E + e] = h[e]; lo[lane * E + e] = l[e]; }
}

// ---- block-wide bitonic sort in LDS, descending, M a power of two ---------------------
__device__ __forceinline__ void block_sort_desc_u64(uint64_t* a, int M) {
  for (int size = 2; size <= M; size <<= 1) {
    for (int d = size >> 1; d > 0; d >>= 1) {
      for (int t = threadIdx.x; t < (M >> 1); t += blockDim.x) {
        const int i = 2 * t - (t & (d - 1));
        const int j = i + d;
        const bool desc = (i & size) == 0;
        const uint64_t x = a[i], y = a[j];
        if ((x < y) == desc && x != y) { a[i] = y; a[j] = x; }
      }
      __syncthreads();
    }
  }
}
// M in {64, 128, 256, 512} (a power of two): one wave sorts in registers -- two block barriers
// instead of the network's log2(M) (log2(M) + 1) / 2 (21 at M = 64); larger M: the block network.
// Called by every thread of the block, after the keys are in LDS and visible (synchronised).
__device__ __forceinline__ void block_sort_desc_u64_fast(uint64_t* a, int M) {
  if (M > 512 || M < 64) { block_sort_desc_u64(a, M); return; }
  if (threadIdx.x < 64) {
    if (M == 64) wave0_sort_lds_u64<1>(a);
    else if (M == 128) wave0_sort_lds_u64<2>(a);
    else if (M == 256) wave0_sort_lds_u64<4>(a);
    else wave0_sort_lds_u64<8>(a);
  }
  __syncthreads();
}

// Pairs (hi, lo) compared lexicographically, descending.
__device__ __forceinline__ void block_sort_desc_pair(uint64_t* hi, uint64_t* lo, int M) {
  for (int size = 2; size <= M; size <<= 1) {
    for (int d = size >> 1; d > 0; d >>= 1) {
      for (int t = threadIdx.x; t < (M >> 1); t += blockDim.x) {
        const int i = 2 * t - (t & (d - 1));
        const int j = i + d;
        const bool desc = (i & size) == 0;
        const uint64_t xh = hi[i], yh = hi[j], xl = lo[i], yl = lo[j];
        const bool x_lt_y = (xh < yh) || (xh == yh && xl < yl);
        const bool x_gt_y = (xh > yh) || (xh == yh && xl > yl);
        if (desc ? x_lt_y : x_gt_y) { hi[i] = yh; hi[j] = xh; lo[i] = yl; lo[j] = xl; }
      }
      __syncthreads();
    }
  }
}
__device__ __forceinline__ void block_sort_desc_pair_fast(uint64_t* hi, uint64_t* lo, int M) {
  if (M > 512 || M < 64) { block_sort_desc_pair(hi, lo, M); return; }
  if (threadIdx.x < 64) {
    if (M == 64) wave0_sort_lds_pair<1>(hi, lo);
    else if (M == 128) wave0_sort_lds_pair<2>(hi, lo);
    else if (M == 256) wave0_sort_lds_pair<4>(hi, lo);
    else wave0_sort_lds_pair<8>(hi, lo);
  }
  __syncthreads();
}

}  // namespace hcr
