// mfma_shape_ab.hip — VERDICT r4 item 1: is QW's dense loop better on v_mfma_f32_32x32x16_f16
// than on v_mfma_f32_16x16x32_f16 on this chip under its held clock?  The QW main loop reduced to
// its matrix part, both shapes at the SAME output tile per wave (32 queries x 32 rows per row
// stage step), the same LDS fragment bytes per flop and the same MFMA cycles per stage:
//   * 8 waves per workgroup (two per SIMD), one workgroup per CU (96 KiB of LDS: two 32-row x
//     768-k stages of random f16 rows in QW's 1 KiB-piece, XOR-swizzled image), 256 workgroups;
//   * each wave holds 32 random unit f16 queries x 768 k as MFMA B fragments (192 VGPRs);
//   * per stage a wave reads 48 KiB of A fragments (48 ds_read_b128) and runs 96 16x16x32 or
//     48 32x32x16 MFMAs (1536 pipe cycles either way) into 16 accumulator VGPRs, one barrier per
//     stage, alternating between the two LDS stages.
// Prints per shape: wall ms, TFLOP/s, the in-kernel clock (s_memtime / s_memrealtime over the
// loop, median over workgroups) and TFLOP/s per GHz.  Random data throughout (zero operands
// raise the clock: MI355X_MICROARCH.md 'DVFS give-back').
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/mfma_shape_ab.hip -o tools/bin/mfma_shape_ab
//   tools/bin/mfma_shape_ab [iters] [rounds] [32 | 64]   (64: QW vs QW64 instead of the two shapes)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define HC(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int KS = 24;                 // 32-deep k-steps (768)
constexpr int STAGE = 2 * KS * 1024;   // 32 rows x 768 k f16 = 48 KiB
constexpr uint32_t SWZ = 0x1320;       // QW's chunk swizzle (ring_common.h V3_SWZ)
__device__ __forceinline__ int slot(int chunk, int row) { return chunk ^ (int)((SWZ >> (((row >> 2) & 3) * 4)) & 3u); }

// QW64: ONE wave per SIMD (4 waves, 256 threads per workgroup), each holding
// 64 queries x 768 k as B fragments (384 VGPRs of the 512-entry file): per stage a wave reads the
// same 48 KiB of A fragments as a QW wave but runs 192 MFMAs on them -- half the LDS read bytes
// per flop.  Same output per workgroup (256 queries x 32 rows per stage), same flops per launch.
__global__ void __launch_bounds__(256, 1)
qw64_kernel(const half8* __restrict__ rows_src, const half8* __restrict__ q_src, int iters,
            float* __restrict__ out, unsigned long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) half8 lds[2 * STAGE / 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 2 * STAGE / 16; i += 256) lds[i] = rows_src[(size_t)blockIdx.x * 16 + i];
  half8 qf[4 * KS];
#pragma unroll
  for (int i = 0; i < 4 * KS; ++i) qf[i] = q_src[((size_t)(blockIdx.x * 4 + wave) * 4 * KS + i) * 64 + lane];
  __syncthreads();
  const uint32_t offA = (lane & 15) * 64 + slot(lane >> 4, lane & 15) * 16;
  const char* lb = reinterpret_cast<const char*>(lds);
  floatx4 acc[2][4] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (lane == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; ++it) {
    const char* st = lb + (it & 1) * STAGE;
    half8 a[2][2];
    a[0][0] = *reinterpret_cast<const half8*>(st + offA);
    a[0][1] = *reinterpret_cast<const half8*>(st + KS * 1024 + offA);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
        a[(ks + 1) & 1][0] = *reinterpret_cast<const half8*>(st + (ks + 1) * 1024 + offA);
        a[(ks + 1) & 1][1] = *reinterpret_cast<const half8*>(st + (KS + ks + 1) * 1024 + offA);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ks & 1][0], qf[n * KS + ks], acc[0][n], 0, 0, 0);
        acc[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ks & 1][1], qf[n * KS + ks], acc[1][n], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (lane == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[(blockIdx.x * 8 + wave) * 2] = t1 - t0;
    clk[(blockIdx.x * 8 + wave) * 2 + 1] = r1 - r0;
  }
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) s += acc[m][n][0] + acc[m][n][1] + acc[m][n][2] + acc[m][n][3];
  out[blockIdx.x * 512 + tid] = s;
}

// QW64 with QW's own fragment pipeline (score_qw.h qw_issue_frags / qw_frag_wait): the A
// fragments of k-step j + 2 are read while those of j feed their 8 MFMAs, counted lgkmcnt
// waits (the plain-C++ loop above leaves the read scheduling -- and 73 waits per stage -- to the
// compiler).
template <int OFF2>
__device__ __forceinline__ void issue2(uint32_t sbase, uint32_t voff, half8 (&av)[2]) {
  uint32_t a;
  asm volatile(
      "v_add_u32 %2, %3, %4\n\t"
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %2 offset:%5"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(a)
      : "s"(sbase), "v"(voff), "n"(OFF2 * 1024)
      : "memory");
}
template <int N>
__device__ __forceinline__ void wait2(half8 (&av)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(av[0]), "+v"(av[1]) : "n"(N) : "memory");
}
__global__ void __launch_bounds__(256, 1)
qw64p_kernel(const half8* __restrict__ rows_src, const half8* __restrict__ q_src, int iters,
             float* __restrict__ out, unsigned long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) half8 lds[2 * STAGE / 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 2 * STAGE / 16; i += 256) lds[i] = rows_src[(size_t)blockIdx.x * 16 + i];
  half8 qf[4 * KS];
#pragma unroll
  for (int i = 0; i < 4 * KS; ++i) qf[i] = q_src[((size_t)(blockIdx.x * 4 + wave) * 4 * KS + i) * 64 + lane];
  __syncthreads();
  const uint32_t offA = (lane & 15) * 64 + slot(lane >> 4, lane & 15) * 16;
  const uint32_t l0 = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)lds);
  floatx4 acc[2][4] = {};
  constexpr int FD = 3;
  unsigned long long t0 = 0, r0 = 0;
  if (lane == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; ++it) {
    const uint32_t st = (uint32_t)__builtin_amdgcn_readfirstlane((int)(l0 + (uint32_t)((it & 1) * STAGE)));
    half8 av[FD][2];
#pragma unroll
    for (int j = 0; j < FD - 1; ++j) issue2<KS>(st + j * 1024, offA, av[j]);
#pragma unroll
    for (int j = 0; j < KS; ++j) {
      if (j + FD - 1 < KS) {
        issue2<KS>(st + (j + FD - 1) * 1024, offA, av[(j + FD - 1) % FD]);
        wait2<2 * (FD - 1)>(av[j % FD]);
      } else if (j + 1 < KS) {
        wait2<2>(av[j % FD]);
      } else {
        wait2<0>(av[j % FD]);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[j % FD][0], qf[n * KS + j], acc[0][n], 0, 0, 0);
        acc[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[j % FD][1], qf[n * KS + j], acc[1][n], 0, 0, 0);
      }
    }
    asm volatile("s_barrier" ::: "memory");
  }
  if (lane == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[(blockIdx.x * 8 + wave) * 2] = t1 - t0;
    clk[(blockIdx.x * 8 + wave) * 2 + 1] = r1 - r0;
  }
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) s += acc[m][n][0] + acc[m][n][1] + acc[m][n][2] + acc[m][n][3];
  out[blockIdx.x * 512 + tid] = s;
}

template <int SHAPE>
__global__ void __launch_bounds__(512, 1)
shape_kernel(const half8* __restrict__ rows_src, const half8* __restrict__ q_src, int iters,
             float* __restrict__ out, unsigned long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) half8 lds[2 * STAGE / 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 2 * STAGE / 16; i += 512) lds[i] = rows_src[(size_t)blockIdx.x * 16 + i];
  // B fragments: 16x16x32 -- lane holds query (l & 15) + 16 n, k = 32 ks + 8 (l >> 4);
  // 32x32x16 -- lane holds query l & 31, k = 16 j + 8 (l >> 5).  192 VGPRs either way.
  half8 qf[2 * KS];
#pragma unroll
  for (int i = 0; i < 2 * KS; ++i) qf[i] = q_src[((size_t)(blockIdx.x * 8 + wave) * 2 * KS + i) * 64 + lane];
  __syncthreads();
  // per-lane A-fragment byte offsets inside a piece pair
  uint32_t offA[2];
  if constexpr (SHAPE == 16) {
    offA[0] = (lane & 15) * 64 + slot(lane >> 4, lane & 15) * 16;          // row block 0; +KS KiB: 1
    offA[1] = offA[0];
  } else {
    // k-step j (16 deep) of piece (rb, j / 2): row l & 15 of row block (l & 31) / 16, chunk
    // 2 (j % 2) + (l >> 5)
    const int rb = (lane & 31) >> 4, r = lane & 15;
    offA[0] = rb * KS * 1024 + r * 64 + slot(lane >> 5, r) * 16;
    offA[1] = rb * KS * 1024 + r * 64 + slot(2 + (lane >> 5), r) * 16;
  }
  const char* lb = reinterpret_cast<const char*>(lds);
  floatx4 acc4[2][2] = {};
  floatx16 acc16 = {};
  unsigned long long t0 = 0, r0 = 0;
  if (lane == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; ++it) {
    const char* st = lb + (it & 1) * STAGE;
    if constexpr (SHAPE == 16) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const half8 a0 = *reinterpret_cast<const half8*>(st + ks * 1024 + offA[0]);
        const half8 a1 = *reinterpret_cast<const half8*>(st + (KS + ks) * 1024 + offA[0]);
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          acc4[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, qf[n * KS + ks], acc4[0][n], 0, 0, 0);
          acc4[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, qf[n * KS + ks], acc4[1][n], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 2 * KS; ++j) {
        const half8 a = *reinterpret_cast<const half8*>(st + (j >> 1) * 1024 + offA[j & 1]);
        acc16 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, qf[j], acc16, 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (lane == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[(blockIdx.x * 8 + wave) * 2] = t1 - t0;
    clk[(blockIdx.x * 8 + wave) * 2 + 1] = r1 - r0;
  }
  float s = 0.f;
  if constexpr (SHAPE == 16) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) s += acc4[m][n][0] + acc4[m][n][1] + acc4[m][n][2] + acc4[m][n][3];
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc16[i];
  }
  out[blockIdx.x * 512 + tid] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const int nwg = 256;
  std::mt19937 gen(5);
  std::normal_distribution<float> nd(0.f, 1.f / std::sqrt(768.f));
  const size_t nrow = (size_t)nwg * 16 + 2 * STAGE / 16 + 64;
  std::vector<_Float16> rows(nrow * 8), qs((size_t)nwg * 8 * 2 * KS * 64 * 8);
  for (auto& v : rows) v = (_Float16)nd(gen);
  for (auto& v : qs) v = (_Float16)nd(gen);
  half8 *d_rows, *d_q;
  float* d_out;
  unsigned long long* d_clk;
  HC(hipMalloc(&d_rows, rows.size() * 2));
  HC(hipMalloc(&d_q, qs.size() * 2));
  HC(hipMalloc(&d_out, (size_t)nwg * 512 * 4));
  HC(hipMalloc(&d_clk, (size_t)nwg * 8 * 2 * 8));
  HC(hipMemcpy(d_rows, rows.data(), rows.size() * 2, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_q, qs.data(), qs.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  const double flops = 2.0 * 32 * 32 * 768 * 8.0 * nwg * iters;   // per launch
  auto run = [&](int shape) {
    HC(hipEventRecord(e0));
    HC(hipMemset(d_clk, 0, (size_t)nwg * 8 * 2 * 8));
    if (shape == 16) hipLaunchKernelGGL(shape_kernel<16>, dim3(nwg), dim3(512), 0, 0, d_rows, d_q, iters, d_out, d_clk);
    else if (shape == 64) hipLaunchKernelGGL(qw64_kernel, dim3(nwg), dim3(256), 0, 0, d_rows, d_q, iters, d_out, d_clk);
    else if (shape == 65) hipLaunchKernelGGL(qw64p_kernel, dim3(nwg), dim3(256), 0, 0, d_rows, d_q, iters, d_out, d_clk);
    else hipLaunchKernelGGL(shape_kernel<32>, dim3(nwg), dim3(512), 0, 0, d_rows, d_q, iters, d_out, d_clk);
    HC(hipGetLastError());
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms = 0.f;
    HC(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> c((size_t)nwg * 16);
    HC(hipMemcpy(c.data(), d_clk, c.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    for (int i = 0; i < nwg * 8; ++i)
      if (c[2 * i + 1]) ghz.push_back((double)c[2 * i] / (double)c[2 * i + 1] * 0.1);   // memrealtime: 100 MHz
    std::sort(ghz.begin(), ghz.end());
    const double g = ghz.empty() ? 0.0 : ghz[ghz.size() / 2];
    const double tf = flops / (ms * 1e-3) / 1e12;
    printf("shape %s  %8.2f ms  %7.1f TFLOP/s  clock %.3f GHz  %6.1f TFLOP/s per GHz  (%.3f of the dense "
           "peak at that clock)\n", shape == 16 ? "16x16x32" : shape == 64 ? "QW64 16x16x32" : shape == 65 ? "QW64 pipelined" : "32x32x16", ms, tf, g, g > 0 ? tf / g : 0.0,
           g > 0 ? tf / (2500.0 * g / 2.4) : 0.0);
    fflush(stdout);
  };
  run(16);                                   // warm-up (clock settles)
  const bool qw64 = argc > 3 && atoi(argv[3]) == 64;   // third argument 64: QW (32 queries per
                                                       // wave) vs QW64 (64 per wave, 1 wave/SIMD)
  for (int r = 0; r < rounds; ++r) {
    run(16);
    if (qw64) { run(64); run(65); } else run(32);
  }
  return 0;
}
