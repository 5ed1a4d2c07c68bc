// Timing-only ablation of score_topk_v3_kernel at the bench shape (10M x 768 f16 rows,
// 1024 queries, k' = 64): build with -DHCR_V3_NO_DMA / -DHCR_V3_NO_MFMA / -DHCR_V3_NO_EPI
// and compare kernel times (outputs are not checked here; tests/test_search_gpu.py does).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../../hc-rag_amd/csrc/score_v5.h"
#include "../../hc-rag_amd/csrc/score_v6.h"
using namespace hcr;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 2; } } while (0)

__global__ void fill_rows(_Float16* r, int64_t n, uint32_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  r[i] = (_Float16)(((int)(x & 0xFFFF) - 32768) * (1.0f / 32768.f) * 0.036f);
}
__global__ void fill_f(float* p, int64_t n, float v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

template <int RT, int QT, int WM, int WN, int NST, bool UNIT = false>
static int run(const char* name, int64_t N, int nq, int reps, bool warm) {
  const int ld = 768, kp = 64, CAP = 512;
  const int nqpad = (nq + QT - 1) / QT * QT, nqb = nqpad / QT;
  const int ntiles = (int)((N + RT - 1) / RT);
  int P = std::max(1, (256 + nqb - 1) / nqb);
  P = std::min(P, ntiles);
  const int nwg = nqb * P;
  const int64_t arows = (N + 255) / 256 * 256 + 512;
  _Float16 *rows, *q; float* inv; uint64_t *buf, *part; uint32_t* tau;
  CK(hipMalloc(&rows, arows * ld * 2)); CK(hipMalloc(&q, (size_t)nqpad * ld * 2));
  CK(hipMalloc(&inv, arows * 4)); CK(hipMalloc(&buf, (size_t)nwg * QT * CAP * 8));
  CK(hipMalloc(&part, (size_t)nqpad * P * kp * 8)); CK(hipMalloc(&tau, nqpad * 4));
  hipLaunchKernelGGL(fill_rows, dim3((unsigned)((arows * ld + 255) / 256)), dim3(256), 0, 0, rows, arows * ld, 1u);
  hipLaunchKernelGGL(fill_rows, dim3((unsigned)((nqpad * ld + 255) / 256)), dim3(256), 0, 0, q, (int64_t)nqpad * ld, 7u);
  hipLaunchKernelGGL(fill_f, dim3((unsigned)((arows + 255) / 256)), dim3(256), 0, 0, inv, arows, 1.0f);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
#ifdef HCR_V3_STAMPS
  uint64_t* dst; CK(hipMalloc(&dst, (size_t)nwg * 8 * 4 * 8)); CK(hipMemset(dst, 0, (size_t)nwg * 8 * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_v3_stamps), &dst, sizeof(dst)));
#endif
  float best = 1e30f, tot = 0.f;
  for (int r = 0; r < reps + 1; ++r) {
    if (!warm || r == 0) CK(hipMemset(tau, 0, nqpad * 4));   // warm: bound left by the last run
    CK(hipEventRecord(e0));
    if constexpr (WM == -1)  // v5 UNIT (256 x 256)
      hipLaunchKernelGGL((score_topk_v5_kernel<_Float16, 512, NST, true>), dim3(nwg), dim3(V3_NT), 0, 0,
                         rows, ld, N, ld / V3_BK, inv, nullptr, q, nqb, P, ntiles, 1, buf, tau, part, kp);
    else if constexpr (WM == -2)  // v5 (256 x 256), inverse-norm path
      hipLaunchKernelGGL((score_topk_v5_kernel<_Float16, 512, NST, false>), dim3(nwg), dim3(V3_NT), 0, 0,
                         rows, ld, N, ld / V3_BK, inv, nullptr, q, nqb, P, ntiles, 1, buf, tau, part, kp);
    else if constexpr (WM == -3)  // v6 (256 x 256, staggered halves)
      hipLaunchKernelGGL((score_topk_v6_kernel<_Float16, 512, NST, UNIT>), dim3(nwg), dim3(V3_NT), 0, 0,
                         rows, ld, N, ld / V3_BK, inv, nullptr, q, nqb, P, ntiles, 1, buf, tau, part, kp);
    else if constexpr (WM == 0)   // v4 (256 x 256)
      hipLaunchKernelGGL((score_topk_v4_kernel<_Float16, 512, NST, UNIT>), dim3(nwg), dim3(V3_NT), 0, 0,
                         rows, ld, N, ld / V3_BK, inv, nullptr, q, nqb, P, ntiles, 1, buf, tau, part, kp);
    else
      hipLaunchKernelGGL((score_topk_v3_kernel<_Float16, 512, RT, QT, (WM ? WM : 2), (WN ? WN : 4), NST>), dim3(nwg), dim3(V3_NT), 0, 0,
                         rows, ld, N, ld / V3_BK, inv, nullptr, q, nqb, P, ntiles, 1, buf, tau, part, kp);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) { best = std::min(best, ms); tot += ms; }
  }
#ifdef HCR_V4_COUNT
  {
    unsigned long long h[4];
    CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_v4_count), sizeof(h)));
    printf("  v4 counts over %d launches: slow entries %llu  appends %llu  epilogues %llu  compactions %llu\n",
           reps + 1, h[0], h[1], h[2], h[3]);
    unsigned long long z[4] = {0, 0, 0, 0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_v4_count), z, sizeof(z)));
  }
#endif
#ifdef HCR_V5_COUNT
  {
    unsigned long long h[4];
    CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_v5_count), sizeof(h)));
    printf("  counts over %d launches: slow blocks %llu  appends %llu  epilogues %llu  compaction-epilogues %llu\n",
           reps + 1, h[0], h[1], h[2], h[3]);
    unsigned long long z[4] = {0, 0, 0, 0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_v5_count), z, sizeof(z)));
  }
#endif
  const double flops = 2.0 * nqpad * N * ld, bytes = (double)N * ld * 2;
  printf("%s%s nq=%d RT=%d QT=%d NST=%d: best %.3f ms avg %.3f ms  %.1f TFLOP/s  %.0f GB/s\n", name, warm ? "(warm bound)" : "", nq, RT, QT, NST,
         best, tot / reps, flops / (best * 1e-3) / 1e12, bytes / (best * 1e-3) / 1e9);
#ifdef HCR_V3_STAMPS
  {
    std::vector<uint64_t> h((size_t)nwg * 8 * 4);
    CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
    double sum[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < h.size(); ++i) sum[i % 4] += (double)h[i];
    const double all = sum[0] + sum[1] + sum[2] + sum[3];
    printf("  stamps (share of wave cycles, last launch): epilogue %.1f%%  wait+barrier %.1f%%  issue(v4: desc+frag reads) %.1f%%  reads+mfma(v4: mfma+dma) %.1f%%  (avg %.0f cyc per wave-step)\n",
           100 * sum[0] / all, 100 * sum[1] / all, 100 * sum[2] / all, 100 * sum[3] / all,
           all / (nwg * 8.0) / ((double)ntiles / P * (ld / V3_BK)));
    hipFree(dst);
  }
#endif
  hipFree(rows); hipFree(q); hipFree(inv); hipFree(buf); hipFree(part); hipFree(tau);
  return 0;
}

int main(int argc, char** argv) {
  const char* name = argc > 1 ? argv[1] : "full";
  const int64_t N = 10000000;
#ifdef HCR_ABL_V5
  if (run<256, 256, -1, 0, 4>("v5unit", N, 1024, 3, false)) return 2;
  if (run<256, 256, -1, 0, 4>("v5unit", N, 1024, 3, true)) return 2;
  if (run<256, 256, -2, 0, 4>("v5inv", N, 1024, 3, false)) return 2;
  if (run<256, 256, -2, 0, 4>("v5inv", N, 1024, 3, true)) return 2;
  if (run<256, 256, -1, 0, 4>("v5unit", N, 256, 3, false)) return 2;
  return 0;
#endif
#ifdef HCR_ABL_V6
  if (run<256, 256, -3, 0, 4>("v6", N, 1024, 3, false)) return 2;
  if (run<256, 256, -3, 0, 4>("v6", N, 1024, 3, true)) return 2;
  if (run<256, 256, -3, 0, 4, true>("v6unit", N, 1024, 3, false)) return 2;
  if (run<256, 256, -3, 0, 4, true>("v6unit", N, 1024, 3, true)) return 2;
#endif
  if (run<256, 256, 0, 0, 4>("v4", N, 1024, 3, false)) return 2;
  if (run<256, 256, 0, 0, 4>("v4", N, 1024, 3, true)) return 2;
  if (run<256, 256, 0, 0, 4, true>("v4unit", N, 1024, 3, false)) return 2;
  if (run<256, 256, 0, 0, 4, true>("v4unit", N, 1024, 3, true)) return 2;
  if (run<256, 256, 0, 0, 4>("v4", N, 256, 3, false)) return 2;
  if (argc > 2) return 0;
  if (run<224, 256, 2, 4, 5>(name, N, 1024, 3, false)) return 2;
  if (run<224, 256, 2, 4, 5>(name, N, 1024, 3, true)) return 2;
  if (run<224, 256, 2, 4, 5>(name, N, 256, 3, false)) return 2;
  if (run<256, 16, 8, 1, 8>(name, N, 16, 3, false)) return 2;
  return 0;
}
