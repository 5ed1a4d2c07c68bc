// Runs the production score_topk224_kernel on a small, ONE-TILE-PER-WORKGROUP shape and
// checks (a) every coarse score against a host recomputation, (b) every partition list
// (top-k' keys of the workgroup's rows, sorted) against the dumped coarse scores.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../hc-rag_amd/csrc/topk_kernels.h"
using namespace hcr;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 2; } } while (0)

static uint32_t ord32h(float f) { uint32_t u; memcpy(&u, &f, 4); return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u); }

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 1000, D = 128, NQ = argc > 2 ? atoi(argv[2]) : 400;
  const int Pwant = argc > 3 ? atoi(argv[3]) : 0;
  const int ld = 128, ksteps = ld / 64, kp = 64;
  const int nqpad = (NQ + 255) / 256 * 256, nqb = nqpad / 256;
  const int ntiles = (N + R2 - 1) / R2;
  int P = Pwant > 0 ? Pwant : std::min((256 + nqb - 1) / nqb, ntiles);
  const int nwg = nqb * P;
  const int CAP = 512;
  const int64_t arows = (N + 255) / 256 * 256 + 512;
  printf("N=%d NQ=%d ntiles=%d nqb=%d P=%d nwg=%d\n", N, NQ, ntiles, nqb, P, nwg);
  srand(3);
  std::vector<_Float16> rows((size_t)arows * ld, (_Float16)0.f), q((size_t)nqpad * ld, (_Float16)0.f);
  std::vector<float> inv(arows, 0.f);
  for (int r = 0; r < N; ++r) {
    double ss = 0;
    for (int d = 0; d < D; ++d) { float x = (rand() / (float)RAND_MAX - 0.5f); rows[(size_t)r * ld + d] = (_Float16)x; ss += (double)(float)rows[(size_t)r * ld + d] * (float)rows[(size_t)r * ld + d]; }
    inv[r] = (float)(1.0 / sqrt(ss));
  }
  for (int i = 0; i < NQ; ++i) for (int d = 0; d < D; ++d) q[(size_t)i * ld + d] = (_Float16)(rand() / (float)RAND_MAX - 0.5f);
  _Float16 *dr, *dq; float *dinv, *ddbg; uint64_t *dbuf, *dpart; uint32_t* dtau;
  CK(hipMalloc(&dr, rows.size() * 2)); CK(hipMalloc(&dq, q.size() * 2)); CK(hipMalloc(&dinv, arows * 4));
  CK(hipMalloc(&ddbg, (size_t)nqpad * N * 4)); CK(hipMalloc(&dbuf, (size_t)nwg * 256 * CAP * 8));
  CK(hipMalloc(&dpart, (size_t)nqpad * P * kp * 8)); CK(hipMalloc(&dtau, nqpad * 4));
  CK(hipMemcpy(dr, rows.data(), rows.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dq, q.data(), q.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dinv, inv.data(), arows * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dtau, 0, nqpad * 4)); CK(hipMemset(ddbg, 0xFF, (size_t)nqpad * N * 4));
  CK(hipMemset(dpart, 0xEE, (size_t)nqpad * P * kp * 8));
  hipLaunchKernelGGL((score_topk224_kernel<_Float16, 512>), dim3(nwg), dim3(NT2), 0, 0,
                     dr, ld, (int64_t)N, ksteps, dinv, nullptr, dq, nqb, P, ntiles, dbuf, dtau, dpart, kp, ddbg);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<float> dbg((size_t)nqpad * N);
  std::vector<uint64_t> part((size_t)nqpad * P * kp);
  CK(hipMemcpy(dbg.data(), ddbg, dbg.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(part.data(), dpart, part.size() * 8, hipMemcpyDeviceToHost));
  // (a) coarse scores
  int bad = 0; double maxerr = 0;
  for (int i = 0; i < NQ; ++i)
    for (int r = 0; r < N; ++r) {
      double s = 0;
      for (int d = 0; d < D; ++d) s += (double)(float)q[(size_t)i * ld + d] * (double)(float)rows[(size_t)r * ld + d];
      s *= inv[r];
      const float g = dbg[(size_t)i * N + r];
      const double e = fabs(g - s);
      if (!(e < 1e-4)) { if (bad < 5) printf("coarse q%d r%d got %g want %g\n", i, r, g, s); ++bad; }
      else maxerr = std::max(maxerr, e);
    }
  printf("(a) coarse scores: %d bad of %d, max err %.3g\n", bad, NQ * N, maxerr);
  // (b) the union of a query's partition lists holds its global top-kp (partition lists
  // may drop keys below the global per-query bound, so they are not compared one by one)
  int badp = 0;
  for (int i = 0; i < NQ; ++i) {
    std::vector<uint64_t> keys, got;
    for (int r = 0; r < N; ++r)
      keys.push_back(((uint64_t)ord32h(dbg[(size_t)i * N + r]) << 32) | (uint64_t)(0xFFFFFFFFu - r));
    for (int p = 0; p < P; ++p)
      for (int j = 0; j < kp; ++j) got.push_back(part[((size_t)i * P + p) * kp + j]);
    std::sort(keys.rbegin(), keys.rend());
    std::sort(got.rbegin(), got.rend());
    for (int j = 0; j < kp && j < N; ++j)
      if (got[j] != keys[j]) { if (badp < 8) printf("union q%d j%d got %016llx want %016llx\n", i, j, (unsigned long long)got[j], (unsigned long long)keys[j]); ++badp; }
  }
  printf("(b) partition unions: %d bad of %d\n", badp, NQ * kp);
  return (bad || badp) ? 1 : 0;
}
