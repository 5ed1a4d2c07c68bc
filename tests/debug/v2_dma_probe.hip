// Fault-safe probe of the 224x256 score kernel's data path (one workgroup, tiny buffers).
// Replays issue_stage() (buffer_load ... lds with source-side XOR swizzle), dumps the LDS
// image, the inverse-norm slot and the MFMA accumulators, and diffs them on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../../hc-rag_amd/csrc/topk_kernels.h"
using namespace hcr;

__global__ void __launch_bounds__(512, 2)
probe(const _Float16* rows, const _Float16* qhat, const float* inv, int ld, int tile,
      char* lds_dump, float* inv_dump, float* acc_dump, int mode, int stg_arg) {
  __shared__ __attribute__((aligned(16))) char lds[L2_TOTAL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  for (int i = tid; i < L2_TOTAL / 4; i += 512) reinterpret_cast<int*>(lds)[i] = 0x7fc00000;
  __syncthreads();
  const int lrow = lane >> 3;
  const int ldb = ld * 2;
  const int voff = lrow * ldb + (((lane & 7) ^ lrow) << 4);
  const char* rows_b = reinterpret_cast<const char*>(rows);
  const __amdgpu_buffer_rsrc_t q_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(qhat), (short)0, Q2 * ldb, 0x00020000);
  const __amdgpu_buffer_rsrc_t inv_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(inv), (short)0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(rows_b + (size_t)tile * R2 * ldb), (short)0, 256 * ldb, 0x00020000);
  const int ks = 0, stg = __builtin_amdgcn_readfirstlane(stg_arg);
  char* sa = lds + stg * STAGE2;
  if (mode == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int grp = wave * 4 + i;
      const int so = grp * 8 * ldb + ks * 128;
      if (grp < R2 / 8) dma16(a_rsrc, sa + grp * 1024, voff, so);
      dma16(q_rsrc, sa + A2_BYTES + grp * 1024, voff, so);
    }
    if (wave == 0) dma16(inv_rsrc, lds + L2_INV + (tile % 3) * 1024, lane * 16, tile * (R2 * 4));
  } else {
    // reference staging through registers (the v1 way) into the same image
    for (int c = tid; c < R2 * 8; c += 512) {
      const int row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(sa + row * 128 + ((ch ^ (row & 7)) << 4)) =
          *reinterpret_cast<const uint4*>(rows_b + ((size_t)tile * R2 + row) * ldb + ch * 16);
    }
    for (int c = tid; c < Q2 * 8; c += 512) {
      const int row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(sa + A2_BYTES + row * 128 + ((ch ^ (row & 7)) << 4)) =
          *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(qhat) + (size_t)row * ldb + ch * 16);
    }
    if (tid < 256) reinterpret_cast<float*>(lds + L2_INV + (tile % 3) * 1024)[tid] = inv[tile * R2 + tid];
  }
  __syncthreads();
  for (int i = tid; i < STAGE2; i += 512) lds_dump[i] = sa[i];
  if (tid < 256) inv_dump[tid] = reinterpret_cast<const float*>(lds + L2_INV + (tile % 3) * 1024)[tid];
  // one K-step of MFMAs exactly as the kernel does
  using V = half8;
  const int fr = lane & 15;
  const int c0 = (lane >> 4) ^ (lane & 7);
  const int offA0 = (wm * (R2 / 2) + fr) * 128 + (c0 << 4);
  const int offA1 = (wm * (R2 / 2) + fr) * 128 + ((c0 ^ 4) << 4);
  const int offB0 = A2_BYTES + (wn * 64 + fr) * 128 + (c0 << 4);
  const int offB1 = A2_BYTES + (wn * 64 + fr) * 128 + ((c0 ^ 4) << 4);
  floatx4 acc[MT2][4];
  for (int m = 0; m < MT2; ++m) for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0, 0, 0, 0};
  for (int kk = 0; kk < 2; ++kk) {
    const int oa = kk ? offA1 : offA0, ob = kk ? offB1 : offB0;
    V bq[4];
    for (int n = 0; n < 4; ++n) bq[n] = *reinterpret_cast<const V*>(sa + ob + n * 16 * 128);
    for (int m = 0; m < MT2; ++m) {
      const V av = *reinterpret_cast<const V*>(sa + oa + m * 16 * 128);
      for (int n = 0; n < 4; ++n) acc[m][n] = MfmaOp<_Float16>::run(av, bq[n], acc[m][n]);
    }
  }
  // acc_dump[row][query] for this K-step (64 dims)
  for (int m = 0; m < MT2; ++m)
    for (int n = 0; n < 4; ++n)
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (R2 / 2) + m * 16 + (lane >> 4) * 4 + r;
        const int q = wn * 64 + n * 16 + fr;
        acc_dump[row * Q2 + q] = acc[m][n][r];
      }
}

int main() {
  const int ld = 64, NR = 3 * 224 + 512, tile = 1;
  std::vector<_Float16> rows((size_t)NR * ld), q((size_t)Q2 * ld);
  std::vector<float> inv(NR);
  srand(1);
  for (auto& x : rows) x = (_Float16)((rand() % 17 - 8) / 8.0f);
  for (auto& x : q) x = (_Float16)((rand() % 17 - 8) / 8.0f);
  for (int i = 0; i < NR; ++i) inv[i] = 1000.0f + i;
  _Float16 *dr, *dq; float *dinv, *dinvd, *dacc; char* dl;
  hipMalloc(&dr, rows.size() * 2); hipMalloc(&dq, q.size() * 2); hipMalloc(&dinv, NR * 4);
  hipMalloc(&dl, STAGE2); hipMalloc(&dinvd, 256 * 4); hipMalloc(&dacc, R2 * Q2 * 4);
  hipMemcpy(dr, rows.data(), rows.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dq, q.data(), q.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dinv, inv.data(), NR * 4, hipMemcpyHostToDevice);
  int bad_total = 0;
  for (int cfg = 0; cfg < 4; ++cfg) {
    const int mode = (cfg & 1) ? 0 : 1, stg = cfg >> 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(512), 0, 0, dr, dq, dinv, ld, tile, dl, dinvd, dacc, mode, stg);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("mode %d: %s\n", mode, hipGetErrorString(e)); return 2; }
    std::vector<char> L(STAGE2); std::vector<float> I(256), A((size_t)R2 * Q2);
    hipMemcpy(L.data(), dl, STAGE2, hipMemcpyDeviceToHost);
    hipMemcpy(I.data(), dinvd, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(A.data(), dacc, A.size() * 4, hipMemcpyDeviceToHost);
    int badA = 0, badB = 0, badI = 0, badM = 0;
    for (int row = 0; row < R2; ++row)
      for (int ch = 0; ch < 8; ++ch)
        if (memcmp(&L[row * 128 + ((ch ^ (row & 7)) << 4)], &rows[((size_t)tile * R2 + row) * ld + ch * 8], 16)) {
          if (badA < 4) printf("mode %d A mismatch row %d chunk %d\n", mode, row, ch);
          ++badA;
        }
    for (int row = 0; row < Q2; ++row)
      for (int ch = 0; ch < 8; ++ch)
        if (memcmp(&L[A2_BYTES + row * 128 + ((ch ^ (row & 7)) << 4)], &q[(size_t)row * ld + ch * 8], 16)) {
          if (badB < 4) printf("mode %d B mismatch row %d chunk %d\n", mode, row, ch);
          ++badB;
        }
    for (int i = 0; i < 256; ++i) if (I[i] != inv[tile * R2 + i]) { if (badI < 4) printf("mode %d inv[%d]=%g want %g\n", mode, i, I[i], inv[tile * R2 + i]); ++badI; }
    for (int row = 0; row < R2; ++row)
      for (int qq = 0; qq < Q2; ++qq) {
        double s = 0;
        for (int d = 0; d < 64; ++d) s += (double)(float)rows[((size_t)tile * R2 + row) * ld + d] * (double)(float)q[(size_t)qq * ld + d];
        if (fabs(s - A[row * Q2 + qq]) > 1e-3) { if (badM < 4) printf("mode %d acc[%d][%d]=%g want %g\n", mode, row, qq, A[row * Q2 + qq], s); ++badM; }
      }
    printf("stage %d mode %d (%s): A-image bad %d/1792, B-image bad %d/2048, inv bad %d/256, acc bad %d/%d\n",
           stg, mode, mode ? "register staging" : "LDS-DMA", badA, badB, badI, badM, R2 * Q2);
    bad_total += badA + badB + badI + badM;
  }
  return bad_total ? 1 : 0;
}
