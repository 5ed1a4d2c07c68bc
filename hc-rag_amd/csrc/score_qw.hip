// score_qw.hip — instantiations and launcher of the wide query-stationary score kernel
// (score_qw.h), in a translation unit of its own (compiles in parallel with the others).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "hcrag.h"
#include "host_common.h"
#define HCR_TOPK_TEMPLATES_ONLY   // the shared non-template kernels live in hcrag_index.hip
#include "score_qw.h"
#include "score_qs_launch.h"

using namespace hcr;

namespace {

// Stage DMA issue spread over the MFMA groups (score_qw.h SPREAD) when the index option does not
// choose: with one query block -- every row stage feeds one workgroup, nothing is lost if
// workgroups drift apart: 10M x 768 B = 256 3.75 vs 3.88 ms, 1M x 384 B = 256 0.266 vs 0.278 ms
// score phase (r05c, interleaved in one process, profiles/r05/) -- and at the barrier with
// several: spread issue lets the query blocks of a row partition drift apart, and FETCH_SIZE
// grows 2.65x for -0.9 % at the headline (r05b/c).  HCR_OPT_QW_DM (0 / 3) overrides per index.
bool qw_spread(int dm, int nqb) {
  const int m = dm >= 0 ? dm : (nqb == 1 ? 3 : 0);
  return m == 3;
}

template <typename TM, int CAP, int KS, int SR, int NST, bool SPREAD, int STG = 0>
void launch_dense(const QsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((score_topk_qw_kernel<TM, CAP, KS, SR, NST, false, SPREAD, STG>), dim3(a.nqb * a.P),
                     dim3(V3_NT), 0, st, static_cast<const TM*>(a.rows), a.ld, a.n_rows,
                     static_cast<const TM*>(a.qhat), a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials,
                     a.pcnt, a.kp);
}

template <typename TM, int CAP, int KS, int SR = qw_sr(KS), int NST = QW_NST>
void launch_t(const QsArgs& a, hipStream_t st) {
  if constexpr (256 % SR == 0) {   // (48-row stages are dense-only: the pre-pass never asks)
    if (a.umax) {                  // the sampling pre-pass (MAXONLY)
      hipLaunchKernelGGL((score_topk_qw_kernel<TM, CAP, KS, SR, NST, true>), dim3(a.nqb * a.P), dim3(V3_NT),
                         0, st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                         a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp, a.tstride, a.umax);
      return;
    }
  }
  const bool spread = qw_spread(a.dm, a.nqb);
  // STG: D = 384 only (QW's plain D = 768 loop already holds 256 VGPRs).  On by default with one
  // accumulator set -- interleaved A/B on one box, score phase (profiles/r05/r05k, r05l):
  // 1M x 384 B = 256 0.2452 (off) / 0.2400 (two sets) / 0.2370 ms (one set); B = 1024 0.7778 /
  // 0.7493 / 0.7454 ms
  if constexpr (KS == 12) {
    const int stg = a.stagger < 0 ? 2 : a.stagger;
    if (stg == 2) {
      if (spread) launch_dense<TM, CAP, KS, SR, NST, true, 2>(a, st);
      else launch_dense<TM, CAP, KS, SR, NST, false, 2>(a, st);
      return;
    }
    if (stg == 1) {
      if (spread) launch_dense<TM, CAP, KS, SR, NST, true, 1>(a, st);
      else launch_dense<TM, CAP, KS, SR, NST, false, 1>(a, st);
      return;
    }
  }
  if (spread) launch_dense<TM, CAP, KS, SR, NST, true>(a, st);
  else launch_dense<TM, CAP, KS, SR, NST, false>(a, st);
}

// Dense-pass stage shape at D = 768: 48 rows (72 KiB) in a 2-deep ring -- one barrier per 48 rows
// instead of per 32 (r04b A/B, 10M x 768 B = 1024, three interleaved rounds on one box: 13.19 /
// 13.26 / 13.20 ms vs 13.21 / 13.38 / 13.30 with 32-row stages in a 3-deep ring) -- for batches
// of several query blocks.  With one query block (B <= 256) every row tile comes from HBM once
// and the 3-deep ring of 32-row stages keeps more of it in flight: 10M x 768 B = 256, 3.855 /
// 3.859 vs 3.880 / 3.879 ms (r04h, two interleaved rounds).  The MAXONLY pre-pass keeps 32-row
// stages (its units are 128 rows).
int dense_sr(int ks, int nqb) {
  return ks == 24 && nqb > 1 ? 48 : qw_sr(ks);
}

template <typename TM, int CAP>
bool by_ks(int ks, const QsArgs& a, hipStream_t st) {
  switch (ks) {
    case 12: launch_t<TM, CAP, 12>(a, st); return true;
    case 24:
      if (!a.umax && dense_sr(24, a.nqb) == 48) launch_t<TM, CAP, 24, 48, 2>(a, st);
      else launch_t<TM, CAP, 24>(a, st);
      return true;
    default: return false;
  }
}

// one candidate capacity: with CAP = 1024 the compaction call's 150 VGPRs make the KS = 24
// kernel spill query fragments in its main loop (those batches, k' > 224, stay on v4)
template <typename TM>
bool by_cap(const QsArgs& a, hipStream_t st) {
  return a.cap == 256 && by_ks<TM, 256>(a.ld / V3_BK, a, st);
}

}  // namespace

bool qw_supported(int ld) { return ld % V3_BK == 0 && qw_sr(ld / V3_BK) > 0; }
int qw_rows(int ld, int nqb) { return dense_sr(ld / V3_BK, nqb); }
int qw_sample_rows(int ld) { return qw_sr(ld / V3_BK); }
int qw_cap(int kp, int ld, int nqb) { return kp + dense_sr(ld / V3_BK, nqb) <= 256 ? 256 : 0; }   // 0: not supported

int launch_qw(int dtype, const QsArgs& a, hipStream_t st) {
  const bool ok = dtype == HCR_F16 ? by_cap<_Float16>(a, st) : by_cap<__bf16>(a, st);
  if (!ok) return hcr_set_errorf(HCR_EINVAL, "internal: no QW kernel for ld=%d cap=%d", a.ld, a.cap);
  HIPC(hipGetLastError());
  return HCR_OK;
}

#ifdef HCR_QW_STAMPS
extern "C" int hcr_debug_qw_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hcr::hcr_qw_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif
