// score_qw1.hip — instantiations and launcher of the one-wave-per-SIMD query-stationary score
// kernel (score_qw1.h), in a translation unit of its own.
#include <hip/hip_runtime.h>

#include "hcrag.h"
#include "host_common.h"
#define HCR_TOPK_TEMPLATES_ONLY   // the shared non-template kernels live in hcrag_index.hip
#include "score_qw1.h"
#include "score_qw1p.h"
#include "score_qs_launch.h"

using namespace hcr;

namespace {

template <typename TM, int KS, bool SPREAD, int NW = QW1_NW, int SR = 0, int NST = 0, int FD = 0>
void launch_t(const QsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((score_topk_qw1_kernel<TM, 256, KS, SPREAD, NW, SR, NST, FD>), dim3(a.nqb * a.P), dim3(NW * 64), 0,
                     st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                     a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
}

// D = 768 tuning shapes (HCR_OPT_QW1_SHAPE): 1 = 4 fragment groups in flight, 2 = 16-row stages
// in a 6-deep ring (5 stages of prefetch), 3 = both
template <typename TM, bool SPREAD>
void launch_768(int shape, const QsArgs& a, hipStream_t st) {
  switch (shape) {
    case 1: launch_t<TM, 24, SPREAD, QW1_NW, 0, 0, 4>(a, st); break;
    case 2: launch_t<TM, 24, SPREAD, QW1_NW, 16, 6, 0>(a, st); break;
    case 3: launch_t<TM, 24, SPREAD, QW1_NW, 16, 6, 4>(a, st); break;
    default: launch_t<TM, 24, SPREAD>(a, st); break;
  }
}

template <typename TM, bool SPREAD>
bool by_ks(int ks, bool nw8, const QsArgs& a, hipStream_t st) {
  switch (ks) {
    case 12:
      if (nw8) launch_t<TM, 12, SPREAD, 8>(a, st);
      else launch_t<TM, 12, SPREAD>(a, st);
      return true;
    case 24: launch_768<TM, SPREAD>(a.nq_blocks, a, st); return true;
    case 32: launch_t<TM, 32, SPREAD>(a, st); return true;
    default: return false;
  }
}

// QW1P (score_qw1p.h): 16-row stages in a 6-deep ring at D = 768, 4-deep at D = 1024, 32-row
// stages 6-deep at D = 384; 3 fragment groups in flight
template <typename TM, int KS, int SR, int NST, int FD>
void launch_p(const QsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((score_topk_qw1p_kernel<TM, 256, KS, SR, NST, FD>), dim3(a.nqb * a.P), dim3(QW1_NW * 64),
                     0, st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                     a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
}
template <typename TM>
bool by_ks_p(int ks, const QsArgs& a, hipStream_t st) {
  if (a.cap != 256) return false;
  switch (ks) {
    case 12: launch_p<TM, 12, 32, 6, 3>(a, st); return true;
    case 24: launch_p<TM, 24, 16, 6, 3>(a, st); return true;
    case 32: launch_p<TM, 32, 16, 4, 4>(a, st); return true;     // (FD must divide NG = 16)
    default: return false;
  }
}

template <typename TM>
bool by_spread(bool spread, bool nw8, const QsArgs& a, hipStream_t st) {
  if (a.cap != 256) return false;
  return spread ? by_ks<TM, true>(a.ld / V3_BK, nw8, a, st) : by_ks<TM, false>(a.ld / V3_BK, nw8, a, st);
}

}  // namespace

bool qw1_supported(int ld) {
  return ld % V3_BK == 0 && (ld / V3_BK == 12 || ld / V3_BK == 24 || ld / V3_BK == 32);
}
int qw1_rows(int ld, int shape) {
  const int ks = ld / V3_BK;
  if (shape == kQw1Pipelined) return ks == 12 ? 32 : 16;
  return ks == 12 ? Qw1Layout<12>::SR : ks == 24 ? (shape >= 2 ? 16 : Qw1Layout<24>::SR) : Qw1Layout<32>::SR;
}
int qw1_queries(int ld) {
  const int ks = ld / V3_BK;
  return ks == 12 ? Qw1Layout<12>::QT : ks == 24 ? Qw1Layout<24>::QT : Qw1Layout<32>::QT;
}
int qw1_cap(int kp, int ld) { return qw1_supported(ld) && kp + qw1_rows(ld, 0) <= 256 ? 256 : 0; }
bool qw1_nw8_supported(int ld) { return ld == 12 * V3_BK; }

int launch_qw1(int dtype, const QsArgs& a, bool spread, bool nw8, hipStream_t st) {
  if (a.nq_blocks == kQw1Pipelined) {
    const bool ok = dtype == HCR_F16 ? by_ks_p<_Float16>(a.ld / V3_BK, a, st) : by_ks_p<__bf16>(a.ld / V3_BK, a, st);
    if (!ok) return hcr_set_errorf(HCR_EINVAL, "internal: no QW1P kernel for ld=%d cap=%d", a.ld, a.cap);
    HIPC(hipGetLastError());
    return HCR_OK;
  }
  if (nw8 && !qw1_nw8_supported(a.ld))
    return hcr_set_errorf(HCR_EINVAL, "internal: no 8-wave QW1 kernel for ld=%d", a.ld);
  const bool ok = dtype == HCR_F16 ? by_spread<_Float16>(spread, nw8, a, st)
                                   : by_spread<__bf16>(spread, nw8, a, st);
  if (!ok) return hcr_set_errorf(HCR_EINVAL, "internal: no QW1 kernel for ld=%d cap=%d", a.ld, a.cap);
  HIPC(hipGetLastError());
  return HCR_OK;
}

#ifdef HCR_QW1_STAMPS
extern "C" int hcr_debug_qw1_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hcr::hcr_qw1_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif
