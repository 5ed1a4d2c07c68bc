// score_qw1.hip — instantiations and launcher of the one-wave-per-SIMD query-stationary score
// kernel (score_qw1.h), in a translation unit of its own.
#include <hip/hip_runtime.h>

#include "hcrag.h"
#include "host_common.h"
#define HCR_TOPK_TEMPLATES_ONLY   // the shared non-template kernels live in hcrag_index.hip
#include "score_qw1.h"
#include "score_qs_launch.h"

using namespace hcr;

namespace {

template <typename TM, int KS, bool SPREAD>
void launch_t(const QsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((score_topk_qw1_kernel<TM, 256, KS, SPREAD>), dim3(a.nqb * a.P), dim3(QW1_NW * 64), 0,
                     st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                     a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
}

template <typename TM, bool SPREAD>
bool by_ks(int ks, const QsArgs& a, hipStream_t st) {
  switch (ks) {
    case 24: launch_t<TM, 24, SPREAD>(a, st); return true;
    case 32: launch_t<TM, 32, SPREAD>(a, st); return true;
    default: return false;
  }
}

template <typename TM>
bool by_spread(bool spread, const QsArgs& a, hipStream_t st) {
  if (a.cap != 256) return false;
  return spread ? by_ks<TM, true>(a.ld / V3_BK, a, st) : by_ks<TM, false>(a.ld / V3_BK, a, st);
}

}  // namespace

bool qw1_supported(int ld) { return ld % V3_BK == 0 && (ld / V3_BK == 24 || ld / V3_BK == 32); }
int qw1_rows(int ld) { return ld / V3_BK == 24 ? Qw1Layout<24>::SR : Qw1Layout<32>::SR; }
int qw1_queries(int ld) { return ld / V3_BK == 24 ? Qw1Layout<24>::QT : Qw1Layout<32>::QT; }
int qw1_cap(int kp, int ld) { return qw1_supported(ld) && kp + qw1_rows(ld) <= 256 ? 256 : 0; }

int launch_qw1(int dtype, const QsArgs& a, bool spread, hipStream_t st) {
  const bool ok = dtype == HCR_F16 ? by_spread<_Float16>(spread, a, st) : by_spread<__bf16>(spread, a, st);
  if (!ok) return hcr_set_errorf(HCR_EINVAL, "internal: no QW1 kernel for ld=%d cap=%d", a.ld, a.cap);
  HIPC(hipGetLastError());
  return HCR_OK;
}
