// score_qw1.hip — instantiations and launcher of the one-wave-per-SIMD query-stationary score
// kernel (score_qw1.h, D = 1024), in a translation unit of its own.
#include <hip/hip_runtime.h>

#include "hcrag.h"
#include "host_common.h"
#define HCR_TOPK_TEMPLATES_ONLY   // the shared non-template kernels live in hcrag_index.hip
#include "score_qw1.h"
#include "score_qs_launch.h"

using namespace hcr;

namespace {

template <typename TM>
void launch_t(const QsArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((score_topk_qw1_kernel<TM, 256, 32>), dim3(a.nqb * a.P), dim3(QW1_NW * 64), 0,
                     st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                     a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
}

}  // namespace

bool qw1_supported(int ld) { return ld == 32 * V3_BK; }
int qw1_rows(int ld) { return Qw1Layout<32>::SR; }
int qw1_queries(int ld) { return Qw1Layout<32>::QT; }
int qw1_cap(int kp, int ld) { return qw1_supported(ld) && kp + qw1_rows(ld) <= 256 ? 256 : 0; }

int launch_qw1(int dtype, const QsArgs& a, hipStream_t st) {
  if (!qw1_supported(a.ld) || a.cap != 256)
    return hcr_set_errorf(HCR_EINVAL, "internal: no QW1 kernel for ld=%d cap=%d", a.ld, a.cap);
  if (dtype == HCR_F16) launch_t<_Float16>(a, st);
  else launch_t<__bf16>(a, st);
  HIPC(hipGetLastError());
  return HCR_OK;
}

#ifdef HCR_QW1_STAMPS
extern "C" int hcr_debug_qw1_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hcr::hcr_qw1_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif
