// score_qw.hip — instantiations and launcher of the wide query-stationary score kernel
// (score_qw.h), in a translation unit of its own (compiles in parallel with the others).
#include <hip/hip_runtime.h>

#include "hcrag.h"
#include "host_common.h"
#define HCR_TOPK_TEMPLATES_ONLY   // the shared non-template kernels live in hcrag_index.hip
#include "score_qw.h"
#include "score_qs_launch.h"

using namespace hcr;

namespace {

template <typename TM, int CAP, int KS, int SR = qw_sr(KS), int NST = QW_NST>
void launch_t(const QsArgs& a, hipStream_t st) {
  if (a.umax)       // the sampling pre-pass (MAXONLY)
    hipLaunchKernelGGL((score_topk_qw_kernel<TM, CAP, KS, SR, NST, true>), dim3(a.nqb * a.P), dim3(V3_NT), 0,
                       st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                       a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp, a.tstride, a.umax);
  else
    hipLaunchKernelGGL((score_topk_qw_kernel<TM, CAP, KS, SR, NST>), dim3(a.nqb * a.P), dim3(V3_NT), 0, st,
                       static_cast<const TM*>(a.rows), a.ld, a.n_rows, static_cast<const TM*>(a.qhat),
                       a.nqb, a.P, a.ntiles, a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
}

template <typename TM, int CAP>
bool by_ks(int ks, const QsArgs& a, hipStream_t st) {
  switch (ks) {
    case 12: launch_t<TM, CAP, 12>(a, st); return true;
    case 24: launch_t<TM, CAP, 24>(a, st); return true;
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
int qw_rows(int ld) { return qw_sr(ld / V3_BK); }
int qw_cap(int kp, int ld) { return kp + qw_sr(ld / V3_BK) <= 256 ? 256 : 0; }   // 0: not supported

int launch_qw(int dtype, const QsArgs& a, hipStream_t st) {
  const bool ok = dtype == HCR_F16 ? by_cap<_Float16>(a, st) : by_cap<__bf16>(a, st);
  if (!ok) return hcr_set_errorf(HCR_EINVAL, "internal: no QW kernel for ld=%d cap=%d", a.ld, a.cap);
  HIPC(hipGetLastError());
  return HCR_OK;
}
