// score_qs.hip — instantiations and launcher of the query-stationary score kernel (score_qs.h),
// in a translation unit of their own so they compile in parallel with hcrag_index.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "hcrag.h"
#include "host_common.h"
#define HCR_TOPK_TEMPLATES_ONLY   // the shared non-template kernels live in hcrag_index.hip
#include "score_qs.h"
#include "score_qs_launch.h"

using namespace hcr;

namespace {

template <typename TM, int CAP, int KS, int NQ, int RT, int NST = (RT == 256 ? 4 : 8), int HS = 2>
void launch_t(const QsArgs& a, hipStream_t st) {
  if (a.unit)
    hipLaunchKernelGGL((score_topk_qs_kernel<TM, CAP, KS, true, NQ, RT, NST, HS>), dim3(a.nqb * a.P),
                       dim3(QS_NW * 64), 0, st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, a.inv32,
                       a.mask, static_cast<const TM*>(a.qhat), a.nqb, a.P, a.ntiles, a.tstride,
                       a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
  else
    hipLaunchKernelGGL((score_topk_qs_kernel<TM, CAP, KS, false, NQ, RT, NST, HS>), dim3(a.nqb * a.P),
                       dim3(QS_NW * 64), 0, st, static_cast<const TM*>(a.rows), a.ld, a.n_rows, a.inv32,
                       a.mask, static_cast<const TM*>(a.qhat), a.nqb, a.P, a.ntiles, a.tstride,
                       a.buf, a.tau_g, a.partials, a.pcnt, a.kp);
}

template <typename TM, int CAP>
bool by_ks(int ks, int nq_blocks, const QsArgs& a, hipStream_t st) {
  if (nq_blocks == 2 && ks == 12 && a.hs == 4) {   // 128-deep stages, 4 x 32 KiB ring
    launch_t<TM, CAP, 12, 2, 128, 4, 4>(a, st);
    return true;
  }
  if (nq_blocks == 2) {            // 256 queries per workgroup on 128-row tiles (KS <= 12)
    switch (ks) {
      case 4: launch_t<TM, CAP, 4, 2, 128>(a, st); return true;
      case 6: launch_t<TM, CAP, 6, 2, 128>(a, st); return true;
      case 12: launch_t<TM, CAP, 12, 2, 128>(a, st); return true;
      default: return false;
    }
  }
  switch (ks) {
    case 4: launch_t<TM, CAP, 4, 1, 256>(a, st); return true;
    case 6: launch_t<TM, CAP, 6, 1, 256>(a, st); return true;
    case 12: launch_t<TM, CAP, 12, 1, 256>(a, st); return true;
    case 16: launch_t<TM, CAP, 16, 1, 256>(a, st); return true;
    case 24: launch_t<TM, CAP, 24, 1, 256>(a, st); return true;
    default: return false;
  }
}

template <typename TM>
bool by_cap(const QsArgs& a, hipStream_t st) {
  const int ks = a.ld / V3_BK;
  if (a.cap == 512) return by_ks<TM, 512>(ks, a.nq_blocks, a, st);
  return by_ks<TM, 1024>(ks, a.nq_blocks, a, st);
}

}  // namespace

bool qs_supported(int ld, int nq_blocks) {
  if (ld % V3_BK) return false;
  const int ks = ld / V3_BK;
  // (ks = 32, ld 1024: the 128 query-fragment VGPRs spill; those batches stay on v3/v4)
  if (nq_blocks == 2) return ks == 4 || ks == 6 || ks == 12;
  return ks == 4 || ks == 6 || ks == 12 || ks == 16 || ks == 24;
}

int qs_cap(int kp) { return kp <= 256 ? 512 : 1024; }   // >= 2 x the 256-row tile

int launch_qs(int dtype, const QsArgs& a, hipStream_t st) {
  const bool ok = dtype == HCR_F16 ? by_cap<_Float16>(a, st) : by_cap<__bf16>(a, st);
  if (!ok) return hcr_set_errorf(HCR_EINVAL, "internal: no QS kernel for ld=%d nq_blocks=%d", a.ld, a.nq_blocks);
  HIPC(hipGetLastError());
  return HCR_OK;
}

#ifdef HCR_QS_STAMPS
extern "C" int hcr_debug_qs_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(hcr::hcr_qs_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif
