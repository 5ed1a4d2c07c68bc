// host_common.h — host-side helpers of libhcrag_hip.so: thread-local error, HIP checks,
// owning device buffer.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <string>

#include "hcrag.h"

int hcr_set_error(int code, const char* msg);    // defined in hcrag_index.hip
int hcr_set_errorf(int code, const char* fmt, ...);
// Drop the rows past `n` of an index (multi.hip: rolls back a failed hcr_multi_add); internal,
// not part of the C ABI.  Rows past the size are never scored; rho stays an upper bound.
struct hcr_index;
int hcr_index_truncate_internal(hcr_index* ix, int64_t n);

#define HIPC(expr)                                                                          \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      return hcr_set_errorf(e_ == hipErrorOutOfMemory ? HCR_ENOMEM : HCR_EHIP, "%s: %s (%s:%d)", \
                            #expr, hipGetErrorString(e_), __FILE__, __LINE__);              \
    }                                                                                       \
  } while (0)

#define CHECK(expr)                \
  do {                             \
    int rc_ = (expr);              \
    if (rc_ != HCR_OK) return rc_; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t want) {
    if (want <= bytes) return HCR_OK;
    if (p) { HIPC(hipFree(p)); p = nullptr; bytes = 0; }
    want = std::max<size_t>(want, 256);
    HIPC(hipMalloc(&p, want));
    // zero-fill on the null stream, then wait for it: callers use their own non-blocking
    // streams, which do not order against the null stream (an unfinished memset would
    // overwrite what the caller's first copy / kernel writes)
    HIPC(hipMemset(p, 0, want));
    HIPC(hipDeviceSynchronize());
    bytes = want;
    return HCR_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};
