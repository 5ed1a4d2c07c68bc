// errors.cpp — the thread-local error message behind hcr_last_error() (include/hcrag.h).
// Plain C++ (no HIP): shared by the HIP library and the host-only sanitizer build of the
// tokenizer (Makefile target `san`).
#include <cstdarg>
#include <cstdio>
#include <string>

#include "hcrag.h"

static thread_local std::string g_err;

int hcr_set_errorf(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hcr_set_error(int code, const char* msg) { return hcr_set_errorf(code, "%s", msg); }

extern "C" const char* hcr_last_error(void) { return g_err.c_str(); }
