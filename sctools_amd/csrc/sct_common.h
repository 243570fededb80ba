// Internal helpers shared by the libsctools_hip.so translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/sctools_hip.h"

namespace sct {

// Thread-local last-error buffer behind sct_last_error().
void set_error(const char* fmt, ...);
const char* last_error();

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return code;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// RAII device buffer for the *_host convenience entry points.
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 1); }
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace sct

#define SCT_HIP(call)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return ::sct::fail(e_ == hipErrorOutOfMemory ? SCT_E_NOMEM : SCT_E_HIP, "%s: %s (%s:%d)", \
                         #call, hipGetErrorString(e_), __FILE__, __LINE__);                  \
  } while (0)

#define SCT_CHECK(cond, ...)                                 \
  do {                                                       \
    if (!(cond)) return ::sct::fail(SCT_E_INVALID, __VA_ARGS__); \
  } while (0)

#define SCT_LAUNCH_CHECK()                                                                      \
  do {                                                                                          \
    hipError_t e_ = hipGetLastError();                                                          \
    if (e_ != hipSuccess)                                                                       \
      return ::sct::fail(SCT_E_HIP, "kernel launch: %s (%s:%d)", hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                             \
  } while (0)
