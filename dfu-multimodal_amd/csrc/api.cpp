// Library-level entry points of libdfu_hip.so: error string, version, zero fill.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "../../include/dfu_hip.h"

static thread_local char g_err[1024] = "";

extern "C" void dfu_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* dfu_last_error_string(void) { return g_err; }

extern "C" int dfu_version(void) { return 1; }

extern "C" int dfu_zero(void* ptr, int64_t bytes, void* stream) {
  if (bytes == 0) return DFU_OK;
  hipError_t e = hipMemsetAsync(ptr, 0, (size_t)bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    dfu_set_error("dfu_zero: %s", hipGetErrorString(e));
    return (int)e;
  }
  return DFU_OK;
}
