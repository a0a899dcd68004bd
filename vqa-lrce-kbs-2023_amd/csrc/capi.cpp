// Error reporting for the C ABI (include/lrce_hip.h): thread-local last-error string.
#include <cstdarg>
#include <cstdio>

#include "lrce_capi.h"

static thread_local char g_err[512] = "";

int lrce_fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int lrce_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lrce_fail(LRCE_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
  return LRCE_OK;
}

extern "C" int lrce_version(void) { return 1; }
extern "C" const char* lrce_last_error(void) { return g_err; }

static const uint64_t* g_rng_offset = nullptr;
extern "C" int lrce_set_rng_offset(const uint64_t* offset) {
  g_rng_offset = offset;
  return LRCE_OK;
}
const uint64_t* lrce_rng_offset() { return g_rng_offset; }
