// Error plumbing and version probes of the C-ABI (include/jmt.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/jmt.h"

namespace jmt {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// per-translation-unit device counters of the bounds-check build (common.h JMT_DCHECK)
static unsigned (*g_bounds[16])(bool) = {};
static int g_nbounds = 0;

int register_bounds_counter(unsigned (*read)(bool reset)) {
  if (g_nbounds < 16) g_bounds[g_nbounds++] = read;
  return g_nbounds;
}

}  // namespace jmt

extern "C" int jmt_abi_version(void) { return JMT_ABI_VERSION; }

// Bounds-check build (`make bounds`, -DJMT_BOUNDS=1): failed device index checks since the last
// reset (synchronises the device); -1 in the default build, which has no checks.
extern "C" long long jmt_bounds_violations(int reset) {
  if (jmt::g_nbounds == 0) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  long long n = 0;
  for (int i = 0; i < jmt::g_nbounds; ++i) n += jmt::g_bounds[i](reset != 0);
  return n;
}
extern "C" const char* jmt_last_error(void) { return jmt::g_err; }
// GEMM (3 dtypes x 4 layouts + split-K reduce) + row ops + CCC + SGD; informational only.
extern "C" int jmt_kernel_count(void) { return 12 + 1 + 8 + 4 + 2 + 4; }
