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

}  // namespace jmt

extern "C" int jmt_abi_version(void) { return JMT_ABI_VERSION; }
extern "C" const char* jmt_last_error(void) { return jmt::g_err; }
// GEMM (3 dtypes x 4 layouts + split-K reduce) + row ops + CCC + SGD; informational only.
extern "C" int jmt_kernel_count(void) { return 12 + 1 + 8 + 4 + 2 + 4; }
