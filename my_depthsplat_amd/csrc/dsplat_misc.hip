// Error reporting and version for the libdsplat_hip.so C ABI (include/dsplat_hip.h).
#include "dsplat_common.h"

namespace {
thread_local char g_err[512] = "";
}

namespace dsplat {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace dsplat

extern "C" {
const char* dsplat_last_error(void) { return g_err; }
int dsplat_abi_version(void) { return 1; }
}
