// Error reporting and version for the libdsplat_hip.so C ABI (include/dsplat_hip.h).
#include "dsplat_common.h"

#include <map>
#include <mutex>
#include <utility>

namespace {
thread_local char g_err[512] = "";
// (kernel, device) -> the dynamic-LDS limit already opted into (hipFuncSetAttribute is a
// per-device setting); guarded, so concurrent callers on different threads / devices are safe
std::mutex g_attr_mu;
std::map<std::pair<const void*, int>, size_t> g_attr;
}

namespace dsplat {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

__global__ void k_zero_u32(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0u;
}

int zero_async(void* p, size_t bytes, hipStream_t st, const char* what) {
  if (bytes == 0) return 0;
  if (bytes % 4 != 0) {
    set_error("%s: zero_async needs a multiple of 4 bytes (%zu)", what, bytes);
    return 1;
  }
  const size_t n = bytes / 4;
  const unsigned blocks = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  k_zero_u32<<<blocks, 256, 0, st>>>(static_cast<uint32_t*>(p), n);
  return check_launch(what);
}

int ensure_dyn_lds(const void* fn, size_t bytes, const char* what) {
  int dev = 0;
  if (int e = check_hip(hipGetDevice(&dev), what)) return e;
  std::lock_guard<std::mutex> lock(g_attr_mu);
  size_t& cur = g_attr[{fn, dev}];
  if (bytes <= cur) return 0;
  if (int e = check_hip(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes), what))
    return e;
  cur = bytes;
  return 0;
}
}  // namespace dsplat

extern "C" {
const char* dsplat_last_error(void) { return g_err; }
int dsplat_abi_version(void) { return 20; }
}
