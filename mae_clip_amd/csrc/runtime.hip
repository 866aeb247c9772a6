// Library-level state: ABI version, thread-local error string, device probe.
#include "common.h"
#include "../../include/maeclip.h"
#include <string.h>

namespace maeclip {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace maeclip

extern "C" int32_t maeclip_abi_version(void) { return MAECLIP_ABI_VERSION; }
extern "C" const char* maeclip_last_error(void) { return maeclip::g_err; }
extern "C" int32_t maeclip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Stream-ordered device timestamp: one lane writes the 100-MHz constant
// REALTIME counter (s_memrealtime, a scalar-cache READ) to *dst with a vector
// store. Bracketing a launch with two of these times it inside a captured HIP
// graph, where torch-ROCm refuses event-record nodes.
namespace {
__global__ void timestamp_kernel(int64_t* dst) {
  if (threadIdx.x == 0) *dst = (int64_t)__builtin_amdgcn_s_memrealtime();
}
}  // namespace

extern "C" int32_t maeclip_timestamp(int64_t* dst, void* stream) {
  MC_CHECK_ARG(dst != nullptr, "maeclip_timestamp: null dst");
  hipLaunchKernelGGL(timestamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dst);
  MC_CHECK_LAUNCH("maeclip_timestamp");
  return 0;
}

extern "C" int64_t maeclip_wallclock_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
  return khz;
}
