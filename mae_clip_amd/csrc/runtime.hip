// Library-level state: ABI version, thread-local error string, plan options,
// device probe.
#include "common.h"
#include "../../include/maeclip.h"
#include <string.h>
#include <stdlib.h>
#include <atomic>
#include <mutex>
#include <unordered_map>

namespace maeclip {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace maeclip

// Plan options (maeclip.h maeclip_set_option): the MAECLIP_<name> environment
// snapshotted once, read by the launch planners through maeclip::option().
namespace {
const char* const g_opt_names[MAECLIP_OPT_COUNT] = {
    "GEMM_BM",   "GEMM_SK",   "GEMM_SPLIT", "GEMM_SPLIT_D", "GEMM_SPLIT_MINK", "GEMM_BM128", "GEMM_GRID",
    "WG_SK",     "ATTN_TWO",  "ATTN_ROWS",  "ATTN_DIAG",    "ATTN_BW16",       "ATTN_FW16"};
std::atomic<int32_t> g_opt[MAECLIP_OPT_COUNT];
std::once_flag g_opt_once;
void opt_init() {
  std::call_once(g_opt_once, [] {
    for (int k = 0; k < MAECLIP_OPT_COUNT; ++k) {
      char name[64];
      snprintf(name, sizeof(name), "MAECLIP_%s", g_opt_names[k]);
      const char* e = getenv(name);
      g_opt[k].store(e && *e ? atoi(e) : -1, std::memory_order_relaxed);
    }
  });
}
}  // namespace

namespace maeclip {
int option(int key, int dflt) {
  opt_init();
  const int v = g_opt[key].load(std::memory_order_relaxed);
  return v < 0 ? dflt : v;
}
}  // namespace maeclip

namespace maeclip {
void allow_lds(const void* kernel, int bytes) {
  if (bytes <= 65536) return;
  static std::mutex mu;
  static std::unordered_map<const void*, int> allowed;
  std::lock_guard<std::mutex> lock(mu);
  int& cur = allowed[kernel];
  if (bytes > cur && hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess)
    cur = bytes;
}
}  // namespace maeclip

extern "C" int32_t maeclip_set_option(int32_t key, int32_t value) {
  if (key < 0 || key >= MAECLIP_OPT_COUNT) return INT32_MIN;
  opt_init();
  return g_opt[key].exchange(value < 0 ? -1 : value, std::memory_order_relaxed);
}
extern "C" int32_t maeclip_get_option(int32_t key) {
  if (key < 0 || key >= MAECLIP_OPT_COUNT) return INT32_MIN;
  opt_init();
  return g_opt[key].load(std::memory_order_relaxed);
}

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
