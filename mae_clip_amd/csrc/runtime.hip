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
