// C-ABI housekeeping entries of libsnrse_hip.so (see include/snrse.h).
#include <hip/hip_runtime.h>

extern "C" int snrse_abi_version(void) { return 1; }

extern "C" const char* snrse_error_string(int code) { return hipGetErrorString((hipError_t)code); }

// Name and gfx target of the current device into `buf` (nul-terminated); returns 0 or a hipError_t.
extern "C" int snrse_device_name(char* buf, int len) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return (int)e;
  int i = 0;
  for (const char* s = prop.gcnArchName; *s && i < len - 1; ++s) buf[i++] = *s;
  if (len > 0) buf[i] = 0;
  return 0;
}

// Library-wide switch behind the "stats_zeroed" option (declared in common.h, set through
// snrse_set_option in conv.hip): statistics buffers arrive already zeroed.
__attribute__((visibility("hidden"))) int g_snrse_stats_zeroed = 0;
