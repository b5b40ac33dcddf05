// Library identity and error strings of the C ABI (include/codenerf.h).
#include "cn_common.h"

extern "C" const char* cn_version(void) {
  return "libcodenerf_hip 0.1 (gfx950; fp32 MFMA field kernel)";
}

extern "C" const char* cn_error_string(int code) {
  if (code == CN_OK) return "success";
  if (code == CN_EINVAL) return "invalid argument (size, pointer or range)";
  if (code == CN_EUNSUPPORTED) return "configuration not implemented by the gfx950 kernels";
  return hipGetErrorString(static_cast<hipError_t>(code));
}
