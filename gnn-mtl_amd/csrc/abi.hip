// Version and error strings of the C-ABI (include/gnnea.h).
#include "common.h"

extern "C" int gnnea_abi_version(void) { return GNNEA_ABI_VERSION; }

extern "C" const char* gnnea_error_string(int code) {
  switch (code) {
    case GNNEA_OK: return "success";
    case GNNEA_EINVAL: return "gnnea: invalid argument";
    case GNNEA_EWORKSPACE: return "gnnea: workspace too small";
    case GNNEA_EALIGN: return "gnnea: misaligned pointer or leading dimension";
    default: break;
  }
  if (code > 0) return hipGetErrorString((hipError_t)code);
  return "gnnea: unknown error";
}
