// Library-level C-ABI entry points (version, error strings).
#include "sv2n_common.h"

extern "C" int sv2n_abi_version(void) { return SV2N_ABI_VERSION; }

extern "C" const char* sv2n_strerror(int code) {
  switch (code) {
    case 0: return "success";
    case SV2N_ERR_ARG: return "sv2n: invalid argument (null pointer or non-positive size)";
    case SV2N_ERR_SHAPE: return "sv2n: unsupported shape (n, heads, layers, widths or LDS budget)";
    case SV2N_ERR_ALIGN: return "sv2n: pointer or leading dimension not 16-byte aligned";
    case SV2N_ERR_WORKSPACE: return "sv2n: workspace too small";
    default: break;
  }
  if (code > 0) return hipGetErrorString((hipError_t)code);
  return "sv2n: unknown error";
}
