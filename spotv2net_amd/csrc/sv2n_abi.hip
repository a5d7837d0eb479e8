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

#ifdef SV2N_CHECK
// make CHECK=1: bound-check violations counted by the instrumented kernels
// since the last call (each translation unit's counter, reset on read); the
// first failing site id (file · 100 + site) goes to *first_site
extern "C" unsigned sv2n_check_hits_tiled(unsigned*);
extern "C" unsigned sv2n_check_hits_fused(unsigned*);
extern "C" unsigned sv2n_check_hits_canon(unsigned*);
extern "C" unsigned sv2n_check_hits_edge(unsigned*);
extern "C" unsigned sv2n_check_hits(unsigned* first_site) {
  (void)hipDeviceSynchronize();
  unsigned tot = 0u, f = 0u;
  for (auto fn : {sv2n_check_hits_tiled, sv2n_check_hits_fused, sv2n_check_hits_canon,
                  sv2n_check_hits_edge}) {
    unsigned s = 0u;
    const unsigned h = fn(&s);
    if (h && !tot) f = s;
    tot += h;
  }
  if (first_site) *first_site = f;
  return tot;
}
#endif
