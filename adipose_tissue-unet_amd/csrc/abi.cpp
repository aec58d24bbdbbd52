// Library-level C ABI: error plumbing and version. Kernels live in the *.hip translation units.
#include <hip/hip_runtime.h>
#include <string>
#include "../../include/adipose_hip.h"

namespace adp {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -2;
  }
  return 0;
}
}  // namespace adp

extern "C" const char* adp_last_error(void) { return adp::g_err.c_str(); }
extern "C" int adp_abi_version(void) { return ADP_ABI_VERSION; }
