// Library-level C ABI: error plumbing and version. Kernels live in the *.hip translation units.
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include "../../include/adipose_hip.h"

namespace adp {
static thread_local std::string g_err;
static thread_local char g_kernel[160] = "";
void set_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_kernel, sizeof(g_kernel), fmt, ap);
  va_end(ap);
}
void set_error(const std::string& msg) { g_err = msg; }
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -2;
  }
  return 0;
}
static std::mutex g_opt_mu;
static std::map<std::string, int>& opts() {
  static std::map<std::string, int> m;
  return m;
}
int option(const char* name, int dflt) {
  std::lock_guard<std::mutex> lk(g_opt_mu);
  auto it = opts().find(name);
  return it == opts().end() ? dflt : it->second;
}
int resident_grid(const void* kernel, int threads, size_t smem) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_pair(kernel, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, smem) != hipSuccess) per = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  const int v = std::max(1, per) * std::max(1, cus);
  cache[key] = v;
  return v;
}
}  // namespace adp

extern "C" int adp_set_option(const char* name, int value) {
  if (!name) return -1;
  std::lock_guard<std::mutex> lk(adp::g_opt_mu);
  if (value == INT_MIN) adp::opts().erase(name);   // back to the built-in default
  else adp::opts()[name] = value;
  return 0;
}

extern "C" const char* adp_last_error(void) { return adp::g_err.c_str(); }
extern "C" const char* adp_last_kernel(void) { return adp::g_kernel; }
extern "C" int adp_abi_version(void) { return ADP_ABI_VERSION; }
