// Library-level C ABI: error plumbing and version. Kernels live in the *.hip translation units.
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>
#include "../../include/adipose_hip.h"

namespace adp {
static thread_local std::string g_err;
static thread_local char g_kernel[160] = "";
static thread_local hipStream_t g_launch_stream = nullptr;

// Per-launch timing of the conv kernels (adp_timing_*): set_kernel, which every conv launcher calls right
// before its main kernel, records a start event on the launch stream; kernel_end, called right after that
// kernel (before any fold / split reduce / bias-sum launch that follows it), records the end event. So the
// pair brackets exactly the kernel rocprofv3 lists under the recorded name.
struct TimedLaunch {
  char name[160];
  hipEvent_t e0, e1;
};
static std::mutex g_time_mu;
static bool g_timing = false;
static std::string g_time_filter;   // (adp_timing_filter: only launches of this kernel name; empty = all)
static bool g_time_open = false;    // a recorded launch waits for its end mark
static std::vector<TimedLaunch> g_timed;
static std::vector<hipEvent_t> g_event_pool;
static hipEvent_t pool_event() {
  hipEvent_t e = nullptr;
  if (!g_event_pool.empty()) {
    e = g_event_pool.back();
    g_event_pool.pop_back();
  } else if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess &&
             hipEventCreate(&e) != hipSuccess) {
    // (timing-only events: no system-scope cache write-back / invalidate when they complete, which both delayed
    //  the next kernel and inflated the measured duration; adp_timing_read reads them after a device sync)
    e = nullptr;
  }
  return e;
}
void set_launch_stream(hipStream_t s) { g_launch_stream = s; }
void set_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_kernel, sizeof(g_kernel), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(g_time_mu);
  g_time_open = false;
  if (!g_timing || (!g_time_filter.empty() && g_time_filter != g_kernel)) return;
  TimedLaunch t{};
  std::snprintf(t.name, sizeof(t.name), "%s", g_kernel);
  t.e0 = pool_event();
  t.e1 = nullptr;
  if (t.e0 && hipEventRecord(t.e0, g_launch_stream) == hipSuccess) {
    g_timed.push_back(t);
    g_time_open = true;
  }
}
void kernel_end() {
  std::lock_guard<std::mutex> lk(g_time_mu);
  if (!g_timing || !g_time_open || g_timed.empty() || g_timed.back().e1) return;
  g_time_open = false;
  hipEvent_t e = pool_event();
  if (e && hipEventRecord(e, g_launch_stream) == hipSuccess) g_timed.back().e1 = e;
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
  // the occupancy depends on the block size and the dynamic LDS as well as the kernel and device
  static std::map<std::tuple<const void*, int, int, size_t>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_tuple(kernel, dev, threads, smem);
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

// the current value of an option (its default when unset: INT_MIN); also the library's report channel for test
// hooks ("tap64_ksplit_last": the split-K factor of the last tap64 launch)
extern "C" int adp_get_option(const char* name) {
  if (!name) return INT_MIN;
  std::lock_guard<std::mutex> lk(adp::g_opt_mu);
  auto it = adp::opts().find(name);
  return it == adp::opts().end() ? INT_MIN : it->second;
}

extern "C" const char* adp_last_error(void) { return adp::g_err.c_str(); }
extern "C" const char* adp_last_kernel(void) { return adp::g_kernel; }
extern "C" int adp_abi_version(void) { return ADP_ABI_VERSION; }

extern "C" int adp_timing(int mode) {
  if (mode < 0 || mode > 2) { adp::set_error("adp_timing: mode 0 (stop), 1 (clear + record) or 2 (stop + clear)"); return -1; }
  std::lock_guard<std::mutex> lk(adp::g_time_mu);
  if (mode != 0) {
    for (auto& t : adp::g_timed) {
      adp::g_event_pool.push_back(t.e0);
      if (t.e1) adp::g_event_pool.push_back(t.e1);
    }
    adp::g_timed.clear();
  }
  adp::g_timing = mode == 1;
  return 0;
}

extern "C" int adp_timing_filter(const char* name) {
  std::lock_guard<std::mutex> lk(adp::g_time_mu);
  adp::g_time_filter = name ? name : "";
  return 0;
}
extern "C" int adp_timing_read(int max, char* names, int name_len, float* ms, int* n) {
  if (!n || (max > 0 && (!names || !ms || name_len < 2))) { adp::set_error("adp_timing_read: bad arguments"); return -1; }
  std::lock_guard<std::mutex> lk(adp::g_time_mu);
  const int cnt = (int)adp::g_timed.size();
  *n = cnt;
  for (int i = 0; i < cnt && i < max; ++i) {
    const auto& t = adp::g_timed[i];
    float v = -1.f;   // -1: no end event (a launcher without kernel_end)
    if (t.e1) {
      if (hipEventSynchronize(t.e1) != hipSuccess || hipEventElapsedTime(&v, t.e0, t.e1) != hipSuccess) {
        adp::set_error("adp_timing_read: event query failed");
        return -2;
      }
    }
    std::snprintf(names + (size_t)i * name_len, name_len, "%s", t.name);
    ms[i] = v;
  }
  return 0;
}
