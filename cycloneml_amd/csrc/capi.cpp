// capi.cpp -- misc C-ABI entry points, error plumbing and scratch buffers.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common.hpp"

namespace cyc {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }
const std::string& get_error() { return g_err; }

int hip_fail(hipError_t e, const char* what, const char* file, int line) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "HIP error %d (%s) in %s at %s:%d", (int)e,
                hipGetErrorString(e), what, file, line);
  set_error(buf);
  if (e == hipErrorOutOfMemory) return CYC_ERR_ALLOC;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return CYC_ERR_NO_DEVICE;
  return CYC_ERR_HIP;
}

int DeviceBuffer::reserve(size_t n) {
  int dev = 0;
  CYC_HIP(hipGetDevice(&dev));
  if (ptr && bytes >= n && device == dev) return CYC_OK;
  release();
  if (n == 0) n = 16;
  CYC_HIP(hipMalloc(&ptr, n));
  bytes = n;
  device = dev;
  return CYC_OK;
}

void DeviceBuffer::release() {
  if (ptr) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (device >= 0 && device != cur) (void)hipSetDevice(device);
    (void)hipFree(ptr);
    if (device >= 0 && device != cur) (void)hipSetDevice(cur);
  }
  ptr = nullptr;
  bytes = 0;
  device = -1;
}

static std::atomic<bool> g_prof{false};
static std::mutex g_prof_mu;
static std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> g_prof_events;

KernelTimer::KernelTimer(const char* n, hipStream_t s) : name(n), st(s) {
  if (!g_prof.load()) return;
  if (hipEventCreate(&e0) != hipSuccess || hipEventRecord(e0, st) != hipSuccess) e0 = nullptr;
}

KernelTimer::~KernelTimer() {
  if (!e0) return;
  hipEvent_t e1 = nullptr;
  if (hipEventCreate(&e1) != hipSuccess || hipEventRecord(e1, st) != hipSuccess) return;
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_prof_events[name].emplace_back(e0, e1);
}

}  // namespace cyc

extern "C" {

int cyc_profile_enable(int enable) {
  cyc::g_prof.store(enable != 0);
  return CYC_OK;
}

int cyc_profile_query(const char* kernel, double* total_ms, int64_t* launches) {
  CYC_REQUIRE(kernel && total_ms && launches, "kernel name and outputs must not be null");
  std::lock_guard<std::mutex> g(cyc::g_prof_mu);
  double tot = 0.0;
  int64_t cnt = 0;
  auto it = cyc::g_prof_events.find(kernel);
  if (it != cyc::g_prof_events.end()) {
    for (auto& e : it->second) {
      CYC_HIP(hipEventSynchronize(e.second));
      float ms = 0.f;
      CYC_HIP(hipEventElapsedTime(&ms, e.first, e.second));
      tot += ms;
      ++cnt;
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    cyc::g_prof_events.erase(it);
  }
  *total_ms = tot;
  *launches = cnt;
  return CYC_OK;
}


const char* cyc_last_error(void) { return cyc::get_error().c_str(); }

int cyc_version(void) { return 100; /* 0.1.0 */ }

int cyc_device_count(int* count) {
  CYC_REQUIRE(count != nullptr, "count must not be null");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    *count = 0;
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  *count = n;
  return CYC_OK;
}

int cyc_set_device(int device) {
  CYC_HIP(hipSetDevice(device));
  return CYC_OK;
}

int cyc_synchronize(void* stream) {
  CYC_HIP(hipStreamSynchronize(cyc::as_stream(stream)));
  return CYC_OK;
}

}  // extern "C"
