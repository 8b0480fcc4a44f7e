// capi.cpp -- misc C-ABI entry points, error plumbing and scratch buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "common.hpp"

namespace cyc {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }
const std::string& get_error() { return g_err; }

// java.lang.Double.toString: shortest digits that round-trip; plain decimal
// for 1e-3 <= |x| < 1e7 with at least one fractional digit ("1.0"), else
// "d.dddE<exp>" ("1.0E10", "2.5E-4"); "NaN", "Infinity", "-0.0".
std::string java_double(double x) {
  if (x != x) return "NaN";
  if (x == __builtin_inf()) return "Infinity";
  if (x == -__builtin_inf()) return "-Infinity";
  if (x == 0.0) return std::signbit(x) ? "-0.0" : "0.0";
  char buf[64];
  int prec = 0;
  for (; prec < 17; ++prec) {
    std::snprintf(buf, sizeof(buf), "%.*e", prec, x);
    if (std::strtod(buf, nullptr) == x) break;
  }
  std::snprintf(buf, sizeof(buf), "%.*e", prec, x);
  // buf = [-]D[.DDD]e[+-]XX
  std::string s(buf);
  std::string sign;
  if (s[0] == '-') {
    sign = "-";
    s = s.substr(1);
  }
  const size_t epos = s.find('e');
  const int exp10 = std::atoi(s.c_str() + epos + 1);
  std::string digits;
  for (size_t i = 0; i < epos; ++i)
    if (s[i] != '.') digits += s[i];
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const double ax = std::fabs(x);
  if (ax >= 1e-3 && ax < 1e7) {
    std::string out;
    if (exp10 >= 0) {
      std::string ip = digits.substr(0, std::min<size_t>(digits.size(), exp10 + 1));
      while ((int)ip.size() < exp10 + 1) ip += '0';
      std::string fp = (int)digits.size() > exp10 + 1 ? digits.substr(exp10 + 1) : "0";
      out = ip + "." + fp;
    } else {
      out = "0." + std::string(-exp10 - 1, '0') + digits;
    }
    return sign + out;
  }
  std::string mant = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0");
  return sign + mant + "E" + std::to_string(exp10);
}

int hip_fail(hipError_t e, const char* what, const char* file, int line) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "HIP error %d (%s) in %s at %s:%d", (int)e,
                hipGetErrorString(e), what, file, line);
  set_error(buf);
  if (e == hipErrorOutOfMemory) return CYC_ERR_ALLOC;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return CYC_ERR_NO_DEVICE;
  return CYC_ERR_HIP;
}

// Deferred frees.  hipFree costs ~0.2 ms of host time per call (measured on
// MI355X: tools/probe/hip_malloc_probe.py) and a plan + row image hold ~50
// buffers, so tearing down one KMeans fit took ~14 ms of its caller's time.
// Released buffers therefore go to one process-wide reaper thread that
// frees them in the background (hipFree itself waits for the device, so no
// buffer is freed under work still in flight); an allocation that fails
// waits for the pending frees and retries.  CYC_SYNC_FREE=1 frees inline.
namespace {
struct Reaper {
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<std::pair<void*, int>> q;
  bool started = false, busy = false, stop = false;
  std::thread th;

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !q.empty(); });
      if (q.empty()) break;   // stop requested and nothing left
      const auto it = q.front();
      q.pop_front();
      busy = true;
      lk.unlock();
      (void)hipSetDevice(it.second);
      (void)hipFree(it.first);
      lk.lock();
      busy = false;
      if (q.empty()) idle.notify_all();
    }
    idle.notify_all();
  }
  void push(void* p, int dev) {
    std::lock_guard<std::mutex> g(mu);
    if (!started) {
      started = true;
      th = std::thread([this] { run(); });
      std::atexit([] { reaper_stop(); });
    }
    q.emplace_back(p, dev);
    cv.notify_one();
  }
  void drain() {
    std::unique_lock<std::mutex> lk(mu);
    idle.wait(lk, [&] { return q.empty() && !busy; });
  }
  static Reaper& get() {
    static Reaper* r = new Reaper();   // never destroyed: exit joins it below
    return *r;
  }
  static void reaper_stop() {
    Reaper& r = get();
    {
      std::lock_guard<std::mutex> g(r.mu);
      r.stop = true;
      r.cv.notify_all();
    }
    if (r.th.joinable()) r.th.join();   // the pending frees, before HIP's own teardown
  }
};
bool sync_free() {
  static const bool v = [] {
    const char* e = std::getenv("CYC_SYNC_FREE");
    return e && e[0] == '1';
  }();
  return v;
}
}  // namespace

int DeviceBuffer::reserve(size_t n) {
  int dev = 0;
  CYC_HIP(hipGetDevice(&dev));
  if (ptr && bytes >= n && device == dev) return CYC_OK;
  release();
  if (n == 0) n = 16;
  hipError_t e = hipMalloc(&ptr, n);
  if (e == hipErrorOutOfMemory && !sync_free()) {
    (void)hipGetLastError();
    Reaper::get().drain();   // the memory of pending frees, then once more
    e = hipMalloc(&ptr, n);
  }
  if (e != hipSuccess) {
    ptr = nullptr;
    return cyc::hip_fail(e, "hipMalloc", __FILE__, __LINE__);
  }
  bytes = n;
  device = dev;
  return CYC_OK;
}

void DeviceBuffer::release() {
  if (ptr) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    const int dev = device >= 0 ? device : cur;
    if (sync_free()) {
      if (dev != cur) (void)hipSetDevice(dev);
      (void)hipFree(ptr);
      if (dev != cur) (void)hipSetDevice(cur);
    } else {
      Reaper::get().push(ptr, dev);
    }
  }
  ptr = nullptr;
  bytes = 0;
  device = -1;
}

static std::atomic<bool> g_prof{false};
static std::mutex g_prof_mu;
static std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> g_prof_events;
static std::set<std::string> g_prof_only;   // empty: every named kernel

KernelTimer::KernelTimer(const char* n, hipStream_t s) : name(n), st(s) {
  if (!g_prof.load()) return;
  {
    std::lock_guard<std::mutex> g(g_prof_mu);
    if (!g_prof_only.empty() && !g_prof_only.count(name)) return;
  }
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

int cyc_profile_only(const char* kernels) {
  std::lock_guard<std::mutex> g(cyc::g_prof_mu);
  cyc::g_prof_only.clear();
  if (!kernels) return CYC_OK;
  std::string all(kernels), cur;
  for (char c : all) {
    if (c == ',') {
      if (!cur.empty()) cyc::g_prof_only.insert(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!cur.empty()) cyc::g_prof_only.insert(cur);
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
