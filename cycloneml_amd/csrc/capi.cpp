// capi.cpp -- misc C-ABI entry points, error plumbing and scratch buffers.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

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

}  // namespace cyc

extern "C" {

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
