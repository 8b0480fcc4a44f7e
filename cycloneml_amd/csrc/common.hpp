// common.hpp -- shared plumbing for libcyclone (gfx950 / MI355X only).
//
// Error model (include/cyclone.h): every extern "C" entry point returns an int
// status and records a thread-local message readable through cyc_last_error().
// Argument checks reproduce the reference's `require` messages so a JVM shim can
// rethrow them as IllegalArgumentException (SURVEY.md 8(b) "Conventions").
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/cyclone.h"

namespace cyc {

void set_error(const std::string& msg);
const std::string& get_error();

// java.lang.Double.toString(x), for `require` messages that interpolate a
// Double (Scala's s"$x").
std::string java_double(double x);

// A hipError_t turned into a CYC_ERR_HIP status with a message.
int hip_fail(hipError_t e, const char* what, const char* file, int line);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Scratch memory grown on demand, one per (device, purpose).  Not thread-safe:
// entry points that use it hold the owning plan's mutex.
struct DeviceBuffer {
  void* ptr = nullptr;
  size_t bytes = 0;
  int device = -1;
  int reserve(size_t n);  // returns CYC_OK or an error status
  void release();
  ~DeviceBuffer() { release(); }
};

// Measurement hook (cyc_profile_enable / cyc_profile_query): brackets one
// launch of a named kernel with HIP events on its stream when enabled.
struct KernelTimer {
  KernelTimer(const char* name, hipStream_t st);
  ~KernelTimer();
  const char* name;
  hipStream_t st;
  hipEvent_t e0 = nullptr;
};

// One-time CSR -> row-blocked CSC transpose (csc.hip): rows in blocks of
// kCscRowBlock; colptr int64[nblocks F + 1] (block-major, then column),
// rowidx int32, cvals fp64; each (block, column)'s rows in increasing order.
constexpr int64_t kCscRowBlock = 1 << 18;
int build_csc(const int64_t* rowptr, const int32_t* colidx, const double* vals, int64_t n, int F,
              int64_t rowBlock,
              DeviceBuffer& colptr, DeviceBuffer& rowidx, DeviceBuffer& cvals, hipStream_t st);

// SparseVector's index requires (ml/linalg/Vectors.scala:617-625) over every
// row of a device CSR (rowptr may start at any base): CYC_ERR_INVALID_ARG
// with the reference's message for the lowest offending row.
int check_csr_indices(const int64_t* rowptr, const int32_t* colidx, int64_t n, int F,
                      hipStream_t st);

// Fixed-margin round-up.
inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Diagnostics (CYC_KMEANS_DUMP=<dir>): the device bytes [p, p + bytes) of
// one call, written to <dir>/<name> after a stream sync.  Never on by
// default; tools/probe/kmeans_state_probe.py reads the files.
// CYCLONE_STRICT_PARITY=1 (cycloneml_amd/config.py): no state carried
// across calls (KMeans bounds, neighbourhoods, incremental sums)
inline bool strict_parity() {
  static const bool on = [] {
    const char* e = std::getenv("CYCLONE_STRICT_PARITY");
    return e && e[0] && e[0] != '0';
  }();
  return on;
}
inline const char* dump_dir() {
  static const char* d = std::getenv("CYC_KMEANS_DUMP");
  return d;
}
inline void dump_dev(const char* name, const void* p, size_t bytes, hipStream_t st) {
  const char* dir = dump_dir();
  if (!dir || !p) return;
  std::vector<char> h(bytes);
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipMemcpy(h.data(), p, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return;
  const std::string path = std::string(dir) + "/" + name;
  if (FILE* f = std::fopen(path.c_str(), "wb")) {
    std::fwrite(h.data(), 1, bytes, f);
    std::fclose(f);
  }
}

// Compute units of the current device (256 on MI355X), for grid sizing.
inline int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return cus;
}

// Split count s in [lo, hi] for a grid of per x s workgroups that runs
// `slots` at a time: the s whose last round is fullest (ties: the smallest),
// so a split-K launch has no near-empty tail round.
inline int64_t balanced_splits(int64_t per, int64_t lo, int64_t hi, int64_t slots) {
  if (hi < lo) hi = lo;
  int64_t best = lo;
  double bestEff = -1.0;
  for (int64_t s = lo; s <= hi; ++s) {
    const int64_t wgs = per * s;
    const int64_t rounds = (wgs + slots - 1) / slots;
    const double eff = (double)wgs / (double)(rounds * slots);
    if (eff > bestEff + 1e-9) {
      bestEff = eff;
      best = s;
    }
  }
  return best;
}

}  // namespace cyc

#define CYC_HIP(expr)                                                     \
  do {                                                                    \
    hipError_t _e = (expr);                                               \
    if (_e != hipSuccess) return cyc::hip_fail(_e, #expr, __FILE__, __LINE__); \
  } while (0)

#define CYC_REQUIRE(cond, msg)                                            \
  do {                                                                    \
    if (!(cond)) {                                                        \
      cyc::set_error(std::string("requirement failed: ") + (msg));        \
      return CYC_ERR_INVALID_ARG;                                         \
    }                                                                     \
  } while (0)

#define CYC_LAUNCH_CHECK(what)                                            \
  do {                                                                    \
    hipError_t _e = hipGetLastError();                                    \
    if (_e != hipSuccess) return cyc::hip_fail(_e, what, __FILE__, __LINE__); \
  } while (0)

// ---------------------------------------------------------------------------
// Device helpers shared by the kernels.
// ---------------------------------------------------------------------------
typedef double cyc_double4 __attribute__((ext_vector_type(4)));

// Non-contracted arithmetic: the reference is JVM code, which never fuses
// a*b+c.  Every translation unit is compiled with -ffp-contract=off and opens
// with `#pragma clang fp contract(off)`; these helpers only name the intent in
// the bit-exact paths (hipcc's __dadd_rn & co. are plain operators here).
#pragma clang fp contract(off)
__device__ __forceinline__ double dsub(double a, double b) { return a - b; }
__device__ __forceinline__ double dmul(double a, double b) { return a * b; }
__device__ __forceinline__ double dadd(double a, double b) { return a + b; }

// mllib/linalg/Vectors.scala:580-587: score = v1(k) - v2(k); sum += score*score
__device__ __forceinline__ double seq_sqdist(const double* __restrict__ a,
                                             const double* __restrict__ b, int d) {
  double s = 0.0;
  for (int j = 0; j < d; ++j) {
    double sc = dsub(a[j], b[j]);
    s = dadd(s, dmul(sc, sc));
  }
  return s;
}

// mllib/linalg/Vectors.scala:500-507 norm(v, 2): sum += v*v; sqrt(sum)
__device__ __forceinline__ double seq_norm2(const double* __restrict__ a, int d) {
  double s = 0.0;
  for (int j = 0; j < d; ++j) s = dadd(s, dmul(a[j], a[j]));
  return __builtin_sqrt(s);  // correctly rounded f64 sqrt on gfx950
}

// ml/impl/Utils.scala:70-80
__device__ __forceinline__ int64_t iut(int64_t i, int64_t j) {
  return (i <= j) ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j;
}
