// kmeans_init.hip -- the executor side of k-means|| initialisation
// (mllib/clustering/KMeans.scala:370-432) on the device.
//
// Each k-means|| step the reference updates the point costs (:392-396, here
// cyc_kmeans_point_cost_dev + a min) and then, per partition, keeps the
// points that pass a Bernoulli draw (:400-404):
//   val rand = new XORShiftRandom(seed ^ (step << 16) ^ index)
//   pointCosts.filter { case (_, c) => rand.nextDouble() < 2.0 * c * k / sumCosts }
// one nextDouble per point, in the partition's order.  XORShiftRandom
// (core/src/main/scala/org/apache/spark/util/random/XORShiftRandom.scala) is
// java.util.Random's nextDouble over the xorshift step
//   x ^= x << 21; x ^= x >>> 35; x ^= x << 4
// with the seed hashed by scala.util.hashing.MurmurHash3.bytesHash (the
// scala-library's published x86_32 MurmurHash3, not in the reference tree).
// The step is linear over GF(2), so the state after m steps is T^m x: the
// host precomputes the 64 matrices T^(2^j) (32 KB, one column per input
// bit), and every thread jumps to its own 64-point run of a partition and
// draws it sequentially -- the same doubles the reference draws, so the
// same points are chosen.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace {

constexpr int kRun = 64;   // points drawn sequentially per thread

__host__ __device__ inline uint64_t xs_step(uint64_t x) {
  x ^= x << 21;
  x ^= x >> 35;
  x ^= x << 4;
  return x;
}

// scala.util.hashing.MurmurHash3.bytesHash (little-endian 4-byte blocks)
uint32_t murmur3_bytes(const uint8_t* data, int n, uint32_t seed) {
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  auto mix = [&](uint32_t h, uint32_t k) {
    k *= 0xCC9E2D51u;
    k = rotl(k, 15);
    k *= 0x1B873593u;
    return h ^ k;
  };
  uint32_t h = seed;
  int i = 0;
  for (; n - i >= 4; i += 4) {
    const uint32_t k = (uint32_t)data[i] | (uint32_t)data[i + 1] << 8 |
                       (uint32_t)data[i + 2] << 16 | (uint32_t)data[i + 3] << 24;
    h = mix(h, k);
    h = rotl(h, 13) * 5 + 0xE6546B64u;
  }
  uint32_t k = 0;
  const int rem = n - i;
  if (rem == 3) k ^= (uint32_t)data[i + 2] << 16;
  if (rem >= 2) k ^= (uint32_t)data[i + 1] << 8;
  if (rem >= 1) {
    k ^= data[i];
    h = mix(h, k);
  }
  h ^= (uint32_t)n;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// y = M x over GF(2), M given by its 64 columns
__host__ __device__ inline uint64_t gf2_apply(const uint64_t* M, uint64_t x) {
  uint64_t y = 0;
  for (int b = 0; b < 64; ++b)
    if ((x >> b) & 1) y ^= M[b];
  return y;
}

// The 64 jump matrices T^(2^j), built once per process.
const uint64_t* jump_matrices_host() {
  static std::vector<uint64_t> J;
  static std::once_flag once;
  std::call_once(once, [] {
    J.resize(64 * 64);
    for (int b = 0; b < 64; ++b) J[b] = xs_step(1ull << b);
    for (int j = 1; j < 64; ++j)
      for (int b = 0; b < 64; ++b) J[j * 64 + b] = gf2_apply(&J[(j - 1) * 64], J[(j - 1) * 64 + b]);
  });
  return J.data();
}

// One thread per 64-point run: binary search of its partition, the jump to
// state 2 q (two draws per point), then the partition's draws in order.
__global__ __launch_bounds__(256) void k_kmpar_sample(
    const double* __restrict__ costs, const int64_t* __restrict__ starts,
    const int64_t* __restrict__ runStart, const uint64_t* __restrict__ state0, int P,
    const uint64_t* __restrict__ jump, double k2, double sumCosts, uint8_t* __restrict__ chosen) {
  __shared__ uint64_t J[64 * 64];
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) J[e] = jump[e];
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= runStart[P]) return;
  int lo = 0, hi = P;   // partition = last p with runStart[p] <= t
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (runStart[mid] <= t) lo = mid; else hi = mid;
  }
  const int p = lo;
  const int64_t q0 = (t - runStart[p]) * kRun;          // first position in the partition
  const int64_t i0 = starts[p] + q0, i1 = min<int64_t>(starts[p + 1], i0 + kRun);
  uint64_t x = state0[p];
  const uint64_t m = 2 * (uint64_t)q0;
  for (int j = 0; j < 64; ++j)
    if ((m >> j) & 1) x = gf2_apply(J + j * 64, x);
  for (int64_t i = i0; i < i1; ++i) {
    x = xs_step(x);
    const uint64_t a = x & ((1ull << 26) - 1);          // next(26)
    x = xs_step(x);
    const uint64_t b = x & ((1ull << 27) - 1);          // next(27)
    const double u = (double)((a << 27) + b) * 0x1p-53;  // java.util.Random.nextDouble
    // rand.nextDouble() < 2.0 * c * k / sumCosts
    chosen[i] = u < 2.0 * costs[i] * k2 / sumCosts ? 1 : 0;
  }
}

}  // namespace

extern "C" {

uint64_t cyc_xorshift_hash_seed(int64_t seed) {
  // XORShiftRandom.hashSeed: ByteBuffer.putLong (big-endian), low then high
  uint8_t b[8];
  for (int i = 0; i < 8; ++i) b[i] = (uint8_t)((uint64_t)seed >> (56 - 8 * i));
  const uint32_t lo = murmur3_bytes(b, 8, 0x3C074A61u);
  const uint32_t hi = murmur3_bytes(b, 8, lo);
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}

int cyc_kmeans_parallel_sample_dev(const double* costs, const int64_t* part_starts,
                                   int32_t num_parts, int32_t first_part_index, int32_t seed,
                                   int32_t step, int32_t k, double sum_costs, uint8_t* chosen,
                                   void* stream) {
  CYC_REQUIRE(part_starts != nullptr && num_parts >= 1, "part_starts must hold num_parts + 1 offsets");
  CYC_REQUIRE(part_starts[0] == 0, "part_starts[0] must be 0");
  for (int p = 0; p < num_parts; ++p)
    CYC_REQUIRE(part_starts[p + 1] >= part_starts[p], "part_starts must be non-decreasing");
  const int64_t n = part_starts[num_parts];
  if (n == 0) return CYC_OK;
  CYC_REQUIRE(costs != nullptr && chosen != nullptr, "costs and chosen must not be null");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  hipStream_t st = cyc::as_stream(stream);
  // per partition: new XORShiftRandom(seed ^ (step << 16) ^ index), the Int
  // widened to Long; the 64-point runs of every partition
  std::vector<uint64_t> s0(num_parts);
  std::vector<int64_t> runs(num_parts + 1, 0);
  for (int p = 0; p < num_parts; ++p) {
    const int32_t idx = first_part_index + p;
    const int32_t init = seed ^ (int32_t)((uint32_t)step << 16) ^ idx;
    s0[p] = cyc_xorshift_hash_seed((int64_t)init);
    runs[p + 1] = runs[p] + (part_starts[p + 1] - part_starts[p] + kRun - 1) / kRun;
  }
  // the jump matrices stay resident for the process (never freed: no
  // device call from a static destructor after the runtime's teardown)
  // (one copy per device: the caller's stream may live on any GPU)
  constexpr int kMaxDev = 64;
  static std::mutex mu;
  static uint64_t* jumps[kMaxDev] = {};
  std::lock_guard<std::mutex> g(mu);
  int rc, dev = 0;
  CYC_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDev) {
    cyc::set_error("device index out of range");
    return CYC_ERR_INVALID_ARG;
  }
  if (!jumps[dev]) {
    CYC_HIP(hipMalloc((void**)&jumps[dev], sizeof(uint64_t) * 64 * 64));
    CYC_HIP(hipMemcpy(jumps[dev], jump_matrices_host(), sizeof(uint64_t) * 64 * 64,
                      hipMemcpyHostToDevice));
  }
  uint64_t* jump = jumps[dev];
  cyc::DeviceBuffer meta;
  const size_t b1 = sizeof(int64_t) * (num_parts + 1), b2 = b1, b3 = sizeof(uint64_t) * num_parts;
  if ((rc = meta.reserve(b1 + b2 + b3))) return rc;
  std::vector<uint8_t> host(b1 + b2 + b3);
  std::memcpy(host.data(), part_starts, b1);
  std::memcpy(host.data() + b1, runs.data(), b2);
  std::memcpy(host.data() + b1 + b2, s0.data(), b3);
  CYC_HIP(hipMemcpyAsync(meta.ptr, host.data(), host.size(), hipMemcpyHostToDevice, st));
  const int64_t threads = runs[num_parts];
  hipLaunchKernelGGL(k_kmpar_sample, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                     costs, (const int64_t*)meta.ptr, (const int64_t*)((char*)meta.ptr + b1),
                     (const uint64_t*)((char*)meta.ptr + b1 + b2), num_parts,
                     (const uint64_t*)jump, (double)k, sum_costs, chosen);
  CYC_LAUNCH_CHECK("k_kmpar_sample");
  CYC_HIP(hipStreamSynchronize(st));   // the staging buffers are freed on return
  return CYC_OK;
}

}  // extern "C"
