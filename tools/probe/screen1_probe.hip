// Time the KMeans one-limb pass (k_screen32<8, 4, 1, false>) on synthetic
// data at the bench's shape (10M rows, d = 256, k = 1024), built with
// -DCYC_PROBE_MODE=bits (kmeans_i8.hip: 2 = no center DMA / waits, 4 = no
// reduction / certification tail, 8 = no row stream) to see which part sets
// its pace.  Results of modes other than 0 are meaningless; only the time is
// read.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize
//     -DCYC_PROBE_MODE=1 -I cycloneml_amd/csrc tools/probe/screen1_probe.hip
//     -L cycloneml_amd -lcyclone -Wl,-rpath,cycloneml_amd -o tools/bin/screen1_m1
#include "../../cycloneml_amd/csrc/kmeans_i8.hip"

#ifndef PROBE_W
#define PROBE_W 4
#endif

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 10000000;
  const int d = 256, k = 1024, S = 8, ktp = k / 32;
  const int64_t rowBytes = 3 * 32 * S;
  std::vector<int8_t> img((size_t)n * rowBytes);
  uint64_t x = 88172645463325252ull;
  for (auto& b : img) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    b = (int8_t)((int)(x % 255) - 127);
  }
  std::vector<int2> meta((size_t)n, int2{0, __builtin_bit_cast(int, 16000.0f)});
  std::vector<double> xnorm((size_t)n, 1000.0), cn(k, 1000.0), g(3 * 64 * ktp, 1.0);
  std::vector<int8_t> cb((size_t)ktp * 3 * S * 1024);
  for (auto& b : cb) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    b = (int8_t)((int)(x % 255) - 127);
  }
  std::vector<float> cq(3 * 64 * ktp);
  for (auto& f : cq) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    f = 1000.0f + (float)(x % 100000);
  }
  cyc::km8::CenterParams P{0, 1, 1.0, k};
  void *dImg, *dMeta, *dXn, *dCb, *dCq, *dG, *dCn, *dP, *dAssign, *dList, *dCnt, *dCr, *dC1, *dCc;
  CK(hipMalloc(&dImg, img.size()));
  CK(hipMalloc(&dMeta, meta.size() * sizeof(int2)));
  CK(hipMalloc(&dXn, n * 8));
  CK(hipMalloc(&dCb, cb.size()));
  CK(hipMalloc(&dCq, cq.size() * 4));
  CK(hipMalloc(&dG, g.size() * 8));
  CK(hipMalloc(&dCn, k * 8));
  CK(hipMalloc(&dP, sizeof(P)));
  CK(hipMalloc(&dAssign, n * 4));
  // sharded appends as the library runs them (kmeans_i8.hpp AppendStage)
  const unsigned scap = cyc::km8::shard_cap(n);
  const size_t cntBytes = sizeof(unsigned) * cyc::km8::kShards * cyc::km8::kShardStride;
  CK(hipMalloc(&dList, (size_t)cyc::km8::kShards * scap * 4));
  CK(hipMalloc(&dCnt, cntBytes));
  CK(hipMalloc(&dCr, (size_t)cyc::km8::kShards * scap * 4));
  CK(hipMalloc(&dC1, (size_t)cyc::km8::kShards * scap * 4 * cyc::km8::kCand1));
  CK(hipMalloc(&dCc, cntBytes));
  CK(hipMemcpy(dImg, img.data(), img.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dMeta, meta.data(), meta.size() * sizeof(int2), hipMemcpyHostToDevice));
  CK(hipMemcpy(dXn, xnorm.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dCb, cb.data(), cb.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dCq, cq.data(), cq.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dG, g.data(), g.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dCn, cn.data(), k * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dP, &P, sizeof(P), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&]() {
    CK(hipMemsetAsync(dCnt, 0, cntBytes, 0));
    CK(hipMemsetAsync(dCc, 0, cntBytes, 0));
    return cyc::km8::launch_screen32<8, PROBE_W, 1, false>(
        dImg, (const int2*)dMeta, (const double*)dXn, n, d, dCb, (const float*)dCq,
        (const double*)dG, (const double*)dCn, (const cyc::km8::CenterParams*)dP, ktp, nullptr,
        nullptr, (int32_t*)dAssign, (int32_t*)dList, (unsigned int*)dCnt, 0, (int32_t*)dCr,
        (int32_t*)dC1, (unsigned int*)dCc, scap);
  };
  for (int i = 0; i < 3; ++i)
    if (launch()) return 1;
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i)
    if (launch()) return 1;
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned int cnt[2] = {0, 0};
  std::vector<unsigned> hc(cntBytes / 4);
  CK(hipMemcpy(hc.data(), dCnt, cntBytes, hipMemcpyDeviceToHost));
  for (int i = 0; i < cyc::km8::kShards; ++i) cnt[0] += hc[(size_t)i * cyc::km8::kShardStride];
  CK(hipMemcpy(hc.data(), dCc, cntBytes, hipMemcpyDeviceToHost));
  for (int i = 0; i < cyc::km8::kShards; ++i) cnt[1] += hc[(size_t)i * cyc::km8::kShardStride];
  std::printf("W %d mode %d: %.3f ms per launch (n %lld; listed %u, candidate rows %u)\n",
              PROBE_W, CYC_PROBE_MODE, ms / reps, (long long)n, cnt[0], cnt[1]);
  return 0;
}
