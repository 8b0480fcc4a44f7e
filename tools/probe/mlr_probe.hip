// Time k_mlr_margins<7> (multinomial LR margins, C = 100, F = 512) on
// synthetic rows, built with -DCYC_MLR_PROBE=bits (logistic.hip: 1 = X for
// chunk 0 only, 2 = no softmax epilogue, 4 = no W DMA) to see which part
// sets its pace.  Results of modes other than 0 are meaningless.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DCYC_MLR_PROBE=1
//     -I cycloneml_amd/csrc tools/probe/mlr_probe.hip -L cycloneml_amd -lcyclone
//     -Wl,-rpath,'$ORIGIN/../../cycloneml_amd' -o tools/bin/mlr_m1
#include "../../cycloneml_amd/csrc/logistic.hip"

#ifndef PROBE_NW
#define PROBE_NW 8
#endif
#ifndef PROBE_DEPHASE
#define PROBE_DEPHASE false
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

__global__ void fill(double* p, int64_t n, double scale, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27;
    p[i] = scale * ((double)(x >> 11) * 0x1p-53 - 0.5);
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 8333333;
  const int F = 512, C = 100, CT = 7, CP = CT * 16;
  double *X, *lab, *coef, *off, *mult, *slabS, *slabMS;
  CK(hipMalloc(&X, (size_t)n * F * 8));
  CK(hipMalloc(&lab, (size_t)n * 8));
  CK(hipMalloc(&coef, (size_t)(C * F + C) * 8));
  CK(hipMalloc(&off, C * 8));
  CK(hipMalloc(&mult, (size_t)n * CP * 8));
  CK(hipMalloc(&slabS, 256 * 8 * 2 * 8));
  CK(hipMalloc(&slabMS, 256 * 8 * CP * 8));   // 2048 waves either way
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, X, n * F, 2.0, 1);
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, coef, (int64_t)C * F + C, 0.1, 2);
  hipLaunchKernelGGL(fill, dim3(1), dim3(128), 0, 0, off, (int64_t)C, 0.1, 3);
  std::vector<double> hl((size_t)n);
  for (int64_t i = 0; i < n; ++i) hl[(size_t)i] = (double)(i % C);
  CK(hipMemcpy(lab, hl.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&]() {
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mlr_margins<CT, PROBE_NW, PROBE_DEPHASE>),
                       dim3(256 * 8 / PROBE_NW), dim3(64 * PROBE_NW), 0, 0, (const double*)X,
                       (const double*)lab, (const double*)nullptr, n, F, C, (const double*)coef,
                       (const double*)off, mult, slabS, slabMS);
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double tf = 2.0 * F * CP * (double)n / (ms / reps * 1e-3) / 1e12;
  std::printf("mlr NW %d dephase %d probe %d: %.3f ms per launch (n %lld), %.1f TF/s on the padded classes\n",
              PROBE_NW, (int)PROBE_DEPHASE, CYC_MLR_PROBE, ms / reps, (long long)n, tf);
  return 0;
}
