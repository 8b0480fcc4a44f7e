// mfma_probe.hip -- microbenchmark of the fp64 matrix / vector rates on gfx950.
// Not part of the product: measures the ceilings the kernels are judged
// against (issue rate and dependent latency of v_mfma_f64_16x16x4_f64, and
// whether fp64 VALU FMAs run beside it).
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void k_mfma(double* out, int iters) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV>
__global__ void k_valu(double* out, int iters) {
  double x[NV];
  for (int i = 0; i < NV; ++i) x[i] = threadIdx.x + i;
  const double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NV; ++i) x[i] = __builtin_fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < NV; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA waves and VALU waves in one workgroup (waves 0..3 MFMA, 4..7 VALU)
__global__ void k_mix(double* out, int iters) {
  const int wave = threadIdx.x >> 6;
  double s = 0;
  if (wave < 4) {
    d4 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    for (int i = 0; i < 4; ++i) s += acc[i][0];
  } else {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < iters * 2; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], 1.0000001, 1e-9);
    for (int i = 0; i < 8; ++i) s += x[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
double timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  double* out;
  hipMalloc(&out, 1024 * 1024 * 8);
  const int iters = 20000;
  const int cus = 256;
  for (int tpb : {256, 512}) {
#define RUN(N)                                                                                \
  {                                                                                           \
    double ms = timeit([&] { hipLaunchKernelGGL(k_mfma<N>, dim3(cus), dim3(tpb), 0, 0, out, iters); }); \
    double flops = 2.0 * 16 * 16 * 4 * N * (double)iters * (tpb / 64) * cus;                  \
    printf("mfma_f64 nacc=%d waves/CU=%d: %.3f ms  %.1f TFLOP/s  %.1f cyc/mfma/SIMD@2.4GHz\n", N, \
           tpb / 64, ms, flops / ms / 1e9, ms * 1e-3 * 2.4e9 / ((double)iters * N * (tpb / 256))); \
  }
    RUN(1) RUN(2) RUN(4) RUN(8)
#undef RUN
  }
  for (int tpb : {256, 512, 1024}) {
    double ms = timeit([&] { hipLaunchKernelGGL(k_valu<8>, dim3(cus), dim3(tpb), 0, 0, out, iters); });
    double flops = 2.0 * 8 * (double)iters * tpb * cus;
    printf("valu_fma_f64 waves/CU=%d: %.3f ms  %.1f TFLOP/s\n", tpb / 64, ms, flops / ms / 1e9);
  }
  {
    double ms = timeit([&] { hipLaunchKernelGGL(k_mix, dim3(cus), dim3(512), 0, 0, out, iters); });
    double fm = 2.0 * 16 * 16 * 4 * 4 * (double)iters * 4 * cus;
    double fv = 2.0 * 8 * (double)iters * 2 * 256 * cus;
    printf("mix (4 mfma waves + 4 valu waves per CU): %.3f ms  mfma %.1f + valu %.1f = %.1f TFLOP/s\n",
           ms, fm / ms / 1e9, fv / ms / 1e9, (fm + fv) / ms / 1e9);
  }
  return 0;
}
