// Probe of v_mfma_f64_4x4x4f64's operand / result layout and issue rate
// (no documentation in the image): A = 1000 + lane, B = lane, so each
// output D = sum over its (A lane, B lane) pairs, decoded on the host.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* out, double* outB, double* outC, long long* cycles) {
  const int lane = threadIdx.x;
  // unit vectors: A has a single 1 at lane la, B all ones -> D shows which
  // outputs lane la's A value reaches
  double d = 0.0;
  for (int la = 0; la < 64; ++la) {
    const double a = lane == la ? 1.0 : 0.0;
    const double b = 1.0 + lane;   // distinguishes B lanes by magnitude
    double acc = 0.0;
    acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc, 0, 0, 0);
    out[la * 64 + lane] = acc;
  }
  for (int lb = 0; lb < 64; ++lb) {
    const double a = 1.0 + lane;
    const double b = lane == lb ? 1.0 : 0.0;
    double acc = 0.0;
    acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc, 0, 0, 0);
    outB[lb * 64 + lane] = acc;
  }
  // rate: 256 independent-ish chained MFMAs
  double a = 1.0 + lane * 1e-3, b = 2.0, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  long long t0 = clock64();
  for (int i = 0; i < 256; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
  }
  long long t1 = clock64();
  typedef double v4d __attribute__((ext_vector_type(4)));
  v4d e = {0, 0, 0, 0};
  long long t2 = clock64();
  for (int i = 0; i < 256; ++i) {
    e = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e, 0, 0, 0);
  }
  long long t3 = clock64();
  outC[lane] = c0 + c1 + c2 + c3 + e[0] + e[1] + e[2] + e[3];
  if (lane == 0) { cycles[0] = t1 - t0; cycles[1] = t3 - t2; }
}

int main() {
  double *o, *ob, *oc;
  long long* cy;
  hipMalloc(&o, 64 * 64 * 8);
  hipMalloc(&ob, 64 * 64 * 8);
  hipMalloc(&oc, 64 * 8);
  hipMalloc(&cy, 16);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o, ob, oc, cy);
  static double h[64 * 64], hb[64 * 64];
  long long hc[2];
  hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  hipMemcpy(hb, ob, sizeof hb, hipMemcpyDeviceToHost);
  hipMemcpy(hc, cy, 16, hipMemcpyDeviceToHost);
  // A lane la reaches outputs {lane: D != 0}; D value = sum of (1 + lane_b) over its B partners
  for (int la = 0; la < 64; ++la) {
    printf("A%02d ->", la);
    for (int l = 0; l < 64; ++l)
      if (h[la * 64 + l] != 0) printf(" %d(%g)", l, h[la * 64 + l]);
    printf("\n");
  }
  for (int lb = 0; lb < 64; ++lb) {
    printf("B%02d ->", lb);
    for (int l = 0; l < 64; ++l)
      if (hb[lb * 64 + l] != 0) printf(" %d(%g)", l, hb[lb * 64 + l]);
    printf("\n");
  }
  printf("cycles 4x4x4 x1024: %lld (%.1f per MFMA), 16x16x4 x256 dependent: %lld (%.1f)\n", hc[0],
         hc[0] / 1024.0, hc[1], hc[1] / 256.0);
  return 0;
}
