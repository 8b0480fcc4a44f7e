// Throughput of wave-aggregated returning atomicAdd on one counter vs spread
// counters (one per block % M, 256 B apart), at the one-limb pass's grid
// shape (n / 128 blocks of 4 waves).  Build: hipcc -O3 --offload-arch=gfx950
// tools/atomic_probe.hip -o tools/atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_probe(unsigned* ctr, int spread, int per_wave,
                                               unsigned* out) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  unsigned* c = ctr + (spread > 1 ? (blockIdx.x % spread) * 64 : 0);
  unsigned acc = 0;
  for (int i = 0; i < per_wave; ++i) {
    // about a fifth of the lanes take part, as in the pass's lists
    if ((lane * 7 + i + blockIdx.x) % 5 == 0) acc += atomicAdd(c, 1u);
  }
  out[(size_t)blockIdx.x * 256 + wave * 64 + lane] = acc;
}

int main() {
  const int blocks = 31250;
  unsigned *ctr, *out;
  hipMalloc(&ctr, 64 * 4096 * 4);
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int spreads[] = {1, 8, 64, 512};
  for (int per : {1, 3}) {
    for (int sp : spreads) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(ctr, 0, 64 * 4096 * 4);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(256), 0, 0, ctr, sp, per, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("atomics/wave=%d spread=%d: %.3f ms (%.1f ns per wave-atomic)\n", per, sp, best,
             best * 1e6 / (blocks * 4.0 * per));
    }
  }
  return 0;
}
