// mfma_i8_layout.hip -- checks the lane maps of v_mfma_i32_32x32x32_i8 with
// exact integer data (not product code).  Assumed: lane l (r = l & 31,
// h = l >> 5) holds A[r][16h + j] and B[16h + j][r], j = 0..15 (bytes of a
// v4i); D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h.
// build: hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_layout.hip -o /tmp/mfma_i8_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[r * 32 + 16 * h + j];
    b[j] = B[(16 * h + j) * 32 + r];
  }
  v4i va, vb;
  __builtin_memcpy(&va, a, 16);
  __builtin_memcpy(&vb, b, 16);
  v16i acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(va, vb, acc, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
    D[row * 32 + col] = acc[reg];
  }
}

int main() {
  signed char hA[1024], hB[1024];
  int ref[1024], got[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) {
    hA[i] = (signed char)(rand() % 255 - 127);
    hB[i] = (signed char)(rand() % 255 - 127);
  }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 32 + j];
      ref[i * 32 + j] = s;
    }
  signed char *dA, *dB;
  int* dD;
  hipMalloc(&dA, 1024);
  hipMalloc(&dB, 1024);
  hipMalloc(&dD, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(got, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; ++i) bad += got[i] != ref[i];
  printf("32x32x32 i8 layout: %d of 1024 wrong\n", bad);
  return bad != 0;
}
