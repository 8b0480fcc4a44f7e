// blokify.hip -- InstanceBlock.blokifyWithMaxMemUsage on the device
// (mllib/src/main/scala/org/apache/spark/ml/feature/Instance.scala:114-187,
// Matrices.fromVectors / getDenseSize / getSparseSize,
// mllib-local/src/main/scala/org/apache/spark/ml/linalg/Matrices.scala:1010-1049,
// 1317-1336).
//
// The reference groups a partition's instances greedily: rows are appended
// until the estimated block size (the smaller of the dense and the CSR
// matrix size, plus labels and -- unless every weight is 1 -- weights)
// reaches maxMemUsage; the row that crosses the limit stays in the block.
// A block is stored dense iff its dense size is below its sparse size
// (fromVectors), counting numNonzeros = values != 0.
//
// Two launches over a device shard:
//   k_row_nnz   -- every row's nonzero count and whether its weight is not 1
//                  (one HBM pass over the values; packed in one int32),
//   k_blocks    -- ONE wave walks the rows in order, 64 at a time (loads one
//                  step ahead), carrying (rows, nnz, all-unit) of the open
//                  block; per step a wave prefix scan gives every lane the
//                  block's size estimate were it to end at that lane, and the
//                  first lane at or over the limit closes the block (several
//                  per step when blocks are shorter than 64 rows).
// Output: block starts (nblocks + 1 entries, the last = n) and a dense flag
// per block; all device.  The walk is sequential by definition (each
// boundary depends on the previous one); at 4 bytes per row it streams a
// 200M-row shard in well under a second, once per fit like the reference's
// persisted blocks.
#include <climits>
#include <mutex>

#include "common.hpp"

namespace {

constexpr int64_t kArrayHeader = 12;

__device__ __forceinline__ int64_t dense_size(int64_t cols, int64_t rows) {
  return 8 * cols * rows + kArrayHeader + 9;                   // Matrices.getDenseSize
}
__device__ __forceinline__ int64_t sparse_size(int64_t nnz, int64_t ptrs) {
  return 8 * nnz + 4 * nnz + 4 * ptrs + kArrayHeader * 3 + 9;  // Matrices.getSparseSize
}
// InstanceBlock.getBlockMemUsage (Instance.scala:114-129)
__device__ __forceinline__ int64_t block_mem(int64_t cols, int64_t rows, int64_t nnz, bool unit) {
  const int64_t m = min(dense_size(cols, rows), sparse_size(nnz, rows + 1));
  return unit ? m + 8 * rows + kArrayHeader * 2 : m + 16 * rows + kArrayHeader * 2;
}

// one thread per row: nnz (values != 0) in bits 0..30, weight != 1 in bit 31
__global__ __launch_bounds__(256) void k_row_nnz(const double* __restrict__ X,
                                                 const int64_t* __restrict__ rowptr,
                                                 const double* __restrict__ vals,
                                                 const double* __restrict__ w, int64_t n, int F,
                                                 uint32_t* __restrict__ packed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t nz = 0;
  if (X) {
    const double* x = X + i * F;
    for (int j = 0; j < F; ++j) nz += x[j] != 0.0;
  } else {
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) nz += vals[k] != 0.0;
  }
  const bool nonunit = w && w[i] != 1.0;
  packed[i] = nz | (nonunit ? 0x80000000u : 0u);
}

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const int64_t o = __shfl_up(v, m);
    if (lane >= m) v += o;
  }
  return v;
}

__global__ __launch_bounds__(64) void k_blocks(const uint32_t* __restrict__ packed, int64_t n,
                                               int F, int64_t maxMem, int64_t* __restrict__ starts,
                                               uint8_t* __restrict__ dense,
                                               int64_t* __restrict__ nblocks) {
  const int lane = threadIdx.x;
  int64_t nb = 0;            // blocks emitted
  int64_t cRows = 0, cNnz = 0, cNonunit = 0;   // the open block before this step
  if (lane == 0) starts[0] = 0;
  uint32_t next = lane < n ? packed[lane] : 0u;
  for (int64_t base = 0; base < n; base += 64) {
    const uint32_t cur = next;
    const int64_t nb2 = base + 64 + lane;
    next = nb2 < n ? packed[nb2] : 0u;            // one step ahead
    const bool valid = base + lane < n;
    const int64_t nzv = valid ? (int64_t)(cur & 0x7fffffffu) : 0;
    const int64_t nuv = valid && (cur >> 31) ? 1 : 0;
    const int64_t rowsIncl = lane + 1;
    const int64_t nzIncl = wave_incl_scan(nzv, lane);
    const int64_t nuIncl = wave_incl_scan(nuv, lane);
    int lo = 0;            // first lane of the open block in this step
    int64_t offRows = 0, offNnz = 0, offNu = 0;   // scan values at lane lo - 1
    while (true) {
      const int64_t rows = cRows + rowsIncl - offRows;
      const int64_t nz = cNnz + nzIncl - offNnz;
      const int64_t nu = cNonunit + nuIncl - offNu;
      const bool over = valid && lane >= lo && block_mem(F, rows, nz, nu == 0) >= maxMem;
      const unsigned long long mask = __ballot(over);
      if (mask == 0ull) break;
      const int b = __ffsll((long long)mask) - 1;      // the row that crosses the limit
      const int64_t bRows = __shfl(rows, b), bNz = __shfl(nz, b);
      if (lane == 0) {
        starts[nb + 1] = base + b + 1;
        dense[nb] = dense_size(F, bRows) < sparse_size(bNz, bRows + 1) ? 1 : 0;
      }
      ++nb;
      cRows = cNnz = cNonunit = 0;
      lo = b + 1;
      offRows = b + 1;
      offNnz = __shfl(nzIncl, b);
      offNu = __shfl(nuIncl, b);
      if (lo >= 64) break;
    }
    // carry the open block's rows of this step (the last lane's scan minus the offset)
    const int last = (int)min<int64_t>(63, n - 1 - base);
    if (lo <= last) {
      cRows += (last + 1) - offRows;
      cNnz += __shfl(nzIncl, last) - offNnz;
      cNonunit += __shfl(nuIncl, last) - offNu;
    }
  }
  if (cRows > 0) {   // the last, partial block
    if (lane == 0) {
      starts[nb + 1] = n;
      dense[nb] = dense_size(F, cRows) < sparse_size(cNnz, cRows + 1) ? 1 : 0;
    }
    ++nb;
  }
  if (lane == 0) *nblocks = nb;
}

std::mutex g_mu;
cyc::DeviceBuffer& scratch() {
  static cyc::DeviceBuffer b;
  return b;
}

}  // namespace

extern "C" int cyc_blokify_dev(const double* X, const int64_t* rowptr, const double* vals,
                               const double* weights, int64_t n, int32_t F, int64_t maxMemUsage,
                               int64_t* starts, uint8_t* dense, int64_t* nblocks, void* stream) {
  CYC_REQUIRE(maxMemUsage > 0, "maxMemUsage > 0");   // Instance.scala:149
  CYC_REQUIRE(n >= 0 && F >= 0, "n >= 0 and numFeatures >= 0");
  CYC_REQUIRE(starts && dense && nblocks, "non-null outputs");
  CYC_REQUIRE(n == 0 || (X != nullptr) != (rowptr != nullptr && vals != nullptr),
              "exactly one of the dense rows or the CSR (rowptr, values)");
  hipStream_t st = cyc::as_stream(stream);
  std::lock_guard<std::mutex> g(g_mu);
  if (n == 0) {
    CYC_HIP(hipMemsetAsync(starts, 0, sizeof(int64_t), st));
    CYC_HIP(hipMemsetAsync(nblocks, 0, sizeof(int64_t), st));
    return CYC_OK;
  }
  if (int rc = scratch().reserve(sizeof(uint32_t) * (size_t)n)) return rc;
  uint32_t* packed = (uint32_t*)scratch().ptr;
  hipLaunchKernelGGL(k_row_nnz, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, rowptr,
                     vals, weights, n, (int)F, packed);
  CYC_LAUNCH_CHECK("k_row_nnz");
  hipLaunchKernelGGL(k_blocks, dim3(1), dim3(64), 0, st, packed, n, (int)F, maxMemUsage, starts,
                     dense, nblocks);
  CYC_LAUNCH_CHECK("k_blocks");
  // the scratch is reused by the next call: finish before the lock drops
  CYC_HIP(hipStreamSynchronize(st));
  return CYC_OK;
}
