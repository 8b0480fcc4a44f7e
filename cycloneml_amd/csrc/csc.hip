// csc.hip -- one-time CSR -> CSC transpose of a resident sparse shard.
//
// The reference's sparse gradient is a row-by-row scatter
// (mllib-local/.../ml/linalg/BLAS.scala:790-804, called from
// BinaryLogisticBlockAggregator.scala:130).  On the GPU a scatter of 64
// random columns per row is fp64-atomic bound, so a prepared shard keeps a
// column-major copy built once (like blokifyWithMaxMemUsage, outside the
// training loop): a stable radix sort of the nonzeros by column (rocPRIM,
// header-only) keeps each column's rows in increasing order, so the
// per-column gradient sums run over the rows in the reference's order.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "common.hpp"

namespace {

// rowOf[p] = r for every nonzero p of row r (wave per row)
__global__ void k_row_of(const int64_t* __restrict__ rowptr, int64_t n,
                         int32_t* __restrict__ rowOf) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = r0; r < n; r += stride)
    for (int64_t p = rowptr[r] + lane; p < rowptr[r + 1]; p += 64) rowOf[p] = (int32_t)r;
}

__global__ void k_gather_csc(const int64_t* __restrict__ perm, int64_t nnz,
                             const int32_t* __restrict__ rowOf, const double* __restrict__ vals,
                             int32_t* __restrict__ rowidx, double* __restrict__ cvals) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nnz;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = perm[q];
    rowidx[q] = rowOf[p];
    cvals[q] = vals[p];
  }
}

// colptr from the sorted column keys: colptr[c] = first q with key >= c.
__global__ void k_colptr(const int32_t* __restrict__ keys, int64_t nnz, int F,
                         int64_t* __restrict__ colptr) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= nnz;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int prev = q == 0 ? -1 : keys[q - 1];
    const int cur = q == nnz ? F : keys[q];
    for (int c = prev + 1; c <= cur; ++c) colptr[c] = q;
  }
}

}  // namespace

namespace cyc {

int build_csc(const int64_t* rowptr, const int32_t* colidx, const double* vals, int64_t n, int F,
              DeviceBuffer& colptr, DeviceBuffer& rowidx, DeviceBuffer& cvals, hipStream_t st) {
  int64_t nnz = 0;
  CYC_HIP(hipMemcpyAsync(&nnz, rowptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  int rc;
  if ((rc = colptr.reserve(sizeof(int64_t) * ((size_t)F + 1))) ||
      (rc = rowidx.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1))) ||
      (rc = cvals.reserve(sizeof(double) * (size_t)std::max<int64_t>(nnz, 1))))
    return rc;
  if (nnz == 0) {
    CYC_HIP(hipMemsetAsync(colptr.ptr, 0, sizeof(int64_t) * ((size_t)F + 1), st));
    return CYC_OK;
  }
  DeviceBuffer keysOut, perm, rowOf, tmp;
  unsigned endBit = 1;
  while (endBit < 31 && (1u << endBit) < (unsigned)F) ++endBit;
  size_t tmpBytes = 0;
  rocprim::counting_iterator<int64_t> pos(0);
  CYC_HIP(rocprim::radix_sort_pairs(nullptr, tmpBytes, colidx, (int32_t*)nullptr, pos,
                                    (int64_t*)nullptr, (size_t)nnz, 0, endBit, st));
  if ((rc = keysOut.reserve(sizeof(int32_t) * (size_t)nnz)) ||
      (rc = perm.reserve(sizeof(int64_t) * (size_t)nnz)) || (rc = tmp.reserve(tmpBytes)))
    return rc;
  CYC_HIP(rocprim::radix_sort_pairs(tmp.ptr, tmpBytes, colidx, (int32_t*)keysOut.ptr, pos,
                                    (int64_t*)perm.ptr, (size_t)nnz, 0, endBit, st));
  tmp.release();
  if ((rc = rowOf.reserve(sizeof(int32_t) * (size_t)nnz))) return rc;
  hipLaunchKernelGGL(k_row_of, dim3(4096), dim3(256), 0, st, rowptr, n, (int32_t*)rowOf.ptr);
  CYC_LAUNCH_CHECK("k_row_of");
  hipLaunchKernelGGL(k_gather_csc, dim3(8192), dim3(256), 0, st, (const int64_t*)perm.ptr, nnz,
                     (const int32_t*)rowOf.ptr, vals, (int32_t*)rowidx.ptr, (double*)cvals.ptr);
  CYC_LAUNCH_CHECK("k_gather_csc");
  hipLaunchKernelGGL(k_colptr, dim3(8192), dim3(256), 0, st, (const int32_t*)keysOut.ptr, nnz, F,
                     (int64_t*)colptr.ptr);
  CYC_LAUNCH_CHECK("k_colptr");
  CYC_HIP(hipStreamSynchronize(st));  // scratch buffers are freed on return
  return CYC_OK;
}

}  // namespace cyc

struct cyc_csc_s {
  int64_t n = 0;
  int F = 0;
  cyc::DeviceBuffer colptr, rowidx, cvals;
};

extern "C" {

int cyc_csc_build_dev(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                      int64_t n, int32_t numFeatures, void* stream, cyc_csc* out) {
  CYC_REQUIRE(out != nullptr && rowptr != nullptr, "output handle and rowptr must not be null");
  CYC_REQUIRE(n >= 0 && numFeatures > 0, "n >= 0 and numFeatures > 0");
  auto* c = new cyc_csc_s();
  c->n = n;
  c->F = numFeatures;
  int rc = cyc::build_csc(rowptr, colidx, vals, n, numFeatures, c->colptr, c->rowidx, c->cvals,
                          cyc::as_stream(stream));
  if (rc) {
    delete c;
    return rc;
  }
  *out = c;
  return CYC_OK;
}

int cyc_csc_destroy(cyc_csc csc) {
  delete csc;
  return CYC_OK;
}

int64_t cyc_csc_rows(cyc_csc csc) { return csc ? csc->n : -1; }

int cyc_csc_arrays(cyc_csc csc, const int64_t** colptr, const int32_t** rowidx,
                   const double** values) {
  CYC_REQUIRE(csc != nullptr, "csc must not be null");
  if (colptr) *colptr = (const int64_t*)csc->colptr.ptr;
  if (rowidx) *rowidx = (const int32_t*)csc->rowidx.ptr;
  if (values) *values = (const double*)csc->cvals.ptr;
  return CYC_OK;
}

}  // extern "C"
