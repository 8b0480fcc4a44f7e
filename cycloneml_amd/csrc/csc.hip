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
//
// Row-blocked: the nonzeros are sorted by (row block, column), row blocks of
// kCscRowBlock rows, so the gradient pass walks one row block at a time and
// its multiplier slice (2 MB) stays in each XCD's L2 while every column
// gathers from it.  colptr has nblocks * F + 1 entries: block b, column c
// is [colptr[b F + c], colptr[b F + c + 1]).
//
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
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

// sort key of nonzero p: (row block, column)
__global__ void k_csc_keys(const int32_t* __restrict__ rowOf, const int32_t* __restrict__ colidx,
                           int64_t nnz, int F, int64_t rowBlock,
                           int64_t* __restrict__ keys) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nnz;
       p += (int64_t)gridDim.x * blockDim.x)
    keys[p] = (int64_t)(rowOf[p] / rowBlock) * F + colidx[p];
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

// colptr from the sorted keys: colptr[key] = first q with keys[q] >= key.
__global__ void k_colptr(const int64_t* __restrict__ keys, int64_t nnz, int64_t nkeys,
                         int64_t* __restrict__ colptr) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= nnz;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prev = q == 0 ? -1 : keys[q - 1];
    const int64_t cur = q == nnz ? nkeys : keys[q];
    for (int64_t c = prev + 1; c <= cur; ++c) colptr[c] = q;
  }
}

// Lowest row whose column indices break SparseVector's requires
// (ml/linalg/Vectors.scala:617-625: first index >= 0, strictly increasing,
// last < size); the host re-derives that row's message.
__global__ void k_check_csr(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
                            int64_t n, int F, unsigned long long* __restrict__ bad) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p0 = rowptr[r] - rowptr[0], p1 = rowptr[r + 1] - rowptr[0];
    bool ok = true;
    int prev = -1;
    for (int64_t p = p0; p < p1; ++p) {
      const int c = colidx[p];
      if (c <= prev || c < 0) { ok = false; break; }
      prev = c;
    }
    if (ok && prev >= F) ok = false;
    if (!ok) atomicMin(bad, (unsigned long long)r);
  }
}

}  // namespace

namespace cyc {

int check_csr_indices(const int64_t* rowptr, const int32_t* colidx, int64_t n, int F,
                      hipStream_t st) {
  if (n <= 0) return CYC_OK;
  DeviceBuffer bad;
  int rc;
  if ((rc = bad.reserve(sizeof(unsigned long long)))) return rc;
  CYC_HIP(hipMemsetAsync(bad.ptr, 0xff, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(k_check_csr, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)),
                     dim3(256), 0, st, rowptr, colidx, n, F, (unsigned long long*)bad.ptr);
  CYC_LAUNCH_CHECK("k_check_csr");
  unsigned long long r = 0;
  CYC_HIP(hipMemcpyAsync(&r, bad.ptr, sizeof(r), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  if (r >= (unsigned long long)n) return CYC_OK;
  int64_t b[3];
  CYC_HIP(hipMemcpy(b, rowptr, sizeof(int64_t), hipMemcpyDeviceToHost));
  CYC_HIP(hipMemcpy(b + 1, rowptr + r, 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<int32_t> idx((size_t)(b[2] - b[1]));
  if (!idx.empty())
    CYC_HIP(hipMemcpy(idx.data(), colidx + (b[1] - b[0]), idx.size() * sizeof(int32_t),
                      hipMemcpyDeviceToHost));
  std::string msg;
  if ((int64_t)idx.size() > F) {
    msg = "You provided " + std::to_string(idx.size()) +
          " indices and values, which exceeds the specified vector size " + std::to_string(F) + ".";
  } else if (idx[0] < 0) {
    msg = "Found negative index: " + std::to_string(idx[0]) + ".";
  } else {
    int prev = -1;
    for (int32_t i : idx) {
      if (prev >= i) {
        msg = "Index " + std::to_string(i) + " follows " + std::to_string(prev) +
              " and is not strictly increasing";
        break;
      }
      prev = i;
    }
    if (msg.empty())
      msg = "Index " + std::to_string(prev) + " out of bounds for vector of size " +
            std::to_string(F);
  }
  set_error("requirement failed: " + msg);
  return CYC_ERR_INVALID_ARG;
}

int build_csc(const int64_t* rowptr, const int32_t* colidx, const double* vals, int64_t n, int F,
              int64_t rowBlock, DeviceBuffer& colptr, DeviceBuffer& rowidx, DeviceBuffer& cvals, hipStream_t st) {
  int64_t nnz = 0;
  CYC_HIP(hipMemcpyAsync(&nnz, rowptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  const int64_t nb = std::max<int64_t>((n + rowBlock - 1) / rowBlock, 1);
  const int64_t nkeys = nb * F;
  int rc;
  if ((rc = colptr.reserve(sizeof(int64_t) * ((size_t)nkeys + 1))) ||
      (rc = rowidx.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1))) ||
      (rc = cvals.reserve(sizeof(double) * (size_t)std::max<int64_t>(nnz, 1))))
    return rc;
  if (nnz == 0) {
    CYC_HIP(hipMemsetAsync(colptr.ptr, 0, sizeof(int64_t) * ((size_t)nkeys + 1), st));
    return CYC_OK;
  }
  DeviceBuffer keys, keysOut, perm, rowOf, tmp;
  if ((rc = rowOf.reserve(sizeof(int32_t) * (size_t)nnz)) ||
      (rc = keys.reserve(sizeof(int64_t) * (size_t)nnz)))
    return rc;
  hipLaunchKernelGGL(k_row_of, dim3(4096), dim3(256), 0, st, rowptr, n, (int32_t*)rowOf.ptr);
  CYC_LAUNCH_CHECK("k_row_of");
  hipLaunchKernelGGL(k_csc_keys, dim3(8192), dim3(256), 0, st, (const int32_t*)rowOf.ptr, colidx,
                     nnz, F, rowBlock, (int64_t*)keys.ptr);
  CYC_LAUNCH_CHECK("k_csc_keys");
  unsigned endBit = 1;
  while (endBit < 63 && ((int64_t)1 << endBit) < nkeys) ++endBit;
  size_t tmpBytes = 0;
  rocprim::counting_iterator<int64_t> pos(0);
  CYC_HIP(rocprim::radix_sort_pairs(nullptr, tmpBytes, (const int64_t*)keys.ptr,
                                    (int64_t*)nullptr, pos, (int64_t*)nullptr, (size_t)nnz, 0,
                                    endBit, st));
  if ((rc = keysOut.reserve(sizeof(int64_t) * (size_t)nnz)) ||
      (rc = perm.reserve(sizeof(int64_t) * (size_t)nnz)) || (rc = tmp.reserve(tmpBytes)))
    return rc;
  CYC_HIP(rocprim::radix_sort_pairs(tmp.ptr, tmpBytes, (const int64_t*)keys.ptr,
                                    (int64_t*)keysOut.ptr, pos, (int64_t*)perm.ptr, (size_t)nnz,
                                    0, endBit, st));
  tmp.release();
  keys.release();
  hipLaunchKernelGGL(k_gather_csc, dim3(8192), dim3(256), 0, st, (const int64_t*)perm.ptr, nnz,
                     (const int32_t*)rowOf.ptr, vals, (int32_t*)rowidx.ptr, (double*)cvals.ptr);
  CYC_LAUNCH_CHECK("k_gather_csc");
  hipLaunchKernelGGL(k_colptr, dim3(8192), dim3(256), 0, st, (const int64_t*)keysOut.ptr, nnz,
                     nkeys, (int64_t*)colptr.ptr);
  CYC_LAUNCH_CHECK("k_colptr");
  CYC_HIP(hipStreamSynchronize(st));  // scratch buffers are freed on return
  return CYC_OK;
}

}  // namespace cyc

struct cyc_csc_s {
  int64_t n = 0;
  int F = 0;
  int64_t rpb = cyc::kCscRowBlock;   // rows per CSC row block
  cyc::DeviceBuffer colptr, rowidx, cvals;
};

extern "C" {

int cyc_csc_build_dev(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                      int64_t n, int32_t numFeatures, void* stream, cyc_csc* out) {
  CYC_REQUIRE(out != nullptr && rowptr != nullptr, "output handle and rowptr must not be null");
  CYC_REQUIRE(n >= 0 && numFeatures > 0, "n >= 0 and numFeatures > 0");
  if (int rc = cyc::check_csr_indices(rowptr, colidx, n, numFeatures, cyc::as_stream(stream)))
    return rc;
  auto* c = new cyc_csc_s();
  c->n = n;
  c->F = numFeatures;
  // rows per row block: the gradient pass keeps one block's multipliers
  // (8 B per row) in L2 (2^17 / 2^19 / 2^20 measured no better in round 1)
  c->rpb = cyc::kCscRowBlock;
  int rc = cyc::build_csc(rowptr, colidx, vals, n, numFeatures, c->rpb, c->colptr, c->rowidx,
                          c->cvals, cyc::as_stream(stream));
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

int32_t cyc_csc_features(cyc_csc csc) { return csc ? csc->F : -1; }

int cyc_csc_blocks(cyc_csc csc, int64_t* rows_per_block, int64_t* nblocks) {
  CYC_REQUIRE(csc != nullptr, "csc must not be null");
  if (rows_per_block) *rows_per_block = csc->rpb;
  if (nblocks) *nblocks = std::max<int64_t>((csc->n + csc->rpb - 1) / csc->rpb, 1);
  return CYC_OK;
}

int cyc_csc_arrays(cyc_csc csc, const int64_t** colptr, const int32_t** rowidx,
                   const double** values) {
  CYC_REQUIRE(csc != nullptr, "csc must not be null");
  if (colptr) *colptr = (const int64_t*)csc->colptr.ptr;
  if (rowidx) *rowidx = (const int32_t*)csc->rowidx.ptr;
  if (values) *values = (const double*)csc->cvals.ptr;
  return CYC_OK;
}

}  // extern "C"
