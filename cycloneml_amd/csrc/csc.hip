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
// Column-sliced CSR (the margin pass): for F beyond what one XCD's L2 holds
// as fp64 coefficients, the columns are cut into S slices of sliceWidth and
// the nonzeros regrouped slice-major, each slice a CSR over all rows
// (rowptrS[s n + r] .. rowptrS[s n + r + 1]), a row's nonzeros in their
// original order.  The margin pass then runs one slice at a time, so the
// coefficients it gathers (2 MB per slice) stay in L2.  Built without a sort:
// per-row counts, one exclusive scan, a per-row stable scatter.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstdlib>

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

// counts[s n + r] = nonzeros of row r in column slice s (8 lanes per row)
__global__ void k_slice_count(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
                              int64_t n, int S, int width, int64_t* __restrict__ counts) {
  const int sub = threadIdx.x & 7;
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 3;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; r < n; r += stride) {
    int cnt[16];
    for (int s = 0; s < S; ++s) cnt[s] = 0;
    const int64_t p1 = rowptr[r + 1];
    for (int64_t p = rowptr[r] + sub; p < p1; p += 8) {
      const int sl = colidx[p] / width;
      for (int s = 0; s < S; ++s) cnt[s] += (sl == s);
    }
    for (int s = 0; s < S; ++s) {
      int c = cnt[s];
      c += __shfl_xor(c, 1);
      c += __shfl_xor(c, 2);
      c += __shfl_xor(c, 4);
      if (sub == 0) counts[(int64_t)s * n + r] = c;
    }
  }
}

// Stable per-row scatter into the slices (one wave per row, 64 nonzeros per
// step; a nonzero's rank among the same slice's earlier ones by ballot).
__global__ void k_slice_scatter(const int64_t* __restrict__ rowptr,
                                const int32_t* __restrict__ colidx,
                                const double* __restrict__ vals, int64_t n, int S, int width,
                                const int64_t* __restrict__ rowptrS, int32_t* __restrict__ colS,
                                double* __restrict__ valS) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += stride) {
    int64_t base[16];
    for (int s = 0; s < S; ++s) base[s] = rowptrS[(int64_t)s * n + r];
    const int64_t p1 = rowptr[r + 1];
    for (int64_t p0 = rowptr[r]; p0 < p1; p0 += 64) {
      const int64_t p = p0 + lane;
      const bool on = p < p1;
      const int c = on ? colidx[p] : 0;
      const int sl = on ? c / width : -1;
      for (int s = 0; s < S; ++s) {
        const unsigned long long m = __ballot(sl == s);
        if (sl == s) {
          const int rank = __popcll(m & ((1ull << lane) - 1ull));
          colS[base[s] + rank] = c;
          valS[base[s] + rank] = vals[p];
        }
        base[s] += __popcll(m);
      }
    }
  }
}

}  // namespace

namespace cyc {

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

int build_slices(const int64_t* rowptr, const int32_t* colidx, const double* vals, int64_t n,
                 int F, int S, int width, DeviceBuffer& rowptrS, DeviceBuffer& colS,
                 DeviceBuffer& valS, hipStream_t st) {
  int64_t nnz = 0;
  CYC_HIP(hipMemcpyAsync(&nnz, rowptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  const int64_t len = (int64_t)S * n;
  int rc;
  DeviceBuffer counts, tmp;
  if ((rc = rowptrS.reserve(sizeof(int64_t) * ((size_t)len + 1))) ||
      (rc = colS.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1))) ||
      (rc = valS.reserve(sizeof(double) * (size_t)std::max<int64_t>(nnz, 1))) ||
      (rc = counts.reserve(sizeof(int64_t) * ((size_t)len + 1))))
    return rc;
  CYC_HIP(hipMemsetAsync(counts.ptr, 0, sizeof(int64_t) * ((size_t)len + 1), st));
  if (n > 0) {
    hipLaunchKernelGGL(k_slice_count, dim3(8192), dim3(256), 0, st, rowptr, colidx, n, S, width,
                       (int64_t*)counts.ptr);
    CYC_LAUNCH_CHECK("k_slice_count");
  }
  size_t tmpBytes = 0;
  CYC_HIP(rocprim::exclusive_scan(nullptr, tmpBytes, (const int64_t*)counts.ptr,
                                  (int64_t*)rowptrS.ptr, (int64_t)0, (size_t)len + 1,
                                  rocprim::plus<int64_t>(), st));
  if ((rc = tmp.reserve(tmpBytes))) return rc;
  CYC_HIP(rocprim::exclusive_scan(tmp.ptr, tmpBytes, (const int64_t*)counts.ptr,
                                  (int64_t*)rowptrS.ptr, (int64_t)0, (size_t)len + 1,
                                  rocprim::plus<int64_t>(), st));
  if (n > 0) {
    hipLaunchKernelGGL(k_slice_scatter, dim3(8192), dim3(256), 0, st, rowptr, colidx, vals, n, S,
                       width, (const int64_t*)rowptrS.ptr, (int32_t*)colS.ptr,
                       (double*)valS.ptr);
    CYC_LAUNCH_CHECK("k_slice_scatter");
  }
  CYC_HIP(hipStreamSynchronize(st));
  return CYC_OK;
}

}  // namespace cyc

struct cyc_csc_s {
  int64_t n = 0;
  int F = 0;
  int64_t rpb = cyc::kCscRowBlock;   // rows per CSC row block
  cyc::DeviceBuffer colptr, rowidx, cvals;
  // column-sliced CSR (S > 1 only)
  int S = 1, width = 0;
  cyc::DeviceBuffer rowptrS, colS, valS;
};

extern "C" {

int cyc_csc_build_dev(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                      int64_t n, int32_t numFeatures, void* stream, cyc_csc* out) {
  CYC_REQUIRE(out != nullptr && rowptr != nullptr, "output handle and rowptr must not be null");
  CYC_REQUIRE(n >= 0 && numFeatures > 0, "n >= 0 and numFeatures > 0");
  auto* c = new cyc_csc_s();
  c->n = n;
  c->F = numFeatures;
  // rows per row block: the gradient pass keeps one block's multipliers
  // (8 B per row) in L2; CYC_CSC_ROWBLOCK_LOG2 overrides (measurement)
  static const int64_t rowBlock = [] {
    const char* e = std::getenv("CYC_CSC_ROWBLOCK_LOG2");
    const int l = e ? std::atoi(e) : 0;
    return (l >= 10 && l <= 24) ? ((int64_t)1 << l) : cyc::kCscRowBlock;
  }();
  c->rpb = rowBlock;
  int rc = cyc::build_csc(rowptr, colidx, vals, n, numFeatures, c->rpb, c->colptr, c->rowidx,
                          c->cvals,
                          cyc::as_stream(stream));
  // slices of at most kSliceCols columns (2 MB of fp64 coefficients)
  c->S = (int)std::min<int64_t>(16, ((int64_t)numFeatures + cyc::kSliceCols - 1) / cyc::kSliceCols);
  if (c->S < 1) c->S = 1;
  c->width = (numFeatures + c->S - 1) / c->S;
  if (rc == CYC_OK && c->S > 1)
    rc = cyc::build_slices(rowptr, colidx, vals, n, numFeatures, c->S, c->width, c->rowptrS,
                           c->colS, c->valS, cyc::as_stream(stream));
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

int cyc_csc_slices(cyc_csc csc, int32_t* nslices, int32_t* width, const int64_t** rowptrS,
                   const int32_t** colS, const double** valS) {
  CYC_REQUIRE(csc != nullptr, "csc must not be null");
  if (nslices) *nslices = csc->S;
  if (width) *width = csc->width;
  if (rowptrS) *rowptrS = (const int64_t*)csc->rowptrS.ptr;
  if (colS) *colS = (const int32_t*)csc->colS.ptr;
  if (valS) *valS = (const double*)csc->valS.ptr;
  return CYC_OK;
}

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
