// kmeans_sparse.hip -- the per-cluster sums of sparse (CSR) points for the
// KMeans plan (kmeans.hip, kmeans_cos.hip), in a fixed order.
//
// The Lloyd body (mllib/clustering/KMeans.scala:296-311) adds every point
// into its cluster's sum with updateClusterSum -- axpy(w, x, sum) for the
// Euclidean measure (DistanceMeasure.scala:189-191), axpy(w / |x|, x, sum)
// for the cosine one (:466-469); the sparse axpy adds a * x_q to sum(col_q)
// (mllib/linalg/BLAS.scala:93-112) -- plus clusterWeightSum(c) += w and
// costAccum += w * cost (:301-304).  Here every nonzero becomes a (cluster *
// d + column, a * x_q) pair, a stable radix sort groups the pairs of one sum
// entry in row order, and rocprim's deterministic reduce-by-key folds each
// group; the rows' (w, w * cost) pairs are grouped by cluster the same way.
// So the sums are bitwise reproducible run to run (the dense path's sort +
// chunk folds, kmeans.hip, give the same guarantee), and agree with the
// reference's per-partition row order to rounding.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "common.hpp"
#include "kmeans_sparse.hpp"

namespace {

__device__ __forceinline__ double dmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double dadd(double a, double b) { return __dadd_rn(a, b); }

// Per nonzero (wave per row): key = cluster * d + column, value = a * x_q
// with a = w (Euclidean) or w / |x| (cosine: xnorm given).
__global__ __launch_bounds__(256) void k_sp_keys(const int64_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ colidx,
                                                 const double* __restrict__ vals,
                                                 const double* __restrict__ w,
                                                 const double* __restrict__ xnorm, int64_t n,
                                                 int d, const int32_t* __restrict__ assign,
                                                 uint64_t* __restrict__ keys,
                                                 double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t q0 = rowptr[0];
  for (int64_t r = wid; r < n; r += nw) {
    const uint64_t base = (uint64_t)assign[r] * (uint64_t)d;
    const double wr = w ? w[r] : 1.0;
    const double a = xnorm ? wr / xnorm[r] : wr;
    for (int64_t q = rowptr[r] + lane; q < rowptr[r + 1]; q += 64) {
      keys[q - q0] = base + (uint64_t)colidx[q];
      out[q - q0] = a == 1.0 ? vals[q] : dmul(a, vals[q]);
    }
  }
}

struct WC {
  double w, c;
};

struct WCAdd {
  __device__ WC operator()(const WC& x, const WC& y) const {
    return WC{dadd(x.w, y.w), dadd(x.c, y.c)};
  }
};

// rows in cluster order (stable): their (w, w * cost)
__global__ void k_sp_rowvals(const uint32_t* __restrict__ perm, int64_t n,
                             const double* __restrict__ w, const double* __restrict__ cost,
                             WC* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = perm[i];
    const double wr = w ? w[r] : 1.0;
    out[i] = WC{wr, dmul(cost[r], wr)};
  }
}

__global__ void k_sp_add_sums(const uint64_t* __restrict__ uniq, const double* __restrict__ agg,
                              const unsigned int* __restrict__ count, double* __restrict__ sums) {
  const unsigned m = *count;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
    sums[uniq[i]] = dadd(sums[uniq[i]], agg[i]);
}

// wsum(c) += w sums, costSum += the clusters' w * cost sums in cluster order
__global__ void k_sp_add_rows(const uint32_t* __restrict__ uniq, const WC* __restrict__ agg,
                              const unsigned int* __restrict__ count, double* __restrict__ wsum,
                              double* __restrict__ costSum) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned m = *count;
  double s = 0.0;
  for (unsigned i = 0; i < m; ++i) {
    wsum[uniq[i]] = dadd(wsum[uniq[i]], agg[i].w);
    s = dadd(s, agg[i].c);
  }
  costSum[0] = dadd(costSum[0], s);
}

unsigned bits_for(uint64_t v) {
  unsigned b = 1;
  while (b < 64 && (v >> b) != 0) ++b;
  return b;
}

}  // namespace

namespace cyc {
namespace kmsparse {

int cluster_sums(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                 const double* w, const double* xnorm, int64_t n, int d, int k,
                 const int32_t* assign, const double* cost, double* sums, double* wsum,
                 double* costSum, hipStream_t st) {
  if (n <= 0) return CYC_OK;
  CYC_REQUIRE(n < ((int64_t)1 << 32), "a sparse KMeans shard holds fewer than 2^32 rows");
  int64_t ends[2];
  CYC_HIP(hipMemcpyAsync(&ends[0], rowptr, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipMemcpyAsync(&ends[1], rowptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  const int64_t nnz = ends[1] - ends[0];
  CYC_REQUIRE(nnz < ((int64_t)1 << 32), "a sparse KMeans shard holds fewer than 2^32 nonzeros");
  DeviceBuffer keys, keysOut, v, vOut, uniq, agg, cnt, tmp, rkeys, rkeysOut, perm, permOut, rv,
      ruq, ragg;
  int rc;
  if ((rc = cnt.reserve(sizeof(unsigned int) * 2))) return rc;
  unsigned int* count = (unsigned int*)cnt.ptr;
  // 1. the sums: nonzeros grouped by (cluster, column), row order kept
  if (nnz > 0) {
    if ((rc = keys.reserve(8 * (size_t)nnz)) || (rc = keysOut.reserve(8 * (size_t)nnz)) ||
        (rc = v.reserve(8 * (size_t)nnz)) || (rc = vOut.reserve(8 * (size_t)nnz)) ||
        (rc = uniq.reserve(8 * (size_t)nnz)) || (rc = agg.reserve(8 * (size_t)nnz)))
      return rc;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 3) / 4, 8192);
    hipLaunchKernelGGL(k_sp_keys, dim3(grid), dim3(256), 0, st, rowptr, colidx, vals, w, xnorm, n,
                       d, assign, (uint64_t*)keys.ptr, (double*)v.ptr);
    CYC_LAUNCH_CHECK("k_sp_keys");
    const unsigned endBit = bits_for((uint64_t)k * (uint64_t)d);
    size_t tb = 0;
    CYC_HIP(rocprim::radix_sort_pairs(nullptr, tb, (const uint64_t*)keys.ptr, (uint64_t*)nullptr,
                                      (const double*)v.ptr, (double*)nullptr, (size_t)nnz, 0,
                                      endBit, st));
    size_t tb2 = 0;
    CYC_HIP(rocprim::deterministic_reduce_by_key(
        nullptr, tb2, (const uint64_t*)keysOut.ptr, (const double*)vOut.ptr, (size_t)nnz,
        (uint64_t*)uniq.ptr, (double*)agg.ptr, count, rocprim::plus<double>(),
        rocprim::equal_to<uint64_t>(), st));
    if ((rc = tmp.reserve(std::max(tb, tb2)))) return rc;
    CYC_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, (const uint64_t*)keys.ptr,
                                      (uint64_t*)keysOut.ptr, (const double*)v.ptr,
                                      (double*)vOut.ptr, (size_t)nnz, 0, endBit, st));
    CYC_HIP(rocprim::deterministic_reduce_by_key(
        tmp.ptr, tb2, (const uint64_t*)keysOut.ptr, (const double*)vOut.ptr, (size_t)nnz,
        (uint64_t*)uniq.ptr, (double*)agg.ptr, count, rocprim::plus<double>(),
        rocprim::equal_to<uint64_t>(), st));
    hipLaunchKernelGGL(k_sp_add_sums, dim3((unsigned)std::min<int64_t>((nnz + 255) / 256, 8192)),
                       dim3(256), 0, st, (const uint64_t*)uniq.ptr, (const double*)agg.ptr,
                       (const unsigned int*)count, sums);
    CYC_LAUNCH_CHECK("k_sp_add_sums");
  }
  // 2. clusterWeightSum and costAccum: rows grouped by cluster, row order kept
  if ((rc = rkeysOut.reserve(4 * (size_t)n)) || (rc = permOut.reserve(4 * (size_t)n)) ||
      (rc = rv.reserve(sizeof(WC) * (size_t)n)) || (rc = ruq.reserve(4 * (size_t)n)) ||
      (rc = ragg.reserve(sizeof(WC) * (size_t)n)))
    return rc;
  rocprim::counting_iterator<uint32_t> pos(0);
  const unsigned endBitK = bits_for((uint64_t)std::max(k - 1, 1));
  size_t tb = 0, tb2 = 0;
  CYC_HIP(rocprim::radix_sort_pairs(nullptr, tb, (const uint32_t*)assign, (uint32_t*)nullptr, pos,
                                    (uint32_t*)nullptr, (size_t)n, 0, endBitK, st));
  CYC_HIP(rocprim::deterministic_reduce_by_key(
      nullptr, tb2, (const uint32_t*)rkeysOut.ptr, (const WC*)rv.ptr, (size_t)n,
      (uint32_t*)ruq.ptr, (WC*)ragg.ptr, count + 1, WCAdd(), rocprim::equal_to<uint32_t>(), st));
  if ((rc = tmp.reserve(std::max(tb, tb2)))) return rc;
  CYC_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, (const uint32_t*)assign,
                                    (uint32_t*)rkeysOut.ptr, pos, (uint32_t*)permOut.ptr,
                                    (size_t)n, 0, endBitK, st));
  hipLaunchKernelGGL(k_sp_rowvals, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)),
                     dim3(256), 0, st, (const uint32_t*)permOut.ptr, n, w, cost, (WC*)rv.ptr);
  CYC_LAUNCH_CHECK("k_sp_rowvals");
  CYC_HIP(rocprim::deterministic_reduce_by_key(
      tmp.ptr, tb2, (const uint32_t*)rkeysOut.ptr, (const WC*)rv.ptr, (size_t)n,
      (uint32_t*)ruq.ptr, (WC*)ragg.ptr, count + 1, WCAdd(), rocprim::equal_to<uint32_t>(), st));
  hipLaunchKernelGGL(k_sp_add_rows, dim3(1), dim3(64), 0, st, (const uint32_t*)ruq.ptr,
                     (const WC*)ragg.ptr, (const unsigned int*)(count + 1), wsum, costSum);
  CYC_LAUNCH_CHECK("k_sp_add_rows");
  // the scratch is freed on return: finish with it first
  CYC_HIP(hipStreamSynchronize(st));
  return CYC_OK;
}

}  // namespace kmsparse
}  // namespace cyc
