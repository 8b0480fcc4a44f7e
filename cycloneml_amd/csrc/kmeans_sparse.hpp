// kmeans_sparse.hpp -- the fixed-order per-cluster sums of sparse points
// (kmeans_sparse.hip) shared by the Euclidean and cosine KMeans plans.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cyc {
namespace kmsparse {

// updateClusterSum over CSR rows (DistanceMeasure.scala:189-191 / :466-469):
// sums(assign[r]) += a_r x_r with a_r = w_r (xnorm == nullptr) or w_r / xnorm[r]
// (cosine); wsum(assign[r]) += w_r; costSum[0] += sum of w_r cost[r].  All
// accumulate; every group of adds is folded in a fixed order (bitwise
// reproducible).  w may be null (unit weights).
int cluster_sums(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                 const double* w, const double* xnorm, int64_t n, int d, int k,
                 const int32_t* assign, const double* cost, double* sums, double* wsum,
                 double* costSum, hipStream_t st);

}  // namespace kmsparse
}  // namespace cyc
