// kmeans_cos.hpp -- CosineDistanceMeasure kernels of the KMeans plan
// (kmeans_cos.hip): the cosine forms of computeStatistics, findClosest,
// updateClusterSum and centroid (mllib/clustering/DistanceMeasure.scala:
// 395-514), driven by the plan in kmeans.hip when its measure is COSINE.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cyc {
namespace kmcos {

// computeStatistics (DistanceMeasure.scala:48-76) with the cosine statistic
// 1 - sqrt(1 - d / 2) (:412-417) of every center pair; packed holds k(k+1)/2
// entries, dmin k scratch keys.  cnorm = the centers' VectorWithNorm norms.
int stats(const double* C, const double* cnorm, int k, int d, double* packed,
          unsigned long long* dmin, hipStream_t st);

// The zero-length assert of distance / updateClusterSum (:454, :467): sets
// flag[0] = 1 if a center norm (when checkCenters) or a row norm is not > 0.
int assert_norms(const double* cnorm, int k, bool checkCenters, const double* xnorm, int64_t n,
                 unsigned long long* flag, hipStream_t st);

// Unit directions of the centers for the i8 screen: V = c / |c|, vnorm =
// |V|.  A center whose given norm is not its computed norm (to 2^-40), or
// is zero / non-finite, gets a NaN row, which turns the screen off.
int centers_unit(const double* C, const double* cnorm, int k, int d, double* V, double* vnorm,
                 hipStream_t st);

// list[0..n) = 0..n-1, *count = n: every row to the exact tier.
int list_all(int32_t* list, unsigned int* count, int64_t n, hipStream_t st);

// The reference loop (findClosest with statistics, :421-447, or without,
// :131-150 when stats == nullptr) for the listed rows; Ct is the transposed
// center copy (d4 x kpad).  cost may be null.
int assign_exact(const double* X, const double* xnorm, int d, const double* C, const double* Ct,
                 int kpad, const double* cnorm, int k, const double* stats, const int32_t* list,
                 const unsigned int* count, int64_t maxRows, int32_t* assign, double* cost,
                 hipStream_t st);

// Sparse (CSR) points: the reference loop for every row (dot(sparse, dense)),
// cost written when non-null (the sums: kmeans_sparse.hpp).
int assign_sparse(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                  const double* xnorm, int64_t n, int d, const double* C, const double* cnorm,
                  int k, const double* stats, int32_t* assign, double* cost, hipStream_t st);

// cost[r] = distance(centers(assign[r]), x_r), the value findClosest returns.
int row_cost(const double* X, int64_t n, int d, const double* C, const double* cnorm,
             const double* xnorm, const int32_t* assign, double* cost, hipStream_t st);

// Per-chunk partial cluster sums of (w / |x|) x (:466-469), weights and
// w * cost over the cluster-sorted rows (the Euclidean plan's chunk layout).
int chunk_sums(const double* X, int d, const double* w, const double* xnorm, const double* cost,
               const int32_t* perm, const int64_t* cstart, const int64_t* chunkStart, int k,
               int64_t maxChunks, double* part, double* pw, double* pc, hipStream_t st);

// centroid (:477-483) and isCenterConverged (:161-166) for every cluster
// with wsum > 0: C, cnorm (= 1.0) updated in place, converged cleared by a
// center that moved by more than epsilon.
int update(double* C, double* cnorm, const double* sums, const double* wsum, int k, int d,
           double epsilon, int32_t* converged, hipStream_t st);

}  // namespace kmcos
}  // namespace cyc
