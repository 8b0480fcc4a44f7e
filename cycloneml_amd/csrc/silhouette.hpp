// silhouette.hpp -- ClusteringEvaluator's Silhouette on the device
// (silhouette.hip), driven by cyc_kmeans_silhouette_{stats,score}_dev in
// kmeans.hip, which sorts the rows by prediction with the plan's counting
// sort first.
//
// Reference: ml/evaluation/ClusteringMetrics.scala -- Silhouette
// .pointSilhouetteCoefficient :66-97 and overallScore :101-103,
// SquaredEuclideanSilhouette :254-400 (computeClusterStats :289-337,
// computeSilhouetteCoefficient :350-366, computeSilhouetteScore :378-399),
// CosineSilhouette :403-600 (computeClusterStats :431-477,
// computeSilhouetteCoefficient :489-504, computeSilhouetteScore :516-547).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cyc {
namespace silh {

// Per-cluster statistics, one flat fp64 buffer of k d + 3 k entries (the
// all-reduce payload of the multi-rank evaluation, treeAggregate's role):
//   [featureSum (k x d) | squaredNormSum (k) | weightSum (k) | rows (k)]
// featureSum is sum_i w_i x_i (Euclidean) or sum_i w_i x_i / |x_i|
// (cosine); squaredNormSum is sum_i |x_i|^2 w_i (0 for cosine); rows counts
// the cluster's rows (a cluster with rows but zero weight is still one of
// the clustersStatsMap keys).
inline int64_t stats_len(int k, int d) { return (int64_t)k * d + 3 * (int64_t)k; }

// pred in [0, k) for every row: bad[0] += rows outside (device); weights
// (nullable) that fail checkNonNegativeWeight's `value >= 0`
// (ml/functions.scala:89-93): *badW = min(*badW, row).
int check_pred(const int32_t* pred, const double* w, int64_t n, int k, unsigned int* bad,
               unsigned long long* badW, hipStream_t st);

// Chunk partials over the rows sorted by cluster (perm, cstart, chunkStart
// as the KMeans counting sort leaves them, kChunk rows per chunk): part
// (chunks x d), pw (weights), pc (squared norms x weights).
int chunk_sums(const double* X, int d, const double* w, const double* xnorm, bool cosine,
               const int32_t* perm, const int64_t* cstart, const int64_t* chunkStart, int k,
               int64_t maxChunks, int kChunk, double* part, double* pw, double* pc,
               hipStream_t st);

// Fold each cluster's chunks in chunk order and add into stats.
int fold(const double* part, const double* pw, const double* pc, const int64_t* cstart,
         const int64_t* chunkStart, int d, int k, double* stats, hipStream_t st);

// Per row the Silhouette coefficient against stats; out[0] += sum_i s_i w_i,
// out[1] += sum_i w_i (fixed-order folds).  scratch: >= 2 ceil(n / 64)
// doubles.
int score(const double* X, const double* xnorm, int64_t n, int d, const int32_t* pred,
          const double* w, int k, bool cosine, const double* stats, double* scratch, double* out,
          hipStream_t st);

}  // namespace silh
}  // namespace cyc
