/*
 * cyclone_oracle.c -- CPU restatement of the reference's MLlib hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * kernels in cycloneml_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never links it.
 *
 * Every function restates one Scala loop of the reference (wmeddie/CycloneML,
 * a Spark 3.3.0-SNAPSHOT MLlib tree mounted at /root/reference) in the same
 * evaluation order.  Compile with -ffp-contract=off: the JVM never fuses
 * a*b+c, so neither may we.  Where the reference calls netlib BLAS
 * (dev.ludovic.netlib 2.2.0, not present in the container) the restatement
 * follows the published netlib reference loops (Fortran BLAS dgemv/dgemm/
 * dspr/ddot/daxpy/dscal), the algorithm JavaBLAS / f2j implement.
 *
 * Parity pinning: see DESIGN.md "Oracle" -- the reference's known-answer
 * tests (RowMatrixSuite gram, KMeansSuite weighted centers, BLASSuite,
 * aggregator suites' naive loops) are committed under tests/golden and
 * checked by tests/test_oracle_golden.py.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Vectors / MLUtils                                                        */
/* ------------------------------------------------------------------------ */

/* mllib/linalg/Vectors.scala:489-514 (p == 2): sum += v*v; sqrt(sum) */
double orc_norm2(const double* x, int64_t n) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += x[i] * x[i];
  return sqrt(s);
}

/* mllib/linalg/Vectors.scala:580-587 dense/dense sqdist:
 *   score = v1(k) - v2(k); squaredDistance += score * score            */
double orc_sqdist(const double* a, const double* b, int64_t n) {
  double s = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    double score = a[k] - b[k];
    s += score * score;
  }
  return s;
}

/* mllib/linalg/Vectors.scala:598-622 sqdist(sparse v1, dense v2) */
double orc_sqdist_sparse_dense(const int32_t* idx, const double* val, int64_t nnz,
                               const double* dense, int64_t n) {
  int64_t kv1 = 0;
  int64_t iv1 = nnz > 0 ? idx[0] : -1;
  double s = 0.0;
  for (int64_t kv2 = 0; kv2 < n; ++kv2) {
    double score;
    if (kv2 != iv1) {
      score = dense[kv2];
    } else {
      score = val[kv1] - dense[kv2];
      if (kv1 < nnz - 1) { kv1 += 1; iv1 = idx[kv1]; }
    }
    s += score * score;
  }
  return s;
}

/* mllib/linalg/BLAS.scala:153-169 dot(sparse x, dense y): sum += xv(k) * y(xi(k)) */
double orc_dot_sparse_dense(const int32_t* idx, const double* val, int64_t nnz,
                            const double* dense) {
  double s = 0.0;
  for (int64_t k = 0; k < nnz; ++k) s += val[k] * dense[idx[k]];
  return s;
}

/* mllib/util/MLUtils.scala:44-50 EPSILON = 2^-52 (the halving loop) */
static double orc_epsilon(void) {
  double eps = 1.0;
  while ((1.0 + (eps / 2.0)) != 1.0) eps /= 2.0;
  return eps;
}

/* mllib/util/MLUtils.scala:533-576 fastSquaredDistance, v1 dense (a center)
 * and v2 sparse (a libsvm point): the norm-trick branch :560-573 with
 * precision = 1e-6.  v1.isInstanceOf[DenseVector] && v2 dense takes sqdist
 * directly (:557-558); that case is orc_sqdist. */
double orc_fast_sqdist_dense_sparse(const double* v1, double norm1,
                                    const int32_t* idx, const double* val, int64_t nnz,
                                    double norm2, int64_t n) {
  const double EPS = orc_epsilon();
  const double precision = 1e-6;
  double sumSquaredNorm = norm1 * norm1 + norm2 * norm2;
  double normDiff = norm1 - norm2;
  double precisionBound1 = 2.0 * EPS * sumSquaredNorm / (normDiff * normDiff + EPS);
  double sqDist;
  if (precisionBound1 < precision) {
    /* dot(v1 dense, v2 sparse) dispatches to dot(sparse, dense) */
    sqDist = sumSquaredNorm - 2.0 * orc_dot_sparse_dense(idx, val, nnz, v1);
  } else {
    double dotValue = orc_dot_sparse_dense(idx, val, nnz, v1);
    /* math.max(x, 0.0): NaN stays NaN, -0.0 becomes 0.0 (java.lang.Math.max) */
    double t = sumSquaredNorm - 2.0 * dotValue;
    sqDist = (t != t) ? t : (t > 0.0 ? t : 0.0);
    double precisionBound2 = EPS * (sumSquaredNorm + 2.0 * fabs(dotValue)) / (sqDist + EPS);
    if (precisionBound2 > precision) {
      sqDist = orc_sqdist_sparse_dense(idx, val, nnz, v1, n);
    }
  }
  return sqDist;
}

/* MLUtils.scala:542-543, the second require of fastSquaredDistance:
 *   require(norm1 >= 0.0 && norm2 >= 0.0, s"Both norms should be greater or
 *   equal to 0.0, found norm1=$norm1, norm2=$norm2")
 * An IllegalArgumentException ends the Spark task, so the first failure is
 * recorded (thread-local, per partition thread) and the loops below stop;
 * the Python wrapper rethrows it with the reference's text.               */
static _Thread_local int g_req_failed = 0;
static _Thread_local double g_req_n1, g_req_n2;

static int orc_require_norms(double norm1, double norm2) {
  if (norm1 >= 0.0 && norm2 >= 0.0) return 1;
  if (!g_req_failed) { g_req_failed = 1; g_req_n1 = norm1; g_req_n2 = norm2; }
  return 0;
}

/* 1 (and the two norms) if a require failed since the last call; clears it */
int orc_take_require_failure(double* norm1, double* norm2) {
  int f = g_req_failed;
  if (f) { *norm1 = g_req_n1; *norm2 = g_req_n2; }
  g_req_failed = 0;
  return f;
}

/* ml/impl/Utils.scala:70-80 indexUpperTriangular */
static inline int64_t orc_iut(int64_t i, int64_t j) {
  return (i <= j) ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j;
}

/* ------------------------------------------------------------------------ */
/* KMeans (dense points, Euclidean)                                          */
/* ------------------------------------------------------------------------ */

/* DistanceMeasure.scala:48-76 computeStatistics + Euclidean :275-277
 * s = 0.25 * distance * distance, distance = sqrt(fastSquaredDistance).
 * packed has k(k+1)/2 entries; k == 1 gives {NaN}.                        */
void orc_kmeans_stats(const double* C, int64_t k, int64_t d, double* packed) {
  if (k == 1) { packed[0] = NAN; return; }
  double* diag = (double*)malloc(sizeof(double) * k);
  double* norms = (double*)malloc(sizeof(double) * k);   /* VectorWithNorm.norm */
  for (int64_t i = 0; i < k; ++i) norms[i] = orc_norm2(C + i * d, d);
  for (int64_t i = 0; i < k; ++i) diag[i] = INFINITY;
  for (int64_t i = 0; i < k; ++i) {
    for (int64_t j = i + 1; j < k; ++j) {
      if (!orc_require_norms(norms[i], norms[j])) { free(diag); free(norms); return; }
      double dist = sqrt(orc_sqdist(C + i * d, C + j * d, d));
      double s = 0.25 * dist * dist;
      packed[orc_iut(i, j)] = s;
      if (s < diag[i]) diag[i] = s;
      if (s < diag[j]) diag[j] = s;
    }
  }
  for (int64_t i = 0; i < k; ++i) packed[orc_iut(i, i)] = diag[i];
  free(diag);
  free(norms);
}

/* DistanceMeasure.scala:282-313 EuclideanDistanceMeasure.findClosest with
 * statistics, dense centers and dense point (fastSquaredDistance == sqdist). */
void orc_find_closest_stats(const double* C, const double* cnorm, int64_t k, int64_t d,
                            const double* stats, const double* x, double xnorm,
                            int32_t* out_idx, double* out_dist) {
  *out_idx = -1;
  *out_dist = NAN;
  if (!orc_require_norms(cnorm[0], xnorm)) return;
  double best = orc_sqdist(C, x, d);
  if (best < stats[0]) { *out_idx = 0; *out_dist = best; return; }
  int64_t bestIndex = 0;
  for (int64_t i = 1; i < k; ++i) {
    double normDiff = cnorm[i] - xnorm;
    double lowerBound = normDiff * normDiff;
    if (lowerBound < best) {
      if (stats[orc_iut(i, bestIndex)] < best) {
        if (!orc_require_norms(cnorm[i], xnorm)) return;
        double dd = orc_sqdist(C + i * d, x, d);
        if (dd < stats[orc_iut(i, i)]) { *out_idx = (int32_t)i; *out_dist = dd; return; }
        if (dd < best) { best = dd; bestIndex = i; }
      }
    }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

/* DistanceMeasure.scala:318-340 findClosest without statistics */
void orc_find_closest(const double* C, const double* cnorm, int64_t k, int64_t d,
                      const double* x, double xnorm, int32_t* out_idx, double* out_dist) {
  double best = INFINITY;
  int64_t bestIndex = 0;
  for (int64_t i = 0; i < k; ++i) {
    double lb = cnorm[i] - xnorm;
    lb = lb * lb;
    if (lb < best) {
      /* a NaN norm never passes lb < best: this require cannot fail here */
      if (!orc_require_norms(cnorm[i], xnorm)) { *out_idx = -1; *out_dist = NAN; return; }
      double dd = orc_sqdist(C + i * d, x, d);
      if (dd < best) { best = dd; bestIndex = i; }
    }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

/* Same as orc_find_closest_stats but the point is sparse (libsvm input,
 * config #1); distances go through the norm trick of MLUtils:560-573. */
void orc_find_closest_stats_sparse(const double* C, const double* cnorm, int64_t k, int64_t d,
                                   const double* stats, const int32_t* idx, const double* val,
                                   int64_t nnz, double xnorm, int32_t* out_idx, double* out_dist) {
  *out_idx = -1;
  *out_dist = NAN;
  if (!orc_require_norms(cnorm[0], xnorm)) return;
  double best = orc_fast_sqdist_dense_sparse(C, cnorm[0], idx, val, nnz, xnorm, d);
  if (best < stats[0]) { *out_idx = 0; *out_dist = best; return; }
  int64_t bestIndex = 0;
  for (int64_t i = 1; i < k; ++i) {
    double normDiff = cnorm[i] - xnorm;
    double lowerBound = normDiff * normDiff;
    if (lowerBound < best) {
      if (stats[orc_iut(i, bestIndex)] < best) {
        if (!orc_require_norms(cnorm[i], xnorm)) return;
        double dd = orc_fast_sqdist_dense_sparse(C + i * d, cnorm[i], idx, val, nnz, xnorm, d);
        if (dd < stats[orc_iut(i, i)]) { *out_idx = (int32_t)i; *out_dist = dd; return; }
        if (dd < best) { best = dd; bestIndex = i; }
      }
    }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

/* DistanceMeasure.scala:318-340 with a SparseVector point: findClosest
 * without statistics, distances through MLUtils.fastSquaredDistance. */
void orc_find_closest_sparse(const double* C, const double* cnorm, int64_t k, int64_t d,
                             const int32_t* idx, const double* val, int64_t nnz, double xnorm,
                             int32_t* out_idx, double* out_dist) {
  double best = INFINITY;
  int64_t bestIndex = 0;
  for (int64_t i = 0; i < k; ++i) {
    double lb = cnorm[i] - xnorm;
    lb = lb * lb;
    if (lb < best) {
      if (!orc_require_norms(cnorm[i], xnorm)) { *out_idx = -1; *out_dist = NAN; return; }
      double dd = orc_fast_sqdist_dense_sparse(C + i * d, cnorm[i], idx, val, nnz, xnorm, d);
      if (dd < best) { best = dd; bestIndex = i; }
    }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

/* DistanceMeasure.pointCost (:152-156) for every row of a dense partition
 * (KMeansModel.computeCost's map, KMeansModel.scala:110-117) plus the
 * partition's RDD.sum fold (sequential, from 0.0).  Returns the sum. */
double orc_point_costs(const double* X, const double* xnorm, int64_t n, int64_t d,
                       const double* C, const double* cnorm, int64_t k, int32_t* assign,
                       double* cost) {
  double sum = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    orc_find_closest(C, cnorm, k, d, X + r * d, xnorm[r], assign + r, cost + r);
    sum += cost[r];
  }
  return sum;
}

/* Same for CSR rows. */
double orc_point_costs_sparse(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                              const double* xnorm, int64_t n, int64_t d, const double* C,
                              const double* cnorm, int64_t k, int32_t* assign, double* cost) {
  double sum = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t q0 = rowptr[r];
    orc_find_closest_sparse(C, cnorm, k, d, colidx + q0, vals + q0, rowptr[r + 1] - q0, xnorm[r],
                            assign + r, cost + r);
    sum += cost[r];
  }
  return sum;
}

/* One Spark partition of the Lloyd iteration body, KMeans.scala:287-306:
 *   (bestCenter, cost) = findClosest(centers, stats, point)
 *   costAccum.add(cost * point.weight)
 *   updateClusterSum = axpy(point.weight, point.vector, sums(bestCenter))
 *   clusterWeightSum(bestCenter) += point.weight
 * sums (k*d), wsum (k) and *cost accumulate (caller zeroes them).
 * assign/dist (optional, may be NULL) receive the per-point findClosest.
 * weights == NULL means unit weights.  netlib daxpy: y(i) = y(i) + da*x(i),
 * and a da == 0 call is a no-op.                                          */
void orc_kmeans_partition(const double* X, const double* xnorm, const double* w,
                          int64_t n, int64_t d, const double* C, const double* cnorm,
                          const double* stats, int64_t k, int32_t* assign, double* dist,
                          double* sums, double* wsum, double* cost) {
  double c = *cost;
  for (int64_t r = 0; r < n; ++r) {
    int32_t bi; double bd;
    orc_find_closest_stats(C, cnorm, k, d, stats, X + r * d, xnorm[r], &bi, &bd);
    if (bi < 0) break;                     /* require failed: the task throws */
    double wt = w ? w[r] : 1.0;
    if (assign) assign[r] = bi;
    if (dist) dist[r] = bd;
    c += bd * wt;
    if (wt != 0.0) {
      double* s = sums + (int64_t)bi * d;
      const double* x = X + r * d;
      for (int64_t j = 0; j < d; ++j) s[j] = s[j] + wt * x[j];
    }
    wsum[bi] += wt;
  }
  *cost = c;
}

/* mllib/linalg/BLAS.scala:63-118 axpy(1.0, sumweight2, sumweight1) merge of
 * reduceByKey (KMeans.scala:308-311), in place: a += b                     */
void orc_axpy(int64_t n, double alpha, const double* x, double* y) {
  if (alpha == 0.0) return;
  for (int64_t i = 0; i < n; ++i) y[i] = y[i] + alpha * x[i];
}

/* KMeans.scala:322-330 + DistanceMeasure.scala:200-203 centroid and
 * :345-350 isCenterConverged (Euclidean: fastSquaredDistance <= eps^2).
 * Updates C/cnorm in place for clusters with wsum > 0; returns 1 if every
 * updated center converged.                                              */
int orc_kmeans_update_centers(double* C, double* cnorm, const double* sums, const double* wsum,
                              int64_t k, int64_t d, double epsilon) {
  int converged = 1;
  double* nc = (double*)malloc(sizeof(double) * d);
  for (int64_t j = 0; j < k; ++j) {
    if (!(wsum[j] > 0)) continue;
    double a = 1.0 / wsum[j];
    for (int64_t t = 0; t < d; ++t) nc[t] = a * sums[j * d + t];
    double nn = orc_norm2(nc, d);
    if (converged && !(orc_sqdist(nc, C + j * d, d) <= epsilon * epsilon)) converged = 0;
    memcpy(C + j * d, nc, sizeof(double) * d);
    cnorm[j] = nn;
  }
  free(nc);
  return converged;
}

/* ------------------------------------------------------------------------ */
/* KMeans, CosineDistanceMeasure (DistanceMeasure.scala:395-514)            */
/* ------------------------------------------------------------------------ */

/* mllib/linalg/BLAS.scala:145-148 dot(dense, dense) = ddot: netlib's loop,
 * dtemp + dx(i)*dy(i) in index order (the unrolled groups add left to right) */
double orc_ddot(const double* x, const double* y, int64_t n) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += x[i] * y[i];
  return s;
}

/* assert(v1.norm > 0 && v2.norm > 0, "Cosine distance is not defined for
 * zero-length vectors.") (:454, and :467 for updateClusterSum): an
 * AssertionError ends the Spark task; recorded like the require above. */
static _Thread_local int g_assert_failed = 0;

static int orc_cos_assert(double n1, double n2) {
  if (n1 > 0 && n2 > 0) return 1;
  g_assert_failed = 1;
  return 0;
}

/* 1 if the cosine assert failed since the last call; clears it */
int orc_take_assert_failure(void) {
  int f = g_assert_failed;
  g_assert_failed = 0;
  return f;
}

/* :453-456 distance(v1, v2) = 1 - dot(v1.vector, v2.vector) / v1.norm / v2.norm */
static double orc_cos_distance(const double* v1, double n1, const double* v2, double n2,
                               int64_t d) {
  return 1.0 - orc_ddot(v1, v2, d) / n1 / n2;
}

/* computeStatistics (:48-76) with the cosine statistic (:412-417):
 * s = 1 - sqrt(1 - distance / 2).  cnorm: the centers' VectorWithNorm norms. */
void orc_cos_stats(const double* C, const double* cnorm, int64_t k, int64_t d, double* packed) {
  if (k == 1) { packed[0] = NAN; return; }
  double* diag = (double*)malloc(sizeof(double) * k);
  for (int64_t i = 0; i < k; ++i) diag[i] = INFINITY;
  for (int64_t i = 0; i < k; ++i) {
    for (int64_t j = i + 1; j < k; ++j) {
      if (!orc_cos_assert(cnorm[i], cnorm[j])) { free(diag); return; }
      double dist = orc_cos_distance(C + i * d, cnorm[i], C + j * d, cnorm[j], d);
      double s = 1.0 - sqrt(1.0 - dist / 2.0);
      packed[orc_iut(i, j)] = s;
      if (s < diag[i]) diag[i] = s;
      if (s < diag[j]) diag[j] = s;
    }
  }
  for (int64_t i = 0; i < k; ++i) packed[orc_iut(i, i)] = diag[i];
  free(diag);
}

/* CosineDistanceMeasure.findClosest with statistics (:421-447) */
void orc_cos_find_closest_stats(const double* C, const double* cnorm, int64_t k, int64_t d,
                                const double* stats, const double* x, double xnorm,
                                int32_t* out_idx, double* out_dist) {
  *out_idx = -1;
  *out_dist = NAN;
  if (!orc_cos_assert(cnorm[0], xnorm)) return;
  double best = orc_cos_distance(C, cnorm[0], x, xnorm, d);
  if (best < stats[0]) { *out_idx = 0; *out_dist = best; return; }
  int64_t bestIndex = 0;
  for (int64_t i = 1; i < k; ++i) {
    if (stats[orc_iut(i, bestIndex)] < best) {
      if (!orc_cos_assert(cnorm[i], xnorm)) return;
      double dd = orc_cos_distance(C + i * d, cnorm[i], x, xnorm, d);
      if (dd < stats[orc_iut(i, i)]) { *out_idx = (int32_t)i; *out_dist = dd; return; }
      if (dd < best) { best = dd; bestIndex = i; }
    }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

/* findClosest without statistics (:131-150), the cosine distance */
void orc_cos_find_closest(const double* C, const double* cnorm, int64_t k, int64_t d,
                          const double* x, double xnorm, int32_t* out_idx, double* out_dist) {
  double best = INFINITY;
  int64_t bestIndex = 0;
  for (int64_t i = 0; i < k; ++i) {
    if (!orc_cos_assert(cnorm[i], xnorm)) { *out_idx = -1; *out_dist = NAN; return; }
    double dd = orc_cos_distance(C + i * d, cnorm[i], x, xnorm, d);
    if (dd < best) { best = dd; bestIndex = i; }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

/* pointCost (:152-156) for every row plus the partition's sum fold. */
double orc_cos_point_costs(const double* X, const double* xnorm, int64_t n, int64_t d,
                           const double* C, const double* cnorm, int64_t k, int32_t* assign,
                           double* cost) {
  double sum = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    orc_cos_find_closest(C, cnorm, k, d, X + r * d, xnorm[r], assign + r, cost + r);
    if (assign[r] < 0) break;
    sum += cost[r];
  }
  return sum;
}

/* One partition of the Lloyd body (KMeans.scala:287-306) with the cosine
 * updateClusterSum (:466-469): axpy(point.weight / point.norm, x, sum). */
void orc_cos_kmeans_partition(const double* X, const double* xnorm, const double* w, int64_t n,
                              int64_t d, const double* C, const double* cnorm,
                              const double* stats, int64_t k, int32_t* assign, double* dist,
                              double* sums, double* wsum, double* cost) {
  double c = *cost;
  for (int64_t r = 0; r < n; ++r) {
    int32_t bi; double bd;
    orc_cos_find_closest_stats(C, cnorm, k, d, stats, X + r * d, xnorm[r], &bi, &bd);
    if (bi < 0) break;                     /* assert failed: the task throws */
    double wt = w ? w[r] : 1.0;
    if (assign) assign[r] = bi;
    if (dist) dist[r] = bd;
    c += bd * wt;
    double a = wt / xnorm[r];
    if (a != 0.0) {                        /* netlib daxpy: da == 0 returns */
      double* s = sums + (int64_t)bi * d;
      const double* x = X + r * d;
      for (int64_t j = 0; j < d; ++j) s[j] = s[j] + a * x[j];
    }
    wsum[bi] += wt;
  }
  *cost = c;
}

/* distance(center dense, point sparse): BLAS.dot(dense, sparse) dispatches
 * to dot(sparse, dense) (mllib/linalg/BLAS.scala:128-134, 153-169) */
static double orc_cos_distance_sparse(const double* c, double nc, const int32_t* idx,
                                      const double* val, int64_t nnz, double nx) {
  return 1.0 - orc_dot_sparse_dense(idx, val, nnz, c) / nc / nx;
}

/* findClosest with (stats != NULL, :421-447) or without (:131-150)
 * statistics for a SparseVector point */
static void orc_cos_find_closest_sparse(const double* C, const double* cnorm, int64_t k,
                                        int64_t d, const double* stats, const int32_t* idx,
                                        const double* val, int64_t nnz, double xnorm,
                                        int32_t* out_idx, double* out_dist) {
  *out_idx = -1;
  *out_dist = NAN;
  double best = INFINITY;
  int64_t bestIndex = 0;
  int64_t i0 = 0;
  if (stats) {
    if (!orc_cos_assert(cnorm[0], xnorm)) return;
    best = orc_cos_distance_sparse(C, cnorm[0], idx, val, nnz, xnorm);
    if (best < stats[0]) { *out_idx = 0; *out_dist = best; return; }
    i0 = 1;
  }
  for (int64_t i = i0; i < k; ++i) {
    if (stats && !(stats[orc_iut(i, bestIndex)] < best)) continue;
    if (!orc_cos_assert(cnorm[i], xnorm)) return;
    double dd = orc_cos_distance_sparse(C + i * d, cnorm[i], idx, val, nnz, xnorm);
    if (stats && dd < stats[orc_iut(i, i)]) { *out_idx = (int32_t)i; *out_dist = dd; return; }
    if (dd < best) { best = dd; bestIndex = i; }
  }
  *out_idx = (int32_t)bestIndex;
  *out_dist = best;
}

double orc_cos_point_costs_sparse(const int64_t* rowptr, const int32_t* colidx,
                                  const double* vals, const double* xnorm, int64_t n, int64_t d,
                                  const double* C, const double* cnorm, int64_t k,
                                  int32_t* assign, double* cost) {
  double sum = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t q0 = rowptr[r];
    orc_cos_find_closest_sparse(C, cnorm, k, d, NULL, colidx + q0, vals + q0, rowptr[r + 1] - q0,
                                xnorm[r], assign + r, cost + r);
    if (assign[r] < 0) break;
    sum += cost[r];
  }
  return sum;
}

/* the Lloyd partition body for SparseVector points: updateClusterSum =
 * mllib BLAS.axpy(w / norm, sparse x, sum) (BLAS.scala:93-112) */
void orc_cos_kmeans_partition_sparse(const int64_t* rowptr, const int32_t* colidx,
                                     const double* vals, const double* xnorm, const double* w,
                                     int64_t n, int64_t d, const double* C, const double* cnorm,
                                     const double* stats, int64_t k, int32_t* assign,
                                     double* dist, double* sums, double* wsum, double* cost) {
  double c = *cost;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t q0 = rowptr[r], nnz = rowptr[r + 1] - q0;
    int32_t bi; double bd;
    orc_cos_find_closest_sparse(C, cnorm, k, d, stats, colidx + q0, vals + q0, nnz, xnorm[r],
                                &bi, &bd);
    if (bi < 0) break;
    double wt = w ? w[r] : 1.0;
    if (assign) assign[r] = bi;
    if (dist) dist[r] = bd;
    c += bd * wt;
    double a = wt / xnorm[r];
    double* s = sums + (int64_t)bi * d;
    for (int64_t q = 0; q < nnz; ++q) {
      if (a == 1.0) s[colidx[q0 + q]] += vals[q0 + q];
      else s[colidx[q0 + q]] += a * vals[q0 + q];
    }
    wsum[bi] += wt;
  }
  *cost = c;
}

/* centroid (:477-483): scal(1/weightSum, sum), norm, scal(1/norm, sum),
 * new VectorWithNorm(sum, 1); isCenterConverged (:161-166): distance(old,
 * new) <= epsilon.  Returns 1 if every updated center converged. */
int orc_cos_update_centers(double* C, double* cnorm, const double* sums, const double* wsum,
                           int64_t k, int64_t d, double epsilon) {
  int converged = 1;
  double* nc = (double*)malloc(sizeof(double) * d);
  for (int64_t j = 0; j < k; ++j) {
    if (!(wsum[j] > 0)) continue;
    double a = 1.0 / wsum[j];
    for (int64_t t = 0; t < d; ++t) nc[t] = a * sums[j * d + t];
    double norm = orc_norm2(nc, d);
    double b = 1.0 / norm;
    for (int64_t t = 0; t < d; ++t) nc[t] = b * nc[t];
    if (converged && !(orc_cos_distance(C + j * d, cnorm[j], nc, 1.0, d) <= epsilon))
      converged = 0;
    memcpy(C + j * d, nc, sizeof(double) * d);
    cnorm[j] = 1.0;
  }
  free(nc);
  return converged;
}

/* ------------------------------------------------------------------------ */
/* ml.impl.Utils                                                            */
/* ------------------------------------------------------------------------ */

/* ml/impl/Utils.scala:91-97 log1pExp */
double orc_log1pexp(double x) {
  if (x > 0) return x + log1p(exp(-x));
  return log1p(exp(x));
}

/* ml/impl/Utils.scala:108-135 strided softmax, in place on arr[offset + step*i] */
void orc_softmax(double* arr, int64_t n, int64_t offset, int64_t step) {
  double maxValue = -1.7976931348623157e308; /* Double.MinValue */
  int64_t end = offset + step * n;
  for (int64_t i = offset; i < end; i += step) {
    double v = arr[i];
    if (isinf(v) && v > 0) {
      for (int64_t t = offset; t < end; t += step) arr[t] = 0.0 * arr[t];
      arr[i] = 1.0;
      return;
    } else if (v > maxValue) {
      maxValue = v;
    }
  }
  double sum = 0.0;
  for (int64_t i = offset; i < end; i += step) {
    double e = exp(arr[i] - maxValue);
    arr[i] = e;
    sum += e;
  }
  double a = 1.0 / sum;
  for (int64_t i = offset; i < end; i += step) arr[i] = a * arr[i];
}

/* ------------------------------------------------------------------------ */
/* Logistic block aggregators                                                */
/* ------------------------------------------------------------------------ */

/* A block as InstanceBlock (ml/feature/Instance.scala:39-106): either dense
 * row-major S x F (values != NULL, rowptr == NULL) or CSR (rowptr/colidx/
 * values, isTransposed = true).  weights == NULL means all-unit weights
 * (Instance.scala:134-138 stores an empty array).                          */
typedef struct {
  int64_t S, F;
  const double* labels;
  const double* weights;
  const double* values;
  const int64_t* rowptr;
  const int32_t* colidx;
} orc_block;

/* margin of row i: netlib dgemv "T" on the row-major block (BLAS.scala:621-631):
 * temp += a(l,i)*x(l) sequentially, y = alpha*temp + y (beta == 1 skips the
 * beta scaling).  CSR: BLAS.scala:777-789 sum += Avals(i) * x(Acols(i)),
 * y = beta*y + sum*alpha.  Both reduce to y + temp for alpha = beta = 1. */
static double orc_row_dot(const orc_block* b, int64_t i, const double* coef) {
  double t = 0.0;
  if (b->rowptr) {
    for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
      t += b->values[p] * coef[b->colidx[p]];
  } else {
    const double* row = b->values + i * b->F;
    for (int64_t f = 0; f < b->F; ++f) t += row[f] * coef[f];
  }
  return t;
}

/* BinaryLogisticBlockAggregator.add, BinaryLogisticBlockAggregator.scala:81-145.
 * coef has F (+1 if fitIntercept) entries; grad (same size), *lossSum,
 * *weightSum accumulate.  scaledMean is used iff fitWithMean.             */
void orc_binary_logistic_add(const orc_block* b, const double* coef, int fitIntercept,
                             int fitWithMean, const double* scaledMean, double* grad,
                             double* lossSum, double* weightSum) {
  const int64_t S = b->S, F = b->F;
  int anyPositive = 0;
  for (int64_t i = 0; i < S; ++i) if (!b->weights || b->weights[i] != 0) anyPositive = 1;
  if (!anyPositive) return;                                     /* :88 */
  double marginOffset = NAN;                                    /* :67-72 */
  if (fitWithMean) {
    double dd = 0.0;                                            /* javaBLAS.ddot */
    for (int64_t f = 0; f < F; ++f) dd += coef[f] * scaledMean[f];
    marginOffset = coef[F] - dd;
  }
  double* arr = (double*)calloc((size_t)S, sizeof(double));
  if (fitIntercept) {
    double off = fitWithMean ? marginOffset : coef[F];
    for (int64_t i = 0; i < S; ++i) arr[i] = off;
  }
  for (int64_t i = 0; i < S; ++i) arr[i] = arr[i] + orc_row_dot(b, i, coef);  /* :97 */
  double localLoss = 0.0, localW = 0.0, multSum = 0.0;
  for (int64_t i = 0; i < S; ++i) {                             /* :104-122 */
    double w = b->weights ? b->weights[i] : 1.0;
    localW += w;
    if (w > 0) {
      double label = b->labels[i];
      double margin = arr[i];
      if (label > 0) localLoss += w * orc_log1pexp(-margin);
      else localLoss += w * (orc_log1pexp(-margin) + margin);
      double mult = w * (1.0 / (1.0 + exp(-margin)) - label);
      arr[i] = mult;
      multSum += mult;
    } else {
      arr[i] = 0.0;
    }
  }
  *lossSum += localLoss;
  *weightSum += localW;
  int allZero = 1;
  for (int64_t i = 0; i < S; ++i) if (arr[i] != 0) { allZero = 0; break; }
  if (!allZero) {
    /* :130 gemv(1.0, A^T, arr, 1.0, grad): netlib dgemv "N" column loop
     * (dense) / BLAS.scala:790-804 CSC scatter (sparse): y(row) += a*(x*alpha) */
    for (int64_t i = 0; i < S; ++i) {
      double t = arr[i];
      if (b->rowptr) {
        double xv = t * 1.0;
        for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
          grad[b->colidx[p]] += b->values[p] * xv;
      } else {
        if (t != 0.0) {
          const double* row = b->values + i * F;
          for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + t * row[f];
        }
      }
    }
    if (fitWithMean) {                                          /* :132-137 javaBLAS.daxpy */
      double a = -multSum;
      if (a != 0.0) for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + a * scaledMean[f];
    }
    if (fitIntercept) grad[F] += multSum;                       /* :139-142 */
  }
  free(arr);
}

/* HingeBlockAggregator.add, ml/optim/aggregator/HingeBlockAggregator.scala:
 * 81-141 (LinearSVC).  Centers whenever it fits an intercept: marginOffset
 * = coef[F] - ddot(coef, scaledMean) (:62-71); per row with weight > 0:
 * y' = label + label - 1, loss = (1 - y' margin) w, counted with the
 * multiplier -y' w only when loss > 0 (:103-117).                        */
void orc_hinge_add(const orc_block* b, const double* coef, int fitIntercept,
                   const double* scaledMean, double* grad, double* lossSum, double* weightSum) {
  const int64_t S = b->S, F = b->F;
  int anyPositive = 0;
  for (int64_t i = 0; i < S; ++i) if (!b->weights || b->weights[i] != 0) anyPositive = 1;
  if (!anyPositive) return;                                     /* :88 */
  double marginOffset = NAN;
  if (fitIntercept) {
    double dd = 0.0;                                            /* javaBLAS.ddot */
    for (int64_t f = 0; f < F; ++f) dd += coef[f] * scaledMean[f];
    marginOffset = coef[F] - dd;
  }
  double* arr = (double*)calloc((size_t)S, sizeof(double));
  if (fitIntercept) for (int64_t i = 0; i < S; ++i) arr[i] = marginOffset;   /* :93 */
  for (int64_t i = 0; i < S; ++i) arr[i] = arr[i] + orc_row_dot(b, i, coef);  /* :94 */
  double localLoss = 0.0, localW = 0.0, multSum = 0.0;
  for (int64_t i = 0; i < S; ++i) {
    double w = b->weights ? b->weights[i] : 1.0;
    localW += w;
    if (w > 0) {
      double label = b->labels[i];
      double labelScaled = label + label - 1.0;
      double loss = (1.0 - labelScaled * arr[i]) * w;
      if (loss > 0) {
        localLoss += loss;
        double mult = -labelScaled * w;
        arr[i] = mult;
        multSum += mult;
      } else {
        arr[i] = 0.0;
      }
    } else {
      arr[i] = 0.0;
    }
  }
  *lossSum += localLoss;
  *weightSum += localW;
  int allZero = 1;
  for (int64_t i = 0; i < S; ++i) if (arr[i] != 0) { allZero = 0; break; }
  if (!allZero) {                                               /* :127 gemv(A^T) */
    for (int64_t i = 0; i < S; ++i) {
      double t = arr[i];
      if (b->rowptr) {
        double xv = t * 1.0;
        for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
          grad[b->colidx[p]] += b->values[p] * xv;
      } else if (t != 0.0) {
        const double* row = b->values + i * F;
        for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + t * row[f];
      }
    }
    if (fitIntercept) {                                         /* :129-137 */
      double a = -multSum;
      if (a != 0.0) for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + a * scaledMean[f];
      grad[F] += multSum;
    }
  }
  free(arr);
}

void orc_hinge_add_dense(int64_t S, int64_t F, const double* X, const double* labels,
                         const double* weights, const double* coef, int fitIntercept,
                         const double* scaledMean, double* grad, double* lossSum,
                         double* weightSum) {
  orc_block b = {S, F, labels, weights, X, NULL, NULL};
  orc_hinge_add(&b, coef, fitIntercept, scaledMean, grad, lossSum, weightSum);
}

void orc_hinge_add_csr(int64_t S, int64_t F, const int64_t* rowptr, const int32_t* colidx,
                       const double* vals, const double* labels, const double* weights,
                       const double* coef, int fitIntercept, const double* scaledMean,
                       double* grad, double* lossSum, double* weightSum) {
  orc_block b = {S, F, labels, weights, vals, rowptr, colidx};
  orc_hinge_add(&b, coef, fitIntercept, scaledMean, grad, lossSum, weightSum);
}

/* HuberBlockAggregator.add, ml/optim/aggregator/HuberBlockAggregator.scala:
 * 80-141.  coef = F linear terms, intercept (fitIntercept), sigma (last);
 * dim = F + 1 (+1).  Centers whenever it fits an intercept (:66-71). */
void orc_huber_add(const orc_block* b, const double* coef, int fitIntercept, double epsilon,
                   const double* scaledMean, double* grad, double* lossSum, double* weightSum) {
  const int64_t S = b->S, F = b->F;
  const int64_t dim = F + (fitIntercept ? 2 : 1);
  int anyPositive = 0;
  for (int64_t i = 0; i < S; ++i) if (!b->weights || b->weights[i] != 0) anyPositive = 1;
  if (!anyPositive) return;                                     /* :87 */
  double marginOffset = NAN;
  if (fitIntercept) {
    double dd = 0.0;
    for (int64_t f = 0; f < F; ++f) dd += coef[f] * scaledMean[f];
    marginOffset = coef[dim - 2] - dd;
  }
  double* arr = (double*)calloc((size_t)S, sizeof(double));
  if (fitIntercept) for (int64_t i = 0; i < S; ++i) arr[i] = marginOffset;   /* :92 */
  for (int64_t i = 0; i < S; ++i) arr[i] = arr[i] + orc_row_dot(b, i, coef);  /* :93 */
  const double sigma = coef[dim - 1];
  double sigmaGradSum = 0.0, localLoss = 0.0, localW = 0.0, multSum = 0.0;
  for (int64_t i = 0; i < S; ++i) {                             /* :103-127 */
    double w = b->weights ? b->weights[i] : 1.0;
    localW += w;
    if (w > 0) {
      double linearLoss = b->labels[i] - arr[i];
      if (fabs(linearLoss) <= sigma * epsilon) {
        localLoss += 0.5 * w * (sigma + pow(linearLoss, 2.0) / sigma);
        double lds = linearLoss / sigma;
        double mult = -1.0 * w * lds;
        arr[i] = mult;
        multSum += mult;
        sigmaGradSum += 0.5 * w * (1.0 - pow(lds, 2.0));
      } else {
        localLoss += 0.5 * w * (sigma + 2.0 * epsilon * fabs(linearLoss) - sigma * epsilon * epsilon);
        double sign = linearLoss >= 0 ? -1.0 : 1.0;
        double mult = w * sign * epsilon;
        arr[i] = mult;
        multSum += mult;
        sigmaGradSum += 0.5 * w * (1.0 - epsilon * epsilon);
      }
    } else {
      arr[i] = 0.0;
    }
  }
  *lossSum += localLoss;
  *weightSum += localW;
  for (int64_t i = 0; i < S; ++i) {                             /* :131 gemv(A^T) */
    double t = arr[i];
    if (b->rowptr) {
      double xv = t * 1.0;
      for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
        grad[b->colidx[p]] += b->values[p] * xv;
    } else if (t != 0.0) {
      const double* row = b->values + i * F;
      for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + t * row[f];
    }
  }
  if (fitIntercept) {                                           /* :133-140 */
    double a = -multSum;
    if (a != 0.0) for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + a * scaledMean[f];
    grad[dim - 2] += multSum;
  }
  grad[dim - 1] += sigmaGradSum;                                /* :142 */
  free(arr);
}

void orc_huber_add_block(int64_t S, int64_t F, const double* X, const int64_t* rowptr,
                         const int32_t* colidx, const double* labels, const double* weights,
                         const double* coef, int fitIntercept, double epsilon,
                         const double* scaledMean, double* grad, double* lossSum,
                         double* weightSum) {
  orc_block b = {S, F, labels, weights, X, rowptr, colidx};
  orc_huber_add(&b, coef, fitIntercept, epsilon, scaledMean, grad, lossSum, weightSum);
}

/* AFTBlockAggregator.add, ml/optim/aggregator/AFTBlockAggregator.scala:76-130.
 * coef = F linear, intercept slot, log(sigma) (dim = F + 2); the block's
 * weights are the censors (NULL: 1.0); weightSum += size. */
void orc_aft_add(const orc_block* b, const double* coef, int fitIntercept,
                 const double* scaledMean, double* grad, double* lossSum, double* weightSum) {
  const int64_t S = b->S, F = b->F, dim = F + 2;
  double marginOffset = NAN;
  if (fitIntercept) {                                           /* :52-58 */
    double dd = 0.0;
    for (int64_t f = 0; f < F; ++f) dd += coef[f] * scaledMean[f];
    marginOffset = coef[dim - 2] - dd;
  }
  const double sigma = exp(coef[dim - 1]);                      /* :86 */
  double* arr = (double*)calloc((size_t)(S > 0 ? S : 1), sizeof(double));
  if (fitIntercept) for (int64_t i = 0; i < S; ++i) arr[i] = marginOffset;
  for (int64_t i = 0; i < S; ++i) arr[i] = arr[i] + orc_row_dot(b, i, coef);  /* :91 */
  double localLoss = 0.0, sigmaGradSum = 0.0, multSum = 0.0;
  for (int64_t i = 0; i < S; ++i) {                             /* :99-110 */
    double ti = b->labels[i];
    double delta = b->weights ? b->weights[i] : 1.0;
    double margin = arr[i];
    double eps = (log(ti) - margin) / sigma;
    double expEps = exp(eps);
    localLoss += delta * log(sigma) - delta * eps + expEps;
    double mult = (delta - expEps) / sigma;
    arr[i] = mult;
    multSum += mult;
    sigmaGradSum += delta + mult * sigma * eps;
  }
  *lossSum += localLoss;
  *weightSum += (double)S;
  for (int64_t i = 0; i < S; ++i) {                             /* :116 gemv(A^T) */
    double t = arr[i];
    if (b->rowptr) {
      double xv = t * 1.0;
      for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
        grad[b->colidx[p]] += b->values[p] * xv;
    } else if (t != 0.0) {
      const double* row = b->values + i * F;
      for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + t * row[f];
    }
  }
  if (fitIntercept) {                                           /* :118-124 */
    double a = -multSum;
    if (a != 0.0) for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + a * scaledMean[f];
    grad[dim - 2] += multSum;
  }
  grad[dim - 1] += sigmaGradSum;                                /* :126 */
  free(arr);
}

void orc_aft_add_block(int64_t S, int64_t F, const double* X, const int64_t* rowptr,
                       const int32_t* colidx, const double* labels, const double* censors,
                       const double* coef, int fitIntercept, const double* scaledMean,
                       double* grad, double* lossSum, double* weightSum) {
  orc_block b = {S, F, labels, censors, X, rowptr, colidx};
  orc_aft_add(&b, coef, fitIntercept, scaledMean, grad, lossSum, weightSum);
}

/* LeastSquaresBlockAggregator.add, ml/optim/aggregator/
 * LeastSquaresBlockAggregator.scala:70-101 (dim = F).  effectiveCoef zeroes
 * the coefficients of features with inverseStd == 0 (:48-55); offset =
 * labelMean / labelStd - javaBLAS.ddot(coef, scaledMean) (:57-62). */
void orc_least_squares_add(const orc_block* b, const double* coef, const double* inverseStd,
                           int fitIntercept, double labelStd, double labelMean,
                           const double* scaledMean, double* grad, double* lossSum,
                           double* weightSum) {
  const int64_t S = b->S, F = b->F;
  int anyPositive = 0;
  for (int64_t i = 0; i < S; ++i) if (!b->weights || b->weights[i] != 0) anyPositive = 1;
  if (!anyPositive) return;                                     /* :77 */
  double* eff = (double*)malloc((size_t)(F > 0 ? F : 1) * sizeof(double));
  for (int64_t f = 0; f < F; ++f) eff[f] = inverseStd[f] != 0 ? coef[f] : 0.0;
  double offset = NAN;
  if (fitIntercept) {
    double dd = 0.0;
    for (int64_t f = 0; f < F; ++f) dd += coef[f] * scaledMean[f];
    offset = labelMean / labelStd - dd;
  }
  double* arr = (double*)calloc((size_t)S, sizeof(double));
  if (fitIntercept) for (int64_t i = 0; i < S; ++i) arr[i] = offset;     /* :84 */
  double a = -1.0 / labelStd;                                   /* :85 javaBLAS.daxpy */
  for (int64_t i = 0; i < S; ++i) arr[i] += a * b->labels[i];
  for (int64_t i = 0; i < S; ++i) arr[i] = arr[i] + orc_row_dot(b, i, eff);  /* :86 */
  double localLoss = 0.0, localW = 0.0;
  for (int64_t i = 0; i < S; ++i) {                             /* :91-99 */
    double w = b->weights ? b->weights[i] : 1.0;
    localW += w;
    double diff = arr[i];
    localLoss += w * diff * diff / 2;
    arr[i] = w * diff;
  }
  *lossSum += localLoss;
  *weightSum += localW;
  for (int64_t i = 0; i < S; ++i) {                             /* :103 gemv(A^T) */
    double t = arr[i];
    if (b->rowptr) {
      double xv = t * 1.0;
      for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
        grad[b->colidx[p]] += b->values[p] * xv;
    } else if (t != 0.0) {
      const double* row = b->values + i * F;
      for (int64_t f = 0; f < F; ++f) grad[f] = grad[f] + t * row[f];
    }
  }
  free(arr);
  free(eff);
}

void orc_least_squares_add_block(int64_t S, int64_t F, const double* X, const int64_t* rowptr,
                                 const int32_t* colidx, const double* labels,
                                 const double* weights, const double* coef,
                                 const double* inverseStd, int fitIntercept, double labelStd,
                                 double labelMean, const double* scaledMean, double* grad,
                                 double* lossSum, double* weightSum) {
  orc_block b = {S, F, labels, weights, X, rowptr, colidx};
  orc_least_squares_add(&b, coef, inverseStd, fitIntercept, labelStd, labelMean, scaledMean, grad,
                        lossSum, weightSum);
}

/* MultinomialLogisticBlockAggregator.add, .scala:101-189 (dense blocks and
 * CSR blocks).  coef: C*F linear part, column-major C x F (coef[f*C + c]),
 * then C intercepts if fitIntercept.  grad has the same layout.            */
void orc_multinomial_logistic_add(const orc_block* b, const double* coef, int64_t C,
                                  int fitIntercept, int fitWithMean, const double* scaledMean,
                                  double* grad, double* lossSum, double* weightSum) {
  const int64_t S = b->S, F = b->F;
  int anyPositive = 0;
  for (int64_t i = 0; i < S; ++i) if (!b->weights || b->weights[i] != 0) anyPositive = 1;
  if (!anyPositive) return;
  const double* linear = coef;               /* linear(c,f) = coef[f*C + c] */
  const double* intercept = fitIntercept ? coef + C * F : NULL;
  double* offset = NULL;
  if (fitWithMean) {
    /* marginOffset :86-92: gemv(-1.0, linear, scaledMean, 1.0, intercept copy):
     * netlib dgemv "N" (C x F col-major): column loop, temp = alpha*x(j),
     * y(i) += temp*a(i,j) */
    offset = (double*)malloc(sizeof(double) * C);
    for (int64_t c = 0; c < C; ++c) offset[c] = intercept[c];
    for (int64_t f = 0; f < F; ++f) {
      if (scaledMean[f] != 0.0) {
        double t = -1.0 * scaledMean[f];
        for (int64_t c = 0; c < C; ++c) offset[c] = offset[c] + t * linear[f * C + c];
      }
    }
  }
  /* mat S x C column-major: arr[c*S + i] */
  double* arr = (double*)calloc((size_t)(S * C), sizeof(double));
  if (fitIntercept) {
    const double* off = fitWithMean ? offset : intercept;
    for (int64_t c = 0; c < C; ++c)
      if (off[c] != 0) for (int64_t i = 0; i < S; ++i) arr[c * S + i] = off[c];
  }
  /* :122 gemm(1.0, A, linear^T, 1.0, mat) -> netlib dgemm("T","T") for dense:
   * c(i,j) = alpha*temp + beta*c(i,j), temp = sum_l a(l,i)*b(j,l) in l order.
   * CSR A: BLAS.scala gemm(SparseMatrix transposed): per (row, col of B)
   * sum += Avals(k) * B(Arows(k), colCounterForB) then C = beta*C + sum*alpha. */
  for (int64_t c = 0; c < C; ++c) {
    for (int64_t i = 0; i < S; ++i) {
      double t = 0.0;
      if (b->rowptr) {
        for (int64_t p = b->rowptr[i]; p < b->rowptr[i + 1]; ++p)
          t += b->values[p] * linear[(int64_t)b->colidx[p] * C + c];
        arr[c * S + i] = 1.0 * arr[c * S + i] + t * 1.0;
      } else {
        const double* row = b->values + i * F;
        for (int64_t f = 0; f < F; ++f) t += row[f] * linear[f * C + c];
        arr[c * S + i] = 1.0 * t + 1.0 * arr[c * S + i];
      }
    }
  }
  double localLoss = 0.0, localW = 0.0;
  for (int64_t i = 0; i < S; ++i) {                              /* :129-142 */
    double w = b->weights ? b->weights[i] : 1.0;
    localW += w;
    if (w > 0) {
      int64_t labelIndex = i + (int64_t)b->labels[i] * S;
      orc_softmax(arr, C, i, S);
      localLoss -= w * log(arr[labelIndex]);
      if (w != 1) for (int64_t c = 0; c < C; ++c) arr[c * S + i] = w * arr[c * S + i];
      arr[labelIndex] -= w;
    } else {
      for (int64_t c = 0; c < C; ++c) arr[c * S + i] = 0.0 * arr[c * S + i];
    }
  }
  *lossSum += localLoss;
  *weightSum += localW;
  /* :153 dgemm("T","T", C, F, S, 1.0, mat, S, A, F, 1.0, grad, C):
   * grad(c, f) = 1.0*temp + 1.0*grad(c,f), temp = sum_s mat(s,c)*A(s,f)   */
  if (b->rowptr) {
    /* :157-161 sparse: linearGradSumMat (F x C) = sm^T x mat via BLAS.gemm
     * with a non-transposed CSC (the transpose of the CSR block): for each
     * column of B (class c) and each CSC column s: Bval = mat(s,c)*alpha,
     * C(row=f) += Avals * Bval; then gradientSumArray(f*C + c) += v.        */
    double* lg = (double*)calloc((size_t)(F * C), sizeof(double));
    for (int64_t c = 0; c < C; ++c) {
      for (int64_t s = 0; s < S; ++s) {
        double bv = arr[c * S + s] * 1.0;
        for (int64_t p = b->rowptr[s]; p < b->rowptr[s + 1]; ++p)
          lg[c * F + b->colidx[p]] += b->values[p] * bv;
      }
    }
    for (int64_t c = 0; c < C; ++c)
      for (int64_t f = 0; f < F; ++f) grad[f * C + c] += lg[c * F + f];
    free(lg);
  } else {
    for (int64_t f = 0; f < F; ++f) {
      for (int64_t c = 0; c < C; ++c) {
        double t = 0.0;
        for (int64_t s = 0; s < S; ++s) t += arr[c * S + s] * b->values[s * F + f];
        grad[f * C + c] = 1.0 * t + 1.0 * grad[f * C + c];
      }
    }
  }
  if (fitIntercept) {                                             /* :165-186 */
    double* ms = (double*)calloc((size_t)C, sizeof(double));
    for (int64_t c = 0; c < C; ++c)
      for (int64_t i = 0; i < S; ++i) ms[c] += arr[c * S + i];
    if (fitWithMean) {
      /* netlib dger(C, F, -1.0, ms, 1, scaledMean, 1, grad, C):
       * for j: if y(j) != 0: temp = alpha*y(j); a(i,j) += x(i)*temp */
      for (int64_t f = 0; f < F; ++f) {
        if (scaledMean[f] != 0.0) {
          double t = -1.0 * scaledMean[f];
          for (int64_t c = 0; c < C; ++c) grad[f * C + c] = grad[f * C + c] + ms[c] * t;
        }
      }
    }
    for (int64_t c = 0; c < C; ++c) grad[C * F + c] = grad[C * F + c] + 1.0 * ms[c];
    free(ms);
  }
  free(arr);
  free(offset);
}

/* Python-friendly entry points (plain pointers, no struct) */
void orc_binary_logistic_add_dense(int64_t S, int64_t F, const double* X, const double* labels,
                                   const double* weights, const double* coef, int fitIntercept,
                                   int fitWithMean, const double* scaledMean, double* grad,
                                   double* lossSum, double* weightSum) {
  orc_block b = {S, F, labels, weights, X, NULL, NULL};
  orc_binary_logistic_add(&b, coef, fitIntercept, fitWithMean, scaledMean, grad, lossSum, weightSum);
}

void orc_binary_logistic_add_csr(int64_t S, int64_t F, const int64_t* rowptr,
                                 const int32_t* colidx, const double* vals, const double* labels,
                                 const double* weights, const double* coef, int fitIntercept,
                                 int fitWithMean, const double* scaledMean, double* grad,
                                 double* lossSum, double* weightSum) {
  orc_block b = {S, F, labels, weights, vals, rowptr, colidx};
  orc_binary_logistic_add(&b, coef, fitIntercept, fitWithMean, scaledMean, grad, lossSum, weightSum);
}

void orc_multinomial_logistic_add_dense(int64_t S, int64_t F, int64_t C, const double* X,
                                        const double* labels, const double* weights,
                                        const double* coef, int fitIntercept, int fitWithMean,
                                        const double* scaledMean, double* grad, double* lossSum,
                                        double* weightSum) {
  orc_block b = {S, F, labels, weights, X, NULL, NULL};
  orc_multinomial_logistic_add(&b, coef, C, fitIntercept, fitWithMean, scaledMean, grad, lossSum,
                               weightSum);
}

void orc_multinomial_logistic_add_csr(int64_t S, int64_t F, int64_t C, const int64_t* rowptr,
                                      const int32_t* colidx, const double* vals,
                                      const double* labels, const double* weights,
                                      const double* coef, int fitIntercept, int fitWithMean,
                                      const double* scaledMean, double* grad, double* lossSum,
                                      double* weightSum) {
  orc_block b = {S, F, labels, weights, vals, rowptr, colidx};
  orc_multinomial_logistic_add(&b, coef, C, fitIntercept, fitWithMean, scaledMean, grad, lossSum,
                               weightSum);
}

/* ------------------------------------------------------------------------ */
/* RowMatrix Gramian / covariance                                            */
/* ------------------------------------------------------------------------ */

/* netlib dspr("U", n, alpha, x, 1, ap) reference loop, called per dense row
 * by mllib/linalg/BLAS.scala:268 (RowMatrix.scala:139-158):
 *   kk = 0; for j: if x(j) != 0: temp = alpha*x(j); k = kk;
 *     for i <= j: ap(k) += x(i)*temp; kk += j + 1                         */
void orc_dspr_upper(int64_t n, double alpha, const double* x, double* ap) {
  int64_t kk = 0;
  for (int64_t j = 0; j < n; ++j) {
    if (x[j] != 0.0) {
      double temp = alpha * x[j];
      int64_t k = kk;
      for (int64_t i = 0; i <= j; ++i, ++k) ap[k] = ap[k] + x[i] * temp;
    }
    kk += j + 1;
  }
}

/* mllib/linalg/BLAS.scala:269-298 spr for a sparse vector */
void orc_spr_sparse(double alpha, const int32_t* idx, const double* val, int64_t nnz, double* U) {
  int64_t colStartIdx = 0, prevCol = 0;
  for (int64_t j = 0; j < nnz; ++j) {
    int64_t col = idx[j];
    colStartIdx += (col - prevCol) * (col + prevCol + 1) / 2;
    double av = alpha * val[j];
    for (int64_t i = 0; i <= j; ++i) U[colStartIdx + idx[i]] += av * val[i];
    prevCol = col;
  }
}

/* RowMatrix.computeGramianMatrix seqOp over one partition (RowMatrix.scala:139-158).
 * mean != NULL gives computeDenseVectorCovariance's seqOp (:171-190):
 * na(index) = ta(index) - means(index); spr(1.0, na, U).                  */
void orc_gramian_partition(const double* X, int64_t rows, int64_t n, const double* mean,
                           double* U) {
  double* na = mean ? (double*)malloc(sizeof(double) * n) : NULL;
  for (int64_t r = 0; r < rows; ++r) {
    const double* x = X + r * n;
    if (mean) {
      for (int64_t t = 0; t < n; ++t) na[t] = x[t] - mean[t];
      x = na;
    }
    orc_dspr_upper(n, 1.0, x, U);
  }
  free(na);
}

/* RowMatrix.scala:845-867 triuToFull (column-major n x n) */
void orc_triu_to_full(int64_t n, const double* U, double* G) {
  int64_t idx = 0;
  for (int64_t col = 0; col < n; ++col) {
    for (int64_t row = 0; row < col; ++row) {
      double v = U[idx++];
      G[col * n + row] = v;
      G[row * n + col] = v;
    }
    G[col * n + col] = U[idx++];
  }
}

/* One partition of the Lloyd body for sparse points (KMeans.scala:299-304):
 * findClosest through the norm trick (orc_find_closest_stats_sparse),
 * costAccum.add(cost * weight), updateClusterSum = mllib BLAS.axpy(weight,
 * sparse x, sum) (mllib/linalg/BLAS.scala:93-112: y(idx) += x or a * x in
 * nnz order) and clusterWeightSum += weight.  CSR rows; w NULL = unit.     */
void orc_kmeans_partition_sparse(const int64_t* rowptr, const int32_t* colidx,
                                 const double* vals, const double* xnorm, const double* w,
                                 int64_t n, int64_t d, const double* C, const double* cnorm,
                                 const double* stats, int64_t k, int32_t* assign, double* dist,
                                 double* sums, double* wsum, double* cost) {
  for (int64_t r = 0; r < n; ++r) {
    const int64_t q0 = rowptr[r], nnz = rowptr[r + 1] - q0;
    int32_t bi;
    double bd;
    orc_find_closest_stats_sparse(C, cnorm, k, d, stats, colidx + q0, vals + q0, nnz, xnorm[r],
                                  &bi, &bd);
    if (bi < 0) break;                     /* require failed: the task throws */
    const double wt = w ? w[r] : 1.0;
    *cost += bd * wt;
    double* y = sums + (int64_t)bi * d;
    if (wt == 1.0) {
      for (int64_t q = 0; q < nnz; ++q) y[colidx[q0 + q]] += vals[q0 + q];
    } else {
      for (int64_t q = 0; q < nnz; ++q) y[colidx[q0 + q]] += wt * vals[q0 + q];
    }
    wsum[bi] += wt;
    if (assign) assign[r] = bi;
    if (dist) dist[r] = bd;
  }
}

/* Vectors.norm(sparse, 2) of each CSR row (stored values in order) */
void orc_row_norms_csr(const int64_t* rowptr, const double* vals, int64_t n, double* out) {
  for (int64_t r = 0; r < n; ++r) {
    double s = 0.0;
    for (int64_t q = rowptr[r]; q < rowptr[r + 1]; ++q) s += vals[q] * vals[q];
    out[r] = sqrt(s);
  }
}

/* ------------------------------------------------------------------------ */
/* Summarizer pre-pass (ml/stat/Summarizer.scala:428-770,                   */
/* ml/stat/MultiClassSummarizer.scala:30-98)                                */
/* ------------------------------------------------------------------------ */

/* SummarizerBuffer state: 8 x F fields (mean, m2n, m2, l1, weightSum, nnz,
 * max, min), then count, totalWeightSum, weightSquareSum, a flag for a weight
 * that failed require(weight >= 0.0) (:472) and that weight.              */
enum { OS_MEAN, OS_M2N, OS_M2, OS_L1, OS_WS, OS_NNZ, OS_MAX, OS_MIN, OS_FIELDS };
#define OS_SCAL 5

/* a fresh buffer, arrays as the first add allocates them (:475-493) */
void orc_summ_init(int64_t F, double* st) {
  memset(st, 0, sizeof(double) * (size_t)(OS_FIELDS * F + OS_SCAL));
  for (int64_t c = 0; c < F; ++c) {
    st[OS_MAX * F + c] = -DBL_MAX; /* Double.MinValue */
    st[OS_MIN * F + c] = DBL_MAX;  /* Double.MaxValue */
  }
}

/* add(nonZeroIterator, size, weight) (:471-546) for one row of nnz (index,
 * value) pairs (idx == NULL: a dense row, index = position).             */
void orc_summ_add_row(int64_t F, double* st, const int32_t* idx, const double* val, int64_t nnz,
                      double w) {
  double* s = st + OS_FIELDS * F;
  if (!(w >= 0.0)) { /* require(weight >= 0.0): the reference throws */
    if (s[3] == 0.0) {
      s[3] = 1.0;
      s[4] = w;
    }
    return;
  }
  if (w == 0.0) return;
  for (int64_t q = 0; q < nnz; ++q) {
    const int64_t c = idx ? idx[q] : q;
    const double v = val[q];
    if (v == 0.0) continue; /* nonZeroIterator */
    if (st[OS_MAX * F + c] < v) st[OS_MAX * F + c] = v;
    if (st[OS_MIN * F + c] > v) st[OS_MIN * F + c] = v;
    const double prevMean = st[OS_MEAN * F + c];
    const double diff = v - prevMean;
    st[OS_MEAN * F + c] = prevMean + w * diff / (st[OS_WS * F + c] + w);
    st[OS_M2N * F + c] += w * (v - st[OS_MEAN * F + c]) * diff;
    st[OS_WS * F + c] += w;
    st[OS_M2 * F + c] += w * v * v;
    st[OS_L1 * F + c] += w * fabs(v);
    st[OS_NNZ * F + c] += 1.0;
  }
  s[1] += w;
  s[2] += w * w;
  s[0] += 1.0;
}

static double orc_jmax(double a, double b) { /* java.lang.Math.max */
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && signbit(a)) return b;
  return a >= b ? a : b;
}
static double orc_jmin(double a, double b) { /* java.lang.Math.min */
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && signbit(b)) return b;
  return a <= b ? a : b;
}

/* a = a.merge(b) (:562-617) */
void orc_summ_merge(int64_t F, double* a, const double* b) {
  double* sa = a + OS_FIELDS * F;
  const double* sb = b + OS_FIELDS * F;
  const double bad = sa[3], badv = sa[4];
  if (sa[1] != 0.0 && sb[1] != 0.0) {
    sa[0] += sb[0];
    sa[1] += sb[1];
    sa[2] += sb[2];
    for (int64_t c = 0; c < F; ++c) {
      const double thisW = a[OS_WS * F + c], otherW = b[OS_WS * F + c];
      const double tot = thisW + otherW;
      if (tot != 0.0) {
        const double dm = b[OS_MEAN * F + c] - a[OS_MEAN * F + c];
        a[OS_MEAN * F + c] += dm * otherW / tot;
        a[OS_M2N * F + c] += b[OS_M2N * F + c] + dm * dm * thisW * otherW / tot;
      }
      a[OS_WS * F + c] = tot;
      a[OS_M2 * F + c] += b[OS_M2 * F + c];
      a[OS_L1 * F + c] += b[OS_L1 * F + c];
      a[OS_MAX * F + c] = orc_jmax(a[OS_MAX * F + c], b[OS_MAX * F + c]);
      a[OS_MIN * F + c] = orc_jmin(a[OS_MIN * F + c], b[OS_MIN * F + c]);
      a[OS_NNZ * F + c] = a[OS_NNZ * F + c] + b[OS_NNZ * F + c];
    }
  } else if (sa[1] == 0.0 && sb[1] != 0.0) {
    memcpy(a, b, sizeof(double) * (size_t)(OS_FIELDS * F + 3));
  }
  if (bad != 0.0) {
    sa[3] = bad;
    sa[4] = badv;
  } else if (sb[3] != 0.0) {
    sa[3] = 1.0;
    sa[4] = sb[4];
  }
}

/* The rows cut into partitions of R rows, each a fresh buffer add()-ed row
 * by row, merged in partition order into out (fresh).  Dense X or CSR.    */
void orc_summarize(int64_t n, int64_t F, const double* X, const int64_t* rowptr,
                   const int32_t* colidx, const double* vals, const double* w, int64_t R,
                   double* out) {
  double* part = (double*)malloc(sizeof(double) * (size_t)(OS_FIELDS * F + OS_SCAL));
  orc_summ_init(F, out);
  for (int64_t p0 = 0; p0 < n; p0 += R) {
    const int64_t p1 = p0 + R < n ? p0 + R : n;
    orc_summ_init(F, part);
    for (int64_t r = p0; r < p1; ++r) {
      const double wr = w ? w[r] : 1.0;
      if (X) orc_summ_add_row(F, part, NULL, X + r * F, F, wr);
      else orc_summ_add_row(F, part, colidx + rowptr[r], vals + rowptr[r],
                            rowptr[r + 1] - rowptr[r], wr);
    }
    orc_summ_merge(F, out, part);
  }
  free(part);
}

/* metrics (:622-769) into out[9 x F]: mean, variance, std, sum, numNonzeros,
 * max, min, normL2, normL1                                                 */
void orc_summ_metrics(int64_t F, const double* st, double* out) {
  const double* s = st + OS_FIELDS * F;
  const double cnt = s[0], TW = s[1], TW2 = s[2];
  const double den = TW - (TW2 / TW);
  for (int64_t c = 0; c < F; ++c) {
    const double mean = st[OS_MEAN * F + c], ws = st[OS_WS * F + c];
    const double nnz = st[OS_NNZ * F + c];
    out[0 * F + c] = mean * (ws / TW);
    double var = 0.0;
    if (den > 0.0) var = orc_jmax((st[OS_M2N * F + c] + mean * mean * ws * (TW - ws) / TW) / den, 0.0);
    out[1 * F + c] = var;
    out[2 * F + c] = sqrt(var);
    out[3 * F + c] = mean * ws;
    out[4 * F + c] = nnz;
    double mx = st[OS_MAX * F + c], mn = st[OS_MIN * F + c];
    if (nnz < cnt && mx < 0.0) mx = 0.0;
    if (nnz < cnt && mn > 0.0) mn = 0.0;
    out[5 * F + c] = mx;
    out[6 * F + c] = mn;
    out[7 * F + c] = sqrt(st[OS_M2 * F + c]);
    out[8 * F + c] = st[OS_L1 * F + c];
  }
}

static int orc_jtoint(double x) { /* Scala Double.toInt */
  if (x != x) return 0;
  if (x >= 2147483647.0) return INT_MAX;
  if (x <= -2147483648.0) return INT_MIN;
  return (int)x;
}

/* MultiClassSummarizer.add over partitions of R rows (:43-56), the
 * partition maps merged in order (:66-79): hist[maxC] class weight sums
 * (classes >= maxC only raise *maxLabel), *invalid, *maxLabel (-1: none). */
void orc_label_summarize(int64_t n, const double* y, const double* w, int64_t R, int64_t maxC,
                         double* hist, int64_t* invalid, int64_t* maxLabel) {
  double* part = (double*)malloc(sizeof(double) * (size_t)maxC);
  for (int64_t c = 0; c < maxC; ++c) hist[c] = 0.0;
  *invalid = 0;
  *maxLabel = -1;
  for (int64_t p0 = 0; p0 < n; p0 += R) {
    const int64_t p1 = p0 + R < n ? p0 + R : n;
    for (int64_t c = 0; c < maxC; ++c) part[c] = 0.0;
    for (int64_t r = p0; r < p1; ++r) {
      const double wr = w ? w[r] : 1.0;
      if (!(wr > 0.0)) continue;
      const double lab = y[r];
      const int li = orc_jtoint(lab);
      if (lab - (double)li != 0.0 || lab < 0) {
        *invalid += 1;
      } else {
        if (li > *maxLabel) *maxLabel = li;
        if (li < maxC) part[li] = part[li] + wr;
      }
    }
    for (int64_t c = 0; c < maxC; ++c) hist[c] = hist[c] + part[c];
  }
  free(part);
}

/* InstanceBlock.blokifyWithMaxMemUsage (ml/feature/Instance.scala:146-180)
 * over rows given by their numNonzeros (values != 0) and weights: rows are
 * appended while the running getBlockMemUsage (:114-129) is below maxMem;
 * the crossing row stays in the block.  Block b = rows [starts[b],
 * starts[b+1]); dense[b] = Matrices.fromVectors's choice (:1010-1049:
 * getDenseSize < getSparseSize, :1317-1336).  Returns the block count. */
static int64_t orc_dense_size(int64_t cols, int64_t rows) { return 8 * cols * rows + 12 + 9; }
static int64_t orc_sparse_size(int64_t nnz, int64_t ptrs) {
  return 8 * nnz + 4 * nnz + 4 * ptrs + 12 * 3 + 9;
}
int64_t orc_blokify(int64_t n, int64_t F, const int64_t* rowNnz, const double* w, int64_t maxMem,
                    int64_t* starts, uint8_t* dense) {
  int64_t nb = 0, r = 0;
  starts[0] = 0;
  while (r < n) {                                   /* iterator.next() */
    int64_t cnt = 0, nnz = 0, mem = 0;
    int unit = 1;
    while (r < n && mem < maxMem) {
      cnt += 1;
      nnz += rowNnz[r];
      unit = unit && (w == NULL || w[r] == 1.0);
      const int64_t ds = orc_dense_size(F, cnt), ss = orc_sparse_size(nnz, cnt + 1);
      const int64_t m = ds < ss ? ds : ss;
      mem = unit ? m + 8 * cnt + 12 * 2 : m + 8 * cnt * 2 + 12 * 2;
      r += 1;
    }
    dense[nb] = orc_dense_size(F, cnt) < orc_sparse_size(nnz, cnt + 1);
    starts[++nb] = r;
  }
  return nb;
}

/* ------------------------------------------------------------------------ */
/* ml/evaluation/ClusteringMetrics.scala: Silhouette (one partition)        */
/* ------------------------------------------------------------------------ */

/* SquaredEuclideanSilhouette (:254-400) or CosineSilhouette (:403-600) over
 * n rows X (n x d) with predictions pred in [0, k) and weights w (NULL =
 * lit(1.0)).  stats (k d + 3 k scratch) receives computeClusterStats' map
 * as [featureSum | squaredNormSum | weightSum | rows]: the seqOp in row
 * order (:310-318 / :451-458; the combOp of one partition is the identity).
 * Then computeSilhouetteCoefficient per row (:350-366 / :489-504 through
 * Silhouette.pointSilhouetteCoefficient :66-97, the other clusters' minimum
 * taken in cluster-id order) and overallScore (:101-103) in row order.
 * Returns 0 and *score, or -1 when fewer than two clusters have rows (the
 * assert :391 / :532).                                                      */
int orc_silhouette(const double* X, int64_t n, int64_t d, const int32_t* pred, const double* w,
                   int64_t k, int cosine, double* stats, double* score) {
  double* fs = stats;
  double* psi = stats + k * d;
  double* W = psi + k;
  double* cnt = W + k;
  double* xn = (double*)malloc(sizeof(double) * (d > 0 ? d : 1));
  memset(stats, 0, sizeof(double) * (size_t)(k * d + 3 * k));
  for (int64_t i = 0; i < n; ++i) {
    const double* x = X + i * d;
    const double wt = w ? w[i] : 1.0;
    const int64_t c = pred[i];
    const double nrm = orc_norm2(x, d);
    double* sum = fs + c * d;
    if (cosine) {
      /* normalizeFeatureUDF: BLAS.scal(1.0 / norm, features) (:528-531) */
      const double a = 1.0 / nrm;
      for (int64_t j = 0; j < d; ++j) xn[j] = a * x[j];
      for (int64_t j = 0; j < d; ++j) sum[j] = sum[j] + wt * xn[j];
    } else {
      /* math.pow(Vectors.norm(features, 2.0), 2.0) (:385-387) */
      const double sq = nrm * nrm;
      for (int64_t j = 0; j < d; ++j) sum[j] = sum[j] + wt * x[j];
      psi[c] = psi[c] + sq * wt;
    }
    W[c] = W[c] + wt;
    cnt[c] = cnt[c] + 1.0;
  }
  int64_t present = 0;
  for (int64_t c = 0; c < k; ++c) present += cnt[c] > 0.0;
  if (present <= 1) {
    free(xn);
    return -1;
  }
  double num = 0.0, den = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const double* x = X + i * d;
    const double wt = w ? w[i] : 1.0;
    const int64_t own = pred[i];
    const double nrm = orc_norm2(x, d);
    const double* v = x;
    double sq = 0.0;
    if (cosine) {
      const double a = 1.0 / nrm;
      for (int64_t j = 0; j < d; ++j) xn[j] = a * x[j];
      v = xn;
    } else {
      sq = nrm * nrm;
    }
    double s;
    if (W[own] == wt) {
      s = 0.0;
    } else {
      double nb = 0.0, cur = 0.0;
      int have = 0;
      for (int64_t c = 0; c < k; ++c) {
        if (!(cnt[c] > 0.0)) continue;
        const double dt = orc_ddot(v, fs + c * d, d);
        const double dist = cosine ? 1.0 - dt / W[c] : sq + psi[c] / W[c] - 2 * dt / W[c];
        if (c == own) {
          cur = dist;
        } else {
          nb = (have && nb <= dist) ? nb : dist;
          have = 1;
        }
      }
      cur = cur * W[own] / (W[own] - wt);
      if (cur < nb) s = 1 - (cur / nb);
      else if (cur > nb) s = (nb / cur) - 1;
      else s = 0.0;
    }
    num = num + s * wt;
    den = den + wt;
  }
  free(xn);
  *score = num / den;
  return 0;
}
