/*
 * cyclone.h -- C ABI of libcyclone, the MI355X (gfx950) backend for the MLlib
 * linear-algebra hot path of wmeddie/CycloneML (Spark 3.3 MLlib).
 *
 * Two layers:
 *   - device-pointer entry points (suffix _dev): operands already resident in
 *     HBM, a HIP stream passed as void*.  These are what a multi-GPU driver
 *     (one process per GPU, RCCL all-reduce of the outputs) calls.
 *   - host-pointer entry points over library-owned resident datasets
 *     (cyc_dataset_*): what a JVM shim (JNI / Panama)
 *     binds in place of the per-partition Scala loops.
 *
 * Conventions
 *   - Every function returns CYC_OK (0) or a CYC_ERR_* code; the message is
 *     thread-local and read with cyc_last_error().  CYC_ERR_INVALID_ARG
 *     carries the reference's `require` text (IllegalArgumentException).
 *   - All floating point is IEEE fp64; indices are int32 (Spark's Int) and row
 *     counts int64.  Dense matrices are row-major (InstanceBlock / an RDD of
 *     DenseVector rows); CSR is (rowptr int64[n+1], colidx int32, values).
 *   - Accumulating outputs (sums, gradients, Gramians, loss/weight sums) are
 *     ADDED to, like the reference aggregators' `add`; zero them first.
 *   - There is no CPU fallback: without a gfx950 device every entry point
 *     returns CYC_ERR_NO_DEVICE.
 *   - Calls on one plan/dataset are serialized by the caller (a plan owns
 *     scratch memory); distinct plans may be used from distinct threads.
 */
#ifndef CYCLONE_H
#define CYCLONE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CYC_OK 0
#define CYC_ERR_INVALID_ARG 1 /* a reference `require` failed              */
#define CYC_ERR_HIP 2         /* HIP runtime error                          */
#define CYC_ERR_ALLOC 3       /* device allocation failed                   */
#define CYC_ERR_UNSUPPORTED 4 /* shape outside what the kernels support     */
#define CYC_ERR_NO_DEVICE 5   /* no usable gfx950 device                    */
#define CYC_ERR_ASSERTION 6   /* a reference `assert` failed (AssertionError) */

/* ------------------------------------------------------------------ misc */
const char* cyc_last_error(void);
int cyc_version(void); /* major*10000 + minor*100 + patch */
int cyc_device_count(int* count);
int cyc_set_device(int device);
int cyc_synchronize(void* stream);

/* Measurement hook (bench.py's roofline): while enabled, every launch of a
 * workload's dominant kernel (k_kmeans_assign, k_gram_tiles, k_mlr_margins,
 * k_mlr_grad, k_binlog_dense, k_binlog_csr) is bracketed by HIP events on the
 * stream it runs on.  query waits for the recorded events of `kernel`,
 * returns their summed time (ms) and count, and forgets them. */
int cyc_profile_enable(int enable);
int cyc_profile_query(const char* kernel, double* total_ms, int64_t* launches);
/* Restrict the timers to the comma-separated kernel names (NULL or "": all
 * of them), so a timed region carries only the events it reads. */
int cyc_profile_only(const char* kernels);

/* ------------------------------------------------------------- vectors */
/* norms[i] = Vectors.norm(row i, 2.0) bit-exactly (mllib/linalg/Vectors.scala:
 * 489-514, sequential sum of squares, correctly rounded sqrt).              */
int cyc_row_norms_dev(const double* X, int64_t n, int32_t d, double* norms, void* stream);

/* ---------------------------------------------------------------- KMeans */
/* Replaces the Lloyd-iteration body of mllib/clustering/KMeans.scala:275-334:
 * DistanceMeasure.computeStatistics[Distributedly] (DistanceMeasure.scala:
 * 48-118), EuclideanDistanceMeasure.findClosest with statistics (:282-313),
 * updateClusterSum / clusterWeightSum / costAccum (KMeans.scala:299-304) and
 * centroid + isCenterConverged (:322-330).  Dense points and centers.
 *
 * Assignments and per-point costs are bit-identical to the reference's
 * findClosest.  Sums/weights/cost are summed in a fixed (deterministic) order
 * that differs from a Spark partitioning, so they agree to ~1e-15 relative.  */
typedef struct cyc_kmeans_plan_s* cyc_kmeans_plan;

int cyc_kmeans_plan_create(int32_t d, int32_t k, int64_t max_rows, cyc_kmeans_plan* plan);
int cyc_kmeans_plan_destroy(cyc_kmeans_plan plan);

/* The plan's DistanceMeasure (DistanceMeasure.decodeFromString,
 * DistanceMeasure.scala:241-247): CYC_DISTANCE_EUCLIDEAN (the default) or
 * CYC_DISTANCE_COSINE (CosineDistanceMeasure, :395-514).  Set it before any
 * other call on the plan; a row image (cyc_kmeans_rows_create) is built for
 * the plan's measure.  With COSINE every call below uses the cosine forms:
 * distance 1 - dot(c, x) / |c| / |x| (:453-456), the statistic
 * 1 - sqrt(1 - d / 2) (:412-417), updateClusterSum axpy(w / |x|, x, sum)
 * (:466-469), the unit-norm centroid whose norm is set to 1.0 (:477-483) and
 * isCenterConverged distance <= epsilon (:161-166); a zero-length (or NaN)
 * norm returns CYC_ERR_ASSERTION with the reference's assert text.  Dense and
 * CSR points (sparse: dot(sparse, dense) and the sparse axpy). */
#define CYC_DISTANCE_EUCLIDEAN 0
#define CYC_DISTANCE_COSINE 1
int cyc_kmeans_plan_set_distance_measure(cyc_kmeans_plan plan, int32_t measure);

/* computeStatistics for the given centers: fills the plan's packed k(k+1)/2
 * statistics (and copies them to stats_out if non-NULL, device memory).
 * With COSINE the centers' norms are computed here (new VectorWithNorm(c),
 * as KMeansModel's lazy statistics do); cyc_kmeans_accumulate_dev uses the
 * cnorm it is given. */
int cyc_kmeans_stats_dev(cyc_kmeans_plan plan, const double* C, double* stats_out, void* stream);

/* Per-fit row image (KMeans.scala:263-270 caches the rows with their norms
 * once per fit; this caches a second view of the same rows): the int8
 * three-limb fixed-point image that the exact-integer screen streams, 3 bytes
 * per (64-padded) element + 8 bytes per row.  Built once from X (n x d device
 * rows); X must not change while the image is used.  For d > 512 the image is
 * empty and the calls below use the bf16 / fp64 screens instead.  Passing the
 * image is optional everywhere (NULL = no i8 tier). */
typedef struct cyc_kmeans_rows_s* cyc_kmeans_rows;
int cyc_kmeans_rows_create(cyc_kmeans_plan plan, const double* X, int64_t n, void* stream,
                           cyc_kmeans_rows* rows);
int cyc_kmeans_rows_destroy(cyc_kmeans_rows rows);
int64_t cyc_kmeans_rows_bytes(cyc_kmeans_rows rows);

/* Carried bounds (Hamerly's, per fit): with a row image, every
 * cyc_kmeans_accumulate_dev call (Euclidean, d <= 256, 96 < k <= 4096)
 * keeps per row an upper bound of its distance to its assigned center and a
 * lower bound to every other center, for the centers of that call.  The next
 * call moves them by each center's drift (triangle inequality) and skips the
 * screen only for rows whose moved bounds still separate the assigned center
 * from every other by more than the reference's rounding slack
 * (2^-29 (|x|^2 + max |c|^2)) -- the pruned reference loop (DistanceMeasure.
 * scala:282-313) returns that same index, so assignments stay bit-identical;
 * every other row is screened as before.  The first call of a fit screens
 * every row.  State of the row image (one fit: one image, one Lloyd loop);
 * cyc_kmeans_assign_dev / point_cost_dev neither use nor change it.
 * set_bounds(rows, 0) turns it off (and either call drops the state; the
 * environment CYC_KMEANS_BOUNDS=0 turns it off for every image).
 * bounds_info: the accumulate calls that used it and the rows they screened
 * (the rest kept their carried assignment); synchronises the device. */
int cyc_kmeans_rows_set_bounds(cyc_kmeans_rows rows, int32_t enable);
int cyc_kmeans_rows_bounds_info(cyc_kmeans_rows rows, int64_t* calls, int64_t* screened_rows);
/* Rows whose bounds failed but whose carried candidate set (the three-limb
 * candidate tier's, with a lower bound for every center outside it) was
 * re-checked instead of a full screen -- certified there or passed on to
 * the screen (and then also counted in screened_rows).  Synchronises. */
int cyc_kmeans_rows_bounds_rechecked(cyc_kmeans_rows rows, int64_t* rechecked_rows);

/* Incremental cluster sums across one fit's cyc_kmeans_accumulate_dev calls
 * on these rows (round 6; on by default, CYC_KMEANS_INCR=0 turns the default
 * off).  Applies with the carried bounds, weights == NULL and cost == NULL
 * (no per-row costs).  The rows object keeps each cluster's sums, count and
 * the sum of squared distances to a reference point.  A call whose moved rows
 * are at most n / 16 updates them by those rows alone.  The cost for the call's
 * centers then comes from Q + 2 (P - c).(S - W P) + W |P - c|^2, with its
 * rounding bounded on the device.  A bound above 2^-40 of the cost, too many
 * moved rows or no prior state run the full pass over every row (which resets
 * the state).  The caller's buffers receive sums, weights and cost either way;
 * the assignments are unaffected.  Replaces nothing in the reference: its
 * KMeans.scala:287-306 re-sums every point.  enable = 0 drops the state. */
int cyc_kmeans_rows_set_incremental(cyc_kmeans_rows rows, int32_t enable);
/* Calls that took the incremental path, and the moved rows they folded, over
 * the object's life.  Synchronises. */
int cyc_kmeans_rows_incremental_info(cyc_kmeans_rows rows, int64_t* incremental_calls,
                                     int64_t* moved_rows);

/* findClosest(centers, stats, point) for n points (stats from the last
 * cyc_kmeans_stats_dev on this plan).  assign[n], cost[n] device outputs.
 * rows: NULL or the image of exactly these X, n.
 * *n_exact_out (host, may be NULL) receives how many points needed the
 * exact-emulation path (ties / near ties the screens cannot separate). */
int cyc_kmeans_assign_dev(cyc_kmeans_plan plan, const double* X, const double* xnorm,
                          cyc_kmeans_rows rows, int64_t n, const double* C, const double* cnorm,
                          int32_t* assign, double* cost, int64_t* n_exact_out, void* stream);

/* findClosest(centers, point) WITHOUT statistics (DistanceMeasure.scala:
 * 318-340): the loop behind DistanceMeasure.pointCost (:152-156), i.e.
 * KMeansModel.computeCost (mllib/clustering/KMeansModel.scala:110-117) and the
 * k-means|| cost updates (KMeans.scala:379-402).  Needs no statistics on the
 * plan.  assign[n] / cost[n] bit-identical to the reference loop (a point no
 * center reaches keeps cost +Infinity, index 0). */
int cyc_kmeans_point_cost_dev(cyc_kmeans_plan plan, const double* X, const double* xnorm,
                              cyc_kmeans_rows rows, int64_t n, const double* C,
                              const double* cnorm, int32_t* assign, double* cost, void* stream);

/* Screening tiers of the last cyc_kmeans_assign_dev call that asked for
 * n_exact_out: rows the first screen (i8 with a row image, else bf16x3) left
 * to the fp64 MFMA screen (all rows when neither runs), and rows left to the
 * exact emulation. */
int cyc_kmeans_last_tiers(cyc_kmeans_plan plan, int64_t* fp64_screen_rows, int64_t* exact_rows);
/* Rows the d <= 256 screen's two-limb i8 pass left to its three-limb pass
 * (rows whose candidate set it could not list) on the last counted assign (-1 when that call ran no two-limb pass).  A
 * statistic of the tiered findClosest; no reference counterpart. */
int cyc_kmeans_last_screen(cyc_kmeans_plan plan, int64_t* three_limb_rows);
/* Rows the two-limb pass handed to its candidate pass (exact fp64 distances
 * to the <= 6 centers its bounds could not exclude) on the last counted
 * assign (-1 when no two-limb pass ran).  Also a tier statistic. */
int cyc_kmeans_last_candidates(cyc_kmeans_plan plan, int64_t* candidate_rows);
/* Of those, the rows the three-limb candidate tier (exact integer limb
 * products over the candidates, k_screen_cands3) could not certify and left
 * to the fp64 candidate pass (-1 when the tier did not run).  A tier
 * statistic; no reference counterpart. */
int cyc_kmeans_last_candidates3(cyc_kmeans_plan plan, int64_t* fp64_rows);
/* The last i8 screen's one-limb pass + two-limb refinement (d <= 256,
 * 96 < k <= 4096): rows the one-limb pass listed with their candidate
 * centers, rows handed to the full two-limb pass, and the candidate centers
 * the refinement screened in total (each wave 32 listed rows); all -1 when
 * that screen ran the two-limb pass over every center.  Statistics of the
 * tiered findClosest; no reference counterpart. */
int cyc_kmeans_last_refine(cyc_kmeans_plan plan, int64_t* listed_rows, int64_t* full_rows,
                           int64_t* union_centers);

/* One partition's contribution to a Lloyd iteration: statistics + assign +
 * per-cluster sums.  sums[k*d] += sum of w*x, wsum[k] += sum of w,
 * cost_sum[0] += sum of w*cost.  weights may be NULL (unit weights).
 * rows: NULL or the image of exactly these X, n.  assign/cost (per-row
 * outputs) may be NULL.  All pointers are device memory.
 * xnorm may be NULL with a Euclidean row image: the image's norms (built
 * with it, in another summation order -- within the screens' margins) serve
 * the screens, and the rows the reference loop itself decides
 * (k_assign_exact) get the reference's Vectors.norm computed there, so the
 * results are the same bits as with the caller's norms (the per-fit norm
 * pass of KMeans.scala:263-270 is then not needed). */
int cyc_kmeans_accumulate_dev(cyc_kmeans_plan plan, const double* X, const double* xnorm,
                              cyc_kmeans_rows rows, const double* weights, int64_t n,
                              const double* C, const double* cnorm, double* sums, double* wsum,
                              double* cost_sum, int32_t* assign, double* cost, void* stream);

/* centroid = scal(1/wsum, sum) and a fresh norm for every cluster with
 * wsum > 0; converged_out (device int32) = 1 iff every such center moved by
 * fastSquaredDistance <= epsilon^2. C and cnorm are updated in place. */
int cyc_kmeans_update_dev(cyc_kmeans_plan plan, double* C, double* cnorm, const double* sums,
                          const double* wsum, double epsilon, int32_t* converged_out,
                          void* stream);

/* ClusteringEvaluator's Silhouette (ml/evaluation/ClusteringEvaluator.scala
 * :106-150 -> ClusteringMetrics.silhouette :48-60): the plan's distance
 * measure selects SquaredEuclideanSilhouette (ClusteringMetrics.scala
 * :254-400) or CosineSilhouette (:403-600).  Replaces the two Spark jobs of
 * computeSilhouetteScore: the aggregateByKey of computeClusterStats and the
 * per-row UDF + overallScore.  Rows X (n x d, plan d) with predictions
 * pred[n] in [0, plan k), weights (nullable = 1.0, each >= 0: the
 * checkNonNegativeWeight require, ml/functions.scala:91), xnorm (nullable:
 * computed) = Vectors.norm(x, 2.0).
 * _stats_dev ADDS this shard's cluster statistics into the device buffer
 * stats[k d + 3 k] = [featureSum (k x d) | squaredNormSum (k) | weightSum
 * (k) | rows (k)] (zero it first; all-reduce it across ranks: the combOp).
 * _score_dev, on the merged stats, ADDS sum_i s_i w_i and sum_i w_i of this
 * shard into partial[2] (device; all-reduce, then the score is
 * partial[0] / partial[1]); fewer than two clusters with rows ->
 * CYC_ERR_ASSERTION "assertion failed: Number of clusters must be greater
 * than one." (:391 / :532). */
int cyc_kmeans_silhouette_stats_dev(cyc_kmeans_plan plan, const double* X, const double* xnorm,
                                    int64_t n, const int32_t* pred, const double* weights,
                                    double* stats, void* stream);
int cyc_kmeans_silhouette_score_dev(cyc_kmeans_plan plan, const double* X, const double* xnorm,
                                    int64_t n, const int32_t* pred, const double* weights,
                                    const double* stats, double* partial, void* stream);

/* Sparse (CSR) points against dense centers: KMeansExample's libsvm input
 * (BASELINE configs[0]).  Distances are MLUtils.fastSquaredDistance's
 * norm-trick branch (MLUtils.scala:533-576: BLAS.dot(sparse, dense), the
 * precision bounds and the Vectors.sqdist(sparse, dense) fallback,
 * Vectors.scala:598-622) and findClosest replays the reference loop, so
 * assignments and costs are bit-identical; the cluster sums use the sparse
 * axpy (mllib BLAS.scala:93-112) with fp64 atomics (order-free to rounding).
 * xnorm = Vectors.norm of the stored values (cyc_row_norms_csr_dev).  The
 * plan's d is numFeatures; plans with d > 1240 serve only these calls. */
int cyc_row_norms_csr_dev(const int64_t* rowptr, const double* vals, int64_t n, double* norms,
                          void* stream);
/* statistics from the last cyc_kmeans_stats_dev on this plan */
int cyc_kmeans_assign_csr_dev(cyc_kmeans_plan plan, const int64_t* rowptr, const int32_t* colidx,
                              const double* vals, const double* xnorm, int64_t n, const double* C,
                              const double* cnorm, int32_t* assign, double* cost, void* stream);
/* findClosest(centers, point) without statistics for CSR rows (pointCost). */
int cyc_kmeans_point_cost_csr_dev(cyc_kmeans_plan plan, const int64_t* rowptr,
                                  const int32_t* colidx, const double* vals, const double* xnorm,
                                  int64_t n, const double* C, const double* cnorm,
                                  int32_t* assign, double* cost, void* stream);
int cyc_kmeans_accumulate_csr_dev(cyc_kmeans_plan plan, const int64_t* rowptr,
                                  const int32_t* colidx, const double* vals, const double* xnorm,
                                  const double* weights, int64_t n, const double* C,
                                  const double* cnorm, double* sums, double* wsum,
                                  double* cost_sum, int32_t* assign, double* cost, void* stream);

/* k-means|| initialisation, the executor side of one step (KMeans.scala:
 * 398-404): chosen[i] = 1 iff the partition's XORShiftRandom(seed ^ (step <<
 * 16) ^ index) draws nextDouble() < 2.0 * costs[i] * k / sum_costs, one draw
 * per point in the partition's order -- the same points the reference keeps.
 * part_starts (HOST, num_parts + 1 offsets from 0): the shard's rows split
 * into Spark partitions; partition p has index first_part_index + p.
 * seed: the Int `new XORShiftRandom(this.seed).nextInt()` (:377).  costs and
 * chosen (uint8) are device arrays of part_starts[num_parts] entries. */
int cyc_kmeans_parallel_sample_dev(const double* costs, const int64_t* part_starts,
                                   int32_t num_parts, int32_t first_part_index, int32_t seed,
                                   int32_t step, int32_t k, double sum_costs, uint8_t* chosen,
                                   void* stream);
/* XORShiftRandom.hashSeed (core/.../util/random/XORShiftRandom.scala:60-66):
 * the generator's initial state for a Long seed (host). */
uint64_t cyc_xorshift_hash_seed(int64_t seed);

/* ------------------------------------------------------ RowMatrix Gramian */
/* Replaces the BLAS.spr seqOp of RowMatrix.computeGramianMatrix
 * (mllib/linalg/distributed/RowMatrix.scala:130-161) and of
 * computeDenseVectorCovariance (:163-220).  U is the packed upper triangle
 * (column-major, U[j(j+1)/2 + i], i <= j) of n(n+1)/2 doubles; the call adds
 * sum_r x_r x_r^T over the dense row-major rows (x_r - mean if mean != NULL).
 * fp64 MFMA syrk, deterministic fixed-order split-K reduction. */
typedef struct cyc_gramian_plan_s* cyc_gramian_plan;

int cyc_gramian_plan_create(int32_t ncols, cyc_gramian_plan* plan);
int cyc_gramian_plan_destroy(cyc_gramian_plan plan);
int cyc_gramian_accumulate_dev(cyc_gramian_plan plan, const double* X, int64_t nrows,
                               const double* mean, double* U, void* stream);
/* U += sum_r x_r x_r^T and sums[c] += sum_r X[r][c] in one pass over the rows
 * (the column sums ride the syrk's diagonal tiles; sums are the same values
 * as cyc_col_sums_dev's to rounding, not the same bits): the uncentred
 * covariance form of RowMatrix.computeCovariance (covariance). */
int cyc_gramian_accumulate_sums_dev(cyc_gramian_plan plan, const double* X, int64_t nrows,
                                    double* U, double* sums, void* stream);
/* sums[c] += sum over rows of X[r][c] (fixed order): the mean pre-pass of
 * RowMatrix.computeCovariance (Statistics.colStats, :456). */
int cyc_col_sums_dev(cyc_gramian_plan plan, const double* X, int64_t nrows, double* sums,
                     void* stream);
/* The same pass with sumsq[c] += sum over rows of X[r][c]^2 beside it (sums
 * bit-identical to cyc_col_sums_dev; sumsq may be NULL): the column
 * variances that choose computeCovariance's form (covariance). */
int cyc_col_moments_dev(cyc_gramian_plan plan, const double* X, int64_t nrows, double* sums,
                        double* sumsq, void* stream);
/* RowMatrix.triuToFull (:845-867): G (n x n column-major) from U. */
int cyc_triu_to_full_dev(int32_t n, const double* U, double* G, void* stream);
/* computeDenseVectorCovariance's finish (:203-217): G = full(U) / (m - 1). */
int cyc_covariance_finalize_dev(int32_t n, const double* U, int64_t m, double* G, void* stream);
/* The same two passes over CSR rows (rowptr int64[nrows + 1], any base;
 * colidx int32 validated as SparseVector indices): the sparse spr branch of
 * BLAS.spr (mllib/linalg/BLAS.scala:269-298) -- the rows are densified in
 * ~1 GiB chunks and go through the fp64 MFMA syrk, mean subtracted when
 * given (the dense-covariance path on CSR rows) -- and the column sums. */
int cyc_gramian_accumulate_csr_dev(cyc_gramian_plan plan, const int64_t* rowptr,
                                   const int32_t* colidx, const double* vals, int64_t nrows,
                                   const double* mean, double* U, void* stream);
int cyc_col_sums_csr_dev(cyc_gramian_plan plan, const int64_t* rowptr, const int32_t* colidx,
                         const double* vals, int64_t nrows, double* sums, void* stream);
int cyc_col_moments_csr_dev(cyc_gramian_plan plan, const int64_t* rowptr, const int32_t* colidx,
                            const double* vals, int64_t nrows, double* sums, double* sumsq,
                            void* stream);
/* RowMatrix.isSparseMatrix (:439-441): *count (device int64) = rows whose
 * sparsity() = 1 - numNonzeros / ncols is below 0.5, over dense X OR CSR
 * (rowptr, vals); the matrix is sparse iff the count (summed over ranks) is 0. */
int cyc_rowmatrix_dense_rows_dev(const double* X, const int64_t* rowptr, const double* vals,
                                 int64_t nrows, int32_t ncols, int64_t* count, void* stream);
/* computeSparseVectorCovariance (:222-246) from the packed Gramian U:
 * G(i, j) = U(i, j) / (m - 1) - (m / (m - 1) * mean(i)) * mean(j), i <= j,
 * mirrored (n x n column-major). */
int cyc_sparse_covariance_finalize_dev(int32_t n, const double* U, int64_t m, const double* mean,
                                       double* G, void* stream);

/* ---------------------------------------------- logistic block aggregators */
/* BinaryLogisticBlockAggregator.add (ml/optim/aggregator/
 * BinaryLogisticBlockAggregator.scala:81-145) and
 * MultinomialLogisticBlockAggregator.add (...Multinomial...scala:101-189)
 * over every block of a device-resident shard (blocks concatenated: dense
 * row-major n x F, or CSR).  Features are already scaled by inverseStd, as
 * in the reference.  Accumulates into grad (same layout as the coefficients:
 * binary F [+1]; multinomial C x F column-major [+ C intercepts]), *lossSum
 * and *weightSum (device doubles), like the aggregator's add + merge.
 * weights may be NULL (all-unit weights, InstanceBlock's empty array). */
typedef struct cyc_logistic_plan_s* cyc_logistic_plan;

/* Column-major copy of a resident CSR shard, built once (outside the
 * training loop, like InstanceBlock.blokifyWithMaxMemUsage,
 * ml/feature/Instance.scala:146-187) by a stable sort of the nonzeros by
 * (row block, column).  Passing it to cyc_binary_logistic_add_csr_dev
 * replaces the gradient's fp64-atomic scatter by per-column sums
 * (deterministic: blocks in order, each block's rows in order).  Costs 12
 * bytes per nonzero + 8 bytes per (row block, column). */
typedef struct cyc_csc_s* cyc_csc;
int cyc_csc_build_dev(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                      int64_t n, int32_t numFeatures, void* stream, cyc_csc* out);
int cyc_csc_destroy(cyc_csc csc);
int64_t cyc_csc_rows(cyc_csc csc);
int32_t cyc_csc_features(cyc_csc csc);
/* The copy is row-blocked (rows_per_block rows per block): colptr has
 * nblocks * numFeatures + 1 entries, block b / column c spanning
 * [colptr[b F + c], colptr[b F + c + 1]) of rowidx / values. */
int cyc_csc_blocks(cyc_csc csc, int64_t* rows_per_block, int64_t* nblocks);
int cyc_csc_arrays(cyc_csc csc, const int64_t** colptr, const int32_t** rowidx,
                   const double** values);

/* Row-block x column-tile layout of a CSR shard (tiles.hip) for the binary
 * aggregators' two sparse gemv (BinaryLogisticBlockAggregator.scala:97,130;
 * ml/linalg/BLAS.scala:764-805): row blocks of cyc_tiles_row_block() = 2048
 * rows, column chunks of <= 2048 columns; each (row block, chunk) segment
 * holds its nonzeros in CSR order as fp64 values + ids, so both gathers run
 * from LDS.  Two entry formats: CYC_TILES_WIDE, 12 bytes per nonzero (32-bit
 * packed row / column ids); CYC_TILES_COMPACT, 10 bytes per entry (16-bit:
 * the column and the row's step from the segment's previous entry; a step of
 * 31 rows or more takes filler entries).  CYC_TILES_AUTO (the default) lets
 * the first append that holds nonzeros choose: compact when its fillers are
 * at most 1/32 of its nonzeros (dense-enough segments, e.g. config 5's 268
 * nonzeros per segment: 1.3 % fillers), wide otherwise; cyc_tiles_set_format
 * fixes one before the first append.  Built by appending CSR rows
 * (rowptr[rows+1] of any base, colidx sorted within a row as in
 * SparseVector, values) in order: every append except the last holds a
 * whole number of row blocks.  Indices are validated with SparseVector's
 * require messages (ml/linalg/Vectors.scala:617-625).  The CSR input is not
 * referenced afterwards (free it: the layout is the shard's only copy).
 * capacity_*: upper bounds for the whole shard; a compact layout reserves a
 * 6.25 % allowance of filler entries on top. */
typedef struct cyc_tiles_s* cyc_tiles;
enum { CYC_TILES_AUTO = 0, CYC_TILES_WIDE = 1, CYC_TILES_COMPACT = 2 };
int cyc_tiles_create(int32_t numFeatures, int64_t capacity_rows, int64_t capacity_nnz,
                     cyc_tiles* out);
int cyc_tiles_set_format(cyc_tiles tiles, int32_t format);
/* the entry format in use (CYC_TILES_AUTO until decided) */
int32_t cyc_tiles_format(cyc_tiles tiles);
int cyc_tiles_append_dev(cyc_tiles tiles, const int64_t* rowptr, const int32_t* colidx,
                         const double* vals, int64_t rows, void* stream);
int cyc_tiles_destroy(cyc_tiles tiles);
int64_t cyc_tiles_rows(cyc_tiles tiles);
int64_t cyc_tiles_nnz(cyc_tiles tiles);
/* entry positions used (= nnz for the wide format; + fillers for compact) */
int64_t cyc_tiles_entries(cyc_tiles tiles);
int32_t cyc_tiles_features(cyc_tiles tiles);
int64_t cyc_tiles_bytes(cyc_tiles tiles);
int32_t cyc_tiles_row_block(void);
/* add() of the plan's binary aggregator over every row of the layout
 * (BinaryLogisticBlockAggregator.scala:81-145, or the Hinge / LeastSquares /
 * Huber / AFT plans' epilogues): labels / weights (AFT: censors; NULL =
 * unit) have cyc_tiles_rows() entries; inverseStd is required by least
 * squares plans (effectiveCoef) and ignored otherwise.  Two passes over the
 * layout (margins, then gradient), deterministic. */
int cyc_binary_add_tiles_dev(cyc_logistic_plan plan, cyc_tiles tiles, const double* labels,
                             const double* weights, const double* coef, const double* inverseStd,
                             const double* scaledMean, double* grad, double* lossSum,
                             double* weightSum, void* stream);

/* HingeBlockAggregator (ml/optim/aggregator/HingeBlockAggregator.scala:
 * 81-141, LinearSVC's loss): the binary kernels with the hinge epilogue
 * (labels {0,1} -> {-1,1}; loss (1 - y' m) w and multiplier -y' w where the
 * loss is positive).  The aggregator centers whenever it fits an intercept
 * (marginOffset, :62-71), so the plan takes fitIntercept only.  Same
 * arguments, layouts and tolerance as the binary logistic entry points. */
int cyc_hinge_plan_create(int32_t numFeatures, int fitIntercept, cyc_logistic_plan* plan);
int cyc_hinge_add_dense_dev(cyc_logistic_plan plan, const double* X, const double* labels,
                            const double* weights, int64_t n, const double* coef,
                            const double* scaledMean, double* grad, double* lossSum,
                            double* weightSum, void* stream);
int cyc_hinge_add_csr_dev(cyc_logistic_plan plan, const int64_t* rowptr, const int32_t* colidx,
                          const double* vals, const double* labels, const double* weights,
                          int64_t n, const double* coef, const double* scaledMean, double* grad,
                          double* lossSum, double* weightSum, cyc_csc csc, void* stream);

/* HuberBlockAggregator (ml/optim/aggregator/HuberBlockAggregator.scala:
 * 41-141, LinearRegression with loss "huber"): the binary kernels with the
 * Huber epilogue.  coef/grad hold F linear terms, the intercept if
 * fitIntercept, then sigma (dim - 1); the aggregator centers whenever it fits
 * an intercept.  epsilon > 1 (LinearRegression's param check). */
int cyc_huber_plan_create(int32_t numFeatures, int fitIntercept, double epsilon,
                          cyc_logistic_plan* plan);
int cyc_huber_add_dense_dev(cyc_logistic_plan plan, const double* X, const double* labels,
                            const double* weights, int64_t n, const double* coef,
                            const double* scaledMean, double* grad, double* lossSum,
                            double* weightSum, void* stream);
int cyc_huber_add_csr_dev(cyc_logistic_plan plan, const int64_t* rowptr, const int32_t* colidx,
                          const double* vals, const double* labels, const double* weights,
                          int64_t n, const double* coef, const double* scaledMean, double* grad,
                          double* lossSum, double* weightSum, cyc_csc csc, void* stream);

/* AFTBlockAggregator (ml/optim/aggregator/AFTBlockAggregator.scala:30-130,
 * AFTSurvivalRegression): the binary kernels with the log-linear survival
 * epilogue.  coef/grad: F linear terms, intercept slot, log(sigma) (dim =
 * F + 2; the intercept gradient stays 0 without fitIntercept).  censors[n]
 * (the reference keeps them in Instance.weight) may be NULL (all 1);
 * labels must be > 0 (checked by the caller, as the reference's require);
 * weightSum counts rows. */
int cyc_aft_plan_create(int32_t numFeatures, int fitIntercept, cyc_logistic_plan* plan);
int cyc_aft_add_dense_dev(cyc_logistic_plan plan, const double* X, const double* labels,
                          const double* censors, int64_t n, const double* coef,
                          const double* scaledMean, double* grad, double* lossSum,
                          double* weightSum, void* stream);
int cyc_aft_add_csr_dev(cyc_logistic_plan plan, const int64_t* rowptr, const int32_t* colidx,
                        const double* vals, const double* labels, const double* censors,
                        int64_t n, const double* coef, const double* scaledMean, double* grad,
                        double* lossSum, double* weightSum, cyc_csc csc, void* stream);

/* LeastSquaresBlockAggregator (ml/optim/aggregator/LeastSquaresBlockAggregator.
 * scala:31-101, LinearRegression's "l-bfgs" loss): the binary kernels with
 * margin (offset or 0) - label/labelStd + x.effectiveCoef, loss w d^2/2 and
 * multiplier w d for every row.  dim = numFeatures (no intercept entry in
 * coef or grad).  coef: the F original coefficients; inverseStd (device, F)
 * zeroes the effective coefficients of constant features (:48-55); the
 * offset labelMean/labelStd - coef.scaledMean (:57-62) uses coef itself.
 * labelStd must be > 0 (the reference's require message). */
int cyc_least_squares_plan_create(int32_t numFeatures, int fitIntercept, double labelStd,
                                  double labelMean, cyc_logistic_plan* plan);
int cyc_least_squares_add_dense_dev(cyc_logistic_plan plan, const double* X,
                                    const double* labels, const double* weights, int64_t n,
                                    const double* coef, const double* inverseStd,
                                    const double* scaledMean, double* grad, double* lossSum,
                                    double* weightSum, void* stream);
int cyc_least_squares_add_csr_dev(cyc_logistic_plan plan, const int64_t* rowptr,
                                  const int32_t* colidx, const double* vals, const double* labels,
                                  const double* weights, int64_t n, const double* coef,
                                  const double* inverseStd, const double* scaledMean,
                                  double* grad, double* lossSum, double* weightSum, cyc_csc csc,
                                  void* stream);

int cyc_logistic_plan_create(int32_t numFeatures, int32_t numClasses, int fitIntercept,
                             int fitWithMean, cyc_logistic_plan* plan);
int cyc_logistic_plan_destroy(cyc_logistic_plan plan);
int cyc_binary_logistic_add_dense_dev(cyc_logistic_plan plan, const double* X,
                                      const double* labels, const double* weights, int64_t n,
                                      const double* coef, const double* scaledMean, double* grad,
                                      double* lossSum, double* weightSum, void* stream);
int cyc_binary_logistic_add_csr_dev(cyc_logistic_plan plan, const int64_t* rowptr,
                                    const int32_t* colidx, const double* vals,
                                    const double* labels, const double* weights, int64_t n,
                                    const double* coef, const double* scaledMean, double* grad,
                                    double* lossSum, double* weightSum, cyc_csc csc,
                                    void* stream);
int cyc_multinomial_logistic_add_dense_dev(cyc_logistic_plan plan, const double* X,
                                           const double* labels, const double* weights,
                                           int64_t n, const double* coef,
                                           const double* scaledMean, double* grad,
                                           double* lossSum, double* weightSum, void* stream);
/* CSR rows (the sparse InstanceBlock branch of :122 and :156-162): margins
 * by a wave per row, gradient over the CSC copy (required: built from these
 * rows by cyc_csc_build_dev), numClasses <= 1024. */
int cyc_multinomial_logistic_add_csr_dev(cyc_logistic_plan plan, const int64_t* rowptr,
                                         const int32_t* colidx, const double* vals,
                                         const double* labels, const double* weights, int64_t n,
                                         const double* coef, const double* scaledMean,
                                         double* grad, double* lossSum, double* weightSum,
                                         cyc_csc csc, void* stream);
/* out[i] = the exponential the dense multinomial margins kernel applies to
 * the softmax terms m - max (Utils.softmax's math.exp, ml/impl/Utils.scala:
 * 127-129): e^x for x <= 0 within a few ulp of libm down to -708.4;
 * subnormal results in (-746, -708.4] (about 1e-13 relative error there);
 * 0 below -746 and at -inf; NaN kept (inputs above 0 are outside its
 * contract).  Exported so its accuracy is
 * testable against the host libm. */
int cyc_softmax_exp_dev(const double* x, int64_t n, double* out, void* stream);

/* ------------------------------------------------ summarizer pre-pass */
/* The first pass of LogisticRegression.train (LogisticRegression.scala:
 * 511-516, Summarizer.getClassificationSummarizers, ml/stat/Summarizer.scala:
 * 228-241) and of RowMatrix/colStats, and the StandardScaler transform of
 * trainImpl (:957-965), over a device-resident shard.
 *
 * SummarizerBuffer (Summarizer.scala:428-770): a buffer is
 * cyc_summarizer_buffer_len(F) = 8 F + 5 doubles (device): per column mean,
 * m2n, m2, l1, weightSum, nnz, max, min (structure of arrays), then count,
 * totalWeightSum, weightSquareSum, a flag set when a row's weight failed
 * `require(weight >= 0.0)` (:472) and that weight.  The rows are cut into
 * partitions (dense: rows_per_partition rows; CSR: the row blocks of the CSC
 * copy), each partition's buffer is add()-ed row by row in the reference's
 * order and the partitions are merged (:562-617) in order.  Buffers of
 * several shards merge with cyc_summarizer_merge_dev, in the given order.
 * metrics (9 x F doubles): mean, variance, std, sum, numNonzeros, max, min,
 * normL2, normL1 (:622-769); count and weightSum are buf[8F], buf[8F+1]. */
int64_t cyc_summarizer_buffer_len(int32_t numFeatures);
int cyc_summarizer_dense_dev(const double* X, const double* weights, int64_t n, int32_t F,
                             int64_t rows_per_partition, double* buf, void* stream);
int cyc_summarizer_csr_dev(cyc_csc csc, const double* weights, double* buf, void* stream);
int cyc_summarizer_merge_dev(int32_t F, const double* bufs, int64_t count, double* out,
                             void* stream);
int cyc_summarizer_metrics_dev(int32_t F, const double* buf, double* metrics, void* stream);
/* MultiClassSummarizer (ml/stat/MultiClassSummarizer.scala:30-98) of the
 * labels: hist[max_classes] = per-class weight sums (classes >= max_classes
 * are counted in max_label only), *invalid = countInvalid, *max_label = the
 * largest valid label (-1: none; numClasses = max_label + 1; call again with
 * a larger max_classes, at most 8192, when it does not fit).  All device. */
int cyc_label_summarizer_dev(const double* labels, const double* weights, int64_t n,
                             int64_t rows_per_partition, int32_t max_classes, double* hist,
                             int64_t* invalid, int32_t* max_label, void* stream);
/* StandardScaler transform with scale only (StandardScaler.scala:261-283),
 * in place: dense values(i) *= scale(i); CSR values(k) *= scale(indices(k)). */
int cyc_scale_columns_dense_dev(double* X, int64_t n, int32_t F, const double* scale,
                                void* stream);
int cyc_scale_columns_csr_dev(const int32_t* colidx, double* vals, int64_t nnz,
                              const double* scale, void* stream);
/* InstanceBlock.blokifyWithMaxMemUsage (ml/feature/Instance.scala:146-187;
 * Matrices.fromVectors's dense-or-sparse choice, Matrices.scala:1010-1049)
 * over one partition's device rows -- dense X (n x F) OR CSR (rowptr, vals),
 * weights optional (null = all 1): starts[0..nblocks] (int64, capacity n + 1,
 * starts[nblocks] = n), dense[b] = 1 iff block b is stored dense, *nblocks;
 * all device.  maxMemUsage <= 0 -> "requirement failed: maxMemUsage > 0".
 * Replaces the per-partition iterator the reference runs on the executor. */
int cyc_blokify_dev(const double* X, const int64_t* rowptr, const double* vals,
                    const double* weights, int64_t n, int32_t F, int64_t maxMemUsage,
                    int64_t* starts, uint8_t* dense, int64_t* nblocks, void* stream);

/* ------------------------------------------- resident datasets (host API) */
/* Layer 2 for a JVM shim: a library-owned HBM copy of one
 * partition's rows, appended once from host blocks (an InstanceBlock's
 * row-major values / CSR arrays, labels and weights, Instance.scala:39-106),
 * then evaluated per iteration with host-pointer model inputs and
 * host-pointer aggregator outputs (ADDED to, like `add`).  The calls wrap
 * the _dev entry points above on the dataset's own stream and return after
 * the outputs are on the host.  Row norms (KMeans) and the CSC copy (sparse
 * binary LR) are built on first use and rebuilt after an append.
 *   cyc_kmeans_iter             KMeans.scala:287-311 (one partition of a Lloyd
 *                               iteration: statistics, findClosest, sums)
 *   cyc_logreg_*_eval           RDDLossFunction.scala:56-70's seqOp over the
 *                               partition's blocks
 *   cyc_gramian, cyc_col_sums   RowMatrix.scala:130-161, :163-220, :456
 * Dense and CSR datasets serve every entry point (CSR Gramian / column sums:
 * the sparse spr rows densified in chunks, cyc_gramian_accumulate_csr_dev). */
typedef struct cyc_dataset_s* cyc_dataset;

int cyc_dataset_dense_create(int32_t numFeatures, int64_t capacity_rows, int has_labels,
                             int has_weights, cyc_dataset* out);
int cyc_dataset_csr_create(int32_t numFeatures, int64_t capacity_rows, int64_t capacity_nnz,
                           int has_labels, int has_weights, cyc_dataset* out);
int cyc_dataset_destroy(cyc_dataset ds);
int64_t cyc_dataset_rows(cyc_dataset ds);
/* X: rows x numFeatures row-major.  labels / weights: `rows` doubles, required
 * iff the dataset was created with them. */
int cyc_dataset_append_dense(cyc_dataset ds, const double* X, const double* labels,
                             const double* weights, int64_t rows);
/* rowptr: rows+1 entries (any base: rowptr[0] is subtracted), colidx in
 * [0, numFeatures), sorted within a row as in SparseVector. */
int cyc_dataset_append_csr(cyc_dataset ds, const int64_t* rowptr, const int32_t* colidx,
                           const double* vals, const double* labels, const double* weights,
                           int64_t rows);

/* centers: k x d row-major.  sums[k*d] += sum w*x, wsum[k] += sum w,
 * cost[0] += sum w*cost; assign_opt (may be NULL) receives the rows'
 * cluster indices. */
int cyc_kmeans_iter(cyc_dataset ds, const double* centers, int32_t k, double* sums, double* wsum,
                    double* cost, int32_t* assign_opt);
/* The same for a DistanceMeasure (CYC_DISTANCE_*, cyc_kmeans_plan_set_distance
 * _measure); center_norms (host, k; may be NULL = computed) are the centers'
 * VectorWithNorm norms -- with COSINE 1.0 after an update (DistanceMeasure.
 * scala:477-483), which the distances divide by. */
int cyc_kmeans_iter_measure(cyc_dataset ds, int32_t measure, const double* centers,
                            const double* center_norms, int32_t k, double* sums, double* wsum,
                            double* cost, int32_t* assign_opt);
int cyc_logreg_binary_eval(cyc_dataset ds, const double* coef, int fitIntercept, int fitWithMean,
                           const double* scaledMean, double* grad, double* lossSum,
                           double* weightSum);
int cyc_logreg_multinomial_eval(cyc_dataset ds, int32_t numClasses, const double* coef,
                                int fitIntercept, int fitWithMean, const double* scaledMean,
                                double* grad, double* lossSum, double* weightSum);
/* U: packed upper n(n+1)/2 (column-major); mean_opt centers the rows. */
/* The other block aggregators over the resident rows, same conventions as
 * cyc_logreg_*_eval (host model in, host state out; grad / lossSum /
 * weightSum accumulate): LinearSVC's HingeBlockAggregator (dim F +
 * fitIntercept), LinearRegression's LeastSquaresBlockAggregator (dim F;
 * inverseStd required) and HuberBlockAggregator (dim F + fitIntercept + 1),
 * AFTSurvivalRegression's AFTBlockAggregator (dim F + 2; the dataset's
 * weights are the censors). */
int cyc_svc_hinge_eval(cyc_dataset ds, const double* coef, int fitIntercept,
                       const double* scaledMean, double* grad, double* lossSum,
                       double* weightSum);
int cyc_linreg_least_squares_eval(cyc_dataset ds, const double* coef, const double* inverseStd,
                                  int fitIntercept, double labelStd, double labelMean,
                                  const double* scaledMean, double* grad, double* lossSum,
                                  double* weightSum);
int cyc_linreg_huber_eval(cyc_dataset ds, const double* params, int fitIntercept, double epsilon,
                          const double* scaledMean, double* grad, double* lossSum,
                          double* weightSum);
int cyc_aft_eval(cyc_dataset ds, const double* coef, int fitIntercept, const double* scaledMean,
                 double* grad, double* lossSum, double* weightSum);
int cyc_gramian(cyc_dataset ds, const double* mean_opt, double* U);
int cyc_col_sums(cyc_dataset ds, double* sums);

/* ----------------------------------------- the aggregation step (RCCL) */
/* One process per GPU, one communicator per process.
 * Replaces RDD.treeAggregate (core/src/main/scala/org/apache/spark/rdd/
 * RDD.scala:1210-1269: seqOp per partition, foldByKey tree levels
 * :1244-1250, driver fold :1267), KMeans' reduceByKey + collectAsMap
 * (mllib/clustering/KMeans.scala:308-311) and the DoubleAccumulator cost by
 * ONE in-place fp64 sum of the flat aggregator state per iteration
 * (gradient | loss | weight, sums | weights | cost, packed Gramian), and
 * TorrentBroadcast of the model (SparkContext.scala:1524) by a broadcast.
 * Rank 0 makes the id with cyc_comm_unique_id and ships the 128 bytes to
 * every rank out of band (e.g. the Spark driver's broadcast); every rank then
 * calls cyc_comm_init with the same id, world size and its own rank and
 * device (collective: it returns once all ranks have joined; it sets the
 * calling thread's current device).  The sum order across ranks is RCCL's
 * (fixed for a topology), like Spark's completion-order fold it is not the
 * 1-GPU order: results agree to ~1e-15 relative.
 * _dev forms: device buffers, enqueued on `stream`.  Host forms: staged
 * through the communicator's own device buffer and stream, synchronous. */
#define CYC_COMM_ID_BYTES 128
typedef struct cyc_comm_s* cyc_comm;
int cyc_comm_unique_id(unsigned char* id /* CYC_COMM_ID_BYTES */);
int cyc_comm_init(const unsigned char* id, int32_t rank, int32_t world, int32_t device,
                  cyc_comm* out);
int cyc_comm_destroy(cyc_comm comm);
int cyc_comm_rank(cyc_comm comm, int32_t* rank, int32_t* world);
int cyc_allreduce_sum_dev(cyc_comm comm, double* buf, int64_t count, void* stream);
int cyc_allreduce_max_dev(cyc_comm comm, double* buf, int64_t count, void* stream);
int cyc_broadcast_dev(cyc_comm comm, double* buf, int64_t count, int32_t root, void* stream);
/* recv[r*count .. (r+1)*count) = rank r's send (the summarizer buffers,
 * merged in rank order by cyc_summarizer_merge_dev) */
int cyc_allgather_dev(cyc_comm comm, const double* send, double* recv, int64_t count,
                      void* stream);
int cyc_allreduce_sum(cyc_comm comm, double* host_buf, int64_t count);
int cyc_broadcast(cyc_comm comm, double* host_buf, int64_t count, int32_t root);

/* ------------------------------------------------------- LIBSVM input */
/* MLUtils.loadLibSVMFile's parse (mllib/util/MLUtils.scala:91-151:
 * parseLibSVMFile, parseLibSVMRecord, computeNumFeatures) on the host, in
 * parallel over line ranges, straight into CSR arrays for the device
 * (KMeansExample's and the sparse LR configs' input format).  Rows keep file
 * order; labels/values are bit-identical to Double.parseDouble; a bad record
 * returns CYC_ERR_INVALID_ARG with the reference's require text.
 * numFeatures <= 0: max(last index of each row, 0) + 1.  Host-only. */
typedef struct cyc_libsvm_s* cyc_libsvm;
int cyc_libsvm_parse(const char* text, int64_t len, int32_t numFeatures, int nthreads,
                     cyc_libsvm* out);
int cyc_libsvm_load_file(const char* path, int32_t numFeatures, int nthreads, cyc_libsvm* out);
int cyc_libsvm_sizes(cyc_libsvm h, int64_t* n, int64_t* nnz, int32_t* numFeatures);
/* host copies: labels[n], rowptr[n+1], colidx[nnz], values[nnz] (any may be NULL) */
int cyc_libsvm_copy(cyc_libsvm h, double* labels, int64_t* rowptr, int32_t* colidx,
                    double* values);
/* device copies (same shapes), synchronous on the stream */
int cyc_libsvm_upload(cyc_libsvm h, double* labels, int64_t* rowptr, int32_t* colidx,
                      double* values, void* stream);
int cyc_libsvm_destroy(cyc_libsvm h);

#ifdef __cplusplus
}
#endif

#endif /* CYCLONE_H */
