// dataset.cpp -- host-pointer layer of the boundary (layer 2):
// a library-owned, HBM-resident copy of one partition's rows plus the
// per-iteration entry points a JVM shim calls in place of the per-partition
// Scala loops:
//
//   cyc_kmeans_iter              KMeans.scala:287-311 (mapPartitions body of
//                                one Lloyd iteration, incl. computeStatistics;
//                                dense or sparse rows)
//   cyc_logreg_binary_eval       RDDLossFunction.scala:56-70 seqOp over the
//                                partition's blocks with
//                                BinaryLogisticBlockAggregator.add (:81-145)
//   cyc_logreg_multinomial_eval  same with MultinomialLogisticBlockAggregator
//                                .add (:101-189)
//   cyc_gramian / cyc_col_sums   RowMatrix.computeGramianMatrix (:130-161),
//                                computeDenseVectorCovariance (:163-220) and
//                                its colStats mean pre-pass (:456)
//
// Rows are appended once (outside the training loop, like
// InstanceBlock.blokifyWithMaxMemUsage + persist, Instance.scala:146-187) and
// stay resident; each call then moves only the model in and the aggregator
// state out.  Derived per-dataset data (row norms for KMeans, the CSC copy
// for the deterministic sparse gradient) is built on first use and dropped
// when rows are appended.  Plans are cached per shape.  Every call runs on
// the dataset's own stream and returns after its outputs are on the host.
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "common.hpp"

struct cyc_dataset_s {
  bool sparse = false;
  int32_t F = 0;
  int64_t cap_rows = 0, cap_nnz = 0;
  int64_t rows = 0, nnz = 0;
  bool has_labels = false, has_weights = false;
  int device = 0;
  hipStream_t st = nullptr;
  cyc::DeviceBuffer X, rowptr, colidx, vals, labels, weights;
  // derived
  cyc::DeviceBuffer xnorm;
  bool xnorm_ok = false;
  std::map<int, cyc_kmeans_rows> krows;   // per-plan row image (built on first use)
  cyc_csc csc = nullptr;
  // plans
  std::map<int, cyc_kmeans_plan> kplans;
  std::map<std::tuple<int, int, int>, cyc_logistic_plan> lplans;
  // hinge / least squares / Huber / AFT plans: (kind, fitIntercept, a, b)
  std::map<std::tuple<int, int, double, double>, cyc_logistic_plan> xplans;
  cyc_gramian_plan gplan = nullptr;
  // model in / state out staging
  cyc::DeviceBuffer in0, in1, in2, out0, out1;
  std::vector<int64_t> rp_tmp;

  ~cyc_dataset_s() {
    for (auto& kv : krows) cyc_kmeans_rows_destroy(kv.second);
    for (auto& kv : kplans) cyc_kmeans_plan_destroy(kv.second);
    for (auto& kv : lplans) cyc_logistic_plan_destroy(kv.second);
    for (auto& kv : xplans) cyc_logistic_plan_destroy(kv.second);
    if (gplan) cyc_gramian_plan_destroy(gplan);
    if (csc) cyc_csc_destroy(csc);
    if (st) (void)hipStreamDestroy(st);
  }
  void invalidate() {
    xnorm_ok = false;
    for (auto& kv : krows) cyc_kmeans_rows_destroy(kv.second);
    krows.clear();
    if (csc) {
      cyc_csc_destroy(csc);
      csc = nullptr;
    }
  }
};

namespace {

int no_device() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  return CYC_OK;
}

int create(bool sparse, int32_t F, int64_t cap_rows, int64_t cap_nnz, int has_labels,
           int has_weights, cyc_dataset* out) {
  CYC_REQUIRE(out != nullptr, "dataset must not be null");
  CYC_REQUIRE(F > 0, "Number of features must be positive");
  CYC_REQUIRE(cap_rows >= 0 && cap_nnz >= 0, "capacities must be non-negative");
  if (int rc = no_device()) return rc;
  auto ds = std::make_unique<cyc_dataset_s>();
  ds->sparse = sparse;
  ds->F = F;
  ds->cap_rows = cap_rows;
  ds->cap_nnz = cap_nnz;
  ds->has_labels = has_labels != 0;
  ds->has_weights = has_weights != 0;
  CYC_HIP(hipGetDevice(&ds->device));
  CYC_HIP(hipStreamCreateWithFlags(&ds->st, hipStreamNonBlocking));
  int rc;
  const size_t R = (size_t)std::max<int64_t>(cap_rows, 1);
  if (sparse) {
    if ((rc = ds->rowptr.reserve(sizeof(int64_t) * (R + 1))) ||
        (rc = ds->colidx.reserve(sizeof(int32_t) * std::max<int64_t>(cap_nnz, 1))) ||
        (rc = ds->vals.reserve(sizeof(double) * std::max<int64_t>(cap_nnz, 1))))
      return rc;
    CYC_HIP(hipMemsetAsync(ds->rowptr.ptr, 0, sizeof(int64_t), ds->st));
  } else if ((rc = ds->X.reserve(sizeof(double) * R * F))) {
    return rc;
  }
  if (ds->has_labels && (rc = ds->labels.reserve(sizeof(double) * R))) return rc;
  if (ds->has_weights && (rc = ds->weights.reserve(sizeof(double) * R))) return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  *out = ds.release();
  return CYC_OK;
}

int append_meta(cyc_dataset ds, const double* labels, const double* weights, int64_t rows) {
  CYC_REQUIRE(!ds->has_labels || labels, "this dataset holds labels: labels must not be null");
  CYC_REQUIRE(!ds->has_weights || weights,
              "this dataset holds weights: weights must not be null");
  if (ds->has_labels)
    CYC_HIP(hipMemcpyAsync((double*)ds->labels.ptr + ds->rows, labels, sizeof(double) * rows,
                           hipMemcpyHostToDevice, ds->st));
  if (ds->has_weights)
    CYC_HIP(hipMemcpyAsync((double*)ds->weights.ptr + ds->rows, weights, sizeof(double) * rows,
                           hipMemcpyHostToDevice, ds->st));
  return CYC_OK;
}

// staging: reserve + upload `count` doubles from host
int upload(cyc::DeviceBuffer& b, const double* h, size_t count, hipStream_t st, double** d) {
  if (int rc = b.reserve(sizeof(double) * std::max<size_t>(count, 1))) return rc;
  *d = (double*)b.ptr;
  if (h && count) CYC_HIP(hipMemcpyAsync(*d, h, sizeof(double) * count, hipMemcpyHostToDevice, st));
  return CYC_OK;
}

int download(double* h, const double* d, size_t count, hipStream_t st) {
  if (h && count) CYC_HIP(hipMemcpyAsync(h, d, sizeof(double) * count, hipMemcpyDeviceToHost, st));
  return CYC_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int ensure_norms(cyc_dataset ds) {
  if (ds->xnorm_ok) return CYC_OK;
  if (int rc = ds->xnorm.reserve(sizeof(double) * std::max<int64_t>(ds->rows, 1))) return rc;
  if (ds->rows) {
    int rc = ds->sparse ? cyc_row_norms_csr_dev((const int64_t*)ds->rowptr.ptr,
                                                (const double*)ds->vals.ptr, ds->rows,
                                                (double*)ds->xnorm.ptr, ds->st)
                        : cyc_row_norms_dev((const double*)ds->X.ptr, ds->rows, ds->F,
                                            (double*)ds->xnorm.ptr, ds->st);
    if (rc) return rc;
  }
  ds->xnorm_ok = true;
  return CYC_OK;
}

cyc_logistic_plan* lplan(cyc_dataset ds, int C, int fi, int fwm, int* rc) {
  auto key = std::make_tuple(C, fi != 0, fwm != 0);
  auto it = ds->lplans.find(key);
  if (it != ds->lplans.end()) return &it->second;
  cyc_logistic_plan p = nullptr;
  if ((*rc = cyc_logistic_plan_create(ds->F, C, fi, fwm, &p))) return nullptr;
  return &(ds->lplans[key] = p);
}

}  // namespace

extern "C" {

int cyc_dataset_dense_create(int32_t numFeatures, int64_t capacity_rows, int has_labels,
                             int has_weights, cyc_dataset* out) {
  return create(false, numFeatures, capacity_rows, 0, has_labels, has_weights, out);
}

int cyc_dataset_csr_create(int32_t numFeatures, int64_t capacity_rows, int64_t capacity_nnz,
                           int has_labels, int has_weights, cyc_dataset* out) {
  return create(true, numFeatures, capacity_rows, capacity_nnz, has_labels, has_weights, out);
}

int cyc_dataset_destroy(cyc_dataset ds) {
  if (ds) {
    DeviceGuard g(ds->device);
    delete ds;
  }
  return CYC_OK;
}

int64_t cyc_dataset_rows(cyc_dataset ds) { return ds ? ds->rows : -1; }

int cyc_dataset_append_dense(cyc_dataset ds, const double* X, const double* labels,
                             const double* weights, int64_t rows) {
  CYC_REQUIRE(ds != nullptr && !ds->sparse, "a dense dataset is required");
  CYC_REQUIRE(rows >= 0 && (rows == 0 || X), "rows must be non-negative and X non-null");
  CYC_REQUIRE(ds->rows + rows <= ds->cap_rows,
              "dataset capacity exceeded: " + std::to_string(ds->rows + rows) + " rows > " +
                  std::to_string(ds->cap_rows));
  if (rows == 0) return CYC_OK;
  DeviceGuard g(ds->device);
  CYC_HIP(hipMemcpyAsync((double*)ds->X.ptr + ds->rows * (size_t)ds->F, X,
                         sizeof(double) * rows * (size_t)ds->F, hipMemcpyHostToDevice, ds->st));
  if (int rc = append_meta(ds, labels, weights, rows)) return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  ds->rows += rows;
  ds->invalidate();
  return CYC_OK;
}

int cyc_dataset_append_csr(cyc_dataset ds, const int64_t* rowptr, const int32_t* colidx,
                           const double* vals, const double* labels, const double* weights,
                           int64_t rows) {
  CYC_REQUIRE(ds != nullptr && ds->sparse, "a CSR dataset is required");
  CYC_REQUIRE(rows >= 0 && rowptr, "rows must be non-negative and rowptr non-null");
  if (rows == 0) return CYC_OK;
  const int64_t base = rowptr[0], nnz = rowptr[rows] - base;
  CYC_REQUIRE(nnz >= 0 && (nnz == 0 || (colidx && vals)), "malformed CSR block");
  CYC_REQUIRE(ds->rows + rows <= ds->cap_rows && ds->nnz + nnz <= ds->cap_nnz,
              "dataset capacity exceeded");
  for (int64_t i = 0; i < rows; ++i)
    CYC_REQUIRE(rowptr[i + 1] >= rowptr[i], "CSR row pointers must be non-decreasing");
  for (int64_t e = 0; e < nnz; ++e)
    CYC_REQUIRE(colidx[e] >= 0 && colidx[e] < ds->F,
                "column index " + std::to_string(colidx[e]) + " out of range [0, " +
                    std::to_string(ds->F) + ")");
  DeviceGuard g(ds->device);
  ds->rp_tmp.resize(rows);
  for (int64_t i = 0; i < rows; ++i) ds->rp_tmp[i] = rowptr[i + 1] - base + ds->nnz;
  CYC_HIP(hipMemcpyAsync((int64_t*)ds->rowptr.ptr + ds->rows + 1, ds->rp_tmp.data(),
                         sizeof(int64_t) * rows, hipMemcpyHostToDevice, ds->st));
  if (nnz) {
    CYC_HIP(hipMemcpyAsync((int32_t*)ds->colidx.ptr + ds->nnz, colidx, sizeof(int32_t) * nnz,
                           hipMemcpyHostToDevice, ds->st));
    CYC_HIP(hipMemcpyAsync((double*)ds->vals.ptr + ds->nnz, vals, sizeof(double) * nnz,
                           hipMemcpyHostToDevice, ds->st));
  }
  if (int rc = append_meta(ds, labels, weights, rows)) return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  ds->rows += rows;
  ds->nnz += nnz;
  ds->invalidate();
  return CYC_OK;
}

int cyc_kmeans_iter(cyc_dataset ds, const double* centers, int32_t k, double* sums, double* wsum,
                    double* cost, int32_t* assign_opt) {
  return cyc_kmeans_iter_measure(ds, CYC_DISTANCE_EUCLIDEAN, centers, nullptr, k, sums, wsum, cost,
                                 assign_opt);
}

int cyc_kmeans_iter_measure(cyc_dataset ds, int32_t measure, const double* centers,
                            const double* center_norms, int32_t k, double* sums, double* wsum,
                            double* cost, int32_t* assign_opt) {
  CYC_REQUIRE(ds != nullptr && centers && sums && wsum && cost, "arguments must not be null");
  CYC_REQUIRE(k >= 1, "Number of clusters must be positive but got " + std::to_string(k));
  // validated before the plan cache: an unknown measure must not reuse a
  // cached Euclidean plan
  CYC_REQUIRE(measure == CYC_DISTANCE_EUCLIDEAN || measure == CYC_DISTANCE_COSINE,
              "distanceMeasure must be one of: euclidean, cosine. " + std::to_string(measure) +
                  " provided.");
  DeviceGuard g(ds->device);
  // plans and row images per (k, measure)
  const int key = k * 2 + (measure == CYC_DISTANCE_COSINE ? 1 : 0);
  cyc_kmeans_plan plan;
  auto it = ds->kplans.find(key);
  if (it != ds->kplans.end()) {
    plan = it->second;
  } else {
    if (int rc = cyc_kmeans_plan_create(ds->F, k, ds->rows, &plan)) return rc;
    if (int rc = cyc_kmeans_plan_set_distance_measure(plan, measure)) {
      cyc_kmeans_plan_destroy(plan);
      return rc;
    }
    ds->kplans[key] = plan;
  }
  if (int rc = ensure_norms(ds)) return rc;
  cyc_kmeans_rows img = nullptr;
  auto ri = ds->krows.find(key);
  if (ds->sparse) {
    // sparse rows: no row image (the screens are dense-only)
  } else if (ri != ds->krows.end()) {
    img = ri->second;
  } else {
    if (int rc = cyc_kmeans_rows_create(plan, (const double*)ds->X.ptr, ds->rows, ds->st, &img))
      return rc;
    ds->krows[key] = img;
  }
  const size_t kd = (size_t)k * ds->F;
  double *dC, *dCn, *dS, *dW;
  int rc;
  if ((rc = upload(ds->in0, centers, kd, ds->st, &dC)) ||
      (rc = upload(ds->in1, nullptr, k, ds->st, &dCn)) ||
      (rc = upload(ds->out0, sums, kd + 1, ds->st, &dS)) ||
      (rc = upload(ds->out1, wsum, k, ds->st, &dW)))
    return rc;
  CYC_HIP(hipMemcpyAsync(dS + kd, cost, sizeof(double), hipMemcpyHostToDevice, ds->st));
  // the centers' VectorWithNorm norms: given (cosine after an update: 1.0),
  // else computed (new VectorWithNorm(center))
  if (center_norms)
    CYC_HIP(hipMemcpyAsync(dCn, center_norms, sizeof(double) * k, hipMemcpyHostToDevice, ds->st));
  else if ((rc = cyc_row_norms_dev(dC, k, ds->F, dCn, ds->st)))
    return rc;
  int32_t* dA = nullptr;
  if (assign_opt) {
    if ((rc = ds->in2.reserve(sizeof(int32_t) * std::max<int64_t>(ds->rows, 1)))) return rc;
    dA = (int32_t*)ds->in2.ptr;
  }
  const double* w = ds->has_weights ? (const double*)ds->weights.ptr : nullptr;
  if (ds->sparse)
    rc = cyc_kmeans_accumulate_csr_dev(plan, (const int64_t*)ds->rowptr.ptr,
                                       (const int32_t*)ds->colidx.ptr, (const double*)ds->vals.ptr,
                                       (const double*)ds->xnorm.ptr, w, ds->rows, dC, dCn, dS, dW,
                                       dS + kd, dA, nullptr, ds->st);
  else
    rc = cyc_kmeans_accumulate_dev(plan, (const double*)ds->X.ptr, (const double*)ds->xnorm.ptr,
                                   img, w, ds->rows, dC, dCn, dS, dW, dS + kd, dA, nullptr, ds->st);
  if (rc) return rc;
  if ((rc = download(sums, dS, kd, ds->st)) || (rc = download(wsum, dW, k, ds->st)) ||
      (rc = download(cost, dS + kd, 1, ds->st)))
    return rc;
  if (assign_opt && ds->rows)
    CYC_HIP(hipMemcpyAsync(assign_opt, dA, sizeof(int32_t) * ds->rows, hipMemcpyDeviceToHost,
                           ds->st));
  CYC_HIP(hipStreamSynchronize(ds->st));
  return CYC_OK;
}

static int logreg_eval(cyc_dataset ds, int32_t C, const double* coef, int fi, int fwm,
                       const double* scaledMean, double* grad, double* lossSum,
                       double* weightSum) {
  CYC_REQUIRE(ds != nullptr && coef && grad && lossSum && weightSum,
              "arguments must not be null");
  CYC_REQUIRE(ds->has_labels, "the dataset holds no labels");
  DeviceGuard g(ds->device);
  int rc = CYC_OK;
  cyc_logistic_plan* plan = lplan(ds, C, fi, fwm, &rc);
  if (!plan) return rc;
  const size_t dim = C == 1 ? (size_t)ds->F + (fi ? 1 : 0) : (size_t)C * (ds->F + (fi ? 1 : 0));
  double *dCoef, *dMean = nullptr, *dG;
  if ((rc = upload(ds->in0, coef, dim, ds->st, &dCoef)) ||
      (rc = upload(ds->out0, grad, dim + 2, ds->st, &dG)))
    return rc;
  if (scaledMean && (rc = upload(ds->in1, scaledMean, ds->F, ds->st, &dMean))) return rc;
  CYC_HIP(hipMemcpyAsync(dG + dim, lossSum, sizeof(double), hipMemcpyHostToDevice, ds->st));
  CYC_HIP(hipMemcpyAsync(dG + dim + 1, weightSum, sizeof(double), hipMemcpyHostToDevice, ds->st));
  const double* w = ds->has_weights ? (const double*)ds->weights.ptr : nullptr;
  const double* y = (const double*)ds->labels.ptr;
  if (C == 1) {
    if (ds->sparse) {
      if (!ds->csc && ds->rows &&
          (rc = cyc_csc_build_dev((const int64_t*)ds->rowptr.ptr, (const int32_t*)ds->colidx.ptr,
                                  (const double*)ds->vals.ptr, ds->rows, ds->F, ds->st, &ds->csc)))
        return rc;
      rc = cyc_binary_logistic_add_csr_dev(*plan, (const int64_t*)ds->rowptr.ptr,
                                           (const int32_t*)ds->colidx.ptr,
                                           (const double*)ds->vals.ptr, y, w, ds->rows, dCoef,
                                           dMean, dG, dG + dim, dG + dim + 1, ds->csc, ds->st);
    } else {
      rc = cyc_binary_logistic_add_dense_dev(*plan, (const double*)ds->X.ptr, y, w, ds->rows,
                                             dCoef, dMean, dG, dG + dim, dG + dim + 1, ds->st);
    }
  } else {
    if (ds->sparse) {
      if (!ds->csc && ds->rows &&
          (rc = cyc_csc_build_dev((const int64_t*)ds->rowptr.ptr, (const int32_t*)ds->colidx.ptr,
                                  (const double*)ds->vals.ptr, ds->rows, ds->F, ds->st, &ds->csc)))
        return rc;
      rc = cyc_multinomial_logistic_add_csr_dev(
          *plan, (const int64_t*)ds->rowptr.ptr, (const int32_t*)ds->colidx.ptr,
          (const double*)ds->vals.ptr, y, w, ds->rows, dCoef, dMean, dG, dG + dim, dG + dim + 1,
          ds->csc, ds->st);
    } else {
    rc = cyc_multinomial_logistic_add_dense_dev(*plan, (const double*)ds->X.ptr, y, w, ds->rows,
                                                dCoef, dMean, dG, dG + dim, dG + dim + 1, ds->st);
    }
  }
  if (rc) return rc;
  if ((rc = download(grad, dG, dim, ds->st)) || (rc = download(lossSum, dG + dim, 1, ds->st)) ||
      (rc = download(weightSum, dG + dim + 1, 1, ds->st)))
    return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  return CYC_OK;
}

// The other block aggregators on the resident rows: kind 1 hinge, 2 least
// squares (a = labelStd, b = labelMean; inverseStd gives effectiveCoef),
// 3 Huber (a = epsilon), 4 AFT (the dataset's weights are the censors).
static int linear_eval(cyc_dataset ds, int kind, const double* coef, size_t dim, int fi,
                       double a, double b, const double* inverseStd, const double* scaledMean,
                       double* grad, double* lossSum, double* weightSum) {
  CYC_REQUIRE(ds != nullptr && coef && grad && lossSum && weightSum,
              "arguments must not be null");
  CYC_REQUIRE(ds->has_labels, "the dataset holds no labels");
  DeviceGuard g(ds->device);
  int rc = CYC_OK;
  const auto key = std::make_tuple(kind, fi != 0, a, b);
  auto it = ds->xplans.find(key);
  if (it == ds->xplans.end()) {
    cyc_logistic_plan p = nullptr;
    if (kind == 1) rc = cyc_hinge_plan_create(ds->F, fi, &p);
    else if (kind == 2) rc = cyc_least_squares_plan_create(ds->F, fi, a, b, &p);
    else if (kind == 3) rc = cyc_huber_plan_create(ds->F, fi, a, &p);
    else rc = cyc_aft_plan_create(ds->F, fi, &p);
    if (rc) return rc;
    it = ds->xplans.emplace(key, p).first;
  }
  cyc_logistic_plan plan = it->second;
  double *dCoef, *dMean = nullptr, *dInv = nullptr, *dG;
  if ((rc = upload(ds->in0, coef, dim, ds->st, &dCoef)) ||
      (rc = upload(ds->out0, grad, dim + 2, ds->st, &dG)))
    return rc;
  if (scaledMean && (rc = upload(ds->in1, scaledMean, ds->F, ds->st, &dMean))) return rc;
  if (inverseStd && (rc = upload(ds->in2, inverseStd, ds->F, ds->st, &dInv))) return rc;
  CYC_HIP(hipMemcpyAsync(dG + dim, lossSum, sizeof(double), hipMemcpyHostToDevice, ds->st));
  CYC_HIP(hipMemcpyAsync(dG + dim + 1, weightSum, sizeof(double), hipMemcpyHostToDevice, ds->st));
  const double* w = ds->has_weights ? (const double*)ds->weights.ptr : nullptr;
  const double* y = (const double*)ds->labels.ptr;
  if (ds->sparse && !ds->csc && ds->rows &&
      (rc = cyc_csc_build_dev((const int64_t*)ds->rowptr.ptr, (const int32_t*)ds->colidx.ptr,
                              (const double*)ds->vals.ptr, ds->rows, ds->F, ds->st, &ds->csc)))
    return rc;
  const int64_t* rp = (const int64_t*)ds->rowptr.ptr;
  const int32_t* ci = (const int32_t*)ds->colidx.ptr;
  const double* vv = (const double*)ds->vals.ptr;
  const double* X = (const double*)ds->X.ptr;
  double *L = dG + dim, *W = dG + dim + 1;
  switch (kind) {
    case 1:
      rc = ds->sparse ? cyc_hinge_add_csr_dev(plan, rp, ci, vv, y, w, ds->rows, dCoef, dMean, dG, L,
                                              W, ds->csc, ds->st)
                      : cyc_hinge_add_dense_dev(plan, X, y, w, ds->rows, dCoef, dMean, dG, L, W,
                                                ds->st);
      break;
    case 2:
      rc = ds->sparse ? cyc_least_squares_add_csr_dev(plan, rp, ci, vv, y, w, ds->rows, dCoef,
                                                      dInv, dMean, dG, L, W, ds->csc, ds->st)
                      : cyc_least_squares_add_dense_dev(plan, X, y, w, ds->rows, dCoef, dInv,
                                                        dMean, dG, L, W, ds->st);
      break;
    case 3:
      rc = ds->sparse ? cyc_huber_add_csr_dev(plan, rp, ci, vv, y, w, ds->rows, dCoef, dMean, dG, L,
                                              W, ds->csc, ds->st)
                      : cyc_huber_add_dense_dev(plan, X, y, w, ds->rows, dCoef, dMean, dG, L, W,
                                                ds->st);
      break;
    default:
      rc = ds->sparse ? cyc_aft_add_csr_dev(plan, rp, ci, vv, y, w, ds->rows, dCoef, dMean, dG, L,
                                            W, ds->csc, ds->st)
                      : cyc_aft_add_dense_dev(plan, X, y, w, ds->rows, dCoef, dMean, dG, L, W,
                                              ds->st);
  }
  if (rc) return rc;
  if ((rc = download(grad, dG, dim, ds->st)) || (rc = download(lossSum, L, 1, ds->st)) ||
      (rc = download(weightSum, W, 1, ds->st)))
    return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  return CYC_OK;
}

int cyc_svc_hinge_eval(cyc_dataset ds, const double* coef, int fitIntercept,
                       const double* scaledMean, double* grad, double* lossSum,
                       double* weightSum) {
  if (!ds) return linear_eval(ds, 1, coef, 0, 0, 0, 0, nullptr, nullptr, grad, lossSum, weightSum);
  return linear_eval(ds, 1, coef, (size_t)ds->F + (fitIntercept ? 1 : 0), fitIntercept, 0.0, 0.0,
                     nullptr, scaledMean, grad, lossSum, weightSum);
}

int cyc_linreg_least_squares_eval(cyc_dataset ds, const double* coef, const double* inverseStd,
                                  int fitIntercept, double labelStd, double labelMean,
                                  const double* scaledMean, double* grad, double* lossSum,
                                  double* weightSum) {
  CYC_REQUIRE(inverseStd != nullptr, "inverseStd must not be null");
  if (!ds) return linear_eval(ds, 2, coef, 0, 0, 0, 0, nullptr, nullptr, grad, lossSum, weightSum);
  return linear_eval(ds, 2, coef, (size_t)ds->F, fitIntercept, labelStd, labelMean, inverseStd,
                     scaledMean, grad, lossSum, weightSum);
}

int cyc_linreg_huber_eval(cyc_dataset ds, const double* params, int fitIntercept, double epsilon,
                          const double* scaledMean, double* grad, double* lossSum,
                          double* weightSum) {
  if (!ds) return linear_eval(ds, 3, params, 0, 0, 0, 0, nullptr, nullptr, grad, lossSum, weightSum);
  return linear_eval(ds, 3, params, (size_t)ds->F + (fitIntercept ? 2 : 1), fitIntercept, epsilon,
                     0.0, nullptr, scaledMean, grad, lossSum, weightSum);
}

int cyc_aft_eval(cyc_dataset ds, const double* coef, int fitIntercept, const double* scaledMean,
                 double* grad, double* lossSum, double* weightSum) {
  if (!ds) return linear_eval(ds, 4, coef, 0, 0, 0, 0, nullptr, nullptr, grad, lossSum, weightSum);
  return linear_eval(ds, 4, coef, (size_t)ds->F + 2, fitIntercept, 0.0, 0.0, nullptr, scaledMean,
                     grad, lossSum, weightSum);
}

int cyc_logreg_binary_eval(cyc_dataset ds, const double* coef, int fitIntercept, int fitWithMean,
                           const double* scaledMean, double* grad, double* lossSum,
                           double* weightSum) {
  return logreg_eval(ds, 1, coef, fitIntercept, fitWithMean, scaledMean, grad, lossSum,
                     weightSum);
}

int cyc_logreg_multinomial_eval(cyc_dataset ds, int32_t numClasses, const double* coef,
                                int fitIntercept, int fitWithMean, const double* scaledMean,
                                double* grad, double* lossSum, double* weightSum) {
  CYC_REQUIRE(numClasses >= 2, "numClasses must be >= 2 for the multinomial aggregator");
  return logreg_eval(ds, numClasses, coef, fitIntercept, fitWithMean, scaledMean, grad, lossSum,
                     weightSum);
}

int cyc_gramian(cyc_dataset ds, const double* mean_opt, double* U) {
  CYC_REQUIRE(ds != nullptr && U, "arguments must not be null");
  DeviceGuard g(ds->device);
  int rc;
  if (!ds->gplan && (rc = cyc_gramian_plan_create(ds->F, &ds->gplan))) return rc;
  const size_t nu = (size_t)ds->F * (ds->F + 1) / 2;
  double *dU, *dM = nullptr;
  if ((rc = upload(ds->out0, U, nu, ds->st, &dU))) return rc;
  if (mean_opt && (rc = upload(ds->in1, mean_opt, ds->F, ds->st, &dM))) return rc;
  rc = ds->sparse
           ? cyc_gramian_accumulate_csr_dev(ds->gplan, (const int64_t*)ds->rowptr.ptr,
                                            (const int32_t*)ds->colidx.ptr,
                                            (const double*)ds->vals.ptr, ds->rows, dM, dU, ds->st)
           : cyc_gramian_accumulate_dev(ds->gplan, (const double*)ds->X.ptr, ds->rows, dM, dU,
                                        ds->st);
  if (rc) return rc;
  if ((rc = download(U, dU, nu, ds->st))) return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  return CYC_OK;
}

int cyc_col_sums(cyc_dataset ds, double* sums) {
  CYC_REQUIRE(ds != nullptr && sums, "arguments must not be null");
  DeviceGuard g(ds->device);
  int rc;
  if (!ds->gplan && (rc = cyc_gramian_plan_create(ds->F, &ds->gplan))) return rc;
  double* dS;
  if ((rc = upload(ds->out1, sums, ds->F, ds->st, &dS))) return rc;
  rc = ds->sparse ? cyc_col_sums_csr_dev(ds->gplan, (const int64_t*)ds->rowptr.ptr,
                                         (const int32_t*)ds->colidx.ptr,
                                         (const double*)ds->vals.ptr, ds->rows, dS, ds->st)
                  : cyc_col_sums_dev(ds->gplan, (const double*)ds->X.ptr, ds->rows, dS, ds->st);
  if (rc) return rc;
  if ((rc = download(sums, dS, ds->F, ds->st))) return rc;
  CYC_HIP(hipStreamSynchronize(ds->st));
  return CYC_OK;
}

}  // extern "C"
