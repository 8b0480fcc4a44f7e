// binary_rows.hpp -- the per-row margin and epilogue shared by the binary
// block aggregators' kernels (logistic.hip: dense / CSR / CSC paths;
// tiles.hip: the row-block x column-tile layout).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cmath>

namespace cyc {

// ml/impl/Utils.scala:91-97
__device__ __forceinline__ double log1p_exp(double x) {
  return x > 0 ? x + log1p(exp(-x)) : log1p(exp(x));
}

// Row margin before the epilogue.  kind 0/1: offset + dot (dgemv "T" with
// beta = 1 on the filled offset); kind 2 (LeastSquaresBlockAggregator.scala:
// 84-86): arr = offset or 0.0, daxpy(-1/labelStd, labels, arr), then + dot.
__device__ __forceinline__ double row_margin(int kind, int fitIntercept, double offset,
                                             double lscale, double label, double dot) {
  if (kind == 2) return ((fitIntercept ? offset : 0.0) + lscale * label) + dot;
  return fitIntercept ? offset + dot : dot;
}

// Per-row epilogue by aggregator kind; returns the multiplier and
// accumulates loss and weight.
//   0 BinaryLogisticBlockAggregator.scala:104-122
//   1 HingeBlockAggregator.scala:103-117 (labels {0,1} scaled to {-1,1};
//     loss (1 - y' m) w and multiplier -y' w only where the loss is > 0)
//   2 LeastSquaresBlockAggregator.scala:90-100 (every row: loss w d d / 2,
//     multiplier w d)
//   3 HuberBlockAggregator.scala:101-127 (quadratic inside sigma * epsilon,
//     linear outside; sgs accumulates sigmaGradSum)
//   4 AFTBlockAggregator.scala:95-108 (log-linear survival; w = censor)
__device__ __forceinline__ double bin_row(int kind, double margin, double w, double label,
                                          double& loss, double& wsum, double& sgs, double sigma,
                                          double eps) {
  if (kind == 4) {
    // AFTBlockAggregator.scala:95-108: w is the censor delta, sigma =
    // exp(log-sigma), every row counts 1 toward weightSum (:110)
    const double e = (log(label) - margin) / sigma;
    const double ee = exp(e);
    loss += w * log(sigma) - w * e + ee;
    const double m = (w - ee) / sigma;
    sgs += w + m * sigma * e;
    wsum += 1.0;
    return m;
  }
  wsum += w;
  if (w > 0 && kind == 3) {
    const double ll = label - margin;
    if (fabs(ll) <= sigma * eps) {
      loss += 0.5 * w * (sigma + ll * ll / sigma);
      const double lds = ll / sigma;
      sgs += 0.5 * w * (1.0 - lds * lds);
      return -1.0 * w * lds;
    }
    loss += 0.5 * w * (sigma + 2.0 * eps * fabs(ll) - sigma * eps * eps);
    sgs += 0.5 * w * (1.0 - eps * eps);
    return w * (ll >= 0 ? -1.0 : 1.0) * eps;
  }
  if (kind == 2) {
    loss += w * margin * margin / 2;
    return w * margin;
  }
  if (w > 0 && kind == 1) {
    const double ls = label + label - 1.0;
    const double l = (1.0 - ls * margin) * w;
    if (l > 0) {
      loss += l;
      return -ls * w;
    }
    return 0.0;
  }
  if (w > 0) {
    if (label > 0) loss += w * log1p_exp(-margin);
    else loss += w * (log1p_exp(-margin) + margin);
    return w * (1.0 / (1.0 + exp(-margin)) - label);
  }
  return 0.0;
}

}  // namespace cyc
