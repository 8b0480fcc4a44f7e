// summarizer.hip -- the LogisticRegression / colStats pre-pass on gfx950.
//
// Replaces, over a device-resident shard:
//   - SummarizerBuffer.add / merge and its metrics (mean, variance, std, sum,
//     count, weightSum, numNonzeros, max, min, normL2, normL1)
//     (mllib/src/main/scala/org/apache/spark/ml/stat/Summarizer.scala:428-770);
//   - MultiClassSummarizer.add / merge / histogram / countInvalid
//     (ml/stat/MultiClassSummarizer.scala:30-98), the label half of
//     Summarizer.getClassificationSummarizers (Summarizer.scala:228-241);
//   - the StandardScaler transform LogisticRegression applies before blokify
//     (ml/feature/StandardScaler.scala:261-283, LogisticRegression.scala:957-965).
//
// The buffer is a per-column Welford recurrence over the NONZERO entries of
// the rows in row order, so it is sequential per column inside a partition.
// Schedule:
//   - the rows are cut into partitions (the shard's Spark partitions); one
//     thread per (partition, column) runs the recurrence over the partition's
//     rows in order.  Dense rows: 256 consecutive columns per workgroup, so
//     every row read is one coalesced 2 KB segment, 8 rows of loads in flight.
//     CSR rows: the row-blocked CSC copy (csc.hip), whose row blocks are the
//     partitions and whose (block, column) runs are exactly one column's
//     nonzeros in row order;
//   - the row-level scalars (count, weight sums) and the label histogram are
//     sequential sums too: one wave per partition streams the weights / labels
//     64 at a time and broadcasts them to a lane-uniform loop;
//   - the partition buffers are folded with merge in partition order, one
//     thread per column (deterministic, no atomics);
//   - a rank's finished buffer is the unit of exchange: ranks all-gather it
//     and merge in rank order (treeAggregate's combOp) -- merge is not a sum,
//     so this is not an all-reduce.
// Buffer layout (doubles): 8 fields x F (structure of arrays: mean, m2n, m2,
// l1, weightSum, nnz, max, min), then count, totalWeightSum, weightSquareSum,
// a flag for a row whose weight failed `require(weight >= 0.0)` (:472) and
// the first such weight.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "common.hpp"

namespace {

enum { kMean = 0, kM2n, kM2, kL1, kWs, kNnz, kMax, kMin, kFields };
constexpr int kScal = 5;   // count, totalWeightSum, weightSquareSum, badFlag, badWeight
constexpr double kDblMax = 1.7976931348623157e308;   // Double.MaxValue
constexpr int kMaxClasses = 8192;                     // LDS histogram of k_label_part

// java.lang.Math.max / min: NaN wins, -0.0 < +0.0
__device__ __forceinline__ double jmax(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && __builtin_signbit(a)) return b;
  return a >= b ? a : b;
}
__device__ __forceinline__ double jmin(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && __builtin_signbit(b)) return b;
  return a <= b ? a : b;
}

// lane j's value, wave-uniform
__device__ __forceinline__ double bcast(double v, int j) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, j);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

struct Col {
  double mean, m2n, m2, l1, ws, nnz, mx, mn;
};

__device__ __forceinline__ void col_init(Col& s) {
  s.mean = s.m2n = s.m2 = s.l1 = s.ws = s.nnz = 0.0;
  s.mx = -kDblMax;   // Double.MinValue (:488)
  s.mn = kDblMax;    // Double.MaxValue (:491)
}

// SummarizerBuffer.add for one nonzero (index, value) of a row of weight
// w > 0 (Summarizer.scala:507-539), the reference's operation order.
__device__ __forceinline__ void col_add(Col& s, double v, double w) {
  if (s.mx < v) s.mx = v;
  if (s.mn > v) s.mn = v;
  const double prev = s.mean;
  const double diff = v - prev;
  s.mean = prev + w * diff / (s.ws + w);
  s.m2n += w * (v - s.mean) * diff;
  s.ws += w;
  s.m2 += w * v * v;
  s.l1 += w * __builtin_fabs(v);
  s.nnz += 1.0;
}

// SummarizerBuffer.merge (:562-617) for one column; tA / tB are the two
// buffers' totalWeightSum.
__device__ __forceinline__ void col_merge(Col& a, double tA, const Col& b, double tB) {
  if (tA != 0.0 && tB != 0.0) {
    const double thisW = a.ws, otherW = b.ws;
    const double tot = thisW + otherW;
    if (tot != 0.0) {
      const double dm = b.mean - a.mean;
      a.mean += dm * otherW / tot;
      a.m2n += b.m2n + dm * dm * thisW * otherW / tot;
    }
    a.ws = tot;
    a.m2 += b.m2;
    a.l1 += b.l1;
    a.mx = jmax(a.mx, b.mx);
    a.mn = jmin(a.mn, b.mn);
    a.nnz = a.nnz + b.nnz;
  } else if (tA == 0.0 && tB != 0.0) {
    a = b;
  }
}

__device__ __forceinline__ void col_load(Col& s, const double* __restrict__ buf, int F, int c) {
  const size_t f = (size_t)F;
  s.mean = buf[kMean * f + c];
  s.m2n = buf[kM2n * f + c];
  s.m2 = buf[kM2 * f + c];
  s.l1 = buf[kL1 * f + c];
  s.ws = buf[kWs * f + c];
  s.nnz = buf[kNnz * f + c];
  s.mx = buf[kMax * f + c];
  s.mn = buf[kMin * f + c];
}

__device__ __forceinline__ void col_store(const Col& s, double* __restrict__ buf, int F, int c) {
  const size_t f = (size_t)F;
  buf[kMean * f + c] = s.mean;
  buf[kM2n * f + c] = s.m2n;
  buf[kM2 * f + c] = s.m2;
  buf[kL1 * f + c] = s.l1;
  buf[kWs * f + c] = s.ws;
  buf[kNnz * f + c] = s.nnz;
  buf[kMax * f + c] = s.mx;
  buf[kMin * f + c] = s.mn;
}

// One thread per (partition, column): the partition's rows in order.
__global__ __launch_bounds__(256) void k_summ_dense(const double* __restrict__ X,
                                                    const double* __restrict__ w, int64_t n, int F,
                                                    int64_t R, int64_t stride,
                                                    double* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int64_t p = blockIdx.y;
  if (c >= F) return;
  const int64_t r0 = p * R, r1 = min(n, r0 + R);
  Col s;
  col_init(s);
  for (int64_t r = r0; r < r1; r += 8) {
    double v[8], wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t rr = min(r + u, r1 - 1);
      v[u] = X[rr * F + c];
      wv[u] = w ? w[rr] : 1.0;
    }
    // rows of weight 0 return early (:473); a negative / NaN weight fails the
    // require (:472) and is reported by k_summ_rows
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (r + u < r1 && wv[u] > 0.0 && v[u] != 0.0) col_add(s, v[u], wv[u]);
  }
  col_store(s, part + p * stride, F, c);
}

// CSR rows through the row-blocked CSC copy: one thread per (block, column),
// the column's nonzeros of the block in row order (row indices are global).
__global__ __launch_bounds__(256) void k_summ_csc(const int64_t* __restrict__ colptr,
                                                  const int32_t* __restrict__ rowidx,
                                                  const double* __restrict__ cv,
                                                  const double* __restrict__ w, int64_t nb, int F,
                                                  int64_t stride, double* __restrict__ part) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;   // b * F + c
  if (e >= nb * F) return;
  const int64_t b = e / F;
  const int c = (int)(e - b * F);
  Col s;
  col_init(s);
  const int64_t k1 = colptr[e + 1];
  for (int64_t k = colptr[e]; k < k1; ++k) {
    const double v = cv[k];
    const double wr = w ? w[rowidx[k]] : 1.0;
    if (wr > 0.0 && v != 0.0) col_add(s, v, wr);
  }
  col_store(s, part + b * stride, F, c);
}

// Row-level scalars of each partition (:472-473, :542-544): count,
// totalWeightSum, weightSquareSum over the rows of weight != 0, and the first
// weight that fails require(weight >= 0.0).  One wave per partition.
__global__ __launch_bounds__(64) void k_summ_rows(const double* __restrict__ w, int64_t n,
                                                  int64_t R, int64_t stride, int F,
                                                  double* __restrict__ part) {
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t r0 = p * R, r1 = min(n, r0 + R);
  double cnt = 0.0, tw = 0.0, tw2 = 0.0, bad = 0.0, badv = 0.0;
  if (!w) {
    for (int64_t r = r0; r < r1; ++r) {   // unit weights: exact integer sums
      tw += 1.0;
      tw2 += 1.0;
      cnt += 1.0;
    }
  } else {
    double nxt = r0 + lane < r1 ? w[r0 + lane] : 0.0;
    for (int64_t b = r0; b < r1; b += 64) {
      const double cur = nxt;
      if (b + 64 + lane < r1) nxt = w[b + 64 + lane];
      const int m = (int)min<int64_t>(64, r1 - b);
      for (int j = 0; j < m; ++j) {
        const double wr = bcast(cur, j);
        if (!(wr >= 0.0)) {
          if (bad == 0.0) {
            bad = 1.0;
            badv = wr;
          }
          continue;
        }
        if (wr == 0.0) continue;
        tw += wr;
        tw2 += wr * wr;
        cnt += 1.0;
      }
    }
  }
  if (lane == 0) {
    double* o = part + p * stride + (size_t)kFields * F;
    o[0] = cnt;
    o[1] = tw;
    o[2] = tw2;
    o[3] = bad;
    o[4] = badv;
  }
}

// out = the P buffers merged in order into an empty buffer; one thread per
// column, every thread folding the scalars the same way.
__global__ __launch_bounds__(256) void k_summ_fold(const double* __restrict__ part, int64_t P,
                                                   int F, int64_t stride,
                                                   double* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= F) return;
  Col a;
  col_init(a);
  double cA = 0.0, tA = 0.0, t2A = 0.0, badA = 0.0, badvA = 0.0;
  for (int64_t p = 0; p < P; ++p) {
    const double* b = part + p * stride;
    const double* sb = b + (size_t)kFields * F;
    const double cB = sb[0], tB = sb[1], t2B = sb[2];
    Col o;
    col_load(o, b, F, c);
    col_merge(a, tA, o, tB);
    if (tA != 0.0 && tB != 0.0) {
      cA += cB;
      tA += tB;
      t2A += t2B;
    } else if (tA == 0.0 && tB != 0.0) {
      cA = cB;
      tA = tB;
      t2A = t2B;
    }
    if (badA == 0.0 && sb[3] != 0.0) {
      badA = 1.0;
      badvA = sb[4];
    }
  }
  col_store(a, out, F, c);
  if (c == 0) {
    double* so = out + (size_t)kFields * F;
    so[0] = cA;
    so[1] = tA;
    so[2] = t2A;
    so[3] = badA;
    so[4] = badvA;
  }
}

// Metrics of a finished buffer (:622-769), 9 x F: mean, variance, std, sum,
// numNonzeros, max, min, normL2, normL1.
__global__ void k_summ_metrics(const double* __restrict__ buf, int F, double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= F) return;
  Col s;
  col_load(s, buf, F, c);
  const double* sc = buf + (size_t)kFields * F;
  const double cnt = sc[0], TW = sc[1], TW2 = sc[2];
  const size_t f = (size_t)F;
  out[0 * f + c] = s.mean * (s.ws / TW);
  // computeVariance (:673-690)
  const double den = TW - (TW2 / TW);
  double var = 0.0;
  if (den > 0.0) var = jmax((s.m2n + s.mean * s.mean * s.ws * (TW - s.ws) / TW) / den, 0.0);
  out[1 * f + c] = var;
  out[2 * f + c] = __builtin_sqrt(var);
  out[3 * f + c] = s.mean * s.ws;
  out[4 * f + c] = s.nnz;
  double mx = s.mx, mn = s.mn;
  if (s.nnz < cnt && mx < 0.0) mx = 0.0;
  if (s.nnz < cnt && mn > 0.0) mn = 0.0;
  out[5 * f + c] = mx;
  out[6 * f + c] = mn;
  out[7 * f + c] = __builtin_sqrt(s.m2);
  out[8 * f + c] = s.l1;
}

// Scala's Double.toInt: NaN -> 0, saturating at the Int range.
__device__ __forceinline__ int jtoint(double x) {
  if (x != x) return 0;
  if (x >= 2147483647.0) return INT_MAX;
  if (x <= -2147483648.0) return INT_MIN;
  return (int)x;
}

// MultiClassSummarizer.add (:43-56) over each partition's rows in order: one
// wave per partition, the per-class weight sums in LDS (maxC doubles), then
// copied to the partition's slab; the invalid count and the largest valid
// label by atomics (order-free integers).  Rows of weight 0 are skipped.
__global__ __launch_bounds__(64) void k_label_part(
    const double* __restrict__ y, const double* __restrict__ w, int64_t n, int64_t R, int maxC,
    double* __restrict__ hist, unsigned long long* __restrict__ inval, int* __restrict__ maxLabel) {
  extern __shared__ double lh[];   // maxC
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  for (int c = lane; c < maxC; c += 64) lh[c] = 0.0;
  __syncthreads();
  const int64_t r0 = p * R, r1 = min(n, r0 + R);
  unsigned long long bad = 0;
  int mx = -1;
  double ny = r0 + lane < r1 ? y[r0 + lane] : 0.0;
  double nw = (w && r0 + lane < r1) ? w[r0 + lane] : 1.0;
  for (int64_t b = r0; b < r1; b += 64) {
    const double cy = ny, cw = nw;
    if (b + 64 + lane < r1) {
      ny = y[b + 64 + lane];
      if (w) nw = w[b + 64 + lane];
    }
    const int m = (int)min<int64_t>(64, r1 - b);
    for (int j = 0; j < m; ++j) {
      const double wr = w ? bcast(cw, j) : 1.0;
      if (!(wr > 0.0)) continue;
      const double lab = bcast(cy, j);
      const int li = jtoint(lab);
      if (lab - (double)li != 0.0 || lab < 0) {
        ++bad;
      } else {
        mx = max(mx, li);
        if (li < maxC && lane == 0) lh[li] = lh[li] + wr;
      }
    }
  }
  __syncthreads();
  double* h = hist + p * (size_t)maxC;
  for (int c = lane; c < maxC; c += 64) h[c] = lh[c];
  if (lane == 0) {
    if (bad) atomicAdd(inval, bad);
    if (mx >= 0) atomicMax(maxLabel, mx);
  }
}

// merge (:66-79) of the partition histograms, in partition order.
__global__ void k_label_fold(const double* __restrict__ hist, int64_t P, int maxC,
                             double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= maxC) return;
  double s = 0.0;
  for (int64_t p = 0; p < P; ++p) s = s + hist[p * (size_t)maxC + c];
  out[c] = s;
}

// StandardScaler.transformDenseWithScale (:261-270): values(i) *= scale(i)
__global__ void k_scale_dense(double* __restrict__ X, int64_t n, int F,
                              const double* __restrict__ scale) {
  const int64_t total = n * (int64_t)F;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x)
    X[e] = X[e] * scale[e % F];
}

// transformSparseWithScale (:272-282): values(i) *= scale(indices(i))
__global__ void k_scale_csr(const int32_t* __restrict__ colidx, double* __restrict__ vals,
                            int64_t nnz, const double* __restrict__ scale) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz;
       e += (int64_t)gridDim.x * blockDim.x)
    vals[e] = vals[e] * scale[colidx[e]];
}

// Partition scratch, one per calling thread (entry points on distinct
// threads may run concurrently, cyclone.h).
cyc::DeviceBuffer& scratch() {
  static thread_local cyc::DeviceBuffer b;
  return b;
}
cyc::DeviceBuffer& scratch2() {
  static thread_local cyc::DeviceBuffer b;
  return b;
}

int fold_into(const double* part, int64_t P, int F, int64_t stride, double* buf, hipStream_t st) {
  hipLaunchKernelGGL(k_summ_fold, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, st, part, P, F,
                     stride, buf);
  CYC_LAUNCH_CHECK("k_summ_fold");
  return CYC_OK;
}

}  // namespace

extern "C" {

int64_t cyc_summarizer_buffer_len(int32_t numFeatures) {
  return numFeatures > 0 ? (int64_t)kFields * numFeatures + kScal : -1;
}

int cyc_summarizer_dense_dev(const double* X, const double* weights, int64_t n, int32_t F,
                             int64_t rows_per_partition, double* buf, void* stream) {
  CYC_REQUIRE(F > 0, "Vector should have dimension larger than zero.");
  CYC_REQUIRE(n >= 0 && rows_per_partition > 0, "n >= 0 and rows_per_partition > 0");
  CYC_REQUIRE(buf != nullptr && (n == 0 || X != nullptr), "X and buf must not be null");
  hipStream_t st = cyc::as_stream(stream);
  const int64_t P = std::max<int64_t>(1, (n + rows_per_partition - 1) / rows_per_partition);
  CYC_REQUIRE(P <= 65535, "at most 65535 partitions per call (raise rows_per_partition)");
  const int64_t stride = (int64_t)kFields * F + kScal;
  if (int rc = scratch().reserve(sizeof(double) * (size_t)(P * stride))) return rc;
  double* part = (double*)scratch().ptr;
  if (n == 0) {
    CYC_HIP(hipMemsetAsync(part, 0, sizeof(double) * (size_t)stride, st));
  } else {
    cyc::KernelTimer timer("k_summ_dense", st);
    hipLaunchKernelGGL(k_summ_dense, dim3((unsigned)((F + 255) / 256), (unsigned)P), dim3(256), 0,
                       st, X, weights, n, F, rows_per_partition, stride, part);
    CYC_LAUNCH_CHECK("k_summ_dense");
    hipLaunchKernelGGL(k_summ_rows, dim3((unsigned)P), dim3(64), 0, st, weights, n,
                       rows_per_partition, stride, F, part);
    CYC_LAUNCH_CHECK("k_summ_rows");
  }
  return fold_into(part, P, F, stride, buf, st);
}

int cyc_summarizer_csr_dev(cyc_csc csc, const double* weights, double* buf, void* stream) {
  CYC_REQUIRE(csc != nullptr && buf != nullptr, "csc and buf must not be null");
  hipStream_t st = cyc::as_stream(stream);
  int64_t R = 0, nb = 0;
  if (int rc = cyc_csc_blocks(csc, &R, &nb)) return rc;
  const int F = cyc_csc_features(csc);
  const int64_t n = cyc_csc_rows(csc);
  CYC_REQUIRE(F > 0, "Vector should have dimension larger than zero.");
  const int64_t P = std::max<int64_t>(1, nb);
  const int64_t stride = (int64_t)kFields * F + kScal;
  if (int rc = scratch().reserve(sizeof(double) * (size_t)(P * stride))) return rc;
  double* part = (double*)scratch().ptr;
  if (n == 0) {
    CYC_HIP(hipMemsetAsync(part, 0, sizeof(double) * (size_t)stride, st));
  } else {
    const int64_t* colptr;
    const int32_t* rowidx;
    const double* cv;
    if (int rc = cyc_csc_arrays(csc, &colptr, &rowidx, &cv)) return rc;
    const int64_t tot = nb * F;
    hipLaunchKernelGGL(k_summ_csc, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, colptr,
                       rowidx, cv, weights, nb, F, stride, part);
    CYC_LAUNCH_CHECK("k_summ_csc");
    hipLaunchKernelGGL(k_summ_rows, dim3((unsigned)P), dim3(64), 0, st, weights, n, R, stride, F,
                       part);
    CYC_LAUNCH_CHECK("k_summ_rows");
  }
  return fold_into(part, P, F, stride, buf, st);
}

int cyc_summarizer_merge_dev(int32_t F, const double* bufs, int64_t count, double* out,
                             void* stream) {
  CYC_REQUIRE(F > 0 && count >= 1 && bufs && out, "F > 0, count >= 1 and non-null buffers");
  const int64_t stride = (int64_t)kFields * F + kScal;
  hipStream_t st = cyc::as_stream(stream);
  // out may alias an input: fold into scratch, then copy
  if (int rc = scratch2().reserve(sizeof(double) * (size_t)stride)) return rc;
  if (int rc = fold_into(bufs, count, F, stride, (double*)scratch2().ptr, st)) return rc;
  CYC_HIP(hipMemcpyAsync(out, scratch2().ptr, sizeof(double) * (size_t)stride,
                         hipMemcpyDeviceToDevice, st));
  return CYC_OK;
}

int cyc_summarizer_metrics_dev(int32_t F, const double* buf, double* metrics, void* stream) {
  CYC_REQUIRE(F > 0 && buf && metrics, "F > 0 and non-null buffers");
  hipLaunchKernelGGL(k_summ_metrics, dim3((unsigned)((F + 255) / 256)), dim3(256), 0,
                     cyc::as_stream(stream), buf, F, metrics);
  CYC_LAUNCH_CHECK("k_summ_metrics");
  return CYC_OK;
}

int cyc_label_summarizer_dev(const double* labels, const double* weights, int64_t n,
                             int64_t rows_per_partition, int32_t max_classes, double* hist,
                             int64_t* invalid, int32_t* max_label, void* stream) {
  CYC_REQUIRE(n >= 0 && rows_per_partition > 0, "n >= 0 and rows_per_partition > 0");
  CYC_REQUIRE(max_classes > 0 && max_classes <= kMaxClasses,
              "max_classes must be in [1, 8192]");
  CYC_REQUIRE(hist && invalid && max_label && (n == 0 || labels), "non-null buffers");
  hipStream_t st = cyc::as_stream(stream);
  const int64_t P = std::max<int64_t>(1, (n + rows_per_partition - 1) / rows_per_partition);
  const size_t hb = sizeof(double) * (size_t)(P * max_classes);
  if (int rc = scratch2().reserve(hb)) return rc;
  double* part = (double*)scratch2().ptr;
  CYC_HIP(hipMemsetAsync(part, 0, hb, st));
  CYC_HIP(hipMemsetAsync(invalid, 0, sizeof(int64_t), st));
  CYC_HIP(hipMemsetAsync(max_label, 0xff, sizeof(int32_t), st));   // -1
  if (n > 0) {
    static bool attr = false;
    if (!attr) {
      CYC_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_label_part),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(sizeof(double) * kMaxClasses)));
      attr = true;
    }
    hipLaunchKernelGGL(k_label_part, dim3((unsigned)P), dim3(64),
                       sizeof(double) * (size_t)max_classes, st, labels, weights, n,
                       rows_per_partition, (int)max_classes, part, (unsigned long long*)invalid,
                       max_label);
    CYC_LAUNCH_CHECK("k_label_part");
  }
  hipLaunchKernelGGL(k_label_fold, dim3((unsigned)((max_classes + 255) / 256)), dim3(256), 0, st,
                     part, P, (int)max_classes, hist);
  CYC_LAUNCH_CHECK("k_label_fold");
  return CYC_OK;
}

int cyc_scale_columns_dense_dev(double* X, int64_t n, int32_t F, const double* scale,
                                void* stream) {
  CYC_REQUIRE(n >= 0 && F > 0 && scale && (n == 0 || X), "n >= 0, F > 0 and non-null buffers");
  if (n == 0) return CYC_OK;
  const int64_t total = n * (int64_t)F;
  const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_scale_dense, dim3(grid), dim3(256), 0, cyc::as_stream(stream), X, n, F,
                     scale);
  CYC_LAUNCH_CHECK("k_scale_dense");
  return CYC_OK;
}

int cyc_scale_columns_csr_dev(const int32_t* colidx, double* vals, int64_t nnz,
                              const double* scale, void* stream) {
  CYC_REQUIRE(nnz >= 0 && scale && (nnz == 0 || (colidx && vals)),
              "nnz >= 0 and non-null buffers");
  if (nnz == 0) return CYC_OK;
  const unsigned grid = (unsigned)std::min<int64_t>((nnz + 255) / 256, 8192);
  hipLaunchKernelGGL(k_scale_csr, dim3(grid), dim3(256), 0, cyc::as_stream(stream), colidx, vals,
                     nnz, scale);
  CYC_LAUNCH_CHECK("k_scale_csr");
  return CYC_OK;
}

}  // extern "C"
