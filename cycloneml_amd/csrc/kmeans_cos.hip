// kmeans_cos.hip -- the CosineDistanceMeasure forms of the KMeans plan
// (mllib/clustering/DistanceMeasure.scala:395-514) on gfx950.
//
// The plan (kmeans.hip) keeps its pipeline and swaps these in:
//   statistics   k_cos_stats_pairs / k_cos_stats_diag: 1 - sqrt(1 - d/2) per
//                center pair, d = 1 - dot(ci, cj) / |ci| / |cj|, the dot a
//                sequential ddot (bit-exact);
//   assignment   the exact-integer i8 screen of kmeans_i8.hip run on UNIT
//                directions (x / |x| rows, c / |c| centers): for unit vectors
//                |u - v|^2 = 2 (1 - cos), so the Euclidean winner the screen
//                certifies is the cosine winner, with the screen's margin
//                (>= ~2^-20 (|u|^2 + |v|^2) ~ 1e-6 in cosine units); rows it
//                cannot certify run k_cos_assign_exact, the reference loop
//                (:421-447, or :131-150 without statistics) restated with the
//                wave-parallel event replay of the Euclidean exact tier;
//   cost, sums   k_cos_row_cost (the distance the loop returns for the chosen
//                center, bit-exact) and k_cos_chunk_sums: axpy(w / |x|, x, sum)
//                (:466-469) over the plan's cluster-sorted chunks;
//   update       k_cos_update: scal(1/w), the norm, scal(1/norm), norm := 1.0
//                (:477-483), isCenterConverged = distance <= epsilon (:161-166).
//
// Why a certified row is the reference's answer.  Let i* be the certified
// center, a = angle(x, i), b = angle(x, i*) < a.  The loop returns early at
// i != i* only if d_i < s(i, i), and skips i* only if s(i*, best) >= d_best.
// By the triangle inequality on angles, s(i, i*) = 1 - cos(angle(i, i*)/2)
// <= 1 - cos((a + b)/2), and cos((a + b)/2) - cos(a) >= (cos b - cos a)/4
// (sin is concave and >= 0 on [0, pi]), so both events need the true gap
// d_i - d_i* to fall below 4x the loop's rounding: ~1e-13 for d_i, and for
// the statistic at most sqrt(d 2^-53) ~ 1.7e-7 (the sqrt of 1 - d/2 near an
// antipodal center pair, d <= 512), below a quarter of the screen's margin.
// The norms the loop divides by are the VectorWithNorm norms: computed ones
// for given centers, 1.0 after an update; a center whose given norm is not
// its computed norm to 2^-40 turns the screen off (every row exact).
#pragma clang fp contract(off)

#include "kmeans_cos.hpp"

#include <algorithm>

#include "common.hpp"

namespace {

constexpr int kT = 32;    // centers per statistics tile side
constexpr int kC = 32;    // dimensions per LDS chunk of the statistics
constexpr int kChunk = 256;   // rows per partial sum (the plan's kChunkRows)

// Order-preserving key of a double (NaN excluded by the caller): unsigned
// key order == numeric order, so atomicMin over keys is a min over values
// that may be negative (a cosine distance rounds to -2^-53 for equal
// directions, making the statistic slightly negative).
__device__ __forceinline__ unsigned long long okey(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double okey_inv(unsigned long long k) {
  return (k >> 63) ? __longlong_as_double((long long)(k & 0x7FFFFFFFFFFFFFFFull))
                   : __longlong_as_double((long long)~k);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

__global__ void k_cos_fill(unsigned long long* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = okey(__builtin_inf());
}

// Pair statistics: one workgroup per 32 x 32 tile of the upper block
// triangle, 2 x 2 pairs per thread, each pair's ddot sequential over the
// dimensions (DistanceMeasure.scala:55-66 with :412-417 and :453-456).
__global__ __launch_bounds__(256) void k_cos_stats_pairs(const double* __restrict__ C,
                                                         const double* __restrict__ cnorm, int k,
                                                         int d, int tps,
                                                         double* __restrict__ packed,
                                                         unsigned long long* __restrict__ dmin) {
  __shared__ double Ci[kT][kC + 1], Cj[kT][kC + 1];
  __shared__ unsigned long long rmin[kT], cmin[kT];
  int t = blockIdx.x, bi = 0;
  while (t >= tps - bi) {
    t -= tps - bi;
    ++bi;
  }
  const int bj = bi + t;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const unsigned long long inf = okey(__builtin_inf());
  if (threadIdx.x < kT) rmin[threadIdx.x] = cmin[threadIdx.x] = inf;
  double s00 = 0.0, s01 = 0.0, s10 = 0.0, s11 = 0.0;
  for (int c0 = 0; c0 < d; c0 += kC) {
    __syncthreads();
    for (int e = threadIdx.x; e < kT * kC; e += 256) {
      const int r = e >> 5, cc = e & 31, col = c0 + cc;
      const int gi = bi * kT + r, gj = bj * kT + r;
      Ci[r][cc] = (gi < k && col < d) ? C[(int64_t)gi * d + col] : 0.0;
      Cj[r][cc] = (gj < k && col < d) ? C[(int64_t)gj * d + col] : 0.0;
    }
    __syncthreads();
    const int lim = min(kC, d - c0);
    for (int cc = 0; cc < lim; ++cc) {
      const double a0 = Ci[ty][cc], a1 = Ci[ty + 16][cc];
      const double b0 = Cj[tx][cc], b1 = Cj[tx + 16][cc];
      s00 = dadd(s00, dmul(a0, b0));
      s01 = dadd(s01, dmul(a0, b1));
      s10 = dadd(s10, dmul(a1, b0));
      s11 = dadd(s11, dmul(a1, b1));
    }
  }
  const double sv[2][2] = {{s00, s01}, {s10, s11}};
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int i = bi * kT + ty + 16 * a, j = bj * kT + tx + 16 * b;
      if (i < k && j < k && j > i) {
        const double dist = 1.0 - sv[a][b] / cnorm[i] / cnorm[j];
        const double v = 1.0 - __builtin_sqrt(1.0 - dist / 2.0);
        packed[iut(i, j)] = v;
        if (!__builtin_isnan(v)) {    // `if (s < diagValues(i))` never keeps a NaN
          const unsigned long long key = okey(v);
          atomicMin(&rmin[ty + 16 * a], key);
          atomicMin(&cmin[tx + 16 * b], key);
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < kT) {
    const int i = bi * kT + threadIdx.x, j = bj * kT + threadIdx.x;
    if (i < k && rmin[threadIdx.x] != inf) atomicMin(&dmin[i], rmin[threadIdx.x]);
    if (j < k && cmin[threadIdx.x] != inf) atomicMin(&dmin[j], cmin[threadIdx.x]);
  }
}

// packed(i, i) = the row minimum (+Infinity when every statistic is NaN);
// k == 1 gives the single NaN of :50.
__global__ void k_cos_stats_diag(int k, double* __restrict__ packed,
                                 const unsigned long long* __restrict__ dmin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  if (k == 1) {
    packed[0] = __builtin_nan("");
    return;
  }
  packed[iut(i, i)] = okey_inv(dmin[i]);
}

__global__ void k_cos_assert(const double* __restrict__ cnorm, int k,
                             const double* __restrict__ xnorm, int64_t n,
                             unsigned long long* __restrict__ flag) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (cnorm)
    for (int64_t i = t0; i < k; i += stride) bad = bad || !(cnorm[i] > 0.0);
  for (int64_t r = t0; r < n; r += stride) bad = bad || !(xnorm[r] > 0.0);
  if (bad) atomicOr(flag, 1ull);
}

// One wave per center.  The computed norm only orients the screen (any
// summation order); the check ties it to the norm the reference divides by.
__global__ __launch_bounds__(256) void k_cos_centers_unit(const double* __restrict__ C,
                                                          const double* __restrict__ cnorm, int k,
                                                          int d, double* __restrict__ V,
                                                          double* __restrict__ vnorm) {
  const int lane = threadIdx.x & 63;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (c >= k) return;
  const double* crow = C + (int64_t)c * d;
  double s = 0.0;
  for (int j = lane; j < d; j += 64) s += crow[j] * crow[j];
  const double t = __builtin_sqrt(wave_sum(s));
  const double g = cnorm[c];
  const bool ok = __builtin_isfinite(t) && t > 0.0 && g > 0.0 &&
                  __builtin_fabs(g - t) <= 0x1p-40 * t;
  double* vrow = V + (int64_t)c * d;
  double s2 = 0.0;
  for (int j = lane; j < d; j += 64) {
    const double v = ok ? crow[j] / t : __builtin_nan("");
    vrow[j] = v;
    s2 += v * v;
  }
  s2 = wave_sum(s2);
  if (lane == 0) vnorm[c] = __builtin_sqrt(s2);
}

__global__ void k_cos_list_all(int32_t* __restrict__ list, unsigned int* __restrict__ count,
                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) list[i] = (int32_t)i;
  if (i == 0) *count = (unsigned int)n;
}

// CosineDistanceMeasure.findClosest (:421-447; stats == nullptr: the base
// findClosest without statistics, :131-150) for the listed rows, one wave
// per row.  As in the Euclidean exact tier (kmeans.hip k_assign_exact): the
// loop state (best, bestIndex) changes only at an event, so 64 consecutive
// centers are measured at once against the current state, a ballot finds
// the first lane whose visit is an event (a return or an update), the state
// advances to it and the lanes after it are re-evaluated (their distances
// reused).  distance(center, x) = 1 - ddot(c, x) / |c| / |x| with the ddot
// sequential over the dimensions, center values from the transposed copy
// (the visiting lanes' loads of one dimension are one coalesced row).
__global__ __launch_bounds__(256) void k_cos_assign_exact(
    const double* __restrict__ X, const double* __restrict__ xnorm, int d,
    const double* __restrict__ C, const double* __restrict__ Ct, int kpad,
    const double* __restrict__ cnorm, int k, const double* __restrict__ stats,
    const int32_t* __restrict__ list, const unsigned int* __restrict__ count,
    int32_t* __restrict__ assign, double* __restrict__ cost) {
  const unsigned cnt = *count;
  const int lane = threadIdx.x & 63;
  const unsigned wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const bool ns = stats == nullptr;
  for (unsigned idx = wid; idx < cnt; idx += nw) {
    const int64_t r = list[idx];
    const double* x = X + r * d;
    const double xn = xnorm[r];
    double best = __builtin_inf();
    if (!ns) {   // :428 bestDistance = distance(centers(0), point)
      double dot = 0.0;
      for (int j = 0; j < d; ++j) dot = dadd(dot, dmul(C[j], x[j]));
      best = 1.0 - dot / cnorm[0] / xn;
    }
    int bi = 0;
    bool done = !ns && best < stats[0];   // :429
    for (int i0 = ns ? 0 : 1; !done && i0 < k; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < k;
      const double sii = (valid && !ns) ? stats[iut(i, i)] : 0.0;
      const double cn = valid ? cnorm[i] : 1.0;
      double dd = 0.0;
      bool have = false;
      int pos = 0;
      for (;;) {
        const bool visit = valid && lane >= pos && (ns || stats[iut(i, bi)] < best);
        if (visit && !have) {
          const double* ci = Ct + i;
          double dot = 0.0;
          for (int j = 0; j < d; ++j) dot = dadd(dot, dmul(ci[(int64_t)j * kpad], x[j]));
          dd = 1.0 - dot / cn / xn;
          have = true;
        }
        const bool brk = !ns && visit && dd < sii;       // :438
        const bool ev = visit && (brk || dd < best);     // :439-442
        const unsigned long long m = __ballot(ev);
        if (!m) break;
        const int f = __ffsll((long long)m) - 1;
        best = __shfl(dd, f);
        bi = i0 + f;
        if (__shfl((int)brk, f)) {
          done = true;
          break;
        }
        pos = f + 1;
      }
    }
    if (lane == 0) {
      assign[r] = bi;
      if (cost) cost[r] = best;
    }
  }
}

// The same loop for SparseVector points (libsvm input): distance(center,
// point) = 1 - dot(c, x) / |c| / |x| with BLAS.dot(dense, sparse) =
// dot(sparse, dense) (mllib/linalg/BLAS.scala:128-134, 153-169), the sum
// over the point's stored entries in order.  Every row (no screen for sparse
// points), one wave per row, grid-stride.
__global__ __launch_bounds__(256) void k_cos_assign_sparse(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const double* __restrict__ vals, const double* __restrict__ xnorm, int64_t n, int d,
    const double* __restrict__ C, const double* __restrict__ cnorm, int k,
    const double* __restrict__ stats, int32_t* __restrict__ assign, double* __restrict__ cost) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const bool ns = stats == nullptr;
  for (int64_t r = wid; r < n; r += nw) {
    const int64_t q0 = rowptr[r], nnz = rowptr[r + 1] - q0;
    const int32_t* idx = colidx + q0;
    const double* val = vals + q0;
    const double xn = xnorm[r];
    auto dist = [&](const double* c, double cn) {
      double dot = 0.0;
      for (int64_t q = 0; q < nnz; ++q) dot = dadd(dot, dmul(val[q], c[idx[q]]));
      return 1.0 - dot / cn / xn;
    };
    double best = ns ? __builtin_inf() : dist(C, cnorm[0]);
    int bi = 0;
    bool done = !ns && best < stats[0];
    for (int i0 = ns ? 0 : 1; !done && i0 < k; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < k;
      const double sii = (valid && !ns) ? stats[iut(i, i)] : 0.0;
      double dd = 0.0;
      bool have = false;
      int pos = 0;
      for (;;) {
        const bool visit = valid && lane >= pos && (ns || stats[iut(i, bi)] < best);
        if (visit && !have) {
          dd = dist(C + (int64_t)i * d, cnorm[i]);
          have = true;
        }
        const bool brk = !ns && visit && dd < sii;
        const bool ev = visit && (brk || dd < best);
        const unsigned long long m = __ballot(ev);
        if (!m) break;
        const int f = __ffsll((long long)m) - 1;
        best = __shfl(dd, f);
        bi = i0 + f;
        if (__shfl((int)brk, f)) {
          done = true;
          break;
        }
        pos = f + 1;
      }
    }
    if (lane == 0) {
      assign[r] = bi;
      if (cost) cost[r] = best;
    }
  }
}

// One thread per row: 256 rows per block, 16-column slices of them staged
// through two padded LDS buffers one slice ahead (coalesced loads, one
// barrier per slice); the dot with the chosen center in column order.
constexpr int kCostRows = 256, kCostCols = 16, kCostStride = kCostCols + 1;
__global__ __launch_bounds__(kCostRows) void k_cos_row_cost(
    const double* __restrict__ X, int64_t n, int d, const double* __restrict__ C,
    const double* __restrict__ cnorm, const double* __restrict__ xnorm,
    const int32_t* __restrict__ assign, double* __restrict__ cost) {
  __shared__ double tile[2][kCostRows * kCostStride];
  const int t = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kCostRows;
  const int64_t myr = row0 + t;
  const int a = myr < n ? assign[myr] : 0;
  const double* crow = C + (int64_t)a * d;
  double v[kCostCols];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < kCostCols; ++i) {
      const int e = t + kCostRows * i, r = e / kCostCols, c = c0 + e % kCostCols;
      const int64_t gr = row0 + r;
      v[i] = (gr < n && c < d) ? __builtin_nontemporal_load(&X[gr * d + c]) : 0.0;
    }
  };
  auto store = [&](double* b) {
#pragma unroll
    for (int i = 0; i < kCostCols; ++i) {
      const int e = t + kCostRows * i;
      b[(e / kCostCols) * kCostStride + e % kCostCols] = v[i];
    }
  };
  double s = 0.0;
  load(0);
  store(tile[0]);
  int buf = 0;
  for (int c0 = 0; c0 < d; c0 += kCostCols) {
    if (c0 + kCostCols < d) load(c0 + kCostCols);
    __syncthreads();   // slice c0 in tile[buf]; every thread done with tile[buf ^ 1]
    const double* row = tile[buf] + t * kCostStride;
    const int lim = min(kCostCols, d - c0);
    for (int c = 0; c < lim; ++c) s = dadd(s, dmul(crow[c0 + c], row[c]));
    if (c0 + kCostCols < d) store(tile[buf ^ 1]);
    buf ^= 1;
  }
  if (myr < n) cost[myr] = 1.0 - s / cnorm[a] / xnorm[myr];
}

// One workgroup per chunk of <= 256 rows of one cluster (rows in their
// original order): thread j sums a_r x_rj over the chunk's rows with
// a_r = w_r / |x_r| (netlib daxpy skips a zero a), 8 rows' loads in flight.
__global__ __launch_bounds__(256) void k_cos_chunk_sums(
    const double* __restrict__ X, int d, const double* __restrict__ w,
    const double* __restrict__ xnorm, const double* __restrict__ cost,
    const int32_t* __restrict__ perm, const int64_t* __restrict__ cstart,
    const int64_t* __restrict__ chunkStart, int k, double* __restrict__ part,
    double* __restrict__ pw, double* __restrict__ pc) {
  __shared__ int32_t rowsS[kChunk];
  __shared__ double coefS[kChunk];
  const int64_t ch = blockIdx.x;
  if (ch >= chunkStart[k]) return;
  int lo = 0, hi = k;   // cluster = last c with chunkStart[c] <= ch
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunkStart[mid] <= ch) lo = mid; else hi = mid;
  }
  const int c = lo;
  const int64_t first = cstart[c] + (ch - chunkStart[c]) * kChunk;
  const int cnt = (int)(min<int64_t>(cstart[c + 1], first + kChunk) - first);
  const int tid = threadIdx.x;
  for (int i = tid; i < cnt; i += 256) {
    const int32_t r = perm[first + i];
    rowsS[i] = r;
    coefS[i] = (w ? w[r] : 1.0) / xnorm[r];   // point.weight / point.norm
  }
  __syncthreads();
  for (int j = tid; j < d; j += 256) {
    double s = 0.0;
    for (int p0 = 0; p0 < cnt; p0 += 8) {
      double xv[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) xv[v] = X[(int64_t)rowsS[min(p0 + v, cnt - 1)] * d + j];
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const double a = coefS[min(p0 + v, cnt - 1)];
        if (p0 + v < cnt && a != 0.0) s = dadd(s, dmul(a, xv[v]));
      }
    }
    part[ch * d + j] = s;
  }
  if (tid == 0) {
    double sw = 0.0, sc = 0.0;
    for (int i = 0; i < cnt; ++i) {
      const int32_t r = rowsS[i];
      const double wt = w ? w[r] : 1.0;
      sw = dadd(sw, wt);                 // clusterWeightSum(bestCenter) += weight
      sc = dadd(sc, dmul(cost[r], wt));  // costAccum.add(cost * weight)
    }
    pw[ch] = sw;
    pc[ch] = sc;
  }
}

// One 64-lane workgroup per center with wsum > 0: lane 0 runs the sequential
// sums (the norm of scal(1/w, sum), then the ddot of the old and new center)
// in index order, then every lane writes its elements.
__global__ __launch_bounds__(64) void k_cos_update(double* __restrict__ C,
                                                   double* __restrict__ cnorm,
                                                   const double* __restrict__ sums,
                                                   const double* __restrict__ wsum, int k, int d,
                                                   double eps, int32_t* __restrict__ converged) {
  __shared__ double ab[2];
  const int c = blockIdx.x, lane = threadIdx.x;
  const double w = wsum[c];
  if (!(w > 0)) return;
  double* crow = C + (int64_t)c * d;
  const double* srow = sums + (int64_t)c * d;
  if (lane == 0) {
    const double a = 1.0 / w;                          // scal(1.0 / weightSum, sum)
    double nn = 0.0;
    for (int j = 0; j < d; ++j) {
      const double v = dmul(a, srow[j]);
      nn = dadd(nn, dmul(v, v));
    }
    const double b = 1.0 / __builtin_sqrt(nn);         // scal(1.0 / norm, sum)
    double dot = 0.0;
    for (int j = 0; j < d; ++j) dot = dadd(dot, dmul(crow[j], dmul(dmul(a, srow[j]), b)));
    // isCenterConverged: distance(old, new) <= epsilon, new.norm = 1
    const double dist = 1.0 - dot / cnorm[c] / 1.0;
    if (!(dist <= eps) && converged) atomicAnd(converged, 0);
    ab[0] = a;
    ab[1] = b;
  }
  __syncthreads();
  const double a = ab[0], b = ab[1];
  for (int j = lane; j < d; j += 64) crow[j] = dmul(dmul(a, srow[j]), b);
  if (lane == 0) cnorm[c] = 1.0;                       // new VectorWithNorm(sum, 1)
}

}  // namespace

namespace cyc {
namespace kmcos {

int stats(const double* C, const double* cnorm, int k, int d, double* packed,
          unsigned long long* dmin, hipStream_t st) {
  const int tps = (k + kT - 1) / kT;
  hipLaunchKernelGGL(k_cos_fill, dim3((k + 255) / 256), dim3(256), 0, st, dmin, k);
  CYC_LAUNCH_CHECK("k_cos_fill");
  hipLaunchKernelGGL(k_cos_stats_pairs, dim3((unsigned)(tps * (tps + 1) / 2)), dim3(256), 0, st, C,
                     cnorm, k, d, tps, packed, dmin);
  CYC_LAUNCH_CHECK("k_cos_stats_pairs");
  hipLaunchKernelGGL(k_cos_stats_diag, dim3((k + 255) / 256), dim3(256), 0, st, k, packed,
                     (const unsigned long long*)dmin);
  CYC_LAUNCH_CHECK("k_cos_stats_diag");
  return CYC_OK;
}

int assert_norms(const double* cnorm, int k, bool checkCenters, const double* xnorm, int64_t n,
                 unsigned long long* flag, hipStream_t st) {
  CYC_HIP(hipMemsetAsync(flag, 0, sizeof(unsigned long long), st));
  const int64_t work = std::max<int64_t>(n, checkCenters ? k : 0);
  if (work == 0) return CYC_OK;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 2048));
  hipLaunchKernelGGL(k_cos_assert, dim3(grid), dim3(256), 0, st, checkCenters ? cnorm : nullptr, k,
                     xnorm, n, flag);
  CYC_LAUNCH_CHECK("k_cos_assert");
  return CYC_OK;
}

int centers_unit(const double* C, const double* cnorm, int k, int d, double* V, double* vnorm,
                 hipStream_t st) {
  hipLaunchKernelGGL(k_cos_centers_unit, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, st, C, cnorm,
                     k, d, V, vnorm);
  CYC_LAUNCH_CHECK("k_cos_centers_unit");
  return CYC_OK;
}

int list_all(int32_t* list, unsigned int* count, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_cos_list_all, dim3((unsigned)((std::max<int64_t>(n, 1) + 255) / 256)),
                     dim3(256), 0, st, list, count, n);
  CYC_LAUNCH_CHECK("k_cos_list_all");
  return CYC_OK;
}

int assign_exact(const double* X, const double* xnorm, int d, const double* C, const double* Ct,
                 int kpad, const double* cnorm, int k, const double* stats, const int32_t* list,
                 const unsigned int* count, int64_t maxRows, int32_t* assign, double* cost,
                 hipStream_t st) {
  KernelTimer timer("k_kmeans_cos_exact", st);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((maxRows + 3) / 4, 4096));
  hipLaunchKernelGGL(k_cos_assign_exact, dim3(grid), dim3(256), 0, st, X, xnorm, d, C, Ct, kpad,
                     cnorm, k, stats, list, count, assign, cost);
  CYC_LAUNCH_CHECK("k_cos_assign_exact");
  return CYC_OK;
}

int assign_sparse(const int64_t* rowptr, const int32_t* colidx, const double* vals,
                  const double* xnorm, int64_t n, int d, const double* C, const double* cnorm,
                  int k, const double* stats, int32_t* assign, double* cost, hipStream_t st) {
  if (n <= 0) return CYC_OK;
  KernelTimer timer("k_kmeans_cos_sparse", st);
  const unsigned grid = (unsigned)std::min<int64_t>((n + 3) / 4, 8192);
  hipLaunchKernelGGL(k_cos_assign_sparse, dim3(grid), dim3(256), 0, st, rowptr, colidx, vals,
                     xnorm, n, d, C, cnorm, k, stats, assign, cost);
  CYC_LAUNCH_CHECK("k_cos_assign_sparse");
  return CYC_OK;
}

int row_cost(const double* X, int64_t n, int d, const double* C, const double* cnorm,
             const double* xnorm, const int32_t* assign, double* cost, hipStream_t st) {
  if (n <= 0) return CYC_OK;
  hipLaunchKernelGGL(k_cos_row_cost, dim3((unsigned)((n + kCostRows - 1) / kCostRows)),
                     dim3(kCostRows), 0, st, X, n, d, C,
                     cnorm, xnorm, assign, cost);
  CYC_LAUNCH_CHECK("k_cos_row_cost");
  return CYC_OK;
}

int chunk_sums(const double* X, int d, const double* w, const double* xnorm, const double* cost,
               const int32_t* perm, const int64_t* cstart, const int64_t* chunkStart, int k,
               int64_t maxChunks, double* part, double* pw, double* pc, hipStream_t st) {
  KernelTimer timer("k_chunk_sums", st);
  hipLaunchKernelGGL(k_cos_chunk_sums, dim3((unsigned)maxChunks), dim3(256), 0, st, X, d, w, xnorm,
                     cost, perm, cstart, chunkStart, k, part, pw, pc);
  CYC_LAUNCH_CHECK("k_cos_chunk_sums");
  return CYC_OK;
}

int update(double* C, double* cnorm, const double* sums, const double* wsum, int k, int d,
           double epsilon, int32_t* converged, hipStream_t st) {
  hipLaunchKernelGGL(k_cos_update, dim3((unsigned)k), dim3(64), 0, st, C, cnorm, sums, wsum, k, d,
                     epsilon, converged);
  CYC_LAUNCH_CHECK("k_cos_update");
  return CYC_OK;
}

}  // namespace kmcos
}  // namespace cyc
