// silhouette.hip -- ClusteringEvaluator's Silhouette (squared Euclidean and
// cosine) over device rows: the per-cluster statistics as fixed-order folds
// over the rows sorted by prediction, then every row's coefficient against
// every cluster's statistics (silhouette.hpp has the reference lines).
//
// The coefficient needs x . Y_c for every row and every cluster -- an n x k
// x d product.  Here a workgroup holds 64 rows; cluster tiles of 64 and
// 16-dim slices of both operands are staged in LDS, each thread keeps 16
// dot accumulators (one row, 16 clusters), and the per-row epilogue (own
// cluster, nearest other cluster) runs on the tile's dots as they finish.
// The evaluation runs once per fitted model, beside a Lloyd loop of many
// iterations; it is not on the timed path.
#include "common.hpp"
#include "silhouette.hpp"

namespace cyc {
namespace silh {
namespace {

// pred outside [0, k) -> bad[0] += 1; a weight that fails `value >= 0`
// (functions.scala:91, NaN included) -> bad[1] = min row index.
__global__ void k_silh_check(const int32_t* __restrict__ pred, const double* __restrict__ w,
                             int64_t n, int k, unsigned int* __restrict__ bad,
                             unsigned long long* __restrict__ badW) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int p = pred[i];
  if (p < 0 || p >= k) atomicAdd(bad, 1u);
  if (w && !(w[i] >= 0.0)) atomicMin(badW, (unsigned long long)i);
}

// One chunk of <= kChunk rows of one cluster (rows in row order): the
// seqOp's `BLAS.axpy(weight, features, featureSum)` per column, and its
// `squaredNormSum + squaredNorm * weight`, `weightSum + weight`
// (ClusteringMetrics.scala:310-318; cosine :451-458 over x * (1 / |x|),
// BLAS.scal :528-531).  The chunk partials are folded in chunk order.
__global__ __launch_bounds__(256) void k_silh_chunk_sums(
    const double* __restrict__ X, int d, const double* __restrict__ w,
    const double* __restrict__ xnorm, int cosine, const int32_t* __restrict__ perm,
    const int64_t* __restrict__ cstart, const int64_t* __restrict__ chunkStart, int k, int kChunk,
    double* __restrict__ part, double* __restrict__ pw, double* __restrict__ pc) {
  const int64_t ch = blockIdx.x;
  if (ch >= chunkStart[k]) return;
  int lo = 0, hi = k;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunkStart[mid] <= ch) lo = mid;
    else hi = mid;
  }
  const int c = lo;
  const int64_t first = cstart[c] + (ch - chunkStart[c]) * kChunk;
  const int64_t last = min<int64_t>(cstart[c + 1], first + kChunk);
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    double s = 0.0;
    for (int64_t p = first; p < last; ++p) {
      const int64_t r = perm[p];
      double x = X[r * d + j];
      if (cosine) x = dmul(x, 1.0 / xnorm[r]);
      s = dadd(s, dmul(w ? w[r] : 1.0, x));
    }
    part[ch * d + j] = s;
  }
  if (threadIdx.x == 0) {
    double sw = 0.0, sq = 0.0;
    for (int64_t p = first; p < last; ++p) {
      const int64_t r = perm[p];
      const double wt = w ? w[r] : 1.0;
      sw = dadd(sw, wt);
      // math.pow(Vectors.norm(features, 2.0), 2.0) (:385-387)
      if (!cosine) sq = dadd(sq, dmul(dmul(xnorm[r], xnorm[r]), wt));
    }
    pw[ch] = sw;
    pc[ch] = sq;
  }
}

// stats += each cluster's chunks folded in chunk order (the combOp's
// BLAS.axpy(1.0, ...) and sums, :319-333), plus its row count.
__global__ __launch_bounds__(256) void k_silh_fold(const double* __restrict__ part,
                                                   const double* __restrict__ pw,
                                                   const double* __restrict__ pc,
                                                   const int64_t* __restrict__ cstart,
                                                   const int64_t* __restrict__ chunkStart, int d,
                                                   int k, double* __restrict__ stats) {
  const int c = blockIdx.x;
  const int64_t a = chunkStart[c], b = chunkStart[c + 1];
  double* fs = stats;
  double* psi = stats + (int64_t)k * d;
  double* W = psi + k;
  double* cnt = W + k;
  if (a == b) return;
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    double s = 0.0;
    for (int64_t ch = a; ch < b; ++ch) s = dadd(s, part[ch * d + j]);
    fs[(int64_t)c * d + j] = dadd(fs[(int64_t)c * d + j], s);
  }
  if (threadIdx.x == 0) {
    double sw = 0.0, sq = 0.0;
    for (int64_t ch = a; ch < b; ++ch) {
      sw = dadd(sw, pw[ch]);
      sq = dadd(sq, pc[ch]);
    }
    psi[c] = dadd(psi[c], sq);
    W[c] = dadd(W[c], sw);
    cnt[c] = dadd(cnt[c], (double)(cstart[c + 1] - cstart[c]));
  }
}

constexpr int SR = 64;   // rows per workgroup
constexpr int SC = 64;   // clusters per tile (16 per wave)
constexpr int SK = 16;   // dims per LDS slice

// Silhouette.pointSilhouetteCoefficient (:66-97) per row over
// SquaredEuclideanSilhouette.computeSilhouetteCoefficient's compute(c) =
// squaredNorm + squaredNormSum / weightSum - 2 dot(x, featureSum) /
// weightSum (:356-361) or CosineSilhouette's 1 - dot(x / |x|,
// normalizedFeatureSum) / weightSum (:495-498), over the clusters present.
// part[2 b], part[2 b + 1]: the block's sum of s w and of w (row order).
__global__ __launch_bounds__(256) void k_silh_score(const double* __restrict__ X,
                                                    const double* __restrict__ xnorm, int64_t n,
                                                    int d, const int32_t* __restrict__ pred,
                                                    const double* __restrict__ w, int k,
                                                    int cosine, const double* __restrict__ stats,
                                                    double* __restrict__ part) {
  __shared__ double Xs[SR][SK + 1];
  __shared__ double Ys[SC][SK + 1];
  __shared__ double sInv[SR];
  __shared__ double rMin[4][SR];
  __shared__ double rOwn[4][SR];
  __shared__ int rHas[4][SR];
  __shared__ double sS[SR], sW[SR];
  const int t = threadIdx.x, r = t & (SR - 1), q = t >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * SR, row = row0 + r;
  const bool ok = row < n;
  const double* fs = stats;
  const double* psi = stats + (int64_t)k * d;
  const double* W = psi + k;
  const double* cnt = W + k;
  const int own = ok ? pred[row] : -1;
  const double nrm = ok ? xnorm[row] : 1.0;
  const double xsq = dmul(nrm, nrm);
  if (q == 0) sInv[r] = 1.0 / nrm;
  double best = __builtin_inf(), ownD = 0.0;
  bool hasBest = false, hasOwn = false;
  for (int c0 = 0; c0 < k; c0 += SC) {
    double acc[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc[u] = 0.0;
    for (int j0 = 0; j0 < d; j0 += SK) {
      __syncthreads();
      for (int e = t; e < SR * SK; e += 256) {
        const int rr = e / SK, kk = e % SK;
        const int64_t gr = row0 + rr;
        const int j = j0 + kk;
        double v = (gr < n && j < d) ? X[gr * d + j] : 0.0;
        if (cosine) v = dmul(v, sInv[rr]);   // BLAS.scal(1.0 / norm, features)
        Xs[rr][kk] = v;
        const int cc = c0 + rr;
        Ys[rr][kk] = (cc < k && j < d) ? fs[(int64_t)cc * d + j] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < SK; ++kk) {
        const double xv = Xs[r][kk];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc[u] = dadd(acc[u], dmul(xv, Ys[q * 16 + u][kk]));
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int c = c0 + q * 16 + u;
      if (!ok || c >= k || !(cnt[c] > 0.0)) continue;
      const double Wc = W[c];
      const double dist = cosine ? dsub(1.0, acc[u] / Wc)
                                 : dsub(dadd(xsq, psi[c] / Wc), dmul(2.0, acc[u]) / Wc);
      if (c == own) {
        ownD = dist;
        hasOwn = true;
      } else {
        // Scala's Set.min: reduceLeft keeping x when x <= y
        best = (hasBest && best <= dist) ? best : dist;
        hasBest = true;
      }
    }
  }
  rMin[q][r] = best;
  rOwn[q][r] = ownD;
  rHas[q][r] = (hasOwn ? 1 : 0) | (hasBest ? 2 : 0);
  __syncthreads();
  if (q == 0) {
    double s = 0.0, wt = 0.0;
    if (ok) {
      double nb = 0.0, cur = 0.0;
      bool hb = false;
      for (int qq = 0; qq < 4; ++qq) {
        if (rHas[qq][r] & 1) cur = rOwn[qq][r];
        if (rHas[qq][r] & 2) {
          nb = (hb && nb <= rMin[qq][r]) ? nb : rMin[qq][r];
          hb = true;
        }
      }
      wt = w ? w[row] : 1.0;
      const double Wo = W[own];
      if (Wo == wt) {
        s = 0.0;   // single-element cluster (:73-75)
      } else {
        const double cd = dmul(cur, Wo) / dsub(Wo, wt);
        if (cd < nb) s = dsub(1.0, cd / nb);
        else if (cd > nb) s = dsub(nb / cd, 1.0);
        else s = 0.0;
      }
      s = dmul(s, wt);   // overallScore: sum(score * weight) (:102)
    }
    sS[r] = s;
    sW[r] = wt;
  }
  __syncthreads();
  if (t == 0) {
    double a = 0.0, b = 0.0;
    for (int i = 0; i < SR; ++i) {
      a = dadd(a, sS[i]);
      b = dadd(b, sW[i]);
    }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// out[0..1] += the blocks' partials, in block order per thread then a tree.
__global__ __launch_bounds__(256) void k_silh_total(const double* __restrict__ part,
                                                    int64_t blocks, double* __restrict__ out) {
  __shared__ double a[256], b[256];
  const int t = threadIdx.x;
  const int64_t per = (blocks + 255) / 256;
  double sa = 0.0, sb = 0.0;
  for (int64_t i = t * per; i < min<int64_t>(blocks, (t + 1) * per); ++i) {
    sa = dadd(sa, part[2 * i]);
    sb = dadd(sb, part[2 * i + 1]);
  }
  a[t] = sa;
  b[t] = sb;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
      a[t] = dadd(a[t], a[t + s]);
      b[t] = dadd(b[t], b[t + s]);
    }
    __syncthreads();
  }
  if (t == 0) {
    out[0] = dadd(out[0], a[0]);
    out[1] = dadd(out[1], b[0]);
  }
}

}  // namespace

int check_pred(const int32_t* pred, const double* w, int64_t n, int k, unsigned int* bad,
               unsigned long long* badW, hipStream_t st) {
  if (n <= 0) return CYC_OK;
  hipLaunchKernelGGL(k_silh_check, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pred, w,
                     n, k, bad, badW);
  CYC_LAUNCH_CHECK("k_silh_check");
  return CYC_OK;
}

int chunk_sums(const double* X, int d, const double* w, const double* xnorm, bool cosine,
               const int32_t* perm, const int64_t* cstart, const int64_t* chunkStart, int k,
               int64_t maxChunks, int kChunk, double* part, double* pw, double* pc,
               hipStream_t st) {
  if (maxChunks <= 0) return CYC_OK;
  hipLaunchKernelGGL(k_silh_chunk_sums, dim3((unsigned)maxChunks), dim3(256), 0, st, X, d, w,
                     xnorm, cosine ? 1 : 0, perm, cstart, chunkStart, k, kChunk, part, pw, pc);
  CYC_LAUNCH_CHECK("k_silh_chunk_sums");
  return CYC_OK;
}

int fold(const double* part, const double* pw, const double* pc, const int64_t* cstart,
         const int64_t* chunkStart, int d, int k, double* stats, hipStream_t st) {
  hipLaunchKernelGGL(k_silh_fold, dim3((unsigned)k), dim3(256), 0, st, part, pw, pc, cstart,
                     chunkStart, d, k, stats);
  CYC_LAUNCH_CHECK("k_silh_fold");
  return CYC_OK;
}

int score(const double* X, const double* xnorm, int64_t n, int d, const int32_t* pred,
          const double* w, int k, bool cosine, const double* stats, double* scratch, double* out,
          hipStream_t st) {
  if (n <= 0) return CYC_OK;
  const int64_t blocks = (n + SR - 1) / SR;
  {
    KernelTimer timer("k_silh_score", st);
    hipLaunchKernelGGL(k_silh_score, dim3((unsigned)blocks), dim3(256), 0, st, X, xnorm, n, d,
                       pred, w, k, cosine ? 1 : 0, stats, scratch);
    CYC_LAUNCH_CHECK("k_silh_score");
  }
  hipLaunchKernelGGL(k_silh_total, dim3(1), dim3(256), 0, st, (const double*)scratch, blocks, out);
  CYC_LAUNCH_CHECK("k_silh_total");
  return CYC_OK;
}

}  // namespace silh
}  // namespace cyc
