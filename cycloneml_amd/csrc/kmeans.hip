// kmeans.hip -- KMeans Lloyd-iteration body on gfx950 (MI355X).
//
// Replaces mllib/clustering/KMeans.scala:275-334 (the mapPartitions body and
// its reduceByKey merge) and DistanceMeasure.scala:48-118, 189-203, 282-350.
//
// Pipeline per iteration (all device-resident, one stream):
//   1. k_center_transpose  C (k x d) -> Ct (d4 x kpad), zero padded: the MFMA
//                          B operand, read straight from L2 (2 MB at k=1024).
//   2. k_stats_pairs/diag  computeStatistics: 0.25*dist^2 packed upper + row
//                          minima, dist = sqrt(sequential sqdist): bit-exact.
//   3. k_kmeans_assign     fp64 MFMA (v_mfma_f64_16x16x4f64) screen of
//                          |x|^2 + |c|^2 - 2 x.c for a 64-row LDS tile against
//                          every center, with a rigorous error margin; a row
//                          whose best center is separated from every other by
//                          more than the margin gets that center and the exact
//                          sequential sqdist (bit-identical to the reference);
//                          other rows are queued for step 4.
//   4. k_assign_exact      the reference's findClosest-with-statistics loop,
//                          restated instruction for instruction, for queued
//                          rows (ties, near ties, NaN/Inf).
//   5. k_hist/k_scan*/k_scatter  stable counting sort of rows by cluster.
//   6. k_chunk_sums/k_reduce_clusters  per-cluster sum of w*x, w, w*cost in a
//                          fixed order (deterministic run to run).
//   7. k_update_centers    centroid = (1/w)*sum, new norm, convergence flag.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "common.hpp"
#include "kmeans_i8.hpp"
#include "kmeans_cos.hpp"
#include "kmeans_sparse.hpp"
#include "silhouette.hpp"

namespace {

constexpr int kWaves = 8;                 // waves per assign workgroup
constexpr int kAssignThreads = kWaves * 64;
constexpr int kSortTile = 4096;           // rows per counting-sort tile
constexpr int kChunkRows = 256;           // rows per deterministic partial sum
constexpr int kMaxK = 8192;               // LDS histogram bound for the sort

// ---------------------------------------------------------------- helpers
// Vectors.norm(dense, 2) (Vectors.scala:489-514): one thread per row, the
// squares summed in column order.  256 rows per block; 16-column slices of
// them staged through two LDS buffers (row stride 17 doubles: the row-wise
// reads hit distinct banks), loaded coalesced (16 consecutive threads read
// one row's 128 bytes) one slice ahead in registers: one barrier per slice.
constexpr int kNormRows = 256, kNormCols = 16, kNormStride = kNormCols + 1;
__global__ __launch_bounds__(kNormRows) void k_row_norms(const double* __restrict__ X, int64_t n,
                                                         int d, double* __restrict__ norms) {
  __shared__ double tile[2][kNormRows * kNormStride];
  const int t = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kNormRows;
  constexpr int PER = kNormRows * kNormCols / kNormRows;   // loads per thread per slice
  double v[PER];
  // element e = t + 256 i of a slice: row e / 16, column e % 16
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = t + kNormRows * i, r = e / kNormCols, c = c0 + e % kNormCols;
      const int64_t gr = row0 + r;
      v[i] = (gr < n && c < d) ? __builtin_nontemporal_load(&X[gr * d + c]) : 0.0;
    }
  };
  auto store = [&](double* b) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = t + kNormRows * i;
      b[(e / kNormCols) * kNormStride + e % kNormCols] = v[i];
    }
  };
  double s = 0.0;
  load(0);
  store(tile[0]);
  int buf = 0;
  for (int c0 = 0; c0 < d; c0 += kNormCols) {
    if (c0 + kNormCols < d) load(c0 + kNormCols);
    __syncthreads();   // slice c0 in tile[buf]; every thread done with tile[buf ^ 1]
    const double* row = tile[buf] + t * kNormStride;
    const int lim = min(kNormCols, d - c0);
    for (int c = 0; c < lim; ++c) s = dadd(s, dmul(row[c], row[c]));
    if (c0 + kNormCols < d) store(tile[buf ^ 1]);
    buf ^= 1;
  }
  const int64_t gr = row0 + t;
  if (gr < n) norms[gr] = __builtin_sqrt(s);
}

__global__ void k_center_transpose(const double* __restrict__ C, int k, int d, int d4, int kpad,
                                   double* __restrict__ Ct) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)d4 * kpad;
  if (idx >= total) return;
  int j = (int)(idx / kpad), i = (int)(idx % kpad);
  Ct[idx] = (i < k && j < d) ? C[(int64_t)i * d + j] : 0.0;
}

constexpr unsigned long long kInfBits = 0x7FF0000000000000ull;   // +Infinity
constexpr int kStT = 32;    // centers per statistics tile side
constexpr int kStC = 32;    // dimensions per LDS chunk of the statistics

__global__ void k_fill_u64(unsigned long long* __restrict__ p, int n, unsigned long long v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}
// k_center_transpose and the statistics' dmin fill in one launch
__global__ void k_center_transpose_fill(const double* __restrict__ C, int k, int d, int d4,
                                        int kpad, double* __restrict__ Ct,
                                        unsigned long long* __restrict__ p, unsigned long long v) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < k) p[idx] = v;
  const int64_t total = (int64_t)d4 * kpad;
  if (idx >= total) return;
  const int j = (int)(idx / kpad), i = (int)(idx % kpad);
  Ct[idx] = (i < k && j < d) ? C[(int64_t)i * d + j] : 0.0;
}
// two counters zeroed by one launch (two fills before)
__global__ void k_zero2(unsigned int* __restrict__ a, unsigned int* __restrict__ b) {
  if (threadIdx.x == 0) *a = 0u;
  if (threadIdx.x == 1 && b) *b = 0u;
}

// computeStatistics pairs (DistanceMeasure.scala:55-66, Euclidean :275-277):
// s = 0.25 * distance * distance, distance = Math.sqrt(sqdist(c_i, c_j)).
// One workgroup per 32 x 32 tile of the upper block triangle: 32-dimension
// chunks of both center tiles in LDS, 2 x 2 pairs per thread, every pair's
// sum sequential over the dimensions in order (bit-exact).  The row minima
// of the diagonal (:62-63) go to dmin as fp64 bit patterns: a statistic is
// >= +0 or NaN, and for those the unsigned bit order is the value order with
// every NaN above +Infinity, so atomicMin never keeps a NaN -- just as the
// reference's `if (s < diagValues(i))` skips it.
__global__ __launch_bounds__(256) void k_stats_pairs(const double* __restrict__ C, int k, int d,
                                                     int tps, double* __restrict__ packed,
                                                     unsigned long long* __restrict__ dmin) {
  __shared__ double Ci[kStT][kStC + 1], Cj[kStT][kStC + 1];
  __shared__ unsigned long long rmin[kStT], cmin[kStT];
  int t = blockIdx.x, bi = 0;
  while (t >= tps - bi) {
    t -= tps - bi;
    ++bi;
  }
  const int bj = bi + t;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  if (threadIdx.x < kStT) rmin[threadIdx.x] = cmin[threadIdx.x] = kInfBits;
  double s00 = 0.0, s01 = 0.0, s10 = 0.0, s11 = 0.0;
  for (int c0 = 0; c0 < d; c0 += kStC) {
    __syncthreads();
    for (int e = threadIdx.x; e < kStT * kStC; e += 256) {
      const int r = e >> 5, cc = e & 31, col = c0 + cc;
      const int gi = bi * kStT + r, gj = bj * kStT + r;
      Ci[r][cc] = (gi < k && col < d) ? C[(int64_t)gi * d + col] : 0.0;
      Cj[r][cc] = (gj < k && col < d) ? C[(int64_t)gj * d + col] : 0.0;
    }
    __syncthreads();
    const int lim = min(kStC, d - c0);
    for (int cc = 0; cc < lim; ++cc) {
      const double a0 = Ci[ty][cc], a1 = Ci[ty + 16][cc];
      const double b0 = Cj[tx][cc], b1 = Cj[tx + 16][cc];
      double q = dsub(a0, b0);
      s00 = dadd(s00, dmul(q, q));
      q = dsub(a0, b1);
      s01 = dadd(s01, dmul(q, q));
      q = dsub(a1, b0);
      s10 = dadd(s10, dmul(q, q));
      q = dsub(a1, b1);
      s11 = dadd(s11, dmul(q, q));
    }
  }
  const double sv[2][2] = {{s00, s01}, {s10, s11}};
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int i = bi * kStT + ty + 16 * a, j = bj * kStT + tx + 16 * b;
      if (i < k && j < k && j > i) {
        const double dist = __builtin_sqrt(sv[a][b]);
        const double v = dmul(dmul(0.25, dist), dist);
        packed[iut(i, j)] = v;
        const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
        atomicMin(&rmin[ty + 16 * a], bits);
        atomicMin(&cmin[tx + 16 * b], bits);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < kStT) {
    const int i = bi * kStT + threadIdx.x, j = bj * kStT + threadIdx.x;
    if (i < k && rmin[threadIdx.x] != kInfBits) atomicMin(&dmin[i], rmin[threadIdx.x]);
    if (j < k && cmin[threadIdx.x] != kInfBits) atomicMin(&dmin[j], cmin[threadIdx.x]);
  }
}

// diagonal (:69-74): packed(i, i) = min over j != i (+Infinity when every
// statistic of the row is NaN); k == 1 gives the single NaN of :50.
__global__ void k_stats_diag(int k, double* __restrict__ packed,
                             const unsigned long long* __restrict__ dmin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  if (k == 1) {
    packed[0] = __builtin_nan("");
    return;
  }
  packed[iut(i, i)] = __longlong_as_double((long long)dmin[i]);
}

// --------------------------------------------------------------- assign
// Screening state of one (row, lane) slot: smallest lower bound L1 with its
// center index I1 and upper bound U1, and the second smallest lower bound L2.
// A row is decided when L2 > U1: every other center is provably farther than
// I1 by more than the combined fp64 error, so the reference's pruned loop
// (whose prunes only skip centers that cannot win) returns I1 as well.
//
// The bounds are kept in fp32 rounded outward (L down, U up): the interval
// only widens, so a decided row is still provably decided; rows whose gap is
// below fp32 resolution (~1e-7 relative) simply go to the exact path.  This
// halves the per-lane state (16 slots per lane) and keeps the kernel in
// registers.
struct Slot {
  float L1, U1, L2;
  int I1;
};

// one fp32 ulp toward -inf / +inf (f finite, not NaN)
__device__ __forceinline__ float ulp_down(float f) {
  int b = __float_as_int(f);
  if (f == 0.0f) return -__int_as_float(1);
  return __int_as_float(f > 0.0f ? b - 1 : b + 1);
}
__device__ __forceinline__ float f_down(double x) {
  float f = (float)x;
  return ((double)f > x) ? ulp_down(f) : f;
}
__device__ __forceinline__ float f_up(double x) {
  float f = (float)x;
  return ((double)f < x) ? -ulp_down(-f) : f;
}

__device__ __forceinline__ void slot_merge(Slot& a, float oL1, float oU1, float oL2, int oI1) {
  float hi = fmaxf(a.L1, oL1);
  float l2 = fminf(hi, fminf(a.L2, oL2));
  if (oL1 < a.L1 || (oL1 == a.L1 && oI1 >= 0 && (a.I1 < 0 || oI1 < a.I1))) {
    a.L1 = oL1;
    a.U1 = oU1;
    a.I1 = oI1;
  }
  a.L2 = l2;
}

// BM rows per workgroup (BM/16 MFMA row tiles per wave); 8 waves split the
// centers in 16-wide slabs.  X tile lives in LDS with a row stride of
// ldsStride doubles (== 2 mod 32: conflict-free ds_read_b64 A fragments).
template <int BM>
__global__ __launch_bounds__(kAssignThreads, 1) void k_kmeans_assign(
    const double* __restrict__ X, const double* __restrict__ xnorm, int64_t n, int d, int d4,
    int ldsStride, const double* __restrict__ Ct, const double* __restrict__ C,
    const double* __restrict__ cnorm, int k, int kpad, double marginFac,
    int32_t* __restrict__ assign, double* __restrict__ cost, int32_t* __restrict__ slowList,
    unsigned int* __restrict__ slowCount, const int32_t* __restrict__ rowList,
    const unsigned int* __restrict__ rowCount) {
  constexpr int T = BM / 16;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Xs = smem;                                   // BM x ldsStride
  double* xnS = Xs + BM * ldsStride;                   // BM
  double* mrg = xnS + BM;                              // kWaves x BM x 4

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Row source: rows row0.. of X (full pass, one block per tile), or the
  // rows an earlier screen queued in rowList (grid-stride over its tiles).
  const int64_t nsrc = rowList ? (int64_t)*rowCount : n;
  for (int64_t blk = blockIdx.x; blk * BM < nsrc; blk += gridDim.x) {
#define CYC_GROW1(i) (rowList ? (int64_t)rowList[row0 + (i)] : row0 + (i))
  const int64_t row0 = blk * BM;
  const int rows = (int)min<int64_t>(BM, nsrc - row0);

  // Stage the BM x d block of X (zero padded to d4 and BM).
  {
    const int total = rows * d;  // < 2^31: BM * d <= 64 * 1240
    for (int e = tid; e < total; e += kAssignThreads) {
      int r = e / d, c = e - r * d;
      Xs[r * ldsStride + c] = X[CYC_GROW1(r) * d + c];
    }
    for (int e = tid; e < BM * d4; e += kAssignThreads) {
      int r = e / d4, c = e - r * d4;
      if (r >= rows || c >= d) Xs[r * ldsStride + c] = 0.0;
    }
    if (tid < BM) xnS[tid] = (tid < rows) ? xnorm[CYC_GROW1(tid)] : 0.0;
  }
  __syncthreads();

  // Per-(row slot, lane) screening state in plain scalar arrays (static
  // indices only, so they stay in registers).
  float sL1[T * 4], sU1[T * 4], sL2[T * 4];
  int sI1[T * 4];
#pragma unroll
  for (int q = 0; q < T * 4; ++q) {
    sL1[q] = sU1[q] = sL2[q] = __builtin_inff();
    sI1[q] = -1;
  }
  unsigned poison = 0;  // bit (4t + r): a NaN reached this slot
  const double* arow = Xs + (lane & 15) * ldsStride + (lane >> 4);
  cyc_double4 acc[T];

  // Screening update for one finished 16-center slab (centers nb .. nb+15).
#define CYC_EPILOGUE(NB, CN)                                                   \
  do {                                                                         \
    const int c_ = (NB) + (lane & 15);                                         \
    if (c_ < k) {                                                              \
      const double cn_ = (CN);                                                 \
      const double cn2_ = cn_ * cn_;                                           \
      _Pragma("unroll") for (int t = 0; t < T; ++t) {                          \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                        \
          const int q = 4 * t + r;                                             \
          const double xn = xnS[t * 16 + (lane >> 4) + 4 * r];                 \
          const double approx = (xn * xn + cn2_) - 2.0 * acc[t][r];            \
          const double sm = xn + cn_;                                          \
          const double M = (sm * sm) * marginFac;                              \
          const double L = approx - M, U = approx + M;                         \
          if (!(L == L) || !(U == U)) poison |= 1u << q;                       \
          if (L < sL1[q]) {                                                    \
            sL2[q] = sL1[q];                                                   \
            sL1[q] = f_down(L);                                                \
            sU1[q] = f_up(U);                                                  \
            sI1[q] = c_;                                                       \
          } else if (L < sL2[q]) {                                             \
            sL2[q] = f_down(L);                                                \
          }                                                                    \
        }                                                                      \
      }                                                                        \
    }                                                                          \
  } while (0)

  const int nslabs = (kpad - wave * 16 + kWaves * 16 - 1) / (kWaves * 16);
  if ((d4 & 15) == 0) {
    // Flat software pipeline over (slab, 16-dim group) steps: the B fragments
    // of step i+1 are in flight while step i's 4 x T MFMAs run.  Two named
    // register buffers keep every index static.
    const int G = d4 / 16;
    const int total = nslabs * G;
    double cn = 0.0;
    double b0[4], b1[4];
#define CYC_LOADB(B, I)                                                             \
  do {                                                                              \
    const int nb_ = wave * 16 + ((I) / G) * (kWaves * 16);                          \
    const double* bc_ = Ct + (int64_t)(((I) % G) * 16 + (lane >> 4)) * kpad + nb_ + \
                        (lane & 15);                                                \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) B[s] = bc_[(int64_t)(s * 4) * kpad]; \
  } while (0)
#define CYC_COMPUTE(B, I)                                                           \
  do {                                                                              \
    const int g_ = (I) % G;                                                         \
    const int nb_ = wave * 16 + ((I) / G) * (kWaves * 16);                          \
    if (g_ == 0) {                                                                  \
      _Pragma("unroll") for (int t = 0; t < T; ++t) acc[t] = cyc_double4{0.0, 0.0, 0.0, 0.0}; \
      const int c0_ = nb_ + (lane & 15);                                            \
      cn = c0_ < k ? cnorm[c0_] : 0.0;                                              \
    }                                                                               \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                 \
      _Pragma("unroll") for (int t = 0; t < T; ++t) {                               \
        const double a_ = arow[t * 16 * ldsStride + g_ * 16 + s * 4];               \
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a_, B[s], acc[t], 0, 0, 0);   \
      }                                                                             \
    }                                                                               \
    if (g_ == G - 1) CYC_EPILOGUE(nb_, cn);                                         \
  } while (0)
    if (total > 0) CYC_LOADB(b0, 0);
    for (int i = 0; i < total; i += 2) {
      if (i + 1 < total) CYC_LOADB(b1, i + 1);
      CYC_COMPUTE(b0, i);
      if (i + 2 < total) CYC_LOADB(b0, i + 2);
      if (i + 1 < total) CYC_COMPUTE(b1, i + 1);
    }
#undef CYC_LOADB
#undef CYC_COMPUTE
  } else {
    for (int nb = wave * 16; nb < kpad; nb += kWaves * 16) {
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] = cyc_double4{0.0, 0.0, 0.0, 0.0};
      const double* bcol = Ct + (int64_t)(lane >> 4) * kpad + nb + (lane & 15);
      for (int kb = 0; kb < d4; kb += 4) {
        const double b = bcol[(int64_t)kb * kpad];
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const double a = arow[t * 16 * ldsStride + kb];
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
        }
      }
      const int c = nb + (lane & 15);
      CYC_EPILOGUE(nb, c < k ? cnorm[c] : 0.0);
    }
  }
#undef CYC_EPILOGUE

  // Reduce each slot over the 16 lanes that hold the same row.
#pragma unroll
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 4 * t + r;
      Slot S{sL1[q], sU1[q], sL2[q], sI1[q]};
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        float oL1 = __shfl_xor(S.L1, m), oU1 = __shfl_xor(S.U1, m), oL2 = __shfl_xor(S.L2, m);
        int oI1 = __shfl_xor(S.I1, m);
        slot_merge(S, oL1, oU1, oL2, oI1);
      }
      sL1[q] = S.L1;
      sU1[q] = S.U1;
      sL2[q] = S.L2;
      sI1[q] = S.I1;
    }
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) poison |= __shfl_xor(poison, m);

  if ((lane & 15) == 0) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = t * 16 + (lane >> 4) + 4 * r;
        double* m = mrg + ((size_t)wave * BM + row) * 4;
        const int q = 4 * t + r;
        m[0] = sL1[q];
        m[1] = sU1[q];
        m[2] = ((poison >> q) & 1u) ? -__builtin_inf() : (double)sL2[q];
        m[3] = (double)sI1[q];
      }
    }
  }
  __syncthreads();

  // One lane per row: merge the 8 waves, then decide or queue.
  if (tid < rows) {
    const int row = tid;
    Slot S{__builtin_inff(), __builtin_inff(), __builtin_inff(), -1};
    for (int w = 0; w < kWaves; ++w) {
      const double* m = mrg + ((size_t)w * BM + row) * 4;
      slot_merge(S, (float)m[0], (float)m[1], (float)m[2], (int)m[3]);
    }
    const int64_t grow = CYC_GROW1(row);
    if (S.I1 >= 0 && S.L2 > S.U1) {
      // Exact fastSquaredDistance(centers(I1), point) = Vectors.sqdist(c, x)
      // (when the caller wants per-row costs; the Lloyd path computes them
      // in k_chunk_sums).
      if (cost) {
        const double* crow = C + (int64_t)S.I1 * d;
        const double* xrow = Xs + row * ldsStride;
        double s = 0.0;
        for (int j = 0; j < d; ++j) {
          double sc = dsub(crow[j], xrow[j]);
          s = dadd(s, dmul(sc, sc));
        }
        cost[grow] = s;
      }
      assign[grow] = S.I1;
    } else {
      unsigned slot = atomicAdd(slowCount, 1u);
      slowList[slot] = (int32_t)grow;
    }
  }
  __syncthreads();   // LDS is restaged by the next tile
  }
#undef CYC_GROW1
}

// Second-generation assign kernel (the default when d4 % 32 == 0 and the
// center norms fit in LDS):
//   - per (row slot, lane) only the lower bounds L1 (best), L2 (second) in
//     fp32 rounded down and the best index; the upper bound of the best
//     center is rebuilt at the end as next_up(L1) + 2 M(best) from its norm,
//     which is >= its true upper bound, so certification stays conservative;
//   - branch-free epilogue (selects), center norms read from LDS (no global
//     load that would force a vmcnt(0) drain of the B prefetch);
//   - B fragments for 32 dims (8 MFMA k-steps) ping-pong between two named
//     register sets, one step ahead.
template <int BM>
__global__ __launch_bounds__(kAssignThreads, 1) void k_kmeans_assign2(
    const double* __restrict__ X, const double* __restrict__ xnorm, int64_t n, int d, int d4,
    int ldsStride, const double* __restrict__ Ct, const double* __restrict__ C,
    const double* __restrict__ cnorm, int k, int kpad, double marginFac,
    int32_t* __restrict__ assign, double* __restrict__ cost, int32_t* __restrict__ slowList,
    unsigned int* __restrict__ slowCount, const int32_t* __restrict__ rowList,
    const unsigned int* __restrict__ rowCount) {
  constexpr int T = BM / 16;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Xs = smem;                      // BM x ldsStride
  double* xnS = Xs + BM * ldsStride;      // BM
  double* mrg = xnS + BM;                 // kWaves x BM x 4
  double* cnS = mrg + kWaves * BM * 4;    // kpad center norms
  double* xqS = cnS + kpad;               // BM: xn^2 (1 - 2 fac)
  // Row source: rows row0.. of X (full pass, one block per tile), or the
  // rows queued in rowList by the bf16 screen (grid-stride over its tiles).
  const int64_t nsrc = rowList ? (int64_t)*rowCount : n;
  for (int64_t blk = blockIdx.x; blk * BM < nsrc; blk += gridDim.x) {
#define CYC_GROW(i) (rowList ? (int64_t)rowList[row0 + (i)] : row0 + (i))
  // Margin M' = 2 fac (|x|^2 + |c|^2) >= fac (|x| + |c|)^2, so the lower bound
  // is L = (xq + cq) - 2 x.c with xq = |x|^2 (1 - 2 fac), cq likewise.
  const double fac2 = 2.0 * marginFac;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
  const int64_t row0 = blk * BM;
  const int rows = (int)min<int64_t>(BM, nsrc - row0);
  {
    const int total = rows * d;
    for (int e = tid; e < total; e += kAssignThreads) {
      int r = e / d, c = e - r * d;
      Xs[r * ldsStride + c] = X[CYC_GROW(r) * d + c];
    }
    for (int e = tid; e < BM * d4; e += kAssignThreads) {
      int r = e / d4, c = e - r * d4;
      if (r >= rows || c >= d) Xs[r * ldsStride + c] = 0.0;
    }
    if (tid < BM) {
      const double xn = (tid < rows) ? xnorm[CYC_GROW(tid)] : 0.0;
      xnS[tid] = xn;
      xqS[tid] = (xn * xn) * (1.0 - fac2);
    }
    for (int c = tid; c < kpad; c += kAssignThreads) cnS[c] = c < k ? cnorm[c] : 0.0;
  }
  __syncthreads();
  // B fragments through a buffer descriptor: per-lane byte offset constant,
  // the (group, k-step, slab) part in an SGPR soffset -> no VALU address math.
  const auto ctR = __builtin_amdgcn_make_buffer_rsrc((void*)Ct, (short)0, d4 * kpad * 8,
                                                     0x00020000);
  const int laneOff = ((lane >> 4) * kpad + (lane & 15)) * 8;

  float sL1[T * 4], sL2[T * 4];
  int sI1[T * 4];
#pragma unroll
  for (int q = 0; q < T * 4; ++q) {
    sL1[q] = sL2[q] = __builtin_inff();
    sI1[q] = -1;
  }
  unsigned poison = 0;
  const double* arow = Xs + (lane & 15) * ldsStride + (lane >> 4);
  cyc_double4 acc[T];
  const int G = d4 / 32;
  const int nslabs = (kpad - wave * 16 + kWaves * 16 - 1) / (kWaves * 16);
  const int total = nslabs * G;
  double b0[8], b1[8];

#define CYC_LOADB(B, I)                                                              \
  do {                                                                               \
    const int nb_ = wave * 16 + ((I) / G) * (kWaves * 16);                           \
    const int so_ = ((((I) % G) * 32) * kpad + nb_) * 8;                             \
    _Pragma("unroll") for (int s = 0; s < 8; ++s)                                    \
      B[s] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(          \
          ctR, laneOff, so_ + s * 32 * kpad, 0));                                    \
  } while (0)
#define CYC_COMPUTE(B, I)                                                            \
  do {                                                                               \
    const int g_ = (I) % G;                                                          \
    if (g_ == 0) {                                                                   \
      _Pragma("unroll") for (int t = 0; t < T; ++t) acc[t] = cyc_double4{0.0, 0.0, 0.0, 0.0}; \
    }                                                                                \
    _Pragma("unroll") for (int s = 0; s < 8; ++s) {                                  \
      _Pragma("unroll") for (int t = 0; t < T; ++t) {                                \
        const double a_ = arow[t * 16 * ldsStride + g_ * 32 + s * 4];                \
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a_, B[s], acc[t], 0, 0, 0);    \
      }                                                                              \
    }                                                                                \
    if (g_ == G - 1) {                                                               \
      const int c_ = wave * 16 + ((I) / G) * (kWaves * 16) + (lane & 15);            \
      const double cn_ = cnS[c_];                                                    \
      const double cq_ = (cn_ * cn_) * (1.0 - fac2);                                 \
      const bool cok_ = c_ < k;                                                      \
      _Pragma("unroll") for (int t = 0; t < T; ++t) {                                \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                              \
          const int q = 4 * t + r;                                                   \
          const double xq = xqS[t * 16 + (lane >> 4) + 4 * r];                       \
          const double L = (xq + cq_) - (acc[t][r] + acc[t][r]);                      \
          poison |= (cok_ && !(L == L)) ? (1u << q) : 0u;                            \
          const float fL = (float)L;   /* f32 rounding mode is toward -inf here */   \
          const bool lt = cok_ && fL < sL1[q];                                       \
          const float l2 = cok_ ? fminf(sL2[q], fL) : sL2[q];                        \
          sL2[q] = lt ? sL1[q] : l2;                                                 \
          sI1[q] = lt ? c_ : sI1[q];                                                 \
          sL1[q] = lt ? fL : sL1[q];                                                 \
        }                                                                            \
      }                                                                              \
    }                                                                                \
  } while (0)
  // MODE.FP_ROUND single-precision bits [1:0] = 2 (toward -inf): every
  // (float) conversion of a lower bound in the loop rounds down.
  __builtin_amdgcn_s_setreg(0x801, 2);
  if (total > 0) CYC_LOADB(b0, 0);
  for (int i = 0; i < total; i += 2) {
    if (i + 1 < total) CYC_LOADB(b1, i + 1);
    CYC_COMPUTE(b0, i);
    if (i + 2 < total) CYC_LOADB(b0, i + 2);
    if (i + 1 < total) CYC_COMPUTE(b1, i + 1);
  }
  __builtin_amdgcn_s_setreg(0x801, 0);   // back to round-to-nearest-even
#undef CYC_LOADB
#undef CYC_COMPUTE

  // Reduce each slot over the 16 lanes that hold the same row.
#pragma unroll
  for (int q = 0; q < T * 4; ++q) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      const float oL1 = __shfl_xor(sL1[q], m), oL2 = __shfl_xor(sL2[q], m);
      const int oI1 = __shfl_xor(sI1[q], m);
      const float hi = fmaxf(sL1[q], oL1);
      sL2[q] = fminf(hi, fminf(sL2[q], oL2));
      const bool take = oL1 < sL1[q] || (oL1 == sL1[q] && oI1 >= 0 && (sI1[q] < 0 || oI1 < sI1[q]));
      sI1[q] = take ? oI1 : sI1[q];
      sL1[q] = take ? oL1 : sL1[q];
    }
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) poison |= __shfl_xor(poison, m);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = 4 * t + r;
        double* m = mrg + ((size_t)wave * BM + t * 16 + (lane >> 4) + 4 * r) * 4;
        m[0] = sL1[q];
        m[1] = ((poison >> q) & 1u) ? -__builtin_inf() : (double)sL2[q];
        m[2] = (double)sI1[q];
      }
    }
  }
  __syncthreads();

  if (tid < rows) {
    const int row = tid;
    float L1 = __builtin_inff(), L2 = __builtin_inff();
    int I1 = -1;
    for (int w = 0; w < kWaves; ++w) {
      const double* m = mrg + ((size_t)w * BM + row) * 4;
      const float oL1 = (float)m[0], oL2 = (float)m[1];
      const int oI1 = (int)m[2];
      const float hi = fmaxf(L1, oL1);
      L2 = fminf(hi, fminf(L2, oL2));
      if (oL1 < L1 || (oL1 == L1 && oI1 >= 0 && (I1 < 0 || oI1 < I1))) {
        L1 = oL1;
        I1 = oI1;
      }
    }
    const int64_t grow = CYC_GROW(row);
    bool decided = false;
    if (I1 >= 0 && L1 == L1 && L1 < __builtin_inff()) {
      const double xn = xnS[row], cn = cnS[I1];
      const double M = (xn * xn + cn * cn) * fac2;
      const double U = (double)(-ulp_down(-L1)) + 2.0 * M * (1.0 + 0x1p-40);
      decided = (double)L2 > U;
    }
    if (decided) {
      if (cost) {
        const double* crow = C + (int64_t)I1 * d;
        const double* xrow = Xs + row * ldsStride;
        double s = 0.0;
        for (int j = 0; j < d; ++j) {
          double sc = dsub(crow[j], xrow[j]);
          s = dadd(s, dmul(sc, sc));
        }
        cost[grow] = s;
      }
      assign[grow] = I1;
    } else {
      unsigned slot = atomicAdd(slowCount, 1u);
      slowList[slot] = (int32_t)grow;
    }
  }
  __syncthreads();   // LDS is restaged by the next tile
  }
#undef CYC_GROW
}

// ---------------------------------------------------- bf16x3 screen (tier 1)
// Third-generation assign (the default where it fits): the screen's dot
// products x.c run on the bf16 matrix cores instead of fp64 ones, 32x the
// MFMA rate, with a rigorous error bound; fp64 only decides.
//
// Split every value v (fp64) into v = vh + vl + ev with vh = bf16(v),
// vl = bf16(v - vh) (the subtraction is exact), |ev| <= 2^-16 |v| (1.0001).
// Then s = xh.ch + xl.ch + xh.cl (three bf16 products per element, f32
// accumulation: v_mfma_f32_16x16x32_bf16 over K = 3 d32) satisfies
//   |x.c - s| <= E = eps (|x|^2 + |c|^2) / 2 + tau,
//   eps = 3.1 * 2^-16 (split) + 2 * 1.03 * (3 d32 + 64) * 2^-23 (f32 sums of
//         up to 3 d32 terms, any faithful/directed rounding, 2x headroom)
//         + 2^-20,
// using sum|x_i||c_i| <= |x||c| <= (|x|^2 + |c|^2)/2, and tau = 2^-58 for
// bf16 / f32 underflow (values are capped at |v| <= 2^56: a row with
// |x| > 2^56 or a NaN goes to the fp64 tier, and a center beyond the cap
// turns the screen off for the launch).  Lower bound of every distance:
//   L_j = xq + cq_j - 2 s_j,  xq = |x|^2 (1 - eps) - 2 tau,  cq = |c|^2 (1 - eps),
// computed with f32 rounding toward -inf (MODE register) so it stays a lower
// bound; the best center's upper bound is L1 + (2 eps + 2^-20)(|x|^2 + |c|^2)
// + 4 tau.  A row whose second-smallest lower bound exceeds that is decided
// exactly as in the fp64 screen (k_kmeans_assign2) and gets the sequential
// fp64 sqdist; every other row is queued for the fp64 screen.
//
// Tiling: 64 rows per workgroup (4 waves, two workgroups per CU), the rows'
// bf16 hi / lo images in LDS; each wave owns every 4th 16-center tile and
// streams its centers' pre-split B fragments (1 KiB per wave-load) from L2,
// TB tiles at a time, each fragment feeding 4 row tiles.
typedef __bf16 cyc_bf16x8 __attribute__((ext_vector_type(8)));
typedef float cyc_float4 __attribute__((ext_vector_type(4)));

constexpr int kS3Waves = 4;
constexpr int kS3Threads = kS3Waves * 64;
constexpr int kS3BM = 64;

__device__ __forceinline__ void split_bf16(double v, unsigned short& h, unsigned short& l) {
  const __bf16 hb = (__bf16)(float)v;
  const double r = v - (double)(float)hb;   // exact: hb is within 2^-8 |v| of v
  const __bf16 lb = (__bf16)(float)r;
  h = __builtin_bit_cast(unsigned short, hb);
  l = __builtin_bit_cast(unsigned short, lb);
}

// Centers -> B fragments of v_mfma_f32_16x16x32_bf16 (lane l of 16-center tile
// ct, k-step ks holds centers ct*16 + (l & 15), dims ks*32 + 8 (l >> 4) + 0..7),
// hi image then lo image per (ct, ks): Cb[((ct KS + ks) 2 + part) 64 + l].
// cq[c] = |c|^2 (1 - eps) rounded down (+inf for padding); screenOk cleared if
// a center is beyond the 2^56 cap or not finite.
__global__ void k_center_split(const double* __restrict__ C, const double* __restrict__ cnorm,
                               int k, int d, int KS, int ktp, double omE, uint4* __restrict__ Cb,
                               float* __restrict__ cq, int* __restrict__ screenOk) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)ktp * KS * 64;
  if (idx < total) {
    const int lane = (int)(idx & 63);
    const int64_t t = idx >> 6;
    const int ks = (int)(t % KS), ct = (int)(t / KS);
    const int c = ct * 16 + (lane & 15), j0 = ks * 32 + 8 * (lane >> 4);
    unsigned short h[8], l[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = j0 + e;
      split_bf16((c < k && j < d) ? C[(int64_t)c * d + j] : 0.0, h[e], l[e]);
    }
    uint4 ph, pl;
    ph.x = h[0] | ((unsigned)h[1] << 16); ph.y = h[2] | ((unsigned)h[3] << 16);
    ph.z = h[4] | ((unsigned)h[5] << 16); ph.w = h[6] | ((unsigned)h[7] << 16);
    pl.x = l[0] | ((unsigned)l[1] << 16); pl.y = l[2] | ((unsigned)l[3] << 16);
    pl.z = l[4] | ((unsigned)l[5] << 16); pl.w = l[6] | ((unsigned)l[7] << 16);
    Cb[((t * 2) + 0) * 64 + lane] = ph;
    Cb[((t * 2) + 1) * 64 + lane] = pl;
  }
  if (idx < (int64_t)ktp * 16) {
    const int c = (int)idx;
    if (c < k) {
      const double cn = cnorm[c];
      if (!(cn <= 0x1p56)) atomicAnd(screenOk, 0);
      cq[c] = f_down((cn * cn) * omE);
    } else {
      cq[c] = __builtin_inff();
    }
  }
}

template <int TB>
__global__ __launch_bounds__(kS3Threads, 2) void k_kmeans_assign3(
    const double* __restrict__ X, const double* __restrict__ xnorm, int64_t n, int d, int KS,
    const uint4* __restrict__ Cb, const float* __restrict__ cq, int ktp,
    const int* __restrict__ screenOk, const double* __restrict__ C,
    const double* __restrict__ cnorm, double omE, double tauL,
    double facU, double tauU, int32_t* __restrict__ assign, double* __restrict__ cost,
    int32_t* __restrict__ list, unsigned int* __restrict__ listCount) {
  constexpr int BM = kS3BM, TA = BM / 16, W = kS3Waves;
  extern __shared__ __attribute__((aligned(16))) uint4 smem3[];
  const int SA = KS * 4 + 1;                       // 16-byte chunks per row (+1 pad)
  uint4* Ah = smem3;                               // BM x SA: bf16 hi image
  uint4* Al = Ah + BM * SA;                        // BM x SA: bf16 lo image
  float* mL1 = (float*)(Al + BM * SA);             // W x BM
  float* mL2 = mL1 + W * BM;                       // W x BM
  int* mI1 = (int*)(mL2 + W * BM);                 // W x BM
  float* xqS = (float*)(mI1 + W * BM);             // BM
  int* exI = (int*)(xqS + BM);                     // BM: decided center or -1
  double* Xd = (double*)smem3;                     // exact phase: 32 x (d + 1), over Ah/Al

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * BM;
  const int rows = (int)min<int64_t>(BM, n - row0);
  if (*screenOk == 0) {
    if (tid < rows) {
      const unsigned slot = atomicAdd(listCount, 1u);
      list[slot] = (int32_t)(row0 + tid);
    }
    return;
  }
  // Stage: one 8-element chunk per thread-step, split into the two images.
  const int chunks = KS * 4;
  for (int e = tid; e < BM * chunks; e += kS3Threads) {
    const int r = e / chunks, ch = e - r * chunks;
    const double* src = X + (row0 + r) * d;
    unsigned short h[8], l[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = ch * 8 + q;
      split_bf16((r < rows && j < d) ? src[j] : 0.0, h[q], l[q]);
    }
    uint4 ph, pl;
    ph.x = h[0] | ((unsigned)h[1] << 16); ph.y = h[2] | ((unsigned)h[3] << 16);
    ph.z = h[4] | ((unsigned)h[5] << 16); ph.w = h[6] | ((unsigned)h[7] << 16);
    pl.x = l[0] | ((unsigned)l[1] << 16); pl.y = l[2] | ((unsigned)l[3] << 16);
    pl.z = l[4] | ((unsigned)l[5] << 16); pl.w = l[6] | ((unsigned)l[7] << 16);
    Ah[r * SA + ch] = ph;
    Al[r * SA + ch] = pl;
  }
  if (tid < BM) {
    const double xn = tid < rows ? xnorm[row0 + tid] : 0.0;
    xqS[tid] = (xn <= 0x1p56) ? f_down((xn * xn) * omE - tauL) : -__builtin_inff();
  }
  __syncthreads();

  float sL1[TA * 4], sL2[TA * 4];
  int sI1[TA * 4];
#pragma unroll
  for (int q = 0; q < TA * 4; ++q) {
    sL1[q] = sL2[q] = __builtin_inff();
    sI1[q] = -1;
  }
  const uint4* ah = Ah + (lane & 15) * SA + (lane >> 4);
  const uint4* al = Al + (lane & 15) * SA + (lane >> 4);
  const int groups = ktp / (W * TB);
  const int total = groups * KS;
  cyc_float4 acc[TA][TB];
  uint4 bh0[TB], bl0[TB], bh1[TB], bl1[TB];
  float cqv[TB];

  // tile tb of group g of this wave: ct = (g TB + tb) W + wave
#define CYC_LOADB3(BH, BL, I)                                                        \
  do {                                                                               \
    const int g_ = (I) / KS, ks_ = (I) - g_ * KS;                                    \
    _Pragma("unroll") for (int tb = 0; tb < TB; ++tb) {                              \
      const int ct_ = (g_ * TB + tb) * W + wave;                                     \
      const uint4* p_ = Cb + ((size_t)(ct_ * KS + ks_) * 2) * 64 + lane;             \
      BH[tb] = p_[0];                                                                \
      BL[tb] = p_[64];                                                               \
    }                                                                                \
  } while (0)
#define CYC_COMPUTE3(BH, BL, I)                                                      \
  do {                                                                               \
    const int g_ = (I) / KS, ks_ = (I) - g_ * KS;                                    \
    if (ks_ == 0) {                                                                  \
      _Pragma("unroll") for (int tb = 0; tb < TB; ++tb) {                            \
        cqv[tb] = cq[((g_ * TB + tb) * W + wave) * 16 + (lane & 15)];                \
        _Pragma("unroll") for (int ta = 0; ta < TA; ++ta)                            \
          acc[ta][tb] = cyc_float4{0.f, 0.f, 0.f, 0.f};                              \
      }                                                                              \
    }                                                                                \
    _Pragma("unroll") for (int ta = 0; ta < TA; ++ta) {                              \
      const cyc_bf16x8 xh_ = __builtin_bit_cast(cyc_bf16x8, ah[ta * 16 * SA + ks_ * 4]); \
      const cyc_bf16x8 xl_ = __builtin_bit_cast(cyc_bf16x8, al[ta * 16 * SA + ks_ * 4]); \
      _Pragma("unroll") for (int tb = 0; tb < TB; ++tb) {                            \
        const cyc_bf16x8 ch_ = __builtin_bit_cast(cyc_bf16x8, BH[tb]);               \
        const cyc_bf16x8 cl_ = __builtin_bit_cast(cyc_bf16x8, BL[tb]);               \
        acc[ta][tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh_, ch_, acc[ta][tb], 0, 0, 0); \
        acc[ta][tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xl_, ch_, acc[ta][tb], 0, 0, 0); \
        acc[ta][tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xh_, cl_, acc[ta][tb], 0, 0, 0); \
      }                                                                              \
    }                                                                                \
    if (ks_ == KS - 1) {                                                             \
      _Pragma("unroll") for (int tb = 0; tb < TB; ++tb) {                            \
        const int c_ = ((g_ * TB + tb) * W + wave) * 16 + (lane & 15);               \
        _Pragma("unroll") for (int ta = 0; ta < TA; ++ta) {                          \
          _Pragma("unroll") for (int r = 0; r < 4; ++r) {                            \
            const int q = 4 * ta + r;                                                \
            const float L = (xqS[ta * 16 + 4 * (lane >> 4) + r] + cqv[tb]) -         \
                            2.0f * acc[ta][tb][r];                                   \
            const bool lt = L < sL1[q];                                              \
            const float l2 = fminf(sL2[q], L);                                       \
            sL2[q] = lt ? sL1[q] : l2;                                               \
            sI1[q] = lt ? c_ : sI1[q];                                               \
            sL1[q] = lt ? L : sL1[q];                                                \
          }                                                                          \
        }                                                                            \
      }                                                                              \
    }                                                                                \
  } while (0)
  // MODE.FP_ROUND single-precision bits [1:0] = 2 (toward -inf) for the
  // bounds (and the f32 accumulation, which the error bound allows).
  __builtin_amdgcn_s_setreg(0x801, 2);
  if (total > 0) CYC_LOADB3(bh0, bl0, 0);
  for (int i = 0; i < total; i += 2) {
    if (i + 1 < total) CYC_LOADB3(bh1, bl1, i + 1);
    CYC_COMPUTE3(bh0, bl0, i);
    if (i + 2 < total) CYC_LOADB3(bh0, bl0, i + 2);
    if (i + 1 < total) CYC_COMPUTE3(bh1, bl1, i + 1);
  }
  __builtin_amdgcn_s_setreg(0x801, 0);
#undef CYC_LOADB3
#undef CYC_COMPUTE3

  // Reduce each slot over the 16 lanes (columns) that hold the same row.
#pragma unroll
  for (int q = 0; q < TA * 4; ++q) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      const float oL1 = __shfl_xor(sL1[q], m), oL2 = __shfl_xor(sL2[q], m);
      const int oI1 = __shfl_xor(sI1[q], m);
      const float hi = fmaxf(sL1[q], oL1);
      sL2[q] = fminf(hi, fminf(sL2[q], oL2));
      const bool take = oL1 < sL1[q] || (oL1 == sL1[q] && oI1 >= 0 && (sI1[q] < 0 || oI1 < sI1[q]));
      sI1[q] = take ? oI1 : sI1[q];
      sL1[q] = take ? oL1 : sL1[q];
    }
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int ta = 0; ta < TA; ++ta) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = 4 * ta + r, row = ta * 16 + 4 * (lane >> 4) + r;
        mL1[wave * BM + row] = sL1[q];
        mL2[wave * BM + row] = sL2[q];
        mI1[wave * BM + row] = sI1[q];
      }
    }
  }
  __syncthreads();
  if (tid < BM) {
    const int row = tid;
    float L1 = __builtin_inff(), L2 = __builtin_inff();
    int I1 = -1;
    for (int w = 0; w < W; ++w) {
      const float oL1 = mL1[w * BM + row], oL2 = mL2[w * BM + row];
      const int oI1 = mI1[w * BM + row];
      const float hi = fmaxf(L1, oL1);
      L2 = fminf(hi, fminf(L2, oL2));
      if (oL1 < L1 || (oL1 == L1 && oI1 >= 0 && (I1 < 0 || oI1 < I1))) {
        L1 = oL1;
        I1 = oI1;
      }
    }
    bool decided = false;
    if (row < rows && I1 >= 0 && L1 > -__builtin_inff() && L1 < __builtin_inff()) {
      const double xn = xnorm[row0 + row], cn = cnorm[I1];
      const double U = (double)L1 + facU * (xn * xn + cn * cn) + tauU;
      decided = (double)L2 > U;
    }
    exI[row] = -1;
    if (row < rows) {
      if (decided) {
        exI[row] = I1;
      } else {
        const unsigned slot = atomicAdd(listCount, 1u);
        list[slot] = (int32_t)(row0 + row);
      }
    }
  }
  __syncthreads();
  if (!cost) {
    if (tid < rows && exI[tid] >= 0) assign[row0 + tid] = exI[tid];
    return;
  }
  // Exact phase: the decided rows' sequential fp64 sqdist, 32 rows at a time
  // staged (coalesced, second read of the tile, from L2 / MALL) over the
  // images' LDS.
  for (int half = 0; half < BM / 32; ++half) {
    const int r0 = half * 32, nr = min(32, rows - r0);
    if (nr <= 0) break;
    for (int e = tid; e < nr * d; e += kS3Threads) {
      const int r = e / d, c = e - r * d;
      Xd[r * (d + 1) + c] = X[(row0 + r0 + r) * d + c];
    }
    __syncthreads();
    if (tid < nr && exI[r0 + tid] >= 0) {
      const int I1 = exI[r0 + tid];
      const double* crow = C + (int64_t)I1 * d;
      const double* xrow = Xd + tid * (d + 1);
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        const double sc = dsub(crow[j], xrow[j]);
        s = dadd(s, dmul(sc, sc));
      }
      assign[row0 + r0 + tid] = I1;
      cost[row0 + r0 + tid] = s;
    }
    __syncthreads();
  }
}

// The exact tier for a short queue (<= kExactCap rows, the usual few): the
// distances of one row to all k centers spread over ceil(k / 256)
// workgroups -- one thread per center, the same sequential sqdist as
// k_assign_exact -- into dist (kExactCap x kpad), then one wave per row
// replays the reference loop over them (k_exact_replay).  One workgroup per
// row streamed all k centers' coordinates through a single CU (~2 MB at
// k = 1024, d = 256: ~80 us for one row); spread over workgroups the queue
// finishes in a few microseconds.  A longer queue takes k_assign_exact.
constexpr int kExactCap = 512;

__global__ __launch_bounds__(256) void k_exact_dist(const double* __restrict__ X, int d,
                                                    const double* __restrict__ Ct, int kpad, int k,
                                                    const int32_t* __restrict__ slowList,
                                                    const unsigned int* __restrict__ slowCount,
                                                    double* __restrict__ dist) {
  __shared__ double xs[1280];
  const unsigned cnt = *slowCount;
  const unsigned idx = blockIdx.y;
  if (cnt > (unsigned)kExactCap || idx >= cnt) return;
  const int tid = threadIdx.x;
  const int c = blockIdx.x * 256 + tid;
  const int64_t r = slowList[idx];
  const double* x = X + r * d;
  const bool xl = d <= 1280;
  if (xl)
    for (int j = tid; j < d; j += 256) xs[j] = x[j];
  __syncthreads();
  const double* xv = xl ? xs : x;
  double acc = 0.0;
  // 16 dimensions' loads out before their adds (the adds are sequential)
  for (int j0 = 0; j0 < d; j0 += 16) {
    double cv[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj)
      cv[jj] = (j0 + jj < d && c < k) ? Ct[(int64_t)(j0 + jj) * kpad + c] : 0.0;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      if (j0 + jj < d) {
        const double sc = dsub(cv[jj], xv[j0 + jj]);
        acc = dadd(acc, dmul(sc, sc));
      }
    }
  }
  if (c < k) dist[(int64_t)idx * kpad + c] = acc;
}

__global__ __launch_bounds__(64) void k_exact_replay(const double* __restrict__ X,
                                                     const double* __restrict__ xnorm, int d,
                                                     int kpad, const double* __restrict__ cnorm,
                                                     int k, const double* __restrict__ stats,
                                                     const int32_t* __restrict__ slowList,
                                                     const unsigned int* __restrict__ slowCount,
                                                     const double* __restrict__ dist,
                                                     int32_t* __restrict__ assign,
                                                     double* __restrict__ cost, int exactNorm) {
  const unsigned cnt = *slowCount;
  const unsigned idx = blockIdx.x;
  if (cnt > (unsigned)kExactCap || idx >= cnt) return;
  const int lane = threadIdx.x;
  const int64_t r = slowList[idx];
  const bool ns = stats == nullptr;
  // the reference's Vectors.norm in index order when the caller's norms are
  // the row image's (k_assign_exact)
  double xn = 0.0;
  if (exactNorm) {
    if (lane == 0) xn = seq_norm2(X + r * d, d);
    xn = __shfl(xn, 0);
  } else {
    xn = xnorm[r];
  }
  const double* dds = dist + (int64_t)idx * kpad;
  double best = __builtin_inf();
  int bi = 0;
  bool done = false;
  int first = 0;
  if (!ns) {
    best = dds[0];                      // :286
    done = best < stats[0];             // :287
    first = 1;
  }
  for (int i0 = first; !done && i0 < k; i0 += 64) {
    const int i = i0 + lane;
    const bool valid = i < k;
    double lb = __builtin_inf(), sii = 0.0, dd = 0.0;
    if (valid) {
      const double nd = dsub(cnorm[i], xn);     // :294-295
      lb = dmul(nd, nd);
      sii = ns ? 0.0 : stats[iut(i, i)];
      dd = dds[i];
    }
    int pos = 0;
    for (;;) {
      const bool visit = valid && lane >= pos && lb < best && (ns || stats[iut(i, bi)] < best);
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

// EuclideanDistanceMeasure.findClosest with statistics, DistanceMeasure.scala:
// 282-313, for the rows the screens could not decide.  One workgroup per
// queued row: the exact sequential sqdist (Vectors.scala:580-587, the same
// operation order as the reference) of every center, 1024 at a time, then
// the replay on one wave.  The reference loop visits centers in order; its
// state (bestDistance, bestIndex) changes only at an update, so the wave
// evaluates 64 consecutive centers at once against the current state: a
// ballot over the lanes whose center the loop would visit finds the first lane
// whose visit changes the state (a `return` at :303 or an update at :304-306),
// the state advances to it, and the lanes after it are re-evaluated against
// the new state (reusing the distances already computed).  Lanes before the
// first event have no side effect in the reference either, so the returned
// (index, distance) is the reference's, bit for bit; distances of centers the
// reference would not visit may be computed speculatively and are discarded.
constexpr int kExactChunk = 1024;   // centers whose distances one pass stages in LDS
constexpr int kExactX = 1280;       // widest row staged in LDS

__global__ __launch_bounds__(256) void k_assign_exact(
    const double* __restrict__ X, const double* __restrict__ xnorm, int d,
    const double* __restrict__ C, const double* __restrict__ Ct, int kpad,
    const double* __restrict__ cnorm, int k,
    const double* __restrict__ stats, const int32_t* __restrict__ slowList,
    const unsigned int* __restrict__ slowCount, int32_t* __restrict__ assign,
    double* __restrict__ cost, int exactNorm, unsigned int skipUpTo) {
  // One workgroup per listed row.  A distance is a pure function of (center,
  // row), so the workgroup first computes Vectors.sqdist(center, x) -- in
  // order j = 0..d-1 (Vectors.scala:580-587) -- for a chunk of 1024 centers
  // at once (thread t: centers t, t + 256, ..; center i read from the
  // transposed copy, coalesced over the threads), and wave 0 then replays the
  // reference loop's visits and events over them.
  __shared__ double xs[kExactX];
  __shared__ double dds[kExactChunk];
  __shared__ int doneS;
  __shared__ double xnS;
  const unsigned cnt = *slowCount;
  if (cnt <= skipUpTo) return;   // the split kernels took the queue
  const int tid = threadIdx.x, lane = tid & 63;
  // stats == nullptr: findClosest(centers, point) (:318-340), best from +inf
  const bool ns = stats == nullptr;
  for (unsigned idx = blockIdx.x; idx < cnt; idx += gridDim.x) {
    const int64_t r = slowList[idx];
    const double* x = X + r * d;
    __syncthreads();   // the previous row's reads of xs / dds / xnS are done
    const bool xl = d <= kExactX;
    if (xl)
      for (int j = tid; j < d; j += 256) xs[j] = x[j];
    const double* xv = xl ? xs : x;
    // exactNorm: the caller's norms are the row image's (any summation
    // order, for the screens' margins); the loop's prune needs the
    // reference's Vectors.norm, in index order (seq_norm2)
    if (exactNorm) {
      __syncthreads();
      if (tid == 0) xnS = seq_norm2(xv, d);
      __syncthreads();
    }
    const double xn = exactNorm ? xnS : xnorm[r];
    double best = __builtin_inf();   // wave 0's replay state
    int bi = 0;
    bool done = false;
    for (int c0 = 0; c0 < k; c0 += kExactChunk) {
      __syncthreads();   // xs written; the previous chunk's replay is done
      double acc[kExactChunk / 256];
#pragma unroll
      for (int u = 0; u < kExactChunk / 256; ++u) acc[u] = 0.0;
      // 16 dimensions' loads go out before their adds (the add chains are
      // sequential; the loads are not)
      for (int j0 = 0; j0 < d; j0 += 16) {
        double cv[16][kExactChunk / 256];
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          const double* row = Ct + (int64_t)(j0 + jj) * kpad + c0 + tid;
#pragma unroll
          for (int u = 0; u < kExactChunk / 256; ++u)
            cv[jj][u] = (j0 + jj < d && c0 + tid + 256 * u < k) ? row[256 * u] : 0.0;
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          if (j0 + jj < d) {
            const double xj = xv[j0 + jj];
#pragma unroll
            for (int u = 0; u < kExactChunk / 256; ++u) {
              const double sc = dsub(cv[jj][u], xj);
              acc[u] = dadd(acc[u], dmul(sc, sc));
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kExactChunk / 256; ++u)
        if (c0 + tid + 256 * u < k) dds[tid + 256 * u] = acc[u];
      __syncthreads();
      if (tid < 64) {
        int first = c0;
        if (c0 == 0 && !ns) {
          best = dds[0];                      // :286
          done = best < stats[0];             // :287
          first = 1;
        }
        const int end = min(k, c0 + kExactChunk);
        for (int i0 = first; !done && i0 < end; i0 += 64) {
          const int i = i0 + lane;
          const bool valid = i < end;
          double lb = __builtin_inf(), sii = 0.0, dd = 0.0;
          if (valid) {
            const double nd = dsub(cnorm[i], xn);     // :294-295
            lb = dmul(nd, nd);
            sii = ns ? 0.0 : stats[iut(i, i)];
            dd = dds[i - c0];
          }
          int pos = 0;
          for (;;) {
            const bool visit = valid && lane >= pos && lb < best && (ns || stats[iut(i, bi)] < best);
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
        if (tid == 0) doneS = done;
      }
      __syncthreads();
      if (doneS) break;
    }
    if (tid == 0) {
      assign[r] = bi;
      if (cost) cost[r] = best;
    }
  }
}

// pointCost of a row no center reaches (NaN/Inf coordinates): findClosest
// without statistics keeps bestDistance = +Infinity (:321-337), while the
// recomputed sqdist to center 0 is NaN or +Infinity.
__global__ void k_nostats_cost_fix(int64_t n, double* __restrict__ cost) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n && __builtin_isnan(cost[r])) cost[r] = __builtin_inf();
}

// MLUtils.fastSquaredDistance's require(norm1 >= 0.0 && norm2 >= 0.0,
// "Both norms should be greater or equal to 0.0, ...") (mllib/util/
// MLUtils.scala:542-543), as a with-statistics Lloyd step meets it:
// computeStatistics (DistanceMeasure.scala:48-76) measures every center pair,
// so a center with a NaN norm fails (k >= 2), and findClosest (:282-287)
// measures (center 0, point) first for every point.  Other centers are only
// measured behind `lowerBound < bestDistance` (:295-297), which a NaN norm
// never passes; findClosest WITHOUT statistics (:318-340) therefore never
// fails.  A norm is NaN iff the vector holds a NaN (Vectors.scala:500-507).
// req[0]: lowest center holding a NaN, req[1]: lowest row with a NaN norm
// (~0 when none; set by the caller); req[2..4] as doubles: norm(c0),
// norm(c1), xnorm[0] -- the values the reference's message interpolates.
__global__ void k_require_norms(const double* __restrict__ C, int k, int d,
                                const double* __restrict__ xnorm, int64_t n,
                                unsigned long long* __restrict__ req) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t kd = (int64_t)k * d;
  for (int64_t i = t0; i < kd; i += stride)
    if (__builtin_isnan(C[i])) atomicMin(&req[0], (unsigned long long)(i / d));
  for (int64_t r = t0; r < n; r += stride)
    if (__builtin_isnan(xnorm[r])) atomicMin(&req[1], (unsigned long long)r);
  double* out = reinterpret_cast<double*>(req + 2);
  if (t0 < 2 && t0 < k) out[t0] = seq_norm2(C + t0 * d, d);
  if (t0 == 2) out[2] = n > 0 ? xnorm[0] : 0.0;
}

// ------------------------------------------------------- counting sort
__global__ void k_hist(const int32_t* __restrict__ assign, int64_t n, int k,
                       int32_t* __restrict__ hist, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  extern __shared__ int32_t cnt[];
  for (int c = threadIdx.x; c < k; c += blockDim.x) cnt[c] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kSortTile;
  const int64_t r1 = min<int64_t>(n, r0 + kSortTile);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) atomicAdd(&cnt[assign[r]], 1);
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += blockDim.x) hist[(int64_t)blockIdx.x * k + c] = cnt[c];
}

// Per cluster: exclusive running offset over the tiles (in place) and the
// total, as a segmented scan (integer sums: any grouping gives the same
// offsets).  1. per (tile segment, cluster) sums; 2. per cluster, the
// segments' exclusive offsets and the total; 3. the offsets inside segments.
constexpr int kScanSegs = 64;

__global__ void k_scan_seg(const int32_t* __restrict__ hist, int tiles, int k, int segT,
                           int32_t* __restrict__ segsum, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  const int c = blockIdx.x * 64 + threadIdx.x, s = blockIdx.y;
  if (c >= k) return;
  const int t0 = s * segT, t1 = min(tiles, t0 + segT);
  int sum = 0;
#pragma unroll 8
  for (int t = t0; t < t1; ++t) sum += hist[(int64_t)t * k + c];
  segsum[(int64_t)s * k + c] = sum;
}

__global__ void k_scan_segoff(int32_t* __restrict__ segsum, int segs, int k,
                              int64_t* __restrict__ total, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= k) return;
  int64_t run = 0;
  for (int s = 0; s < segs; ++s) {
    const int32_t h = segsum[(int64_t)s * k + c];
    segsum[(int64_t)s * k + c] = (int32_t)run;
    run += h;
  }
  total[c] = run;
}

__global__ void k_scan_apply(int32_t* __restrict__ hist, int tiles, int k, int segT,
                             const int32_t* __restrict__ segoff, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  const int c = blockIdx.x * 64 + threadIdx.x, s = blockIdx.y;
  if (c >= k) return;
  const int t0 = s * segT, t1 = min(tiles, t0 + segT);
  int32_t run = segoff[(int64_t)s * k + c];
  for (int t = t0; t < t1; ++t) {
    const int32_t h = hist[(int64_t)t * k + c];
    hist[(int64_t)t * k + c] = run;
    run += h;
  }
}

// Single block: cluster start offsets and chunk start offsets (exclusive scans).
__global__ void k_scan_clusters(const int64_t* __restrict__ total, int k,
                                int64_t* __restrict__ cstart, int64_t* __restrict__ chunkStart,
                                const int* __restrict__ gate) {
  if (gate && !*gate) return;
  __shared__ int64_t s_rows[1024], s_chunks[1024];
  const int tid = threadIdx.x;
  const int per = (k + 1023) / 1024;
  int64_t rows = 0, chunks = 0;
  for (int q = 0; q < per; ++q) {
    int c = tid * per + q;
    if (c < k) {
      rows += total[c];
      chunks += (total[c] + kChunkRows - 1) / kChunkRows;
    }
  }
  s_rows[tid] = rows;
  s_chunks[tid] = chunks;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int64_t a = tid >= off ? s_rows[tid - off] : 0, b = tid >= off ? s_chunks[tid - off] : 0;
    __syncthreads();
    s_rows[tid] += a;
    s_chunks[tid] += b;
    __syncthreads();
  }
  int64_t rbase = tid ? s_rows[tid - 1] : 0, cbase = tid ? s_chunks[tid - 1] : 0;
  for (int q = 0; q < per; ++q) {
    int c = tid * per + q;
    if (c < k) {
      cstart[c] = rbase;
      chunkStart[c] = cbase;
      rbase += total[c];
      cbase += (total[c] + kChunkRows - 1) / kChunkRows;
    }
  }
  if (tid == 1023) {
    cstart[k] = s_rows[1023];
    chunkStart[k] = s_chunks[1023];
  }
}

// One wave per tile, rows in order: perm[cstart[c] + tileOffset[c] + rank] = row.
// Tiles by XCD: block b runs on XCD b % 8 and takes tile (b % 8) * per +
// b / 8, so each XCD walks a contiguous range of tiles.  A cluster's rows
// from consecutive tiles land side by side in perm; with consecutive tiles
// on one XCD their 4-byte writes meet in that XCD's L2 instead of partial
// lines from eight L2s (the grid is 8 * per blocks; the spare ones leave).
__global__ void k_scatter(const int32_t* __restrict__ assign, int64_t n, int k,
                          const int32_t* __restrict__ tileOff, const int64_t* __restrict__ cstart,
                          int32_t* __restrict__ perm, int64_t tiles, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  extern __shared__ int64_t pos[];
  const int64_t per = ((int64_t)gridDim.x + 7) / 8;
  const int64_t tile = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (tile >= tiles) return;
  const int lane = threadIdx.x;
  const int kb = 32 - __builtin_clz((unsigned)max(k - 1, 1));   // bits of a cluster index
  for (int c = lane; c < k; c += 64) pos[c] = cstart[c] + tileOff[tile * k + c];
  __syncthreads();
  const int64_t r0 = tile * kSortTile;
  const int64_t r1 = min<int64_t>(n, r0 + kSortTile);
  // the tile's assignments loaded up front (one latency, not one per 64
  // rows: 124 -> ~30 us at 10M rows), then the stable in-order walk
  constexpr int PER = kSortTile / 64;
  int cv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int64_t r = r0 + i * 64 + lane;
    cv[i] = (r < r1) ? assign[r] : -1;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int64_t r = r0 + i * 64 + lane;
    const int c = cv[i];
    // the lanes holding the same cluster: one ballot per bit of the index
    unsigned long long m = __ballot(c >= 0);
    for (int b = 0; b < kb; ++b) {
      const bool bit = (c >> b) & 1;
      const unsigned long long bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
    const int prior = __popcll(m & ((1ull << lane) - 1));
    const int last = 63 - __clzll(m);
    int64_t p = (c >= 0) ? pos[c] + prior : 0;
    __builtin_amdgcn_wave_barrier();
    if (c >= 0) {
      perm[p] = (int32_t)r;
      if (last == lane) pos[c] = p + 1;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Partial sums of up to kChunkRows rows of one cluster, rows in index order
// (updateClusterSum, DistanceMeasure.scala:189-191: axpy(w, x, sum)), their
// weights, and each row's cost = fastSquaredDistance(center, row) = the
// sequential Vectors.sqdist (Vectors.scala:580-587) that findClosest returns
// for the chosen center, summed as w * cost (KMeans.scala:302) in row order.
// The cost is fused here because the rows are read anyway: thread j holds
// dims j, j+256, ... (NJ of them) and writes (c_j - x_j)^2 of G rows to LDS;
// G threads then run the G sequential sums.  costOut (may be NULL) receives
// the per-row costs.
template <int NJ>
__global__ __launch_bounds__(256) void k_chunk_sums(
    const double* __restrict__ X, int d, const double* __restrict__ w,
    const double* __restrict__ C, const int32_t* __restrict__ perm,
    const int64_t* __restrict__ cstart, const int64_t* __restrict__ chunkStart, int k,
    double* __restrict__ part, double* __restrict__ pw, double* __restrict__ pc,
    double* __restrict__ costOut) {
  constexpr int G = 16;
  __shared__ double sq[G * (NJ * 256 + 1)];
  __shared__ double rcost[G];
  const int64_t ch = blockIdx.x;
  if (ch >= chunkStart[k]) return;
  int lo = 0, hi = k;   // cluster = last c with chunkStart[c] <= ch
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunkStart[mid] <= ch) lo = mid; else hi = mid;
  }
  const int c = lo;
  const int64_t first = cstart[c] + (ch - chunkStart[c]) * kChunkRows;
  const int64_t last = min<int64_t>(cstart[c + 1], first + kChunkRows);
  const int tid = threadIdx.x;
  constexpr int SQS = NJ * 256 + 1;
  double s[NJ], cj[NJ];
#pragma unroll
  for (int q = 0; q < NJ; ++q) {
    const int j = tid + 256 * q;
    s[q] = 0.0;
    cj[q] = j < d ? C[(int64_t)c * d + j] : 0.0;
  }
  double sw = 0.0, sc = 0.0;
  for (int64_t g0 = first; g0 < last; g0 += G) {
    const int gn = (int)min<int64_t>(G, last - g0);
    for (int pp = 0; pp < gn; ++pp) {
      const int64_t r = perm[g0 + pp];
      const double wr = w ? w[r] : 1.0;
#pragma unroll
      for (int q = 0; q < NJ; ++q) {
        const int j = tid + 256 * q;
        if (j < d) {
          const double x = X[r * d + j];
          s[q] = w ? dadd(s[q], dmul(wr, x)) : dadd(s[q], x);
          const double df = dsub(cj[q], x);
          sq[pp * SQS + j] = dmul(df, df);
        }
      }
    }
    __syncthreads();
    if (tid < gn) {
      double t = 0.0;
      for (int j = 0; j < d; ++j) t = dadd(t, sq[tid * SQS + j]);
      rcost[tid] = t;
      if (costOut) costOut[perm[g0 + tid]] = t;
    }
    __syncthreads();
    if (tid == 0) {
      for (int pp = 0; pp < gn; ++pp) {
        const double wt = w ? w[perm[g0 + pp]] : 1.0;
        sw = dadd(sw, wt);
        sc = dadd(sc, dmul(rcost[pp], wt));
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NJ; ++q) {
    const int j = tid + 256 * q;
    if (j < d) part[ch * d + j] = s[q];
  }
  if (tid == 0) {
    pw[ch] = sw;
    pc[ch] = sc;
  }
}

// The Lloyd path when no per-row costs are requested: thread j accumulates
// both sum_r w x_rj and sum_r w (c_j - x_rj)^2 over the chunk's rows, and the
// chunk's cost is one fixed-order block reduction of the latter.  The cost
// total then differs from summing the rows' sequential sqdist values only
// in rounding order (all terms positive, ~1e-16 relative; the bar is 1e-10),
// and the pass is a plain HBM stream: 8 rows' loads in flight per thread.
template <int NJ>
__global__ __launch_bounds__(256) void k_chunk_sums_fast(
    const double* __restrict__ X, int d, const double* __restrict__ w,
    const double* __restrict__ C, const int32_t* __restrict__ perm,
    const int64_t* __restrict__ cstart, const int64_t* __restrict__ chunkStart, int k,
    double* __restrict__ part, double* __restrict__ pw, double* __restrict__ pc,
    const double* __restrict__ xnorm, double* __restrict__ pa, const int* __restrict__ gate) {
  __shared__ int32_t rowsS[kChunkRows];
  __shared__ double red[256], reda[256];
  if (gate && !*gate) return;
  const int64_t ch = blockIdx.x;
  if (ch >= chunkStart[k]) return;
  int lo = 0, hi = k;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunkStart[mid] <= ch) lo = mid; else hi = mid;
  }
  const int c = lo;
  const int64_t first = cstart[c] + (ch - chunkStart[c]) * kChunkRows;
  const int cnt = (int)(min<int64_t>(cstart[c + 1], first + kChunkRows) - first);
  const int tid = threadIdx.x;
  for (int i = tid; i < cnt; i += 256) rowsS[i] = perm[first + i];
  __syncthreads();
  double s[NJ], q[NJ], cj[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    s[u] = q[u] = 0.0;
    cj[u] = j < d ? C[(int64_t)c * d + j] : 0.0;
  }
  for (int p0 = 0; p0 < cnt; p0 += 8) {
    double xv[8][NJ];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int64_t r = rowsS[min(p0 + v, cnt - 1)];
#pragma unroll
      for (int u = 0; u < NJ; ++u) {
        const int j = tid + 256 * u;
        // nontemporal: the rows are read once per iteration
        xv[v][u] = j < d ? __builtin_nontemporal_load(&X[r * d + j]) : 0.0;
      }
    }
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      if (p0 + v < cnt) {
        const double wr = w ? w[rowsS[p0 + v]] : 1.0;
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
          const double x = xv[v][u];
          const double df = dsub(cj[u], x);
          if (w) {
            s[u] = dadd(s[u], dmul(wr, x));
            q[u] = dadd(q[u], dmul(wr, dmul(df, df)));
          } else {
            s[u] = dadd(s[u], x);
            q[u] = dadd(q[u], dmul(df, df));
          }
        }
      }
    }
  }
  double qt = 0.0;
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    if (j < d) part[ch * d + j] = s[u];
    qt = dadd(qt, q[u]);
  }
  red[tid] = qt;
  // pa (incremental sums' error scale): the chunk's sum of w |x| (wave-order
  // norms are enough, it only sizes a bound)
  if (pa) reda[tid] = tid < cnt ? (w ? dmul(w[rowsS[tid]], xnorm[rowsS[tid]]) : xnorm[rowsS[tid]])
                                : 0.0;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      red[tid] = dadd(red[tid], red[tid + off]);
      if (pa) reda[tid] = dadd(reda[tid], reda[tid + off]);
    }
    __syncthreads();
  }
  if (tid == 0) {
    double sw = 0.0;
    if (w) {
      for (int i = 0; i < cnt; ++i) sw = dadd(sw, w[rowsS[i]]);
    } else {
      sw = (double)cnt;
    }
    pw[ch] = sw;
    pc[ch] = red[0];
    if (pa) pa[ch] = reda[0];
  }
}

// Same without the fused cost (d > 1024): costs come from k_row_cost.
__global__ void k_chunk_sums_nocost(const double* __restrict__ X, int d,
                                    const double* __restrict__ w,
                                    const double* __restrict__ cost,
                                    const int32_t* __restrict__ perm,
                                    const int64_t* __restrict__ cstart,
                                    const int64_t* __restrict__ chunkStart, int k,
                                    double* __restrict__ part, double* __restrict__ pw,
                                    double* __restrict__ pc) {
  const int64_t ch = blockIdx.x;
  if (ch >= chunkStart[k]) return;
  int lo = 0, hi = k;
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (chunkStart[mid] <= ch) lo = mid; else hi = mid;
  }
  const int c = lo;
  const int64_t first = cstart[c] + (ch - chunkStart[c]) * kChunkRows;
  const int64_t last = min<int64_t>(cstart[c + 1], first + kChunkRows);
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    double s = 0.0;
    if (w) {
      for (int64_t p = first; p < last; ++p) {
        const int64_t r = perm[p];
        s = dadd(s, dmul(w[r], X[r * d + j]));
      }
    } else {
      for (int64_t p = first; p < last; ++p) s = dadd(s, X[(int64_t)perm[p] * d + j]);
    }
    part[ch * d + j] = s;
  }
  if (threadIdx.x == 0) {
    double sw = 0.0, sc = 0.0;
    for (int64_t p = first; p < last; ++p) {
      const int64_t r = perm[p];
      const double wt = w ? w[r] : 1.0;
      sw = dadd(sw, wt);
      sc = dadd(sc, dmul(cost[r], wt));
    }
    pw[ch] = sw;
    pc[ch] = sc;
  }
}

// cost[r] = Vectors.sqdist(C[assign[r]], X[r]) (Vectors.scala:580-587): the
// distance findClosest returns for the chosen center.  One thread per row,
// the rows staged as in k_row_norms (256 rows, 16-column slices through two
// padded LDS buffers one slice ahead); the centers (L2-resident) read per
// thread.
__global__ __launch_bounds__(kNormRows) void k_row_cost(const double* __restrict__ X, int64_t n,
                                                        int d, const double* __restrict__ C,
                                                        const int32_t* __restrict__ assign,
                                                        double* __restrict__ cost) {
  __shared__ double tile[2][kNormRows * kNormStride];
  const int t = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kNormRows;
  const int64_t myr = row0 + t;
  const double* crow = myr < n ? C + (int64_t)assign[myr] * d : C;
  constexpr int PER = kNormCols;   // loads per thread per slice
  double v[PER];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = t + kNormRows * i, r = e / kNormCols, c = c0 + e % kNormCols;
      const int64_t gr = row0 + r;
      v[i] = (gr < n && c < d) ? __builtin_nontemporal_load(&X[gr * d + c]) : 0.0;
    }
  };
  auto store = [&](double* b) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = t + kNormRows * i;
      b[(e / kNormCols) * kNormStride + e % kNormCols] = v[i];
    }
  };
  double s = 0.0;
  load(0);
  store(tile[0]);
  int buf = 0;
  for (int c0 = 0; c0 < d; c0 += kNormCols) {
    if (c0 + kNormCols < d) load(c0 + kNormCols);
    __syncthreads();   // slice c0 in tile[buf]; every thread done with tile[buf ^ 1]
    const double* row = tile[buf] + t * kNormStride;
    const int lim = min(kNormCols, d - c0);
    for (int c = 0; c < lim; ++c) {
      const double df = dsub(crow[c0 + c], row[c]);
      s = dadd(s, dmul(df, df));
    }
    if (c0 + kNormCols < d) store(tile[buf ^ 1]);
    buf ^= 1;
  }
  if (myr < n) cost[myr] = s;
}

// Fold a cluster's chunks in chunk order and add into the caller's sums.
// fS / fW / fA (optional, the incremental sums' state): the cluster's own
// sums, weight and sum of w |x| (from pa) stored besides.
__global__ void k_reduce_clusters(const double* __restrict__ part, const double* __restrict__ pw,
                                  const double* __restrict__ pc,
                                  const int64_t* __restrict__ chunkStart, int d,
                                  double* __restrict__ sums, double* __restrict__ wsum,
                                  double* __restrict__ ccost, const double* __restrict__ pa,
                                  double* __restrict__ fS, double* __restrict__ fW,
                                  double* __restrict__ fA, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  const int c = blockIdx.x;
  const int64_t a = chunkStart[c], b = chunkStart[c + 1];
  if (a == b) {
    if (threadIdx.x == 0) ccost[c] = 0.0;
    if (fS) {
      for (int j = threadIdx.x; j < d; j += blockDim.x) fS[(int64_t)c * d + j] = 0.0;
      if (threadIdx.x == 0) fW[c] = fA[c] = 0.0;
    }
    return;
  }
  // chunk order kept; 16 chunks' loads in flight per step
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    double s = 0.0;
    int64_t ch = a;
    for (; ch + 16 <= b; ch += 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = part[(ch + u) * d + j];
#pragma unroll
      for (int u = 0; u < 16; ++u) s = dadd(s, v[u]);
    }
    for (; ch < b; ++ch) s = dadd(s, part[ch * d + j]);
    sums[(int64_t)c * d + j] = dadd(sums[(int64_t)c * d + j], s);
    if (fS) fS[(int64_t)c * d + j] = s;
  }
  // the weight and cost folds on two other waves (pa on a third)
  const int tw = 64 % blockDim.x, tc = 128 % blockDim.x, ta = 192 % blockDim.x;
  if (fS && threadIdx.x == ta && ta != tw && ta != tc) {
    double s = 0.0;
    for (int64_t ch = a; ch < b; ++ch) s = dadd(s, pa[ch]);
    fA[c] = s;
  }
  if (threadIdx.x == tw || threadIdx.x == tc) {
    const double* src = threadIdx.x == tw ? pw : pc;
    double s = 0.0;
    int64_t ch = a;
    for (; ch + 8 <= b; ch += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[ch + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) s = dadd(s, v[u]);
    }
    for (; ch < b; ++ch) s = dadd(s, src[ch]);
    if (threadIdx.x == tw) {
      wsum[c] = dadd(wsum[c], s);
      if (fS) fW[c] = s;
    } else {
      ccost[c] = s;
    }
  }
}

// Single block, fixed-shape tree: cost_sum += sum_c ccost[c].
__global__ void k_cost_total(const double* __restrict__ ccost, int k, double* __restrict__ out,
                             const int* __restrict__ gate) {
  if (gate && !*gate) return;
  __shared__ double s[256];
  double a = 0.0;
  for (int c = threadIdx.x; c < k; c += 256) a = dadd(a, ccost[c]);
  s[threadIdx.x] = a;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) s[threadIdx.x] = dadd(s[threadIdx.x], s[threadIdx.x + off]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = dadd(out[0], s[0]);
}

// ------------------------------------------------- incremental cluster sums
// (round 6) With the carried bounds most rows keep their center from one
// Lloyd call of a fit to the next, so the cluster sums change only by the
// rows that moved.  The row image's owner keeps, per cluster c, the sums S_c,
// weight W_c (unit weights: the count), member count N_c, a reference point
// P_c (the centers of the last full pass) with Q_c = sum |x - P_c|^2 over the
// members, and A_c = sum |x| (error scale).  A call with few moved rows
// (<= n / kIncMovedFrac) updates them by the moved rows alone (subtracted
// from the old cluster, added to the new, in row order: each cluster's
// workgroup picks its entries from the row-ordered moved list) and takes the cost
// for the call's centers c from
//   sum_x |x - c|^2 = Q_c + 2 (P_c - c).(S_c - W_c P_c) + W_c |P_c - c|^2,
// which is exact algebra; the rounding of every term is bounded on the device
// (ES_c, EQ_c and the correction's own).  When the bound
// exceeds 2^-40 of the cost, a moved count is too large, or no state exists,
// the call runs the full pass over every row instead (the sort by cluster and
// k_chunk_sums_fast), which resets the state.  Gates: gate[0] = 1 runs the
// full pass, gate[1] = 1 the incremental one; exactly one is set.
constexpr int kIncRows = 2048;       // rows per k_inc_moved workgroup
constexpr int kIncMovedFrac = 16;    // at most n / 16 moved rows take the incremental path
                                     // (kIncSplit workgroups fold a cluster's entries: a large
                                     // churn concentrates on a few clusters)

// The rows whose assignment differs from prev (then prev = assign): per
// kIncRows-row block, in row order, into tmpRow / tmpOld at the block's base;
// the block's count in bcount[block].
__global__ __launch_bounds__(256) void k_inc_moved(const int32_t* __restrict__ assign,
                                                   int32_t* __restrict__ prev, int64_t n,
                                                   int32_t* __restrict__ tmpRow,
                                                   int32_t* __restrict__ tmpOld,
                                                   unsigned int* __restrict__ bcount) {
  constexpr int IT = kIncRows / 256;
  __shared__ unsigned wc[IT * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kIncRows;
  unsigned long long masks[IT];
  int32_t olds[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int64_t r = base + it * 256 + tid;
    bool moved = false;
    olds[it] = -1;
    if (r < n) {
      const int32_t a = assign[r], b = prev[r];
      moved = a != b;
      olds[it] = b;
      if (moved) prev[r] = a;
    }
    masks[it] = __builtin_amdgcn_ballot_w64(moved);
    if (lane == 0) wc[it * 4 + wave] = (unsigned)__builtin_popcountll(masks[it]);
  }
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    unsigned before = 0;
    for (int j = 0; j < it * 4 + wave; ++j) before += wc[j];
    if ((masks[it] >> lane) & 1ull) {
      const int64_t pos = base + before + (unsigned)__builtin_popcountll(masks[it] & below);
      tmpRow[pos] = (int32_t)(base + it * 256 + tid);
      tmpOld[pos] = olds[it];
    }
  }
  if (tid == 0) {
    unsigned total = 0;
    for (int j = 0; j < IT * 4; ++j) total += wc[j];
    bcount[blockIdx.x] = total;
  }
}

// Single block: bcount[0..nb) -> exclusive offsets, bcount[nb] = *count = the
// moved rows; the gates (incremental when valid and count <= mcap); *movedCum
// += count on the incremental path.
__global__ __launch_bounds__(1024) void k_inc_scan(unsigned int* __restrict__ bcount, int64_t nb,
                                                   unsigned int* __restrict__ count, int valid,
                                                   int64_t mcap, int* __restrict__ gate,
                                                   unsigned long long* __restrict__ movedCum) {
  __shared__ unsigned part[1024];
  const int t = threadIdx.x;
  const int64_t per = (nb + 1023) / 1024;
  const int64_t a = min<int64_t>(nb, t * per), e = min<int64_t>(nb, a + per);
  unsigned s = 0;
  for (int64_t i = a; i < e; ++i) s += bcount[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const unsigned v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  unsigned run = t ? part[t - 1] : 0u;
  for (int64_t i = a; i < e; ++i) {
    const unsigned c = bcount[i];
    bcount[i] = run;
    run += c;
  }
  if (t == 1023) {
    const unsigned total = part[1023];
    bcount[nb] = total;
    *count = total;
    const int inc = valid && (int64_t)total <= mcap;
    gate[0] = inc ? 0 : 1;
    gate[1] = inc ? 1 : 0;
    if (inc) *movedCum += (unsigned long long)total;
  }
}

// The blocks' moved rows behind their offsets, with their new and old
// clusters (incremental path only).
__global__ __launch_bounds__(256) void k_inc_gather(const int32_t* __restrict__ tmpRow,
                                                    const int32_t* __restrict__ tmpOld,
                                                    const unsigned int* __restrict__ bcount,
                                                    const int32_t* __restrict__ assign,
                                                    int32_t* __restrict__ movedRow,
                                                    int32_t* __restrict__ movedNew,
                                                    int32_t* __restrict__ movedOld,
                                                    const int* __restrict__ gate) {
  if (!gate[1]) return;
  const int64_t b = blockIdx.x, base = b * kIncRows;
  const unsigned off = bcount[b], cnt = bcount[b + 1] - off;
  for (unsigned i = threadIdx.x; i < cnt; i += 256) {
    const int32_t r = tmpRow[base + i];
    movedRow[off + i] = r;
    movedNew[off + i] = assign[r];
    movedOld[off + i] = tmpOld[base + i];
  }
}

// Block sum of NV doubles per thread (fixed tree, results in every thread).
template <int NV>
__device__ __forceinline__ void inc_block_sum(double (&v)[NV], double* red) {
  const int tid = threadIdx.x;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) red[i * 256 + tid] = v[i];
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
#pragma unroll
      for (int i = 0; i < NV; ++i) red[i * 256 + tid] = dadd(red[i * 256 + tid], red[i * 256 + tid + off]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[i * 256];
}

// kIncSplit workgroups per cluster, each over one contiguous slice of the
// moved list: the cluster's entries there (the moved rows that left or
// joined it) picked in list order -- kIncScan entries per thread per step,
// compacted in order through LDS -- and folded into a partial (sums per
// dimension; the cost terms, count and norm sums as scalars).  Unit weights.
constexpr int kIncScan = 8;
constexpr int kIncSplit = 8;
constexpr int kIncPs = 6;   // scalars per partial: dq, |dq|, count, sum |x| signed, sum |x|, entries
template <int NJ>
__global__ __launch_bounds__(256) void k_inc_part(
    const double* __restrict__ X, int d, const double* __restrict__ xnorm,
    const int32_t* __restrict__ movedRow, const int32_t* __restrict__ movedNew,
    const int32_t* __restrict__ movedOld, const unsigned int* __restrict__ count,
    const double* __restrict__ P, double* __restrict__ pds, double* __restrict__ psc,
    const int* __restrict__ gate) {
  if (!gate[1]) return;
  constexpr int B = 256 * kIncScan;
  __shared__ int32_t rowsS[B];
  __shared__ float sgS[B];
  __shared__ unsigned wcS[kIncScan * 4];
  __shared__ double red[5 * 256];
  const int c = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned m = *count;
  const unsigned s0 = (unsigned)((uint64_t)m * g / kIncSplit);
  const unsigned s1 = (unsigned)((uint64_t)m * (g + 1) / kIncSplit);
  int64_t ent = 0;
  double ds[NJ], dq[NJ], dqa[NJ], pj[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    ds[u] = dq[u] = dqa[u] = 0.0;
    pj[u] = j < d ? P[(int64_t)c * d + j] : 0.0;
  }
  double tN = 0.0, tA = 0.0, tAbs = 0.0;   // this thread's entries: count, sum |x|
  const unsigned long long below = (1ull << lane) - 1ull;
  for (unsigned base = s0; base < s1; base += B) {
    int nw[kIncScan], ol[kIncScan];
#pragma unroll
    for (int q = 0; q < kIncScan; ++q) {
      const unsigned i = base + q * 256 + tid;
      nw[q] = i < s1 ? movedNew[i] : -1;
      ol[q] = i < s1 ? movedOld[i] : -1;
    }
    unsigned long long mk[kIncScan];
    __syncthreads();   // the previous batch's entries are folded
#pragma unroll
    for (int q = 0; q < kIncScan; ++q) {
      mk[q] = __builtin_amdgcn_ballot_w64(nw[q] == c || ol[q] == c);
      if (lane == 0) wcS[q * 4 + wave] = (unsigned)__builtin_popcountll(mk[q]);
    }
    __syncthreads();
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < kIncScan; ++q) {
      unsigned before = 0;
      for (int j = 0; j < q * 4 + wave; ++j) before += wcS[j];
      if ((mk[q] >> lane) & 1ull) {
        const unsigned pos = before + (unsigned)__builtin_popcountll(mk[q] & below);
        rowsS[pos] = movedRow[base + q * 256 + tid];
        sgS[pos] = nw[q] == c ? 1.0f : -1.0f;
      }
    }
    for (int j = 0; j < kIncScan * 4; ++j) cnt += (int)wcS[j];
    __syncthreads();
    ent += cnt;
    for (int e = tid; e < cnt; e += 256) {
      const bool add = sgS[e] > 0.0f;
      const double xn = xnorm[rowsS[e]];
      tN += add ? 1.0 : -1.0;
      tA = add ? dadd(tA, xn) : dsub(tA, xn);
      tAbs = dadd(tAbs, xn);
    }
    for (int p0 = 0; p0 < cnt; p0 += 8) {
      double xv[8][NJ];
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const int64_t r = rowsS[min(p0 + v, cnt - 1)];
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
          const int j = tid + 256 * u;
          xv[v][u] = j < d ? X[r * d + j] : 0.0;
        }
      }
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        if (p0 + v < cnt) {
          const bool add = sgS[p0 + v] > 0.0f;
#pragma unroll
          for (int u = 0; u < NJ; ++u) {
            const double x = xv[v][u];
            const double df = dsub(pj[u], x);
            const double t = dmul(df, df);
            ds[u] = add ? dadd(ds[u], x) : dsub(ds[u], x);
            dq[u] = add ? dadd(dq[u], t) : dsub(dq[u], t);
            dqa[u] = dadd(dqa[u], t);
          }
        }
      }
    }
  }
  double r1[5] = {0.0, 0.0, tN, tA, tAbs};
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    r1[0] = dadd(r1[0], dq[u]);
    r1[1] = dadd(r1[1], dqa[u]);
  }
  inc_block_sum<5>(r1, red);
  const int64_t slot = (int64_t)c * kIncSplit + g;
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    if (j < d) pds[slot * d + j] = ds[u];
  }
  if (tid < 5) psc[slot * kIncPs + tid] = r1[tid];
  if (tid == 5) psc[slot * kIncPs + 5] = (double)ent;
}

// One workgroup per cluster: its partials summed in slice order, folded into
// the state; then its cost for the call's centers C and the bound of that
// cost's rounding (cerr), cbad = 1 when the state's error grew past 2^-38 of
// the sum of the members' norms.
template <int NJ>
__global__ __launch_bounds__(256) void k_inc_combine(
    int d, const double* __restrict__ C, const double* __restrict__ pds,
    const double* __restrict__ psc, double* __restrict__ S, const double* __restrict__ P,
    double* __restrict__ W, double* __restrict__ Q, int64_t* __restrict__ N,
    double* __restrict__ A, double* __restrict__ ES, double* __restrict__ EQ,
    double* __restrict__ ccost, double* __restrict__ cerr, int* __restrict__ cbad,
    const int* __restrict__ gate) {
  if (!gate[1]) return;
  __shared__ double red[4 * 256];
  const int c = blockIdx.x, tid = threadIdx.x;
  double r1[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  int64_t ent = 0;
  double ds[NJ], pj[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    ds[u] = 0.0;
    pj[u] = j < d ? P[(int64_t)c * d + j] : 0.0;
  }
  for (int g = 0; g < kIncSplit; ++g) {
    const int64_t slot = (int64_t)c * kIncSplit + g;
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int j = tid + 256 * u;
      if (j < d) ds[u] = dadd(ds[u], pds[slot * d + j]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) r1[i] = dadd(r1[i], psc[slot * kIncPs + i]);
    ent += (int64_t)psc[slot * kIncPs + 5];
  }
  const int64_t nNew = N[c] + (int64_t)r1[2];
  const bool empty = nNew <= 0;
  const double wNew = empty ? 0.0 : (double)nNew;    // unit weights: the count
  double sv[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    const double s0 = j < d ? S[(int64_t)c * d + j] : 0.0;
    sv[u] = empty ? 0.0 : (ent ? dadd(s0, ds[u]) : s0);
    if (j < d && ent) S[(int64_t)c * d + j] = sv[u];
  }
  // the cost's terms for the call's centers
  double r2[4] = {0.0, 0.0, 0.0, 0.0};   // |S|^2, D.V, |D|^2, |P|^2
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int j = tid + 256 * u;
    if (j < d) {
      const double D = dsub(pj[u], C[(int64_t)c * d + j]);
      const double V = dsub(sv[u], dmul(wNew, pj[u]));
      r2[0] = dadd(r2[0], dmul(sv[u], sv[u]));
      r2[1] = dadd(r2[1], dmul(D, V));
      r2[2] = dadd(r2[2], dmul(D, D));
      r2[3] = dadd(r2[3], dmul(pj[u], pj[u]));
    }
  }
  inc_block_sum<4>(r2, red);
  if (tid == 0) {
    double q = Q[c], a = A[c], es = ES[c], eq = EQ[c];
    if (empty) {
      q = a = es = eq = 0.0;
    } else if (ent) {
      const double nS = sqrt(r2[0]) * (1.0 + 0x1p-50);
      q = dadd(q, r1[0]);
      a = dadd(a, r1[3]);
      // a slice's entries sum sequentially, then the slices and (for the
      // cost terms) the dimensions and the block tree: <= ent + kIncSplit
      // + 16 roundings per term
      es += 0x1p-52 * ((double)(ent + kIncSplit + 1) * r1[4] + nS);
      eq += 0x1p-52 * ((double)(ent + kIncSplit + 16) * r1[1] + fabs(q));
    }
    N[c] = empty ? 0 : nNew;
    W[c] = wNew;
    Q[c] = q;
    A[c] = a;
    ES[c] = es;
    EQ[c] = eq;
    double cost = 0.0, err = 0.0;
    int bad = 0;
    if (!empty) {
      const double nS = sqrt(r2[0]) * (1.0 + 0x1p-50), nD = sqrt(r2[2]) * (1.0 + 0x1p-50),
                   nP = sqrt(r2[3]) * (1.0 + 0x1p-50);
      cost = dadd(q, dadd(dmul(2.0, r2[1]), dmul(wNew, r2[2])));
      const double sv2 = nS + wNew * nP;
      // the correction's own rounding: D and V (one rounding each, the
      // 2^-51 term), the dot's and |D|^2's sums (<= NJ + 8 + 2 <= 14
      // roundings of terms bounded by |D| |V|, |D|^2: 2 x 16 x 2^-53 <=
      // 2^-47, taken as 2^-46)
      err = eq + 2.0 * nD * (es + 0x1p-51 * sv2) + 0x1p-46 * (nD * sv2 + wNew * r2[2]) +
            0x1p-50 * fabs(cost);
      bad = !(es <= 0x1p-38 * a) || !(fabs(cost) < INFINITY) || !(err < INFINITY);
    }
    ccost[c] = cost;
    cerr[c] = err;
    cbad[c] = bad;
  }
}

// Single block: the clusters' costs and error bounds summed in a fixed
// tree; the incremental result stands when no cluster is flagged and the
// bound is within 2^-40 of the cost, else the gates switch to the full pass.
__global__ __launch_bounds__(256) void k_inc_check(const double* __restrict__ ccost,
                                                   const double* __restrict__ cerr,
                                                   const int* __restrict__ cbad, int k,
                                                   int* __restrict__ gate,
                                                   double* __restrict__ tot,
                                                   unsigned long long* __restrict__ incCum) {
  if (!gate[1]) return;
  __shared__ double red[3 * 256];
  double v[3] = {0.0, 0.0, 0.0};
  for (int c = threadIdx.x; c < k; c += 256) {
    v[0] = dadd(v[0], ccost[c]);
    v[1] += cerr[c];
    v[2] += cbad[c] ? 1.0 : 0.0;
  }
  inc_block_sum<3>(v, red);
  if (threadIdx.x == 0) {
    const bool ok = v[2] == 0.0 && v[1] <= 0x1p-40 * fabs(v[0]) && fabs(v[0]) < INFINITY;
    tot[0] = v[0];
    tot[1] = v[1];
    if (ok) {
      *incCum += 1ull;
    } else {
      gate[0] = 1;
      gate[1] = 0;
    }
  }
}

// After the check (one launch, k_inc_finish): the incremental result into
// the caller's buffers (gate[1]: sums += S, wsum += W, cost_sum += the
// checked total); after a full pass (gate[0]) its fresh sums are the state
// (written by k_reduce_clusters), P = C, Q = the clusters' costs, N = the
// counts, and the error bounds of the full pass's own summation (<= 256
// rows per chunk partial, the block tree, then the chunk fold).  The two
// read and write disjoint buffers, so one after the other or side by side
// is the same.
__global__ __launch_bounds__(256) void k_inc_finish(
    const double* __restrict__ C, int d, double* __restrict__ P, const double* __restrict__ ccost,
    const int64_t* __restrict__ total, const int64_t* __restrict__ chunkStart,
    double* __restrict__ Q, int64_t* __restrict__ N, const double* __restrict__ A,
    double* __restrict__ ES, double* __restrict__ EQ, const double* __restrict__ S,
    const double* __restrict__ W, const double* __restrict__ tot, double* __restrict__ sums,
    double* __restrict__ wsum, double* __restrict__ costSum, const int* __restrict__ gate) {
  const int c = blockIdx.x;
  if (gate[0]) {
    for (int j = threadIdx.x; j < d; j += 256) P[(int64_t)c * d + j] = C[(int64_t)c * d + j];
    if (threadIdx.x == 0) {
      const double f = 0x1p-52 * (double)(300 + (chunkStart[c + 1] - chunkStart[c]));
      Q[c] = ccost[c];
      N[c] = total[c];
      ES[c] = f * A[c];
      EQ[c] = f * fabs(ccost[c]);
    }
  }
  if (gate[1]) {
    for (int j = threadIdx.x; j < d; j += 256)
      sums[(int64_t)c * d + j] = dadd(sums[(int64_t)c * d + j], S[(int64_t)c * d + j]);
    if (threadIdx.x == 0) {
      wsum[c] = dadd(wsum[c], W[c]);
      if (c == 0) costSum[0] = dadd(costSum[0], tot[0]);
    }
  }
}

constexpr int kUpdLds = 3072;   // widest center staged in LDS by k_update_centers

// centroid (DistanceMeasure.scala:200-203: scal(1/w, sum); new VectorWithNorm)
// and isCenterConverged (:345-350).  One 64-lane workgroup per center: the
// elementwise part in parallel, then lane 0 runs the two sequential sums (the
// moved distance and the new norm, in index order) from LDS.  The caller sets
// *converged = 1 first; a center that moved clears it.
__global__ __launch_bounds__(64) void k_update_centers(
    double* __restrict__ C, double* __restrict__ cnorm, const double* __restrict__ sums,
    const double* __restrict__ wsum, int k, int d, double eps2, int32_t* __restrict__ converged) {
  extern __shared__ double upd[];   // 2 d (d <= kUpdLds)
  const int c = blockIdx.x, lane = threadIdx.x;
  const double w = wsum[c];
  if (!(w > 0)) return;
  const double a = 1.0 / w;
  double* crow = C + (int64_t)c * d;
  const double* srow = sums + (int64_t)c * d;
  if (d > kUpdLds) {
    // wide (sparse-input) centers: lane 0 reads both rows in order first
    if (lane == 0) {
      double moved = 0.0, nn = 0.0;
      for (int j = 0; j < d; ++j) {
        const double v = dmul(a, srow[j]);
        const double sc = dsub(v, crow[j]);
        moved = dadd(moved, dmul(sc, sc));
        nn = dadd(nn, dmul(v, v));
      }
      cnorm[c] = __builtin_sqrt(nn);
      if (!(moved <= eps2) && converged) atomicAnd(converged, 0);
    }
    __syncthreads();
    for (int j = lane; j < d; j += 64) crow[j] = dmul(a, srow[j]);
    return;
  }
  for (int j = lane; j < d; j += 64) {
    const double v = dmul(a, srow[j]);
    const double sc = dsub(v, crow[j]);
    upd[j] = dmul(sc, sc);
    upd[d + j] = dmul(v, v);
    crow[j] = v;
  }
  __syncthreads();
  if (lane == 0) {
    double moved = 0.0, nn = 0.0;
    for (int j = 0; j < d; ++j) {
      moved = dadd(moved, upd[j]);
      nn = dadd(nn, upd[d + j]);
    }
    cnorm[c] = __builtin_sqrt(nn);
    if (!(moved <= eps2) && converged) atomicAnd(converged, 0);
  }
}

// ------------------------------------------------------------ sparse points
// KMeansExample's input (BASELINE configs[0]) is libsvm, i.e. SparseVector
// points against dense centers: fastSquaredDistance then takes the norm-trick
// branch (MLUtils.scala:560-573) with BLAS.dot(sparse, dense)
// (mllib/linalg/BLAS.scala:153-169) and the sqdist(sparse, dense) fallback
// (Vectors.scala:598-622).  These kernels restate that path for CSR rows.

// Vectors.norm(sparse, 2) (Vectors.scala:489-514 over the stored values)
__global__ void k_row_norms_csr(const int64_t* __restrict__ rowptr,
                                const double* __restrict__ vals, int64_t n,
                                double* __restrict__ norms) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  double s = 0.0;
  for (int64_t q = rowptr[r]; q < rowptr[r + 1]; ++q) s = dadd(s, dmul(vals[q], vals[q]));
  norms[r] = __builtin_sqrt(s);
}

// java.lang.Math.max(a, 0.0): NaN stays NaN, -0.0 becomes +0.0
__device__ __forceinline__ double jmax0(double a) {
  if (a != a) return a;
  return a > 0.0 ? a : 0.0;
}

// MLUtils.fastSquaredDistance(v1 = dense center, norm1, v2 = sparse point,
// norm2) with precision 1e-6 (:533-576), the reference's operation order.
__device__ double fast_sqdist_ds(const double* __restrict__ c, double norm1,
                                 const int32_t* __restrict__ idx,
                                 const double* __restrict__ val, int64_t nnz, double norm2,
                                 int d) {
  const double EPS = 0x1p-52;                         // MLUtils.EPSILON (:44-50)
  const double sumSq = dadd(dmul(norm1, norm1), dmul(norm2, norm2));
  const double nd = dsub(norm1, norm2);
  const double pb1 = dmul(dmul(2.0, EPS), sumSq) / dadd(dmul(nd, nd), EPS);
  double dot = 0.0;                                   // dot(sparse, dense), nnz order
  for (int64_t q = 0; q < nnz; ++q) dot = dadd(dot, dmul(val[q], c[idx[q]]));
  if (pb1 < 1e-6) return dsub(sumSq, dmul(2.0, dot));
  double sq = jmax0(dsub(sumSq, dmul(2.0, dot)));
  const double pb2 = dmul(EPS, dadd(sumSq, dmul(2.0, __builtin_fabs(dot)))) / dadd(sq, EPS);
  if (pb2 > 1e-6) {                                   // Vectors.sqdist(sparse, dense)
    int64_t kv1 = 0;
    int iv1 = nnz > 0 ? idx[0] : -1;
    double t = 0.0;
    for (int kv2 = 0; kv2 < d; ++kv2) {
      double score;
      if (kv2 != iv1) {
        score = c[kv2];
      } else {
        score = dsub(val[kv1], c[kv2]);
        if (kv1 < nnz - 1) {
          ++kv1;
          iv1 = idx[kv1];
        }
      }
      t = dadd(t, dmul(score, score));
    }
    sq = t;
  }
  return sq;
}

// EuclideanDistanceMeasure.findClosest with statistics (DistanceMeasure.scala:
// 282-313) for sparse rows: the wave-parallel replay of k_assign_exact with
// fastSquaredDistance as the distance.  Every row takes this path (the
// screens are dense-only); one wave per row, grid-stride.
__global__ __launch_bounds__(256) void k_assign_sparse(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const double* __restrict__ vals, const double* __restrict__ xnorm, int64_t n, int d,
    const double* __restrict__ C, const double* __restrict__ cnorm, int k,
    const double* __restrict__ stats, int32_t* __restrict__ assign, double* __restrict__ cost) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wid; r < n; r += nw) {
    const int64_t q0 = rowptr[r], nnz = rowptr[r + 1] - q0;
    const int32_t* idx = colidx + q0;
    const double* val = vals + q0;
    const double xn = xnorm[r];
    // stats == nullptr: findClosest(centers, point) (:318-340), best from +inf
    const bool ns = stats == nullptr;
    double best = ns ? __builtin_inf() : fast_sqdist_ds(C, cnorm[0], idx, val, nnz, xn, d);   // :286
    int bi = 0;
    bool done = !ns && best < stats[0];                                       // :287
    for (int i0 = ns ? 0 : 1; !done && i0 < k; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < k;
      double lb = __builtin_inf(), sii = 0.0;
      if (valid) {
        const double ndf = dsub(cnorm[i], xn);                         // :294-295
        lb = dmul(ndf, ndf);
        sii = ns ? 0.0 : stats[iut(i, i)];
      }
      double dd = 0.0;
      bool have = false;
      int pos = 0;
      for (;;) {
        const bool visit = valid && lane >= pos && lb < best && (ns || stats[iut(i, bi)] < best);
        if (visit && !have) {
          dd = fast_sqdist_ds(C + (int64_t)i * d, cnorm[i], idx, val, nnz, xn, d);
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

}  // namespace

// ------------------------------------------------------------------ plan
struct cyc_kmeans_plan_s {
  int d = 0, k = 0, d4 = 0, kpad = 0, bm = 0, ldsStride = 0;
  int measure = CYC_DISTANCE_EUCLIDEAN;   // DistanceMeasure of the plan
  // cosine: unit center directions for the screen, their norms, computed
  // center norms (statistics without given norms)
  cyc::DeviceBuffer cosV, cosVn, cosCn;
  bool dense_ok = true;     // d fits the LDS-resident dense assign kernels (d <= 1240)
  int variant = 1;          // 2: k_kmeans_assign2 (fp64 screen), 3: bf16x3 screen
  int ldsStride2 = 0;
  size_t assignLds2 = 0;
  // bf16x3 screen (variant 3): k-steps of 32 dims, padded 16-center tiles,
  // center tiles per wave group, LDS bytes, error-bound constants
  int ks3 = 0, ktp3 = 0;
  static constexpr int tb3 = 2;
  size_t lds3 = 0;
  double omE3 = 1.0, tauL3 = 0.0, facU3 = 0.0, tauU3 = 0.0;
  int64_t lastTier2 = 0;    // rows the bf16 screen queued (last counted call)
  int64_t lastExact = 0;    // rows the fp64 screen queued (last counted call)
  int64_t lastLimb3 = -1;   // rows the two-limb i8 pass left to the three-limb pass (-1: none)
  int64_t lastCands = -1;   // rows the two-limb i8 pass left to the candidate pass
  int64_t lastCands2 = -1;  // rows the three-limb candidate tier left to the fp64 pass
  bool cands3 = false;      // the last cand_args enabled the three-limb candidate tier
  cyc::DeviceBuffer cb3, cq3, ok3, list3, list3Count;
  // i8 exact-integer screen (kmeans_i8.hip), used with a row image
  int ktp8 = 0;
  // cb8: the center image (fragments, then the center-major copy, d <= 256)
  cyc::DeviceBuffer cb8, cq8, g8, prm8, scr8, list8Count;   // list8 = slowList (idle then)
  // candidate pass of the d <= 256 screen (kmeans_i8.hpp CandArgs)
  cyc::DeviceBuffer candRows, cands, candCount;
  // the rows the three-limb candidate tier leaves to the fp64 pass
  cyc::DeviceBuffer candRows2, cands2, candCount2;
  // the one-limb pass + two-limb refinement (kmeans_i8.hpp RefineArgs)
  cyc::DeviceBuffer cand1Rows, cand1, cand1Count, fullList, fullCount;
  // the screens' sharded append stage (kmeans_i8.hpp AppendStage)
  cyc::DeviceBuffer stgRowsA, stgRowsB, stgCandRows, stgCands, stgCounts;
  bool lastRefined = false;  // the last i8 screen ran the refinement path
  int64_t max_rows = 0;
  size_t assignLds = 0;
  std::mutex mu;
  cyc::DeviceBuffer ct, stats, dmin, segsum, slowList, slowCount, assignTmp, costTmp;
  cyc::DeviceBuffer hist, total, cstart, chunkStart, perm, part, pw, pc, ccost;
  cyc::DeviceBuffer exactDist;   // k_exact_dist's distances (kExactCap x kpad)
  // require(norm1 >= 0.0 && norm2 >= 0.0) check (k_require_norms): device
  // result, its pinned host copy and the event that marks the copy landed
  cyc::DeviceBuffer req;
  // ClusteringEvaluator's Silhouette (silhouette.hpp): check flags, row
  // norms, per-block score partials
  cyc::DeviceBuffer silFlags, silNorms, silPart;
  unsigned long long* reqHost = nullptr;
  hipEvent_t reqEv = nullptr;
  ~cyc_kmeans_plan_s() {
    if (reqHost) (void)hipHostFree(reqHost);
    if (reqEv) (void)hipEventDestroy(reqEv);
  }
};

// Per-fit row image for the i8 screen (cyc_kmeans_rows_create).
struct cyc_kmeans_rows_s {
  const double* X = nullptr;
  int64_t n = 0;
  int d = 0;
  bool usable = false;     // d <= 512
  bool cosine = false;     // image of the unit directions x / |x|
  cyc::DeviceBuffer img, meta, unorm;   // unorm: |x / |x|| per row (cosine); |x| (Euclidean:
                                        // any summation order, the screens' margins)
  // Carried bounds of one fit's Lloyd iterations (kmeans_i8.hpp Bounds):
  // cyc_kmeans_accumulate_dev screens only the rows they cannot certify.
  // State: per row (ub, lb) and the assignment they certify (bAssign), the
  // centers they refer to (bCp, k x d); valid once a call has written them.
  bool bEnabled = true;    // cyc_kmeans_rows_set_bounds (CYC_KMEANS_BOUNDS=0: off by default)
  bool bValid = false;
  int bk = 0;
  cyc::DeviceBuffer bnd, bAssign, bCp, bDelta, bCcs, bPrm, bTmp, bCount, bList, bListCount, bCum;
  cyc::DeviceBuffer bTmp2, bCount2;   // the filter's state-1 list (k8::Bounds::collected)
  // carried candidate sets (kmeans_i8.hpp Bounds): outside bound, sets,
  // per-row state, the re-check list, its count and running total
  cyc::DeviceBuffer bLnc, bSets, bState, bRc, bRcCount, bRcCum;
  // the centers' neighbourhoods for the state-3 re-checks (k_center_nbrs)
  cyc::DeviceBuffer bNbr, bNbrR;
  int64_t bCalls = 0, bFullRows = 0;   // bounded calls; rows of their full (first) screens
  // Incremental cluster sums (k_inc_*; with the carried bounds, unit
  // weights, no per-row costs): the assignment the state refers to (iPrev),
  // the per-cluster state S, P, W, Q, N, A, ES, EQ, and the scratch of the
  // moved-row list and its sort by cluster.  iCum: moved rows and calls that
  // took the incremental path (two 64-bit counters).
  bool iEnabled = true;    // cyc_kmeans_rows_set_incremental (CYC_KMEANS_INCR=0: off)
  bool iValid = false;
  int ik = 0;
  cyc::DeviceBuffer iPrev, iTmpRow, iTmpOld, iBcount, iCount, iGate, iMovedRow, iMovedNew,
      iMovedOld, iS, iP, iW, iQ, iN, iA, iES, iEQ, iCost, iErr, iBad, iTot, iCum, iPa, iPds, iPsc;
};

namespace {

int pick_bm(int d4, int& stride, size_t& lds) {
  const int cands[3] = {64, 32, 16};
  const int maxbm = 64;
  for (int bm : cands) {
    if (bm > maxbm) continue;
    int s = d4 + ((2 - d4 % 32) + 32) % 32;  // stride == 2 (mod 32)
    size_t bytes = ((size_t)bm * s + bm + (size_t)kWaves * bm * 4) * sizeof(double);
    if (bytes <= 160 * 1024) {
      stride = s;
      lds = bytes;
      return bm;
    }
  }
  return 0;
}

template <int BM>
int launch_assign(cyc_kmeans_plan p, const double* X, const double* xnorm, int64_t n,
                  const double* C, const double* cnorm, int32_t* assign, double* cost,
                  hipStream_t st, const int32_t* rowList = nullptr,
                  const unsigned int* rowCount = nullptr) {
  static bool attr_set = false;
  if (!attr_set) {
    CYC_HIP(hipFuncSetAttribute((const void*)k_kmeans_assign<BM>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CYC_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_kmeans_assign2<BM>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const double marginFac = (double)(p->d + 16) * 0x1p-46;
  // list mode (rows queued by the bf16 screen): persistent grid over the queue
  const int64_t blocks = rowList ? std::min<int64_t>((n + BM - 1) / BM, 1024) : (n + BM - 1) / BM;
  cyc::KernelTimer timer(rowList ? "k_kmeans_assign_fp64" : "k_kmeans_assign", st);
#define CYC_A2()                                                                              \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_kmeans_assign2<BM>), dim3((unsigned)blocks), dim3(kAssignThreads), \
                     p->assignLds2, st, X, xnorm, n, p->d, p->d4, p->ldsStride2,               \
                     (const double*)p->ct.ptr, C, cnorm, p->k, p->kpad, marginFac, assign, cost, \
                     (int32_t*)p->slowList.ptr, (unsigned int*)p->slowCount.ptr, rowList, rowCount)
  if (p->variant == 2 || p->variant == 3) CYC_A2();
  else
  hipLaunchKernelGGL(k_kmeans_assign<BM>, dim3((unsigned)blocks), dim3(kAssignThreads),
                     p->assignLds, st, X, xnorm, n, p->d, p->d4, p->ldsStride,
                     (const double*)p->ct.ptr, C, cnorm, p->k, p->kpad, marginFac, assign, cost,
                     (int32_t*)p->slowList.ptr, (unsigned int*)p->slowCount.ptr, rowList,
                     rowCount);
  CYC_LAUNCH_CHECK("k_kmeans_assign");
  return CYC_OK;
}

int do_stats(cyc_kmeans_plan p, const double* C, hipStream_t st) {
  const int k = p->k, d = p->d;
  const int tps = (k + kStT - 1) / kStT;
  unsigned long long* dmin = (unsigned long long*)p->dmin.ptr;
  if (p->dense_ok) {
    const int64_t total = std::max<int64_t>((int64_t)p->d4 * p->kpad, k);
    hipLaunchKernelGGL(k_center_transpose_fill, dim3((unsigned)((total + 255) / 256)), dim3(256),
                       0, st, C, k, d, p->d4, p->kpad, (double*)p->ct.ptr, dmin, kInfBits);
    CYC_LAUNCH_CHECK("k_center_transpose_fill");
  } else {
    hipLaunchKernelGGL(k_fill_u64, dim3((k + 255) / 256), dim3(256), 0, st, dmin, k, kInfBits);
    CYC_LAUNCH_CHECK("k_fill_u64");
  }
  hipLaunchKernelGGL(k_stats_pairs, dim3((unsigned)(tps * (tps + 1) / 2)), dim3(256), 0, st, C, k,
                     d, tps, (double*)p->stats.ptr, dmin);
  CYC_LAUNCH_CHECK("k_stats_pairs");
  hipLaunchKernelGGL(k_stats_diag, dim3((k + 255) / 256), dim3(256), 0, st, k,
                     (double*)p->stats.ptr, (const unsigned long long*)dmin);
  CYC_LAUNCH_CHECK("k_stats_diag");
  return CYC_OK;
}

template <int TB>
int launch_assign3(cyc_kmeans_plan p, const double* X, const double* xnorm, int64_t n,
                   const double* C, const double* cnorm, int32_t* assign, double* cost,
                   hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    CYC_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_kmeans_assign3<TB>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  cyc::KernelTimer timer("k_kmeans_assign", st);
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_kmeans_assign3<TB>), dim3((unsigned)((n + kS3BM - 1) / kS3BM)),
                     dim3(kS3Threads), p->lds3, st, X, xnorm, n, p->d, p->ks3,
                     (const uint4*)p->cb3.ptr, (const float*)p->cq3.ptr, p->ktp3,
                     (const int*)p->ok3.ptr, C, cnorm, p->omE3, p->tauL3, p->facU3, p->tauU3,
                     assign, cost, (int32_t*)p->list3.ptr, (unsigned int*)p->list3Count.ptr);
  CYC_LAUNCH_CHECK("k_kmeans_assign3");
  return CYC_OK;
}

// The candidate pass's buffers and arguments (d <= 256 screens only).
int cand_args(cyc_kmeans_plan p, int64_t n, const double* X, const double* xnorm,
              const double* C, const double* cnorm, bool unit, cyc::km8::CandArgs& ca,
              bool& use) {
  use = cyc::km8::uses32(p->d);
  if (!use) return CYC_OK;
  int rc;
  if ((rc = p->candRows.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = p->cands.reserve(sizeof(int32_t) * (size_t)n * cyc::km8::kCandMax)) ||
      (rc = p->candCount.reserve(64)))
    return rc;
  // Euclidean: a 2^-30 relative gap is far above fp64 rounding; the cosine
  // plan keeps the screen's own 2^-19 (the statistic's sqrt, kmeans_cos.hip)
  ca = cyc::km8::CandArgs{X, xnorm, C, cnorm, p->k, unit, unit ? 0x1p-19 : 0x1p-30,
                          (int32_t*)p->candRows.ptr, (int32_t*)p->cands.ptr,
                          (unsigned int*)p->candCount.ptr};
  // the three-limb candidate tier (CYC_KMEANS_CANDS3=0: every candidate row
  // straight to the fp64 pass)
  const char* e3 = std::getenv("CYC_KMEANS_CANDS3");
  p->cands3 = !(e3 && e3[0] == '0');
  if (p->cands3) {
    if ((rc = p->candRows2.reserve(sizeof(int32_t) * (size_t)n)) ||
        (rc = p->cands2.reserve(sizeof(int32_t) * (size_t)n * cyc::km8::kCandMax)) ||
        (rc = p->candCount2.reserve(64)))
      return rc;
    ca.candRows2 = (int32_t*)p->candRows2.ptr;
    ca.cands2 = (int32_t*)p->cands2.ptr;
    ca.candCount2 = (unsigned int*)p->candCount2.ptr;
  }
  return CYC_OK;
}

// The one-limb pass + two-limb refinement of the d <= 256 screen, for k >
// 96 (below that the two-limb pass over every center is as cheap) and k <=
// 4096 (the refinement's union bitmap).
int refine_args(cyc_kmeans_plan p, int64_t n, bool useCa, cyc::km8::RefineArgs& ra, bool& use) {
  const int kstride = cyc::km8::tiles32(p->k) * 32;
  use = useCa && p->k > 96 && kstride <= 4096 && std::getenv("CYC_KMEANS_NO_REFINE") == nullptr;
  p->lastRefined = use;
  if (!use) return CYC_OK;
  int rc;
  if ((rc = p->cand1Rows.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = p->cand1.reserve(sizeof(int32_t) * (size_t)n * cyc::km8::kCand1)) ||
      (rc = p->cand1Count.reserve(64)) ||
      (rc = p->fullList.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = p->fullCount.reserve(64)))
    return rc;
  ra = cyc::km8::RefineArgs{kstride, (int32_t*)p->cand1Rows.ptr, (int32_t*)p->cand1.ptr,
                            (unsigned int*)p->cand1Count.ptr, (int32_t*)p->fullList.ptr,
                            (unsigned int*)p->fullCount.ptr};
  return CYC_OK;
}

// Carried bounds for a Lloyd call (cyc_kmeans_accumulate_dev): Euclidean
// rows with an image whose screen runs the one-limb pass (refine_args).
bool bounds_on(cyc_kmeans_plan p, cyc_kmeans_rows rows) {
  static const bool envOff = [] {
    const char* e = std::getenv("CYC_KMEANS_BOUNDS");
    return e && e[0] == '0';
  }();
  return rows && rows->usable && !rows->cosine && rows->bEnabled && !envOff &&
         !cyc::strict_parity() &&
         p->measure == CYC_DISTANCE_EUCLIDEAN && cyc::km8::uses32(p->d) && p->k > 96 &&
         cyc::km8::tiles32(p->k) * 32 <= 4096 && std::getenv("CYC_KMEANS_NO_REFINE") == nullptr;
}

// CYC_KMEANS_NBR=0: no neighbourhood re-checks (state 3)
bool nbrOff() {
  static const bool off = [] {
    const char* e = std::getenv("CYC_KMEANS_NBR");
    return e && e[0] == '0';
  }();
  return off || cyc::strict_parity();
}

// Moves the bounds to the centers C (the drift against the last call's,
// then Cp = C) and lists the rows they cannot certify; bd for the screen.
// The first call of a fit (or after a change of k) screens every row.
int bounds_prepare(cyc_kmeans_plan p, cyc_kmeans_rows rows, const double* C,
                   const double* xnorm, int64_t n, hipStream_t st, cyc::km8::Bounds& bd) {
  namespace k8 = cyc::km8;
  const int k = p->k, d = p->d;
  int rc;
  if ((rc = rows->bnd.reserve(sizeof(float2) * (size_t)n)) ||
      (rc = rows->bAssign.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->bCp.reserve(sizeof(double) * (size_t)k * d)) ||
      (rc = rows->bDelta.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->bCcs.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->bPrm.reserve(sizeof(k8::DriftParams))) ||
      (rc = rows->bTmp.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->bCount.reserve(sizeof(unsigned int) * (size_t)(k8::bounds_blocks(n) + 1))) ||
      (rc = rows->bTmp2.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->bCount2.reserve(sizeof(unsigned int) * (size_t)(k8::bounds_blocks(n) + 1))) ||
      (rc = rows->bList.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->bListCount.reserve(64)) ||
      (rc = rows->bLnc.reserve(sizeof(float) * (size_t)n)) ||
      (rc = rows->bSets.reserve(sizeof(int32_t) * (size_t)n * k8::kCandMax)) ||
      (rc = rows->bState.reserve((size_t)n)) ||
      (rc = rows->bRc.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->bRcCount.reserve(64)) ||
      (rc = rows->bNbr.reserve(sizeof(int32_t) * (size_t)k * k8::kCandMax)) ||
      (rc = rows->bNbrR.reserve(sizeof(float) * (size_t)k)))
    return rc;
  if (!rows->bCum.ptr) {
    if ((rc = rows->bCum.reserve(64)) || (rc = rows->bRcCum.reserve(64))) return rc;
    CYC_HIP(hipMemsetAsync(rows->bCum.ptr, 0, 8, st));
    CYC_HIP(hipMemsetAsync(rows->bRcCum.ptr, 0, 8, st));
  }
  const bool carry = rows->bValid && rows->bk == k;
  rows->bValid = false;   // until the screen has written the bounds
  if ((rc = k8::centers_drift(C, (double*)rows->bCp.ptr, k, d, (double*)rows->bDelta.ptr,
                              (double*)rows->bCcs.ptr, (k8::DriftParams*)rows->bPrm.ptr, st)))
    return rc;
  bd = k8::Bounds{(float2*)rows->bnd.ptr, nullptr, nullptr};
  bd.lnc = (float*)rows->bLnc.ptr;
  bd.sets = (int32_t*)rows->bSets.ptr;
  bd.state = (unsigned char*)rows->bState.ptr;
  bd.dp = (const k8::DriftParams*)rows->bPrm.ptr;
  bd.tmp = (int32_t*)rows->bTmp.ptr;
  bd.bcount = (unsigned int*)rows->bCount.ptr;
  bd.list = (int32_t*)rows->bList.ptr;
  bd.listCount = (unsigned int*)rows->bListCount.ptr;
  bd.cum = (unsigned long long*)rows->bCum.ptr;
  bd.n = n;
  if (carry) {
    // kept rows, the re-check list (screen: the re-check, then the state-1
    // rows collected into bList for the one-limb pass; with the two-phase
    // re-check the filter lists its state-1 rows there itself and the
    // re-check appends its failures)
    const bool two = k8::recheck_two_phase();
    if ((rc = k8::bounds_filter((const int32_t*)rows->bAssign.ptr, (float2*)rows->bnd.ptr,
                                bd.lnc, bd.state, xnorm, n, k, (const double*)rows->bDelta.ptr,
                                bd.dp, bd.tmp, bd.bcount, (int32_t*)rows->bRc.ptr,
                                (unsigned int*)rows->bRcCount.ptr,
                                (unsigned long long*)rows->bRcCum.ptr,
                                nbrOff() ? nullptr : (const double*)p->stats.ptr,
                                (int32_t*)rows->bNbr.ptr, (float*)rows->bNbrR.ptr, st,
                                two ? (int32_t*)rows->bTmp2.ptr : nullptr,
                                two ? (unsigned int*)rows->bCount2.ptr : nullptr,
                                two ? bd.list : nullptr, two ? bd.listCount : nullptr,
                                two ? bd.cum : nullptr)))
      return rc;
    bd.collected = two;
    if (!nbrOff()) {
      bd.nbr = (const int32_t*)rows->bNbr.ptr;
      bd.nbrR = (const float*)rows->bNbrR.ptr;
    }
    static const int dumpCall = [] {
      const char* e = std::getenv("CYC_KMEANS_DUMP_CALL");
      return e ? std::atoi(e) : 10;
    }();
    if (cyc::dump_dir() && rows->bCalls == dumpCall) {
      bd.dump = 1;
      cyc::dump_dev("state_filter", rows->bState.ptr, (size_t)n, st);
      cyc::dump_dev("bnd", rows->bnd.ptr, sizeof(float2) * (size_t)n, st);
      cyc::dump_dev("lnc", rows->bLnc.ptr, sizeof(float) * (size_t)n, st);
      cyc::dump_dev("assign", rows->bAssign.ptr, sizeof(int32_t) * (size_t)n, st);
      cyc::dump_dev("nbrR", rows->bNbrR.ptr, sizeof(float) * (size_t)k, st);
      cyc::dump_dev("nbr", rows->bNbr.ptr, sizeof(int32_t) * (size_t)k * k8::kCandMax, st);
      cyc::dump_dev("delta", rows->bDelta.ptr, sizeof(double) * (size_t)k, st);
      cyc::dump_dev("prm", rows->bPrm.ptr, sizeof(k8::DriftParams), st);
    }
    bd.rcRows = (const int32_t*)rows->bRc.ptr;
    bd.rcCount = (const unsigned int*)rows->bRcCount.ptr;
    bd.rowsIn = bd.list;
    bd.rowsInCount = bd.listCount;
  } else {
    // a full screen: no carried sets yet (NaN outside bounds)
    CYC_HIP(hipMemsetAsync(bd.lnc, 0xff, sizeof(float) * (size_t)n, st));
    rows->bFullRows += n;
  }
  return CYC_OK;
}

// The screens' sharded append stage for n rows (with the candidate pass);
// CYC_KMEANS_NO_STAGE=1 appends straight to the lists (one counter each).
int stage_args(cyc_kmeans_plan p, int64_t n, bool useCa, cyc::km8::AppendStage& sg, bool& use) {
  use = useCa && std::getenv("CYC_KMEANS_NO_STAGE") == nullptr;
  if (!use) return CYC_OK;
  namespace k8 = cyc::km8;
  const unsigned cap = k8::shard_cap(n);
  const size_t ent = (size_t)cap * k8::kShards;
  const size_t cbytes = sizeof(unsigned int) * k8::kSets * k8::kShards * k8::kShardStride;
  int rc;
  if ((rc = p->stgRowsA.reserve(sizeof(int32_t) * ent)) ||
      (rc = p->stgRowsB.reserve(sizeof(int32_t) * ent)) ||
      (rc = p->stgCandRows.reserve(sizeof(int32_t) * ent)) ||
      (rc = p->stgCands.reserve(sizeof(int32_t) * ent * k8::kCand1)) ||
      (rc = p->stgCounts.reserve(cbytes)))
    return rc;
  sg = k8::AppendStage{(int32_t*)p->stgRowsA.ptr, (int32_t*)p->stgRowsB.ptr,
                       (int32_t*)p->stgCandRows.ptr, (int32_t*)p->stgCands.ptr,
                       (unsigned int*)p->stgCounts.ptr, cap};
  return CYC_OK;
}

// The exact tier over the plan's slow queue: the split kernels for a queue of
// <= kExactCap rows, k_assign_exact for a longer one; known = the queue's
// length when the host has it (-1: decided on the device, both enqueued).
int launch_exact(cyc_kmeans_plan p, const double* X, const double* xnorm, int64_t n,
                 const double* C, const double* cnorm, const double* statsArg, int32_t* assign,
                 double* cost, bool approxNorm, int64_t known, hipStream_t st) {
  cyc::KernelTimer timer("k_kmeans_exact", st);
  const int k = p->k, kpad = p->kpad;
  const unsigned* cnt = (const unsigned*)p->slowCount.ptr;
  static const bool splitOff = [] {   // CYC_KMEANS_EXACT_SPLIT=0: k_assign_exact alone
    const char* e = std::getenv("CYC_KMEANS_EXACT_SPLIT");
    return e && e[0] == '0';
  }();
  const bool split = !splitOff && p->d <= 1280 && (known < 0 || known <= kExactCap);
  if (split) {
    int rc;
    if ((rc = p->exactDist.reserve(sizeof(double) * (size_t)kExactCap * kpad))) return rc;
    const unsigned rowsMax = (unsigned)std::min<int64_t>(known < 0 ? n : known, kExactCap);
    hipLaunchKernelGGL(k_exact_dist, dim3((unsigned)((k + 255) / 256), rowsMax), dim3(256), 0, st,
                       X, p->d, (const double*)p->ct.ptr, kpad, k, (const int32_t*)p->slowList.ptr,
                       cnt, (double*)p->exactDist.ptr);
    CYC_LAUNCH_CHECK("k_exact_dist");
    hipLaunchKernelGGL(k_exact_replay, dim3(rowsMax), dim3(64), 0, st, X, xnorm, p->d, kpad, cnorm,
                       k, statsArg, (const int32_t*)p->slowList.ptr, cnt,
                       (const double*)p->exactDist.ptr, assign, cost, approxNorm ? 1 : 0);
    CYC_LAUNCH_CHECK("k_exact_replay");
    if (known >= 0) return CYC_OK;
  }
  // the long queue (or no split): one workgroup per row, grid-stride
  const unsigned grid = known >= 0 ? (unsigned)std::min<int64_t>(known, 4096)
                                   : (unsigned)std::min<int64_t>((n + 3) / 4, 2048);
  hipLaunchKernelGGL(k_assign_exact, dim3(grid), dim3(256), 0, st, X, xnorm, p->d, C,
                     (const double*)p->ct.ptr, kpad, cnorm, k, statsArg,
                     (const int32_t*)p->slowList.ptr, cnt, assign, cost, approxNorm ? 1 : 0,
                     split ? (unsigned)kExactCap : 0u);
  CYC_LAUNCH_CHECK("k_assign_exact");
  return CYC_OK;
}

int do_assign(cyc_kmeans_plan p, const double* X, const double* xnorm, cyc_kmeans_rows rows,
              int64_t n, const double* C, const double* cnorm, int32_t* assign, double* cost,
              int64_t* n_exact_out, hipStream_t st, bool nostats = false,
              const cyc::km8::Bounds* bd = nullptr, bool approxNorm = false) {
  // nostats: findClosest(centers, point) (DistanceMeasure.scala:318-340); the
  // screens certify only rows whose winner both loops return, so only the
  // exact tier differs (no statistics prunes, best starts at +inf)
  const double* statsArg = nostats ? nullptr : (const double*)p->stats.ptr;
  const bool i8 = rows && rows->usable;
  // slowCount (and list3Count for the i8 tier) zeroed by one launch
  hipLaunchKernelGGL(k_zero2, dim3(1), dim3(64), 0, st, (unsigned int*)p->slowCount.ptr,
                     i8 ? (unsigned int*)p->list3Count.ptr : nullptr);
  CYC_LAUNCH_CHECK("k_zero2");
  int rc = CYC_OK;
  const int32_t* rowList = nullptr;
  const unsigned int* rowCount = nullptr;
  if (i8) {
    // tier 1: exact-integer i8 screen over every row; undecided rows -> list3
    if ((rc = cyc::km8::centers_prepare(C, cnorm, p->k, p->d, p->ktp8, p->cb8.ptr,
                                        (float*)p->cq8.ptr, (double*)p->g8.ptr,
                                        (cyc::km8::CenterParams*)p->prm8.ptr,
                                        (double*)p->scr8.ptr, st)))
      return rc;
    cyc::km8::CandArgs ca;
    bool useCa = false;
    if ((rc = cand_args(p, n, X, nullptr, C, cnorm, false, ca, useCa))) return rc;
    cyc::km8::RefineArgs ra;
    bool useRa = false;
    if ((rc = refine_args(p, n, useCa, ra, useRa))) return rc;
    cyc::km8::AppendStage sg;
    bool useSg = false;
    if ((rc = stage_args(p, n, useCa, sg, useSg))) return rc;
    if ((rc = cyc::km8::screen(rows->img.ptr, (const int2*)rows->meta.ptr, xnorm, n, p->d,
                               p->cb8.ptr, (const float*)p->cq8.ptr, (const double*)p->g8.ptr,
                               cnorm, (const cyc::km8::CenterParams*)p->prm8.ptr, p->ktp8,
                               assign, (int32_t*)p->list3.ptr, (unsigned int*)p->list3Count.ptr,
                               (int32_t*)p->slowList.ptr, (unsigned int*)p->list8Count.ptr, st,
                               useCa ? &ca : nullptr, useRa ? &ra : nullptr,
                               useSg ? &sg : nullptr, bd)))
      return rc;
    rowList = (const int32_t*)p->list3.ptr;
    rowCount = (const unsigned int*)p->list3Count.ptr;
  } else if (p->variant == 3) {
    // tier 1: bf16x3 screen over every row; undecided rows -> list3
    CYC_HIP(hipMemsetAsync(p->list3Count.ptr, 0, sizeof(unsigned int), st));
    CYC_HIP(hipMemsetAsync(p->ok3.ptr, 1, sizeof(int), st));
    const int64_t tot = (int64_t)p->ktp3 * p->ks3 * 64;
    hipLaunchKernelGGL(k_center_split, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, C,
                       cnorm, p->k, p->d, p->ks3, p->ktp3, p->omE3, (uint4*)p->cb3.ptr,
                       (float*)p->cq3.ptr, (int*)p->ok3.ptr);
    CYC_LAUNCH_CHECK("k_center_split");
    rc = launch_assign3<2>(p, X, xnorm, n, C, cnorm, assign, cost, st);
    if (rc) return rc;
    rowList = (const int32_t*)p->list3.ptr;
    rowCount = (const unsigned int*)p->list3Count.ptr;
  }
  // tier 2: fp64 MFMA screen (every row, or the queued ones).  Queued rows
  // (a few thousand after the i8 tiers) go 16 to a workgroup: a 64-row
  // tile kept ~50 CUs busy for ~110 us each (CYC_KMEANS_LIST_BM=0: the
  // plan's tile); the dynamic LDS stays the plan's (64-row) size, which
  // covers 16 rows
  static const bool list16 = [] {
    const char* e = std::getenv("CYC_KMEANS_LIST_BM");
    return !(e && e[0] == '0');
  }();
  if (rowList && list16 && p->bm >= 16) {
    rc = launch_assign<16>(p, X, xnorm, n, C, cnorm, assign, cost, st, rowList, rowCount);
  } else switch (p->bm) {
    case 64: rc = launch_assign<64>(p, X, xnorm, n, C, cnorm, assign, cost, st, rowList, rowCount); break;
    case 32: rc = launch_assign<32>(p, X, xnorm, n, C, cnorm, assign, cost, st, rowList, rowCount); break;
    default: rc = launch_assign<16>(p, X, xnorm, n, C, cnorm, assign, cost, st, rowList, rowCount); break;
  }
  if (rc) return rc;
  // Exact emulation of the reference loop for undecided rows.  The queue
  // length is read back only when the caller asks for it; otherwise a
  // grid-stride launch drains whatever the queue holds without a host sync.
  unsigned int h_slow = 0, h_tier2 = 0, h_limb3 = 0, h_cand = 0, h_cand2 = 0;
  if (n_exact_out) {
    const bool twoPass = rows && rows->usable && cyc::km8::uses32(p->d);
    CYC_HIP(hipMemcpyAsync(&h_slow, p->slowCount.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    if (rowCount)
      CYC_HIP(hipMemcpyAsync(&h_tier2, rowCount, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    if (twoPass) {
      CYC_HIP(hipMemcpyAsync(&h_limb3, p->list8Count.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
      CYC_HIP(hipMemcpyAsync(&h_cand, p->candCount.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
      if (p->cands3)
        CYC_HIP(hipMemcpyAsync(&h_cand2, p->candCount2.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    }
    CYC_HIP(hipStreamSynchronize(st));
    *n_exact_out = h_slow;
    p->lastTier2 = rowCount ? (int64_t)h_tier2 : n;
    p->lastExact = h_slow;
    p->lastLimb3 = twoPass ? (int64_t)h_limb3 : -1;
    p->lastCands = twoPass ? (int64_t)h_cand : -1;
    p->lastCands2 = twoPass && p->cands3 ? (int64_t)h_cand2 : -1;
    if (h_slow)
      return launch_exact(p, X, xnorm, n, C, cnorm, statsArg, assign, cost, approxNorm,
                          (int64_t)h_slow, st);
    return CYC_OK;
  }
  return launch_exact(p, X, xnorm, n, C, cnorm, statsArg, assign, cost, approxNorm, -1, st);
}

// Enqueue k_require_norms and the copy of its result; require_check reads it
// after the rest of the call is enqueued, so the host waits only for this
// early, short kernel (its result lands long before the assign finishes).
int require_enqueue(cyc_kmeans_plan p, const double* C, const double* xnorm, int64_t n,
                    hipStream_t st) {
  int rc;
  if ((rc = p->req.reserve(5 * sizeof(unsigned long long)))) return rc;
  if (!p->reqHost) CYC_HIP(hipHostMalloc((void**)&p->reqHost, 5 * sizeof(unsigned long long)));
  if (!p->reqEv) CYC_HIP(hipEventCreateWithFlags(&p->reqEv, hipEventDisableTiming));
  CYC_HIP(hipMemsetAsync(p->req.ptr, 0xff, 2 * sizeof(unsigned long long), st));
  const int64_t work = std::max<int64_t>(n, (int64_t)p->k * p->d);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 2048));
  hipLaunchKernelGGL(k_require_norms, dim3(grid), dim3(256), 0, st, C, p->k, p->d, xnorm, n,
                     (unsigned long long*)p->req.ptr);
  CYC_LAUNCH_CHECK("k_require_norms");
  CYC_HIP(hipMemcpyAsync(p->reqHost, p->req.ptr, 5 * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, st));
  CYC_HIP(hipEventRecord(p->reqEv, st));
  return CYC_OK;
}

// The IllegalArgumentException the reference raises first, if any:
// computeStatistics' pair loop (i < j, DistanceMeasure.scala:55-66) meets
// (0, m) for the lowest NaN center m > 0, or (0, 1) when center 0 is NaN;
// with k == 1 there are no statistics and the first point meets center 0;
// otherwise the first NaN-norm point meets center 0 (norm2 = NaN).
int require_check(cyc_kmeans_plan p, int64_t n, const double* Xrow0 = nullptr) {
  CYC_HIP(hipEventSynchronize(p->reqEv));
  const unsigned long long cbad = p->reqHost[0], rbad = p->reqHost[1];
  double* v = reinterpret_cast<double*>(p->reqHost + 2);
  if (Xrow0 && n > 0 && cbad == 0 && !(p->k >= 2)) {
    // the message's norm2 is row 0's Vectors.norm: the image's norms (in
    // another summation order) stand in for the caller's, so recompute it
    std::vector<double> x0((size_t)p->d);
    CYC_HIP(hipMemcpy(x0.data(), Xrow0, sizeof(double) * (size_t)p->d, hipMemcpyDeviceToHost));
    double sq = 0.0;
    for (int j = 0; j < p->d; ++j) sq = sq + x0[j] * x0[j];
    v[2] = std::sqrt(sq);
  }
  const double nan = __builtin_nan("");
  auto fail = [](double n1, double n2) {
    cyc::set_error("requirement failed: Both norms should be greater or equal to 0.0, found "
                   "norm1=" + cyc::java_double(n1) + ", norm2=" + cyc::java_double(n2));
    return CYC_ERR_INVALID_ARG;
  };
  if (p->k >= 2 && cbad < (unsigned long long)p->k) return cbad == 0 ? fail(nan, v[1]) : fail(v[0], nan);
  if (n > 0 && cbad == 0) return fail(nan, v[2]);
  if (rbad < (unsigned long long)n) return fail(v[0], nan);
  return CYC_OK;
}

int ensure_rows(cyc_kmeans_plan p, int64_t n) {
  if (n <= p->max_rows && p->slowList.ptr) return CYC_OK;
  int rc;
  if ((rc = p->slowList.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(n, 1)))) return rc;
  if ((rc = p->list3.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(n, 1)))) return rc;
  p->max_rows = std::max(p->max_rows, n);
  return CYC_OK;
}

// ------------------------------------------------------------ cosine plan
bool is_cos(cyc_kmeans_plan p) { return p->measure == CYC_DISTANCE_COSINE; }

// The zero-length assert of CosineDistanceMeasure.distance (DistanceMeasure.
// scala:453-456): enqueued first, read by cos_check at the end of the call.
// Every center norm is checked when checkCenters (computeStatistics measures
// every pair for k >= 2; findClosest measures center 0, and without
// statistics every center, for each point), every row norm when n > 0.
int cos_enqueue(cyc_kmeans_plan p, const double* cnorm, bool checkCenters, const double* xnorm,
                int64_t n, hipStream_t st) {
  int rc;
  if ((rc = p->req.reserve(5 * sizeof(unsigned long long)))) return rc;
  if (!p->reqHost) CYC_HIP(hipHostMalloc((void**)&p->reqHost, 5 * sizeof(unsigned long long)));
  if (!p->reqEv) CYC_HIP(hipEventCreateWithFlags(&p->reqEv, hipEventDisableTiming));
  if ((rc = cyc::kmcos::assert_norms(cnorm, p->k, checkCenters, xnorm, n,
                                     (unsigned long long*)p->req.ptr, st)))
    return rc;
  CYC_HIP(hipMemcpyAsync(p->reqHost, p->req.ptr, sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, st));
  CYC_HIP(hipEventRecord(p->reqEv, st));
  return CYC_OK;
}

int cos_check(cyc_kmeans_plan p) {
  CYC_HIP(hipEventSynchronize(p->reqEv));
  if (p->reqHost[0]) {
    cyc::set_error("assertion failed: Cosine distance is not defined for zero-length vectors.");
    return CYC_ERR_ASSERTION;
  }
  return CYC_OK;
}

int cos_transpose(cyc_kmeans_plan p, const double* C, hipStream_t st) {
  const int64_t total = (int64_t)p->d4 * p->kpad;
  hipLaunchKernelGGL(k_center_transpose, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     C, p->k, p->d, p->d4, p->kpad, (double*)p->ct.ptr);
  CYC_LAUNCH_CHECK("k_center_transpose");
  return CYC_OK;
}

int cos_stats(cyc_kmeans_plan p, const double* C, const double* cnorm, hipStream_t st) {
  return cyc::kmcos::stats(C, cnorm, p->k, p->d, (double*)p->stats.ptr,
                           (unsigned long long*)p->dmin.ptr, st);
}

// CosineDistanceMeasure.findClosest for n dense rows: the i8 screen on the
// unit directions (row image built for cosine), then the reference loop for
// every row it leaves (every row without an image).
int cos_assign(cyc_kmeans_plan p, const double* X, const double* xnorm, cyc_kmeans_rows rows,
               int64_t n, const double* C, const double* cnorm, int32_t* assign, double* cost,
               int64_t* n_exact_out, hipStream_t st, bool nostats) {
  int rc;
  if ((rc = cos_transpose(p, C, st))) return rc;
  int32_t* list = (int32_t*)p->list3.ptr;
  unsigned int* count = (unsigned int*)p->list3Count.ptr;
  const bool screen = rows && rows->usable && p->ktp8 > 0;
  if (screen) {
    if ((rc = p->cosV.reserve(sizeof(double) * (size_t)p->k * p->d)) ||
        (rc = p->cosVn.reserve(sizeof(double) * (size_t)p->k)))
      return rc;
    double* V = (double*)p->cosV.ptr;
    double* Vn = (double*)p->cosVn.ptr;
    if ((rc = cyc::kmcos::centers_unit(C, cnorm, p->k, p->d, V, Vn, st))) return rc;
    CYC_HIP(hipMemsetAsync(count, 0, sizeof(unsigned int), st));
    cyc::km8::CandArgs ca;
    bool useCa = false;
    if ((rc = cand_args(p, n, X, xnorm, V, Vn, true, ca, useCa))) return rc;
    cyc::km8::AppendStage sg;
    bool useSg = false;
    if ((rc = stage_args(p, n, useCa, sg, useSg))) return rc;
    if ((rc = cyc::km8::centers_prepare(V, Vn, p->k, p->d, p->ktp8, p->cb8.ptr,
                                        (float*)p->cq8.ptr, (double*)p->g8.ptr,
                                        (cyc::km8::CenterParams*)p->prm8.ptr,
                                        (double*)p->scr8.ptr, st)) ||
        (rc = cyc::km8::screen(rows->img.ptr, (const int2*)rows->meta.ptr,
                               (const double*)rows->unorm.ptr, n, p->d, p->cb8.ptr,
                               (const float*)p->cq8.ptr, (const double*)p->g8.ptr, Vn,
                               (const cyc::km8::CenterParams*)p->prm8.ptr, p->ktp8, assign, list,
                               count, (int32_t*)p->slowList.ptr,
                               (unsigned int*)p->list8Count.ptr, st, useCa ? &ca : nullptr,
                               nullptr, useSg ? &sg : nullptr)))
      return rc;
  } else if ((rc = cyc::kmcos::list_all(list, count, n, st))) {
    return rc;
  }
  int64_t maxRows = n;
  if (n_exact_out) {
    unsigned int h = 0, h3 = 0, hc = 0, hc2 = 0;
    const bool twoPass = screen && cyc::km8::uses32(p->d);
    CYC_HIP(hipMemcpyAsync(&h, count, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    if (twoPass) {
      CYC_HIP(hipMemcpyAsync(&h3, p->list8Count.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
      CYC_HIP(hipMemcpyAsync(&hc, p->candCount.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
      if (p->cands3)
        CYC_HIP(hipMemcpyAsync(&hc2, p->candCount2.ptr, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    }
    CYC_HIP(hipStreamSynchronize(st));
    *n_exact_out = h;
    p->lastTier2 = h;   // no fp64 screen tier: the screen's leftovers are exact
    p->lastExact = h;
    p->lastLimb3 = twoPass ? (int64_t)h3 : -1;
    p->lastCands = twoPass ? (int64_t)hc : -1;
    p->lastCands2 = twoPass && p->cands3 ? (int64_t)hc2 : -1;
    maxRows = h;
  }
  if (maxRows == 0) return CYC_OK;
  return cyc::kmcos::assign_exact(X, xnorm, p->d, C, (const double*)p->ct.ptr, p->kpad, cnorm,
                                  p->k, nostats ? nullptr : (const double*)p->stats.ptr, list,
                                  count, maxRows, assign, cost, st);
}

}  // namespace

namespace {

// Counting sort of rows 0..n by assign[] into the plan's perm (stable: row
// order kept within a cluster), with cstart (k + 1 cluster offsets) and
// chunkStart (k + 1 offsets of kChunkRows-row chunks); part / pw / pc
// reserved for maxChunks chunks of d columns.
int sort_clusters(cyc_kmeans_plan p, const int32_t* assign, int64_t n, int d, hipStream_t st,
                  int64_t& maxChunks, const int* gate = nullptr) {
  const int k = p->k;
  int rc;
  const int tiles = (int)((n + kSortTile - 1) / kSortTile);
  maxChunks = (n + kChunkRows - 1) / kChunkRows + k;
  if ((rc = p->hist.reserve(sizeof(int32_t) * (size_t)tiles * k)) ||
      (rc = p->total.reserve(sizeof(int64_t) * (size_t)k)) ||
      (rc = p->cstart.reserve(sizeof(int64_t) * (size_t)(k + 1))) ||
      (rc = p->chunkStart.reserve(sizeof(int64_t) * (size_t)(k + 1))) ||
      (rc = p->perm.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = p->part.reserve(sizeof(double) * (size_t)maxChunks * d)) ||
      (rc = p->pw.reserve(sizeof(double) * (size_t)maxChunks)) ||
      (rc = p->pc.reserve(sizeof(double) * (size_t)maxChunks)) ||
      (rc = p->ccost.reserve(sizeof(double) * (size_t)k)))
    return rc;
  int32_t* hist = (int32_t*)p->hist.ptr;
  hipLaunchKernelGGL(k_hist, dim3(tiles), dim3(256), sizeof(int32_t) * k, st, assign, n, k, hist,
                     gate);
  CYC_LAUNCH_CHECK("k_hist");
  {
    const int segT = (tiles + std::min(kScanSegs, tiles) - 1) / std::min(kScanSegs, tiles);
    const int segs = (tiles + segT - 1) / segT;
    if ((rc = p->segsum.reserve(sizeof(int32_t) * (size_t)segs * k))) return rc;
    int32_t* segsum = (int32_t*)p->segsum.ptr;
    hipLaunchKernelGGL(k_scan_seg, dim3((unsigned)((k + 63) / 64), (unsigned)segs), dim3(64), 0, st,
                       (const int32_t*)hist, tiles, k, segT, segsum, gate);
    CYC_LAUNCH_CHECK("k_scan_seg");
    hipLaunchKernelGGL(k_scan_segoff, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, st, segsum,
                       segs, k, (int64_t*)p->total.ptr, gate);
    CYC_LAUNCH_CHECK("k_scan_segoff");
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)((k + 63) / 64), (unsigned)segs), dim3(64), 0,
                       st, hist, tiles, k, segT, (const int32_t*)segsum, gate);
    CYC_LAUNCH_CHECK("k_scan_apply");
  }
  hipLaunchKernelGGL(k_scan_clusters, dim3(1), dim3(1024), 0, st, (const int64_t*)p->total.ptr, k,
                     (int64_t*)p->cstart.ptr, (int64_t*)p->chunkStart.ptr, gate);
  CYC_LAUNCH_CHECK("k_scan_clusters");
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)(8 * (((int64_t)tiles + 7) / 8))), dim3(64),
                     sizeof(int64_t) * k, st, assign, n, k, hist, (const int64_t*)p->cstart.ptr,
                     (int32_t*)p->perm.ptr, (int64_t)tiles, gate);
  CYC_LAUNCH_CHECK("k_scatter");
  return CYC_OK;
}

bool inc_on(cyc_kmeans_rows rows) {
  static const bool envOff = [] {
    const char* e = std::getenv("CYC_KMEANS_INCR");
    return e && e[0] == '0';
  }();
  return rows->iEnabled && !envOff && !cyc::strict_parity();
}

// The Lloyd call's cluster sums, weights and cost through the incremental
// state (k_inc_*) or, when the device decides so, the full pass; both paths
// are enqueued and gated on the device (no host round trip).  assign: the
// call's assignment (the bounds' bAssign).
int inc_accumulate(cyc_kmeans_plan p, cyc_kmeans_rows rows, const double* X,
                   const double* xnorm, const int32_t* assign, int64_t n, const double* C,
                   double* sums, double* wsum, double* cost_sum, hipStream_t st) {
  const int k = p->k, d = p->d, nj = (d + 255) / 256;
  const int64_t nb = (n + kIncRows - 1) / kIncRows;
  const int64_t mcap = n / kIncMovedFrac;
  const size_t kd = (size_t)k * d;
  int rc;
  const bool fresh = rows->iPrev.ptr == nullptr;
  if ((rc = rows->iPrev.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->iTmpRow.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->iTmpOld.reserve(sizeof(int32_t) * (size_t)n)) ||
      (rc = rows->iBcount.reserve(sizeof(unsigned int) * (size_t)(nb + 1))) ||
      (rc = rows->iCount.reserve(64)) || (rc = rows->iGate.reserve(64)) ||
      (rc = rows->iMovedRow.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(mcap, 1))) ||
      (rc = rows->iMovedNew.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(mcap, 1))) ||
      (rc = rows->iMovedOld.reserve(sizeof(int32_t) * (size_t)std::max<int64_t>(mcap, 1))) ||
      (rc = rows->iS.reserve(sizeof(double) * kd)) || (rc = rows->iP.reserve(sizeof(double) * kd)) ||
      (rc = rows->iPds.reserve(sizeof(double) * kd * kIncSplit)) ||
      (rc = rows->iPsc.reserve(sizeof(double) * (size_t)k * kIncSplit * kIncPs)) ||
      (rc = rows->iW.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iQ.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iN.reserve(sizeof(int64_t) * (size_t)k)) ||
      (rc = rows->iA.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iES.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iEQ.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iCost.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iErr.reserve(sizeof(double) * (size_t)k)) ||
      (rc = rows->iBad.reserve(sizeof(int) * (size_t)k)) || (rc = rows->iTot.reserve(64)) ||
      (rc = rows->iCum.reserve(64)))
    return rc;
  if (fresh) {
    CYC_HIP(hipMemsetAsync(rows->iPrev.ptr, 0xff, sizeof(int32_t) * (size_t)n, st));
    CYC_HIP(hipMemsetAsync(rows->iCum.ptr, 0, 16, st));
  }
  const int valid = rows->iValid && rows->ik == k ? 1 : 0;
  rows->iValid = false;   // until this call has completed
  int* gate = (int*)rows->iGate.ptr;
  unsigned long long* cum = (unsigned long long*)rows->iCum.ptr;
  const unsigned int* cnt = (const unsigned int*)rows->iCount.ptr;
  {
    cyc::KernelTimer timer("k_kmeans_inc", st);
    hipLaunchKernelGGL(k_inc_moved, dim3((unsigned)nb), dim3(256), 0, st, assign,
                       (int32_t*)rows->iPrev.ptr, n, (int32_t*)rows->iTmpRow.ptr,
                       (int32_t*)rows->iTmpOld.ptr, (unsigned int*)rows->iBcount.ptr);
    CYC_LAUNCH_CHECK("k_inc_moved");
    hipLaunchKernelGGL(k_inc_scan, dim3(1), dim3(1024), 0, st, (unsigned int*)rows->iBcount.ptr,
                       nb, (unsigned int*)rows->iCount.ptr, valid, mcap, gate, cum);
    CYC_LAUNCH_CHECK("k_inc_scan");
    hipLaunchKernelGGL(k_inc_gather, dim3((unsigned)nb), dim3(256), 0, st,
                       (const int32_t*)rows->iTmpRow.ptr, (const int32_t*)rows->iTmpOld.ptr,
                       (const unsigned int*)rows->iBcount.ptr, assign,
                       (int32_t*)rows->iMovedRow.ptr, (int32_t*)rows->iMovedNew.ptr,
                       (int32_t*)rows->iMovedOld.ptr, (const int*)gate);
    CYC_LAUNCH_CHECK("k_inc_gather");
#define CYC_IF(NJ)                                                                               \
  do {                                                                                           \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_inc_part<NJ>), dim3((unsigned)k, kIncSplit), dim3(256), 0, \
                     st, X, d, xnorm, (const int32_t*)rows->iMovedRow.ptr,                        \
                     (const int32_t*)rows->iMovedNew.ptr, (const int32_t*)rows->iMovedOld.ptr,   \
                     cnt, (const double*)rows->iP.ptr, (double*)rows->iPds.ptr,                 \
                     (double*)rows->iPsc.ptr, (const int*)gate);                                 \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_inc_combine<NJ>), dim3((unsigned)k), dim3(256), 0, st, d, C, \
                     (const double*)rows->iPds.ptr, (const double*)rows->iPsc.ptr,              \
                     (double*)rows->iS.ptr, (const double*)rows->iP.ptr, (double*)rows->iW.ptr,  \
                     (double*)rows->iQ.ptr, (int64_t*)rows->iN.ptr, (double*)rows->iA.ptr,       \
                     (double*)rows->iES.ptr, (double*)rows->iEQ.ptr, (double*)rows->iCost.ptr,   \
                     (double*)rows->iErr.ptr, (int*)rows->iBad.ptr, (const int*)gate);         \
  } while (0)
    if (nj == 1) CYC_IF(1);
    else if (nj == 2) CYC_IF(2);
    else CYC_IF(4);
#undef CYC_IF
    CYC_LAUNCH_CHECK("k_inc_part / k_inc_combine");
    hipLaunchKernelGGL(k_inc_check, dim3(1), dim3(256), 0, st, (const double*)rows->iCost.ptr,
                       (const double*)rows->iErr.ptr, (const int*)rows->iBad.ptr, k, gate,
                       (double*)rows->iTot.ptr, cum + 1);
    CYC_LAUNCH_CHECK("k_inc_check");
  }
  // the full pass (gate[0]): the counting sort, chunk sums, cluster folds,
  // and the state reset from them
  int64_t maxChunks = 0;
  if ((rc = sort_clusters(p, assign, n, d, st, maxChunks, gate))) return rc;
  if ((rc = rows->iPa.reserve(sizeof(double) * (size_t)maxChunks))) return rc;
  {
    cyc::KernelTimer timer("k_chunk_sums", st);
#define CYC_CSF(NJ)                                                                              \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_chunk_sums_fast<NJ>), dim3((unsigned)maxChunks), dim3(256), 0, \
                     st, X, d, (const double*)nullptr, C, (const int32_t*)p->perm.ptr,          \
                     (const int64_t*)p->cstart.ptr, (const int64_t*)p->chunkStart.ptr, k,       \
                     (double*)p->part.ptr, (double*)p->pw.ptr, (double*)p->pc.ptr, xnorm,        \
                     (double*)rows->iPa.ptr, (const int*)gate)
    if (nj == 1) CYC_CSF(1);
    else if (nj == 2) CYC_CSF(2);
    else CYC_CSF(4);
#undef CYC_CSF
    CYC_LAUNCH_CHECK("k_chunk_sums");
  }
  hipLaunchKernelGGL(k_reduce_clusters, dim3(k), dim3(256), 0, st, (const double*)p->part.ptr,
                     (const double*)p->pw.ptr, (const double*)p->pc.ptr,
                     (const int64_t*)p->chunkStart.ptr, d, sums, wsum, (double*)p->ccost.ptr,
                     (const double*)rows->iPa.ptr, (double*)rows->iS.ptr, (double*)rows->iW.ptr,
                     (double*)rows->iA.ptr, (const int*)gate);
  CYC_LAUNCH_CHECK("k_reduce_clusters");
  hipLaunchKernelGGL(k_cost_total, dim3(1), dim3(256), 0, st, (const double*)p->ccost.ptr, k,
                     cost_sum, (const int*)gate);
  CYC_LAUNCH_CHECK("k_cost_total");
  hipLaunchKernelGGL(k_inc_finish, dim3(k), dim3(256), 0, st, C, d, (double*)rows->iP.ptr,
                     (const double*)p->ccost.ptr, (const int64_t*)p->total.ptr,
                     (const int64_t*)p->chunkStart.ptr, (double*)rows->iQ.ptr,
                     (int64_t*)rows->iN.ptr, (const double*)rows->iA.ptr, (double*)rows->iES.ptr,
                     (double*)rows->iEQ.ptr, (const double*)rows->iS.ptr,
                     (const double*)rows->iW.ptr, (const double*)rows->iTot.ptr, sums, wsum,
                     cost_sum, (const int*)gate);
  CYC_LAUNCH_CHECK("k_inc_finish");
  return CYC_OK;
}

}  // namespace

extern "C" {

int cyc_row_norms_dev(const double* X, int64_t n, int32_t d, double* norms, void* stream) {
  CYC_REQUIRE(n >= 0 && d > 0, "n >= 0 and d > 0");
  if (n == 0) return CYC_OK;
  hipLaunchKernelGGL(k_row_norms, dim3((unsigned)((n + kNormRows - 1) / kNormRows)),
                     dim3(kNormRows), 0, cyc::as_stream(stream), X, n, d, norms);
  CYC_LAUNCH_CHECK("k_row_norms");
  return CYC_OK;
}

int cyc_kmeans_plan_create(int32_t d, int32_t k, int64_t max_rows, cyc_kmeans_plan* plan) {
  CYC_REQUIRE(plan != nullptr, "plan must not be null");
  CYC_REQUIRE(d > 0, "Number of features must be positive");
  CYC_REQUIRE(k >= 1, "Number of clusters must be positive but got " + std::to_string(k));
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  if (k > kMaxK) {
    cyc::set_error("k > 8192 is not supported by the device counting sort");
    return CYC_ERR_UNSUPPORTED;
  }
  auto* p = new cyc_kmeans_plan_s();
  p->d = d;
  p->k = k;
  p->d4 = (int)cyc::round_up(d, 4);
  p->kpad = (int)cyc::round_up(k, 16);
  p->bm = pick_bm(p->d4, p->ldsStride, p->assignLds);
  // variant 2: row stride d4 + 1 (== 1 mod 16 doubles: the two 16-lane
  // halves of a ds_read2_b64 fragment read hit distinct banks)
  p->ldsStride2 = p->d4 + 1;
  p->assignLds2 = p->assignLds + sizeof(double) * ((size_t)p->kpad + p->bm) -
                  sizeof(double) * (size_t)p->bm * (p->ldsStride - p->ldsStride2);
  p->variant = ((p->d4 % 32) == 0 && p->assignLds2 <= 160 * 1024) ? 2 : 1;
  // bf16x3 screen in front of the fp64 one where its LDS tile fits
  p->ks3 = (int)((d + 31) / 32);
  p->lds3 = (size_t)2 * kS3BM * (p->ks3 * 4 + 1) * 16 + (size_t)kS3Waves * kS3BM * 12 +
            (size_t)kS3BM * 8;
  const bool fits3 = p->variant == 2 && p->lds3 <= 160 * 1024;
  if (fits3) p->variant = 3;
  // test hook (tests/test_kmeans_gpu.py): the screen tier a plan uses
  // without a row image -- 1 fp64 screen, 2 fp64 screen with the
  // conflict-free stride, 3 bf16x3 screen in front of it
  if (const char* v = std::getenv("CYC_KMEANS_ASSIGN")) {
    const int want = std::atoi(v);
    if (want == 1 || (p->d4 % 32 == 0 && p->assignLds2 <= 160 * 1024 && want >= 2 && want <= 3 &&
                      (want != 3 || fits3)))
      p->variant = want;
  }
  {
    p->ktp3 = (int)cyc::round_up((k + 15) / 16, kS3Waves * p->tb3);
    const double d32 = 32.0 * p->ks3;
    const double eps = 3.1 * 0x1p-16 + 2.0 * 1.03 * (3.0 * d32 + 64.0) * 0x1p-23 + 0x1p-20;
    const double tau = 0x1p-58;
    p->omE3 = 1.0 - eps;
    p->tauL3 = 2.0 * tau;
    p->facU3 = (2.0 * eps + 0x1p-20) * (1.0 + 0x1p-20);
    p->tauU3 = 4.0 * tau;
  }
  // d > 1240: no LDS-resident dense assign; the plan still serves sparse rows
  p->dense_ok = p->bm != 0;
  int rc;
  if (p->variant == 3 &&
      ((rc = p->cb3.reserve((size_t)p->ktp3 * p->ks3 * 2 * 64 * 16)) ||
       (rc = p->cq3.reserve(sizeof(float) * (size_t)p->ktp3 * 16)) ||
       (rc = p->ok3.reserve(64)))) {
    delete p;
    return rc;
  }
  if ((rc = p->list3Count.reserve(64))) {
    delete p;
    return rc;
  }
  if (d <= cyc::km8::kMaxD) {
    const int ks8 = cyc::km8::ksteps(d);
    p->ktp8 = (int)cyc::round_up((k + 15) / 16, cyc::km8::kWaves);
    if ((rc = p->cb8.reserve((size_t)p->ktp8 * ks8 * 3 * 64 * 16 * 2)) ||
        (rc = p->cq8.reserve(sizeof(float) * (size_t)p->ktp8 * 48)) ||
        (rc = p->g8.reserve(sizeof(double) * (size_t)p->ktp8 * 48)) ||
        (rc = p->list8Count.reserve(64)) ||
        (rc = p->prm8.reserve(sizeof(cyc::km8::CenterParams))) ||
        (rc = p->scr8.reserve(sizeof(double) * 2 * (size_t)k))) {
      delete p;
      return rc;
    }
  }
  if ((p->dense_ok && (rc = p->ct.reserve(sizeof(double) * (size_t)p->d4 * p->kpad))) ||
      (rc = p->stats.reserve(sizeof(double) * ((size_t)k * (k + 1) / 2))) ||
      (rc = p->dmin.reserve(sizeof(unsigned long long) * (size_t)k)) ||
      (rc = p->slowCount.reserve(64)) || (rc = ensure_rows(p, std::max<int64_t>(max_rows, 1)))) {
    delete p;
    return rc;
  }
  *plan = p;
  return CYC_OK;
}

int cyc_kmeans_last_tiers(cyc_kmeans_plan p, int64_t* fp64_screen_rows, int64_t* exact_rows) {
  CYC_REQUIRE(p != nullptr && fp64_screen_rows && exact_rows, "arguments must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  *fp64_screen_rows = p->lastTier2;
  *exact_rows = p->lastExact;
  return CYC_OK;
}

int cyc_kmeans_last_screen(cyc_kmeans_plan p, int64_t* three_limb_rows) {
  CYC_REQUIRE(p != nullptr && three_limb_rows, "arguments must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  *three_limb_rows = p->lastLimb3;
  return CYC_OK;
}

int cyc_kmeans_last_candidates(cyc_kmeans_plan p, int64_t* candidate_rows) {
  CYC_REQUIRE(p != nullptr && candidate_rows, "arguments must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  *candidate_rows = p->lastCands;
  return CYC_OK;
}

int cyc_kmeans_last_candidates3(cyc_kmeans_plan p, int64_t* fp64_rows) {
  CYC_REQUIRE(p != nullptr && fp64_rows, "arguments must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  *fp64_rows = p->lastCands2;
  return CYC_OK;
}

int cyc_kmeans_last_refine(cyc_kmeans_plan p, int64_t* listed_rows, int64_t* full_rows,
                           int64_t* union_centers) {
  CYC_REQUIRE(p != nullptr && listed_rows && full_rows && union_centers,
              "arguments must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  *listed_rows = *full_rows = *union_centers = -1;
  if (!p->lastRefined) return CYC_OK;
  unsigned int h[3] = {0, 0, 0};
  CYC_HIP(hipMemcpy(h, p->cand1Count.ptr, sizeof(unsigned int), hipMemcpyDeviceToHost));
  CYC_HIP(hipMemcpy(h + 1, p->fullCount.ptr, 2 * sizeof(unsigned int), hipMemcpyDeviceToHost));
  *listed_rows = h[0];
  *full_rows = h[1];
  *union_centers = h[2];
  return CYC_OK;
}

int cyc_kmeans_plan_destroy(cyc_kmeans_plan plan) {
  delete plan;
  return CYC_OK;
}

int cyc_kmeans_plan_set_distance_measure(cyc_kmeans_plan p, int32_t measure) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  // DistanceMeasure.decodeFromString (DistanceMeasure.scala:241-247)
  CYC_REQUIRE(measure == CYC_DISTANCE_EUCLIDEAN || measure == CYC_DISTANCE_COSINE,
              "distanceMeasure must be one of: euclidean, cosine. " + std::to_string(measure) +
                  " provided.");
  std::lock_guard<std::mutex> g(p->mu);
  p->measure = measure;
  return CYC_OK;
}

int cyc_kmeans_stats_dev(cyc_kmeans_plan p, const double* C, double* stats_out, void* stream) {
  CYC_REQUIRE(p != nullptr && C != nullptr, "plan and centers must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  int rc;
  if (is_cos(p)) {
    // new VectorWithNorm(center): norms computed here (KMeansModel.scala:47-56)
    if ((rc = p->cosCn.reserve(sizeof(double) * (size_t)p->k))) return rc;
    const double* cn = (const double*)p->cosCn.ptr;
    hipLaunchKernelGGL(k_row_norms, dim3((unsigned)((p->k + kNormRows - 1) / kNormRows)),
                       dim3(kNormRows), 0, st, C, (int64_t)p->k, p->d, (double*)p->cosCn.ptr);
    CYC_LAUNCH_CHECK("k_row_norms");
    if ((rc = cos_enqueue(p, cn, p->k >= 2, nullptr, 0, st))) return rc;
    if (p->dense_ok && (rc = cos_transpose(p, C, st))) return rc;
    if ((rc = cos_stats(p, C, cn, st))) return rc;
  } else {
    if ((rc = require_enqueue(p, C, nullptr, 0, st))) return rc;
    if ((rc = do_stats(p, C, st))) return rc;
  }
  if (stats_out)
    CYC_HIP(hipMemcpyAsync(stats_out, p->stats.ptr, sizeof(double) * ((size_t)p->k * (p->k + 1) / 2),
                           hipMemcpyDeviceToDevice, st));
  return is_cos(p) ? cos_check(p) : require_check(p, 0);
}

int cyc_kmeans_rows_create(cyc_kmeans_plan p, const double* X, int64_t n, void* stream,
                           cyc_kmeans_rows* out) {
  CYC_REQUIRE(p != nullptr && out != nullptr, "plan and out must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(X != nullptr || n == 0, "X must not be null");
  auto* r = new cyc_kmeans_rows_s();
  r->X = X;
  r->n = n;
  r->d = p->d;
  r->usable = p->d <= cyc::km8::kMaxD && p->ktp8 > 0;
  r->cosine = is_cos(p);
  if (r->usable && n > 0) {
    int rc;
    hipStream_t st = cyc::as_stream(stream);
    if ((rc = r->img.reserve((size_t)n * cyc::km8::image_row_bytes(p->d))) ||
        (rc = r->meta.reserve(sizeof(int2) * (size_t)n))) {
      delete r;
      return rc;
    }
    if (r->cosine) {
      // the image of x / |x|, and |x / |x|| for the screen's margins
      cyc::DeviceBuffer xn;
      if ((rc = r->unorm.reserve(sizeof(double) * (size_t)n)) ||
          (rc = xn.reserve(sizeof(double) * (size_t)n))) {
        delete r;
        return rc;
      }
      hipLaunchKernelGGL(k_row_norms, dim3((unsigned)((n + kNormRows - 1) / kNormRows)),
                         dim3(kNormRows), 0, st, X, n, p->d, (double*)xn.ptr);
      CYC_LAUNCH_CHECK("k_row_norms");
      rc = cyc::km8::rows_quantize(X, n, p->d, r->img.ptr, (int2*)r->meta.ptr, st,
                                   (const double*)xn.ptr, (double*)r->unorm.ptr);
      if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = CYC_ERR_HIP;   // xn freed here
    } else {
      // with the image, the norms in any summation order (a wave sum): what
      // the screens need when the caller passes no norms (accumulate_dev)
      if ((rc = r->unorm.reserve(sizeof(double) * (size_t)n))) {
        delete r;
        return rc;
      }
      rc = cyc::km8::rows_quantize(X, n, p->d, r->img.ptr, (int2*)r->meta.ptr, st, nullptr,
                                   (double*)r->unorm.ptr);
    }
    if (rc) {
      delete r;
      return rc;
    }
  }
  *out = r;
  return CYC_OK;
}

int cyc_kmeans_rows_destroy(cyc_kmeans_rows rows) {
  delete rows;
  return CYC_OK;
}

int64_t cyc_kmeans_rows_bytes(cyc_kmeans_rows rows) {
  return rows ? (int64_t)(rows->img.bytes + rows->meta.bytes) : 0;
}

int cyc_kmeans_rows_set_bounds(cyc_kmeans_rows rows, int32_t enable) {
  CYC_REQUIRE(rows != nullptr, "rows must not be null");
  rows->bEnabled = enable != 0;
  rows->bValid = false;   // a re-enabled fit starts from a full screen
  return CYC_OK;
}

int cyc_kmeans_rows_set_incremental(cyc_kmeans_rows rows, int32_t enable) {
  CYC_REQUIRE(rows != nullptr, "rows must not be null");
  rows->iEnabled = enable != 0;
  rows->iValid = false;   // the next call runs the full pass
  return CYC_OK;
}

int cyc_kmeans_rows_incremental_info(cyc_kmeans_rows rows, int64_t* incremental_calls,
                                     int64_t* moved_rows) {
  CYC_REQUIRE(rows != nullptr && incremental_calls != nullptr && moved_rows != nullptr,
              "arguments must not be null");
  unsigned long long cum[2] = {0, 0};
  if (rows->iCum.ptr) {
    CYC_HIP(hipDeviceSynchronize());
    CYC_HIP(hipMemcpy(cum, rows->iCum.ptr, sizeof(cum), hipMemcpyDeviceToHost));
  }
  *incremental_calls = (int64_t)cum[1];
  *moved_rows = (int64_t)cum[0];
  return CYC_OK;
}

int cyc_kmeans_rows_bounds_rechecked(cyc_kmeans_rows rows, int64_t* rechecked_rows) {
  CYC_REQUIRE(rows != nullptr && rechecked_rows != nullptr, "arguments must not be null");
  unsigned long long cum = 0;
  if (rows->bRcCum.ptr) {
    CYC_HIP(hipDeviceSynchronize());
    CYC_HIP(hipMemcpy(&cum, rows->bRcCum.ptr, sizeof(cum), hipMemcpyDeviceToHost));
  }
  *rechecked_rows = (int64_t)cum;
  return CYC_OK;
}

int cyc_kmeans_rows_bounds_info(cyc_kmeans_rows rows, int64_t* calls, int64_t* screened_rows) {
  CYC_REQUIRE(rows != nullptr && calls != nullptr && screened_rows != nullptr,
              "arguments must not be null");
  unsigned long long cum = 0;
  if (rows->bCum.ptr) {
    CYC_HIP(hipDeviceSynchronize());   // the counter is added on the callers' streams
    CYC_HIP(hipMemcpy(&cum, rows->bCum.ptr, sizeof(cum), hipMemcpyDeviceToHost));
  }
  *calls = rows->bCalls;
  *screened_rows = rows->bFullRows + (int64_t)cum;
  return CYC_OK;
}

namespace {
int check_rows(cyc_kmeans_plan p, cyc_kmeans_rows rows, const double* X, int64_t n) {
  CYC_REQUIRE(rows == nullptr || (rows->X == X && rows->n == n && rows->d == p->d),
              "the row image was built for other rows (cyc_kmeans_rows_create)");
  CYC_REQUIRE(rows == nullptr || rows->cosine == is_cos(p),
              "the row image was built for another distance measure");
  return CYC_OK;
}
}  // namespace

int cyc_kmeans_assign_dev(cyc_kmeans_plan p, const double* X, const double* xnorm,
                          cyc_kmeans_rows rows, int64_t n, const double* C, const double* cnorm,
                          int32_t* assign, double* cost, int64_t* n_exact_out, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(assign != nullptr && cost != nullptr, "assign and cost must not be null");
  if (n_exact_out) *n_exact_out = 0;
  if (n == 0) return CYC_OK;
  if (int rc = check_rows(p, rows, X, n)) return rc;
  if (!p->dense_ok) {
    cyc::set_error("d > 1240 is not supported by the LDS-resident assign kernel (dense rows)");
    return CYC_ERR_UNSUPPORTED;
  }
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  int rc = ensure_rows(p, n);
  if (rc) return rc;
  if (is_cos(p)) {
    if ((rc = cos_enqueue(p, cnorm, true, xnorm, n, st)) ||
        (rc = cos_assign(p, X, xnorm, rows, n, C, cnorm, assign, nullptr, n_exact_out, st, false)) ||
        (rc = cyc::kmcos::row_cost(X, n, p->d, C, cnorm, xnorm, assign, cost, st)))
      return rc;
    return cos_check(p);
  }
  if ((rc = require_enqueue(p, C, xnorm, n, st))) return rc;
  if ((rc = do_assign(p, X, xnorm, rows, n, C, cnorm, assign, nullptr, n_exact_out, st))) return rc;
  hipLaunchKernelGGL(k_row_cost, dim3((unsigned)((n + kNormRows - 1) / kNormRows)),
                     dim3(kNormRows), 0, st, X, n, p->d, C,
                     (const int32_t*)assign, cost);
  CYC_LAUNCH_CHECK("k_row_cost");
  return require_check(p, n);
}

int cyc_kmeans_point_cost_dev(cyc_kmeans_plan p, const double* X, const double* xnorm,
                              cyc_kmeans_rows rows, int64_t n, const double* C,
                              const double* cnorm, int32_t* assign, double* cost, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(assign != nullptr && cost != nullptr, "assign and cost must not be null");
  if (n == 0) return CYC_OK;
  if (int rc = check_rows(p, rows, X, n)) return rc;
  if (!p->dense_ok) {
    cyc::set_error("d > 1240 is not supported by the LDS-resident assign kernel (dense rows)");
    return CYC_ERR_UNSUPPORTED;
  }
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  int rc = ensure_rows(p, n);
  if (rc) return rc;
  if (is_cos(p)) {
    if ((rc = cos_enqueue(p, cnorm, true, xnorm, n, st)) ||
        (rc = cos_assign(p, X, xnorm, rows, n, C, cnorm, assign, nullptr, nullptr, st, true)) ||
        (rc = cyc::kmcos::row_cost(X, n, p->d, C, cnorm, xnorm, assign, cost, st)))
      return rc;
    // a row no center beats +Infinity for keeps it (:136-148)
    hipLaunchKernelGGL(k_nostats_cost_fix, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                       cost);
    CYC_LAUNCH_CHECK("k_nostats_cost_fix");
    return cos_check(p);
  }
  // the fp64 screen reads the transposed centers, which cyc_kmeans_stats_dev
  // would otherwise build: no statistics are needed here
  const int64_t total = (int64_t)p->d4 * p->kpad;
  hipLaunchKernelGGL(k_center_transpose, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     C, p->k, p->d, p->d4, p->kpad, (double*)p->ct.ptr);
  CYC_LAUNCH_CHECK("k_center_transpose");
  if ((rc = do_assign(p, X, xnorm, rows, n, C, cnorm, assign, nullptr, nullptr, st, true)))
    return rc;
  hipLaunchKernelGGL(k_row_cost, dim3((unsigned)((n + kNormRows - 1) / kNormRows)),
                     dim3(kNormRows), 0, st, X, n, p->d, C,
                     (const int32_t*)assign, cost);
  CYC_LAUNCH_CHECK("k_row_cost");
  hipLaunchKernelGGL(k_nostats_cost_fix, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                     cost);
  CYC_LAUNCH_CHECK("k_nostats_cost_fix");
  return CYC_OK;
}

int cyc_kmeans_accumulate_dev(cyc_kmeans_plan p, const double* X, const double* xnorm,
                              cyc_kmeans_rows rows, const double* weights, int64_t n,
                              const double* C, const double* cnorm, double* sums, double* wsum,
                              double* cost_sum, int32_t* assign, double* cost, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(sums && wsum && cost_sum, "sums, wsum and cost_sum must not be null");
  if (n == 0) return CYC_OK;
  if (int rc = check_rows(p, rows, X, n)) return rc;
  if (!p->dense_ok) {
    cyc::set_error("d > 1240 is not supported by the LDS-resident assign kernel (dense rows)");
    return CYC_ERR_UNSUPPORTED;
  }
  // xnorm == NULL: the row image's norms for the screens (Euclidean), the
  // reference's own norms computed where its loop needs them (k_assign_exact)
  const bool approxNorm = xnorm == nullptr;
  CYC_REQUIRE(!approxNorm || (rows && rows->usable && !rows->cosine && rows->unorm.ptr),
              "xnorm may be null only with a Euclidean row image (cyc_kmeans_rows_create)");
  if (approxNorm) xnorm = (const double*)rows->unorm.ptr;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  const int k = p->k, d = p->d;
  int rc = ensure_rows(p, n);
  if (rc) return rc;
  // carried bounds: the assignment lives in the row image's state and is
  // copied to the caller's array after the screen
  const bool useBnd = bounds_on(p, rows);
  int32_t* const userAssign = assign;
  if (useBnd) {
    assign = (int32_t*)nullptr;
  } else if (!assign) {
    if ((rc = p->assignTmp.reserve(sizeof(int32_t) * (size_t)n))) return rc;
    assign = (int32_t*)p->assignTmp.ptr;
  }
  const bool cosm = is_cos(p);
  if (cosm) {
    if ((rc = cos_enqueue(p, cnorm, true, xnorm, n, st)) || (rc = cos_stats(p, C, cnorm, st)) ||
        (rc = cos_assign(p, X, xnorm, rows, n, C, cnorm, assign, nullptr, nullptr, st, false)))
      return rc;
  } else {
    if ((rc = require_enqueue(p, C, xnorm, n, st))) return rc;
    if ((rc = do_stats(p, C, st))) return rc;
    cyc::km8::Bounds bd{};
    if (useBnd) {
      if ((rc = bounds_prepare(p, rows, C, xnorm, n, st, bd))) return rc;
      assign = (int32_t*)rows->bAssign.ptr;
    }
    if ((rc = do_assign(p, X, xnorm, rows, n, C, cnorm, assign, nullptr, nullptr, st, false,
                        useBnd ? &bd : nullptr, approxNorm)))
      return rc;
    if (useBnd) {
      rows->bValid = true;
      rows->bk = k;
      ++rows->bCalls;
      if (userAssign)
        CYC_HIP(hipMemcpyAsync(userAssign, assign, sizeof(int32_t) * (size_t)n,
                               hipMemcpyDeviceToDevice, st));
    }
  }
  const int nj = (d + 255) / 256;
  // incremental cluster sums (k_inc_*): with the carried bounds, unit
  // weights and no per-row costs asked for
  const bool useInc = useBnd && inc_on(rows) && !cost && !weights && nj <= 4;
  if (rows && !useInc) rows->iValid = false;
  if (useInc) {
    if ((rc = inc_accumulate(p, rows, X, xnorm, assign, n, C, sums, wsum, cost_sum, st)))
      return rc;
    rc = require_check(p, n, approxNorm ? X : nullptr);
    rows->iValid = rc == CYC_OK;
    rows->ik = k;
    return rc;
  }
  // d > 1024: per-row costs first (k_chunk_sums fuses them for d <= 1024);
  // cosine: always (the cost is a ddot, summed per row)
  if (cosm) {
    if (!cost) {
      if ((rc = p->costTmp.reserve(sizeof(double) * (size_t)n))) return rc;
      cost = (double*)p->costTmp.ptr;
    }
    if ((rc = cyc::kmcos::row_cost(X, n, d, C, cnorm, xnorm, assign, cost, st))) return rc;
  } else if (nj > 4) {
    if (!cost) {
      if ((rc = p->costTmp.reserve(sizeof(double) * (size_t)n))) return rc;
      cost = (double*)p->costTmp.ptr;
    }
    hipLaunchKernelGGL(k_row_cost, dim3((unsigned)((n + kNormRows - 1) / kNormRows)),
                     dim3(kNormRows), 0, st, X, n, d, C,
                       (const int32_t*)assign, cost);
    CYC_LAUNCH_CHECK("k_row_cost");
  }

  int64_t maxChunks = 0;
  if ((rc = sort_clusters(p, assign, n, d, st, maxChunks))) return rc;
  // Number of chunks is data dependent; launch the upper bound and let the
  // surplus blocks (ch >= chunkStart[k]) exit.
  if (cosm) {
    if ((rc = cyc::kmcos::chunk_sums(X, d, weights, xnorm, cost, (const int32_t*)p->perm.ptr,
                                     (const int64_t*)p->cstart.ptr,
                                     (const int64_t*)p->chunkStart.ptr, k, maxChunks,
                                     (double*)p->part.ptr, (double*)p->pw.ptr,
                                     (double*)p->pc.ptr, st)))
      return rc;
  } else {
    cyc::KernelTimer timer("k_chunk_sums", st);
    const dim3 grid((unsigned)maxChunks);
#define CYC_CS(NJ)                                                                              \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_chunk_sums<NJ>), grid, dim3(256), 0, st, X, d, weights, C, \
                     (const int32_t*)p->perm.ptr, (const int64_t*)p->cstart.ptr,               \
                     (const int64_t*)p->chunkStart.ptr, k, (double*)p->part.ptr,               \
                     (double*)p->pw.ptr, (double*)p->pc.ptr, cost)
#define CYC_CSF(NJ)                                                                              \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_chunk_sums_fast<NJ>), grid, dim3(256), 0, st, X, d, weights, \
                     C, (const int32_t*)p->perm.ptr, (const int64_t*)p->cstart.ptr,             \
                     (const int64_t*)p->chunkStart.ptr, k, (double*)p->part.ptr,                \
                     (double*)p->pw.ptr, (double*)p->pc.ptr, (const double*)nullptr,             \
                     (double*)nullptr, (const int*)nullptr)
    if (!cost && nj == 1) CYC_CSF(1);
    else if (!cost && nj == 2) CYC_CSF(2);
    else if (!cost && nj <= 4) CYC_CSF(4);
    else if (nj == 1) CYC_CS(1);
    else if (nj == 2) CYC_CS(2);
    else if (nj <= 4) CYC_CS(4);
    else
      hipLaunchKernelGGL(k_chunk_sums_nocost, grid, dim3(256), 0, st, X, d, weights,
                         (const double*)cost, (const int32_t*)p->perm.ptr,
                         (const int64_t*)p->cstart.ptr, (const int64_t*)p->chunkStart.ptr, k,
                         (double*)p->part.ptr, (double*)p->pw.ptr, (double*)p->pc.ptr);
#undef CYC_CS
#undef CYC_CSF
    CYC_LAUNCH_CHECK("k_chunk_sums");
  }
  hipLaunchKernelGGL(k_reduce_clusters, dim3(k), dim3(256), 0, st, (const double*)p->part.ptr,
                     (const double*)p->pw.ptr, (const double*)p->pc.ptr,
                     (const int64_t*)p->chunkStart.ptr, d, sums, wsum, (double*)p->ccost.ptr,
                     (const double*)nullptr, (double*)nullptr, (double*)nullptr, (double*)nullptr,
                     (const int*)nullptr);
  CYC_LAUNCH_CHECK("k_reduce_clusters");
  hipLaunchKernelGGL(k_cost_total, dim3(1), dim3(256), 0, st, (const double*)p->ccost.ptr, k,
                     cost_sum, (const int*)nullptr);
  CYC_LAUNCH_CHECK("k_cost_total");
  return cosm ? cos_check(p) : require_check(p, n, approxNorm ? X : nullptr);
}

int cyc_kmeans_update_dev(cyc_kmeans_plan p, double* C, double* cnorm, const double* sums,
                          const double* wsum, double epsilon, int32_t* converged_out,
                          void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(epsilon >= 0, "epsilon must be nonnegative");
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  if (converged_out) CYC_HIP(hipMemsetD32Async((hipDeviceptr_t)converged_out, 1, 1, st));
  if (is_cos(p))
    return cyc::kmcos::update(C, cnorm, sums, wsum, p->k, p->d, epsilon, converged_out, st);
  hipLaunchKernelGGL(k_update_centers, dim3((unsigned)p->k), dim3(64),
                     p->d <= kUpdLds ? sizeof(double) * 2 * (size_t)p->d : 0, st, C, cnorm, sums, wsum, p->k, p->d,
                     epsilon * epsilon, converged_out);
  CYC_LAUNCH_CHECK("k_update_centers");
  return CYC_OK;
}


// ---------------------------------------------------------------------------
// ClusteringEvaluator's Silhouette (ml/evaluation/ClusteringMetrics.scala,
// silhouette.hpp): the plan's measure picks SquaredEuclideanSilhouette
// (CYC_DISTANCE_EUCLIDEAN) or CosineSilhouette.
// ---------------------------------------------------------------------------
namespace {

// pred in [0, k) and checkNonNegativeWeight over the rows (host sync).
int sil_check(cyc_kmeans_plan p, const int32_t* pred, const double* w, int64_t n,
              hipStream_t st) {
  int rc;
  if ((rc = p->silFlags.reserve(16))) return rc;
  unsigned int* bad = (unsigned int*)p->silFlags.ptr;
  unsigned long long* badW = (unsigned long long*)((char*)p->silFlags.ptr + 8);
  CYC_HIP(hipMemsetAsync(bad, 0, 8, st));
  CYC_HIP(hipMemsetAsync(badW, 0xff, 8, st));
  if ((rc = cyc::silh::check_pred(pred, w, n, p->k, bad, badW, st))) return rc;
  unsigned long long h[2] = {0, 0};
  CYC_HIP(hipMemcpyAsync(h, p->silFlags.ptr, 16, hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  if ((unsigned int)h[0] != 0u) {
    cyc::set_error("requirement failed: predictions must lie in [0, k) for k = " +
                   std::to_string(p->k));
    return CYC_ERR_INVALID_ARG;
  }
  if (h[1] != ~0ull) {
    double v = 0.0;
    CYC_HIP(hipMemcpy(&v, w + h[1], sizeof(double), hipMemcpyDeviceToHost));
    // ml/functions.scala:91
    cyc::set_error("requirement failed: illegal weight value: " + cyc::java_double(v) +
                   ". weight must be >= 0.0.");
    return CYC_ERR_INVALID_ARG;
  }
  return CYC_OK;
}

// Vectors.norm(features, 2.0) per row (given, or into the plan's buffer).
int sil_norms(cyc_kmeans_plan p, const double* X, const double* xnorm, int64_t n, hipStream_t st,
              const double*& out) {
  if (xnorm) {
    out = xnorm;
    return CYC_OK;
  }
  int rc;
  if ((rc = p->silNorms.reserve(sizeof(double) * (size_t)n))) return rc;
  if ((rc = cyc_row_norms_dev(X, n, p->d, (double*)p->silNorms.ptr, st))) return rc;
  out = (const double*)p->silNorms.ptr;
  return CYC_OK;
}

}  // namespace

int cyc_kmeans_silhouette_stats_dev(cyc_kmeans_plan p, const double* X, const double* xnorm,
                                    int64_t n, const int32_t* pred, const double* weights,
                                    double* stats, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(stats != nullptr, "stats must not be null");
  if (n == 0) return CYC_OK;
  CYC_REQUIRE(X != nullptr && pred != nullptr, "X and pred must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  int rc;
  const double* xn = nullptr;
  if ((rc = sil_check(p, pred, weights, n, st)) || (rc = sil_norms(p, X, xnorm, n, st, xn)))
    return rc;
  int64_t maxChunks = 0;
  if ((rc = sort_clusters(p, pred, n, p->d, st, maxChunks))) return rc;
  if ((rc = cyc::silh::chunk_sums(X, p->d, weights, xn, is_cos(p), (const int32_t*)p->perm.ptr,
                                  (const int64_t*)p->cstart.ptr,
                                  (const int64_t*)p->chunkStart.ptr, p->k, maxChunks, kChunkRows,
                                  (double*)p->part.ptr, (double*)p->pw.ptr, (double*)p->pc.ptr,
                                  st)))
    return rc;
  return cyc::silh::fold((const double*)p->part.ptr, (const double*)p->pw.ptr,
                         (const double*)p->pc.ptr, (const int64_t*)p->cstart.ptr,
                         (const int64_t*)p->chunkStart.ptr, p->d, p->k, stats, st);
}

int cyc_kmeans_silhouette_score_dev(cyc_kmeans_plan p, const double* X, const double* xnorm,
                                    int64_t n, const int32_t* pred, const double* weights,
                                    const double* stats, double* partial, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(stats != nullptr && partial != nullptr, "stats and partial must not be null");
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  const int k = p->k, d = p->d;
  // clustersStatsMap.size > 1 (ClusteringMetrics.scala:391 / :532): the
  // clusters with rows, over every rank's rows once stats are merged
  std::vector<double> cnt((size_t)k);
  CYC_HIP(hipMemcpyAsync(cnt.data(), stats + (int64_t)k * d + 2 * (int64_t)k,
                         sizeof(double) * (size_t)k, hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  int present = 0;
  for (int c = 0; c < k; ++c) present += cnt[(size_t)c] > 0.0 ? 1 : 0;
  if (present <= 1) {
    cyc::set_error("assertion failed: Number of clusters must be greater than one.");
    return CYC_ERR_ASSERTION;
  }
  if (n == 0) return CYC_OK;
  CYC_REQUIRE(X != nullptr && pred != nullptr, "X and pred must not be null");
  int rc;
  const double* xn = nullptr;
  if ((rc = sil_check(p, pred, weights, n, st)) || (rc = sil_norms(p, X, xnorm, n, st, xn)))
    return rc;
  if ((rc = p->silPart.reserve(sizeof(double) * 2 * (size_t)((n + 63) / 64)))) return rc;
  return cyc::silh::score(X, xn, n, d, pred, weights, k, is_cos(p), stats,
                          (double*)p->silPart.ptr, partial, st);
}


int cyc_row_norms_csr_dev(const int64_t* rowptr, const double* vals, int64_t n, double* norms,
                          void* stream) {
  CYC_REQUIRE(n >= 0 && (n == 0 || (rowptr && norms)), "n >= 0 and non-null buffers");
  if (n == 0) return CYC_OK;
  hipLaunchKernelGGL(k_row_norms_csr, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     cyc::as_stream(stream), rowptr, vals, n, norms);
  CYC_LAUNCH_CHECK("k_row_norms_csr");
  return CYC_OK;
}

namespace {
int sparse_assign(cyc_kmeans_plan p, const int64_t* rowptr, const int32_t* colidx,
                  const double* vals, const double* xnorm, int64_t n, const double* C,
                  const double* cnorm, int32_t* assign, double* cost, hipStream_t st,
                  bool nostats = false) {
  const unsigned grid = (unsigned)std::min<int64_t>((n + 3) / 4, 8192);
  cyc::KernelTimer timer("k_kmeans_assign_sparse", st);
  hipLaunchKernelGGL(k_assign_sparse, dim3(grid), dim3(256), 0, st, rowptr, colidx, vals, xnorm,
                     n, p->d, C, cnorm, p->k, nostats ? nullptr : (const double*)p->stats.ptr,
                     assign, cost);
  CYC_LAUNCH_CHECK("k_assign_sparse");
  return CYC_OK;
}
}  // namespace

int cyc_kmeans_assign_csr_dev(cyc_kmeans_plan p, const int64_t* rowptr, const int32_t* colidx,
                              const double* vals, const double* xnorm, int64_t n, const double* C,
                              const double* cnorm, int32_t* assign, double* cost, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(assign != nullptr && cost != nullptr, "assign and cost must not be null");
  if (n == 0) return CYC_OK;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  int rc;
  if (is_cos(p)) {
    if ((rc = cos_enqueue(p, cnorm, true, xnorm, n, st)) ||
        (rc = cyc::kmcos::assign_sparse(rowptr, colidx, vals, xnorm, n, p->d, C, cnorm, p->k,
                                        (const double*)p->stats.ptr, assign, cost, st)))
      return rc;
    return cos_check(p);
  }
  if ((rc = require_enqueue(p, C, xnorm, n, st))) return rc;
  if ((rc = sparse_assign(p, rowptr, colidx, vals, xnorm, n, C, cnorm, assign, cost, st)))
    return rc;
  return require_check(p, n);
}

int cyc_kmeans_point_cost_csr_dev(cyc_kmeans_plan p, const int64_t* rowptr,
                                  const int32_t* colidx, const double* vals, const double* xnorm,
                                  int64_t n, const double* C, const double* cnorm,
                                  int32_t* assign, double* cost, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(assign != nullptr && cost != nullptr, "assign and cost must not be null");
  if (n == 0) return CYC_OK;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  if (is_cos(p)) {
    int rc;
    if ((rc = cos_enqueue(p, cnorm, true, xnorm, n, st)) ||
        (rc = cyc::kmcos::assign_sparse(rowptr, colidx, vals, xnorm, n, p->d, C, cnorm, p->k,
                                        nullptr, assign, cost, st)))
      return rc;
    hipLaunchKernelGGL(k_nostats_cost_fix, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                       cost);
    CYC_LAUNCH_CHECK("k_nostats_cost_fix");
    return cos_check(p);
  }
  return sparse_assign(p, rowptr, colidx, vals, xnorm, n, C, cnorm, assign, cost, st, true);
}

int cyc_kmeans_accumulate_csr_dev(cyc_kmeans_plan p, const int64_t* rowptr,
                                  const int32_t* colidx, const double* vals, const double* xnorm,
                                  const double* weights, int64_t n, const double* C,
                                  const double* cnorm, double* sums, double* wsum,
                                  double* cost_sum, int32_t* assign, double* cost, void* stream) {
  CYC_REQUIRE(p != nullptr, "plan must not be null");
  CYC_REQUIRE(n >= 0, "n >= 0");
  CYC_REQUIRE(sums && wsum && cost_sum, "sums, wsum and cost_sum must not be null");
  if (n == 0) return CYC_OK;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  int rc;
  if (!assign) {
    if ((rc = p->assignTmp.reserve(sizeof(int32_t) * (size_t)n))) return rc;
    assign = (int32_t*)p->assignTmp.ptr;
  }
  if (!cost) {
    if ((rc = p->costTmp.reserve(sizeof(double) * (size_t)n))) return rc;
    cost = (double*)p->costTmp.ptr;
  }
  if (is_cos(p)) {
    if ((rc = cos_enqueue(p, cnorm, true, xnorm, n, st)) || (rc = cos_stats(p, C, cnorm, st)) ||
        (rc = cyc::kmcos::assign_sparse(rowptr, colidx, vals, xnorm, n, p->d, C, cnorm, p->k,
                                        (const double*)p->stats.ptr, assign, cost, st)) ||
        (rc = cyc::kmsparse::cluster_sums(rowptr, colidx, vals, weights, xnorm, n, p->d, p->k,
                                          assign, cost, sums, wsum, cost_sum, st)))
      return rc;
    return cos_check(p);
  }
  if ((rc = require_enqueue(p, C, xnorm, n, st))) return rc;
  if ((rc = do_stats(p, C, st))) return rc;
  if ((rc = sparse_assign(p, rowptr, colidx, vals, xnorm, n, C, cnorm, assign, cost, st)))
    return rc;
  if ((rc = cyc::kmsparse::cluster_sums(rowptr, colidx, vals, weights, nullptr, n, p->d, p->k,
                                        assign, cost, sums, wsum, cost_sum, st)))
    return rc;
  return require_check(p, n);
}

}  // extern "C"
