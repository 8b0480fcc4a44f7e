// logistic.hip -- LogisticRegression block aggregators on gfx950 (MI355X).
//
// Binary:      ml/optim/aggregator/BinaryLogisticBlockAggregator.scala:81-145
// Multinomial: ml/optim/aggregator/MultinomialLogisticBlockAggregator.scala:101-189
// Merge:       DifferentiableLossAggregator.scala:49-59 (gradientSum, lossSum,
//              weightSum add up; done here in a fixed order, deterministic
//              except the sparse binary gradient, see below).
//
// The device holds all blocks of a shard as one matrix (InstanceBlock rows
// concatenated: dense row-major n x F, or CSR); one call is the whole
// treeAggregate seqOp over the shard.
//
// Kernels
//   k_binlog_dense<FPL>  HBM-bound: one wave per row stream, each lane holds
//                        FPL coefficients and FPL gradient accumulators in
//                        registers; margin by a fixed-shape wave reduction,
//                        loss/multiplier epilogue, grad += mult * x.  One pass
//                        over X.  Per-wave partials folded in wave order.
//   k_binlog_csr         one wave per row: coef gathered by column index,
//                        gradient scattered with hardware fp64 atomics
//                        (global_atomic_add_f64).  One pass over the CSR.
//   k_mlr_margins<CT>    margins = X W^T on fp64 MFMA (16x16x4), X staged in
//                        LDS 64 x 64 at a time, W (C x F, 410 KB) read from
//                        L2; softmax / loss / multiplier epilogue in
//                        registers (cross-lane max and sum); writes the
//                        multiplier matrix (n x CP) and per-wave partials.
//   k_mlr_grad<CT>       grad^T (CP x F) = mult^T X on fp64 MFMA, split-K
//                        over rows, 16-row chunks of both operands in LDS,
//                        partial tiles to slabs folded in fixed order.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <mutex>

#include "binary_rows.hpp"
#include "common.hpp"
#include "tiles.hpp"

namespace {

using cyc::bin_row;
using cyc::log1p_exp;
using cyc::row_margin;

__device__ __forceinline__ double wave_sum_bcast(double s) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  return __shfl(s, 0);  // every lane takes lane 0's association order
}

template <int FPL>
__global__ __launch_bounds__(256) void k_binlog_dense(
    const double* __restrict__ X, const double* __restrict__ labels,
    const double* __restrict__ weights, int64_t n, int F, const double* __restrict__ coef,
    int fitIntercept, int kind, double offset, double lscale, double sigma, double eps, int64_t rowsPerWave, double* __restrict__ slabG,
    double* __restrict__ slabS) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = gw * rowsPerWave;
  const int64_t r1 = min<int64_t>(n, r0 + rowsPerWave);
  double cf[FPL], g[FPL];
#pragma unroll
  for (int j = 0; j < FPL; ++j) {
    const int f = lane + 64 * j;
    cf[j] = f < F ? coef[f] : 0.0;
    g[j] = 0.0;
  }
  double loss = 0.0, wsum = 0.0, msum = 0.0, sgs = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const double* xr = X + r * F;
    double x[FPL];
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < FPL; ++j) {
      const int f = lane + 64 * j;
      x[j] = f < F ? xr[f] : 0.0;
      s += x[j] * cf[j];
    }
    const double dot = wave_sum_bcast(s);
    const double margin = row_margin(kind, fitIntercept, offset, lscale, labels[r], dot);
    const double w = weights ? weights[r] : 1.0;
    const double mult = bin_row(kind, margin, w, labels[r], loss, wsum, sgs, sigma, eps);
    msum += mult;
    if (mult != 0.0) {
#pragma unroll
      for (int j = 0; j < FPL; ++j) g[j] += mult * x[j];
    }
  }
#pragma unroll
  for (int j = 0; j < FPL; ++j) {
    const int f = lane + 64 * j;
    if (f < F) slabG[gw * F + f] = g[j];
  }
  if (lane == 0) {
    slabS[gw * 4 + 0] = loss;
    slabS[gw * 4 + 1] = wsum;
    slabS[gw * 4 + 2] = msum;
    slabS[gw * 4 + 3] = sgs;
  }
}

__global__ __launch_bounds__(256) void k_binlog_csr(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const double* __restrict__ vals, const double* __restrict__ labels,
    const double* __restrict__ weights, int64_t n, const double* __restrict__ coef,
    int fitIntercept, int kind, double offset, double lscale, double sigma, double eps, int64_t rowsPerWave, double* __restrict__ gradAcc,
    double* __restrict__ slabS) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = gw * rowsPerWave;
  const int64_t r1 = min<int64_t>(n, r0 + rowsPerWave);
  double loss = 0.0, wsum = 0.0, msum = 0.0, sgs = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t p0 = rowptr[r], p1 = rowptr[r + 1];
    // first 64 nonzeros stay in registers for the scatter
    const int64_t q = p0 + lane;
    double v0 = 0.0;
    int c0 = 0;
    if (q < p1) {
      v0 = vals[q];
      c0 = colidx[q];
    }
    double s = (q < p1) ? v0 * coef[c0] : 0.0;
    for (int64_t p = q + 64; p < p1; p += 64) s += vals[p] * coef[colidx[p]];
    const double dot = wave_sum_bcast(s);
    const double margin = row_margin(kind, fitIntercept, offset, lscale, labels[r], dot);
    const double w = weights ? weights[r] : 1.0;
    const double mult = bin_row(kind, margin, w, labels[r], loss, wsum, sgs, sigma, eps);
    msum += mult;
    if (mult != 0.0) {
      if (q < p1) unsafeAtomicAdd(&gradAcc[c0], v0 * mult);
      for (int64_t p = q + 64; p < p1; p += 64) unsafeAtomicAdd(&gradAcc[colidx[p]], vals[p] * mult);
    }
  }
  if (lane == 0) {
    slabS[gw * 4 + 0] = loss;
    slabS[gw * 4 + 1] = wsum;
    slabS[gw * 4 + 2] = msum;
    slabS[gw * 4 + 3] = sgs;
  }
}

// Pass 2: gradient by columns from the CSC copy, grad[f] = sum over the
// column's rows (row order) of vals * mult[row]; one wave per column run,
// fixed-shape reduction, no atomics (deterministic).  The reference scatters
// the same products into grad[f] row by row (BLAS.scala:790-804).
__global__ __launch_bounds__(256) void k_binlog_csc_grad(
    const int64_t* __restrict__ colptr, const int32_t* __restrict__ rowidx,
    const double* __restrict__ cvals, const double* __restrict__ mult, int F,
    int colsPerWave, double* __restrict__ gradAcc) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t c0 = gw * colsPerWave;
  const int64_t c1 = min<int64_t>(F, c0 + colsPerWave);
  for (int64_t c = c0; c < c1; ++c) {
    const int64_t q0 = colptr[c], q1 = colptr[c + 1];
    double s = 0.0;
    for (int64_t q = q0 + lane; q < q1; q += 64) s += cvals[q] * mult[rowidx[q]];
    s = wave_sum_bcast(s);
    if (lane == 0) gradAcc[c] = s;
  }
}

// Pass 1, grouped: a wave takes 64 consecutive rows at a time, 8 lanes per
// row (8 rows per round, each row's nonzeros strided over its 8 lanes and
// summed by a 3-step butterfly), then hands row i's partial dot to lane i so
// the per-row epilogue (log1p/exp, BinaryLogisticBlockAggregator.scala:
// 104-122) runs once per row instead of once per lane; dots[r] receives the
// multiplier, written coalesced.
constexpr int CSR_IT = 2;   // nonzeros per lane per chunk (16 loads in flight)
constexpr int RP = 8;       // rows per pass
__global__ __launch_bounds__(256) void k_binlog_csr_mult8(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const double* __restrict__ vals, const double* __restrict__ labels,
    const double* __restrict__ weights, int64_t n, const double* __restrict__ coef,
    int fitIntercept, int kind, double offset, double lscale, double sigma, double eps,
    double* __restrict__ dots, double* __restrict__ slabS) {
  const int lane = threadIdx.x & 63, sub = lane & 7, grp = lane >> 3;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  double loss = 0.0, wsum = 0.0, msum = 0.0, sgs = 0.0;
  for (int64_t g0 = gw * 64; g0 < n; g0 += nw * 64) {
    // row bounds of the 64 rows by one coalesced load, then shuffles
    const int64_t myr = g0 + lane < n ? g0 + lane : n;
    const int64_t rp0 = rowptr[myr];
    const int64_t rp1 = rowptr[myr + 1 < n ? myr + 1 : n];
    // the 8 rounds advance together in 16-nonzero chunks (8 lanes x 2 per
    // row): each chunk issues all 16 index/value loads, then the 16 gathers,
    // then the products, so every chunk has 16 loads in flight per lane and
    // the dependent index->coefficient latency is paid once per chunk rather
    // than once per nonzero.  A lane's products still add in ascending
    // nonzero order (sub, sub+8, sub+16, ...), as the single-row loop did.
    // RP rows per pass (8 / RP passes per round group) bound the live state.
    int64_t maxlen = rp1 - rp0;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
      const int64_t o = __shfl_xor(maxlen, m);
      maxlen = o > maxlen ? o : maxlen;
    }
    double mydot = 0.0;
#pragma unroll
    for (int h = 0; h < 8; h += RP) {
      int64_t beg[RP], end[RP];
      double sr[RP];
#pragma unroll
      for (int rr = 0; rr < RP; ++rr) {
        beg[rr] = __shfl(rp0, (h + rr) * 8 + grp);
        end[rr] = __shfl(rp1, (h + rr) * 8 + grp);
        sr[rr] = 0.0;
      }
      for (int64_t k = 0; k < maxlen; k += 8 * CSR_IT) {
        int ci[RP][CSR_IT];
        double vv[RP][CSR_IT], cf[RP][CSR_IT];
#pragma unroll
        for (int rr = 0; rr < RP; ++rr)
#pragma unroll
          for (int it = 0; it < CSR_IT; ++it) {
            const int64_t p = beg[rr] + k + sub + 8 * it;
            const bool ok = p < end[rr];
            ci[rr][it] = ok ? __builtin_nontemporal_load(colidx + p) : -1;
            vv[rr][it] = ok ? __builtin_nontemporal_load(vals + p) : 0.0;
          }
#pragma unroll
        for (int rr = 0; rr < RP; ++rr)
#pragma unroll
          for (int it = 0; it < CSR_IT; ++it) cf[rr][it] = ci[rr][it] >= 0 ? coef[ci[rr][it]] : 0.0;
#pragma unroll
        for (int rr = 0; rr < RP; ++rr)
#pragma unroll
          for (int it = 0; it < CSR_IT; ++it)
            if (ci[rr][it] >= 0) sr[rr] += vv[rr][it] * cf[rr][it];
      }
#pragma unroll
      for (int rr = 0; rr < RP; ++rr) {
        double s = sr[rr];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        const double v = __shfl(s, 8 * (lane & 7));
        if ((lane >> 3) == h + rr) mydot = v;
      }
    }
    const int64_t row = g0 + lane;
    if (row < n) {
      const double margin = row_margin(kind, fitIntercept, offset, lscale, labels[row], mydot);
      const double w = weights ? weights[row] : 1.0;
      const double m = bin_row(kind, margin, w, labels[row], loss, wsum, sgs, sigma, eps);
      msum += m;
      dots[row] = m;
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    loss += __shfl_xor(loss, m);
    wsum += __shfl_xor(wsum, m);
    msum += __shfl_xor(msum, m);
    sgs += __shfl_xor(sgs, m);
  }
  if (lane == 0) {
    slabS[gw * 4 + 0] = loss;
    slabS[gw * 4 + 1] = wsum;
    slabS[gw * 4 + 2] = msum;
    slabS[gw * 4 + 3] = sgs;
  }
}

// Pass 2 over one row block of the row-blocked CSC (csc.hip): 16 lanes per
// column, products vals * mult[row] (the block's 2 MB multiplier slice stays
// in L2), fixed 4-step butterfly, gradAcc[c] = (first ? 0 : gradAcc[c]) + s.
// Deterministic: blocks in order, a block's rows in order within each lane.
constexpr int LPC = 32, IT = 1, CPG = 4;   // lanes per group of CPG columns
__global__ __launch_bounds__(256) void k_binlog_csc_grad_blk(
    const int64_t* __restrict__ colptrB, const int32_t* __restrict__ rowidx,
    const double* __restrict__ cvals, const double* __restrict__ mult, int F, int first,
    double* __restrict__ gradAcc) {
  // LPC lanes per group of CPG consecutive columns; the first LPC*IT
  // nonzeros of each column are loaded before any gather (all in flight)
  const int sub = threadIdx.x & (LPC - 1), lane = threadIdx.x & 63, gbase = lane & (64 - LPC);
  const int64_t c0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPC) * CPG;
  const int64_t ci = c0 + (sub < CPG + 1 ? sub : CPG);
  const int64_t cp = colptrB[ci < F ? ci : (int64_t)F];
  int64_t b[CPG + 1];
#pragma unroll
  for (int i = 0; i <= CPG; ++i) b[i] = __shfl(cp, gbase + i);
  int ri[CPG][IT];
  double vv[CPG][IT], mm[CPG][IT];
#pragma unroll
  for (int i = 0; i < CPG; ++i)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int64_t q = b[i] + sub + LPC * it;
      const bool ok = c0 + i < F && q < b[i + 1];
      ri[i][it] = ok ? __builtin_nontemporal_load(rowidx + q) : -1;
      vv[i][it] = ok ? __builtin_nontemporal_load(cvals + q) : 0.0;
    }
#pragma unroll
  for (int i = 0; i < CPG; ++i)
#pragma unroll
    for (int it = 0; it < IT; ++it) mm[i][it] = ri[i][it] >= 0 ? mult[ri[i][it]] : 0.0;
  double mine = 0.0;
#pragma unroll
  for (int i = 0; i < CPG; ++i) {
    double s = vv[i][0] * mm[i][0];
#pragma unroll
    for (int it = 1; it < IT; ++it) s += vv[i][it] * mm[i][it];
    if (c0 + i < F)
      for (int64_t q = b[i] + sub + LPC * IT; q < b[i + 1]; q += LPC)
        s += __builtin_nontemporal_load(cvals + q) * mult[__builtin_nontemporal_load(rowidx + q)];
#pragma unroll
    for (int m = LPC / 2; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (sub == i) mine = s;
  }
  if (sub < CPG && c0 + sub < F) gradAcc[c0 + sub] = first ? mine : gradAcc[c0 + sub] + mine;
}

// Fold per-wave scalars in wave order: out3 = {loss, wsum, msum}.
__global__ void k_fold_scalars(const double* __restrict__ slabS, int64_t waves, int width,
                               double* __restrict__ out) {
  __shared__ double sh[256];
  for (int c = 0; c < width; ++c) {
    double a = 0.0;
    const int64_t per = (waves + 255) / 256;
    const int64_t w0 = threadIdx.x * per, w1 = min<int64_t>(waves, w0 + per);
    for (int64_t w = w0; w < w1; ++w) a += slabS[w * width + c];
    sh[threadIdx.x] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int i = 0; i < 256; ++i) t += sh[i];
      out[c] = t;
    }
    __syncthreads();
  }
}

// grad[f] += sum_w slabG[w][f] (or += gradAcc[f]); then the fitWithMean
// correction (daxpy(-multiplierSum, scaledMean), :132-137) and the intercept
// (:139-142).  scal = {loss, wsum, msum}.
__global__ void k_binlog_fold(const double* __restrict__ slabG, int64_t waves,
                              const double* __restrict__ gradAcc, int F,
                              const double* __restrict__ scal, int fitIntercept, int fitWithMean,
                              int sigmaIdx, const double* __restrict__ scaledMean,
                              double* __restrict__ grad, double* __restrict__ lossSum,
                              double* __restrict__ weightSum) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  const double msum = scal[2];
  if (f < F) {
    double s = 0.0;
    if (slabG) {
      for (int64_t w = 0; w < waves; ++w) s += slabG[w * F + f];
    } else {
      s = gradAcc[f];
    }
    double gf = grad[f] + s;
    if (fitWithMean) gf = gf + (-msum) * scaledMean[f];
    grad[f] = gf;
  }
  if (f == 0) {
    if (fitIntercept) grad[F] += msum;
    if (sigmaIdx >= 0) grad[sigmaIdx] += scal[3];   // Huber :138
    *lossSum += scal[0];
    *weightSum += scal[1];
  }
}

// marginOffset (Binary :67-72): coef[F] - sum_f coef[f]*scaledMean[f]
// marginOffset: coef[F] - ddot(coef, scaledMean) (Binary :67-72, Hinge
// :62-71), or for least squares (:57-62) labelMean / labelStd - ddot(...)
// (base passed in, useBase = 1).
// One 1024-thread workgroup: thread t sums its contiguous stretch of the
// products in index order, then a fixed tree -- deterministic (the
// reference's sequential ddot order is not pinned below 1e-10 anyway).
constexpr int kOffParts = 256;                 // partial sums of the offset dot

// stage 1: part p sums the products of its contiguous range, lane-strided
// (coalesced), each thread in index order, then a fixed shuffle / wave tree
__global__ __launch_bounds__(256) void k_binlog_offset_part(const double* __restrict__ coef,
                                                            const double* __restrict__ sm, int F,
                                                            double* __restrict__ part) {
  __shared__ double sh[4];
  const int t = threadIdx.x;
  const int64_t per = ((int64_t)F + kOffParts - 1) / kOffParts;
  const int64_t f0 = blockIdx.x * per, f1 = std::min<int64_t>(F, f0 + per);
  double dd = 0.0;
  for (int64_t f = f0 + t; f < f1; f += 256) dd += coef[f] * sm[f];
  for (int m = 32; m >= 1; m >>= 1) dd += __shfl_xor(dd, m);
  if ((t & 63) == 0) sh[t >> 6] = dd;
  __syncthreads();
  if (t == 0) part[blockIdx.x] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

// stage 2: the parts in order; out = (base or intercept) - dot
__global__ void k_binlog_offset(const double* __restrict__ part, const double* __restrict__ coef,
                                int F, int useBase, double base, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < kOffParts; ++i) s += part[i];
  out[0] = (useBase ? base : coef[F]) - s;
}

// LeastSquaresBlockAggregator.effectiveCoef (:48-55): coefficient or 0.0
// where the feature's inverseStd is 0.
__global__ void k_effective_coef(const double* __restrict__ coef,
                                 const double* __restrict__ inverseStd, int F,
                                 double* __restrict__ out) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < F) out[f] = inverseStd[f] != 0 ? coef[f] : 0.0;
}

// --------------------------------------------------------- multinomial
// marginOffset (Multinomial :86-92): intercept + gemv(-1.0, linear, scaledMean)
// with netlib dgemv "N" column order.
__global__ void k_mlr_offset(const double* __restrict__ coef, const double* __restrict__ sm,
                             int F, int C, double* __restrict__ off) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double o = coef[(int64_t)C * F + c];
  for (int f = 0; f < F; ++f) {
    if (sm[f] != 0.0) {
      const double t = -1.0 * sm[f];
      o = o + t * coef[(int64_t)f * C + c];
    }
  }
  off[c] = o;
}

typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef int v2i32 __attribute__((ext_vector_type(2)));

// tools/probe/mlr_probe.hip builds k_mlr_margins with parts removed to time
// them (results then meaningless): bits 1 = X loaded for chunk 0 only, 2 = no
// softmax epilogue, 4 = no W DMA, 8 = no multiplier stores, 16 = no exp.
// 0 in the library.
#ifndef CYC_MLR_PROBE
#define CYC_MLR_PROBE 0
#endif
// k_mlr_margins: waves per workgroup; dephased workgroup pairs (see the kernel)
#ifndef CYC_MLR_NW
#define CYC_MLR_NW 8
#endif
#ifndef CYC_MLR_DEPHASE
#define CYC_MLR_DEPHASE false
#endif

// 2^(j/32), j = 0..31, correctly rounded (exp_neg's table)
__constant__ double kExp2Tab[32] = {
    1.0, 1.0218971486541166, 1.0442737824274138, 1.0671404006768237,
    1.0905077326652577, 1.1143867425958924, 1.1387886347566916, 1.1637248587775775,
    1.189207115002721, 1.215247359980469, 1.241857812073484, 1.2690509571917332,
    1.2968395546510096, 1.3252366431597413, 1.3542555469368927, 1.383909881963832,
    1.4142135623730951, 1.4451808069770467, 1.4768261459394993, 1.5091644275934228,
    1.5422108254079407, 1.5759808451078865, 1.6104903319492543, 1.645755478153965,
    1.681792830507429, 1.718619298122478, 1.7562521603732995, 1.7947090750031072,
    1.8340080864093424, 1.8741676341103, 1.9152065613971474, 1.9571441241754002};

// e^x for x <= 0 (the softmax terms m - max): x = (32 e + j) ln2/32 + r with
// |r| <= ln2/64 (Cody-Waite, a 38-bit high part), e^x = 2^e 2^(j/32) e^r,
// e^r by its degree-6 Taylor polynomial (truncation < 2^-57 relative),
// 2^(j/32) from the LDS table T: within a few ulp, against Math.exp's 1 ulp
// in the reference -- far inside the aggregator's 1e-10 bar -- at 15 f64
// VALU where the libm exp takes ~23.  Below -708.4 the result is subnormal:
// the final ldexp rounds it onto the subnormal grid (a second rounding, and
// past kd = 2^15 the reduction's high product is no longer exact: a relative
// error of ~1e-13 there), so a label whose probability is subnormal keeps
// the reference's finite -log(p).  Below -746 (where e^x rounds to 0 in any
// libm) it returns 0, so -inf gives 0; NaN stays NaN.  tests/
// test_logistic_gpu.py sweeps it against the host libm.
__device__ __forceinline__ double exp_neg(double x, const double* __restrict__ T) {
  // a select, not a branch (a branch here splits the softmax epilogue's wave)
  const bool under = x < -746.0;
  x = under ? -746.0 : x;
  const double kd = __builtin_rint(x * 46.16624130844683);   // 32 / ln2
  double r = __builtin_fma(kd, -0.021660849392446835, x);
  r = __builtin_fma(kd, -5.145609244655338e-14, r);
  const int k = (int)kd;
  double q = 1.0 / 720.0;
  q = __builtin_fma(q, r, 1.0 / 120.0);
  q = __builtin_fma(q, r, 1.0 / 24.0);
  q = __builtin_fma(q, r, 1.0 / 6.0);
  q = __builtin_fma(q, r, 0.5);
  q = __builtin_fma(q, r, 1.0);
  q = __builtin_fma(q, r, 1.0);
  double e = __builtin_ldexp(T[k & 31] * q, k >> 5);
  asm volatile("" : "+v"(e));   // computed on every lane (no branch around it)
  return under ? 0.0 : e;
}

// exp_neg over an array (cyc_softmax_exp_dev: its accuracy test)
__global__ void k_softmax_exp(const double* __restrict__ x, int64_t n, double* __restrict__ out) {
  __shared__ double T[32];
  if (threadIdx.x < 32) T[threadIdx.x] = kExp2Tab[threadIdx.x];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = exp_neg(x[i], T);
}

// a row-16 DPP move of a double (both halves; all lanes active)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

constexpr int MR = 256;    // rows per margin tile, at most (8 waves x 32 rows)
constexpr int MK = 16;     // features per LDS chunk

// margins = X W^T (+ offset) for 256-row tiles, 16-feature chunks, on
// v_mfma_f64_16x16x4f64: 2 row tiles x CT class tiles of 16x16 per wave;
// softmax / loss / multiplier epilogue in registers.  Persistent over tiles,
// one 8-wave workgroup per CU.
// X goes from HBM straight into registers in the MFMA A layout -- lane (row
// r = l & 15, group g = l >> 4) holds features f0 + 4g .. 4g + 3 of its row
// for k-steps 0..3 (the contraction order within a chunk is permuted: 128
// contiguous bytes per row per chunk, two dwordx4 loads per lane per row
// tile) -- loaded one chunk ahead into a second register set: no LDS, no
// barrier for X.  W chunks (16 features x C classes, contiguous in coef,
// 12.8 KB at C = 100) are DMA'd into two LDS buffers (buffer_load ... lds,
// 1 KiB pieces spread over the waves, one chunk ahead; no registers), one
// barrier per chunk.  Padding classes read the next coefficients (finite;
// their margins are never used) or zero past the end of coef.
// (The last class tile on v_mfma_f64_4x4x4f64, as k_mlr_grad does, measured
// 4-5 % slower here at C = 100, with or without sched_barrier fences.)
// NW waves per workgroup (32 NW rows per tile; NW = 4: two workgroups per
// CU); DEPHASE: the workgroups whose index bit 0 differs from bit 8 start
// half a tile late, so the two workgroups of a CU (consecutive indices, or
// i and i + 256) run their softmax epilogues while the other one's MFMAs
// keep the matrix pipe busy.
template <int CT, int NW = 8, bool DEPHASE = false>
__global__ __launch_bounds__(64 * NW, 2) void k_mlr_margins(
    const double* __restrict__ X, const double* __restrict__ labels,
    const double* __restrict__ weights, int64_t n, int F, int C, const double* __restrict__ coef,
    const double* __restrict__ offset, double* __restrict__ mult, double* __restrict__ slabS,
    double* __restrict__ slabMS) {
  constexpr int MR = 32 * NW, MT = 64 * NW;
  constexpr int CP = CT * 16;
  static_assert(MK == 16, "the A layout covers 16 features per chunk");
  constexpr int WBUF = MK * CP + 128;   // doubles per W buffer (whole 1 KiB pieces)
  // the two W buffers, then exp_neg's table and the per-class offsets (never
  // DMA targets)
  __shared__ __attribute__((aligned(16))) double Ws[2][WBUF + 32 + CP];
  double* const expT = Ws[1] + WBUF;
  double* const offS = expT + 32;
  __shared__ double plS[MR];   // each wave's 32 label probabilities of a tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4;
  const int64_t tiles = (n + MR - 1) / MR;
  const int nch = (F + MK - 1) / MK;
  if constexpr (DEPHASE) {
    // half a tile at ~2 GHz with two waves per SIMD sharing the pipe:
    // nch chunks x 8 CT MFMAs x 64 cycles, on the 100 MHz constant clock
    if (((blockIdx.x ^ (blockIdx.x >> 8)) & 1) != 0) {
      const int64_t ticks = (int64_t)nch * 8 * CT * 64 / 20;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks)
        __builtin_amdgcn_s_sleep(32);
    }
  }
  // read after a barrier: the epilogue reads them by ds_read, so none of
  // its waits is a vmcnt that would also drain the multiplier stores
  if (threadIdx.x < 32) expT[threadIdx.x] = kExp2Tab[threadIdx.x];
  if (threadIdx.x < CP) offS[threadIdx.x] = (offset && (int)threadIdx.x < C) ? offset[threadIdx.x] : 0.0;
  double loss = 0.0, wsum = 0.0;
  double ms[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) ms[ct] = 0.0;
  // Loads go through buffer descriptors: 32-bit offsets; rows past n read
  // as zero (out-of-range offsets).  Host guarantees MR * F * 8 < 2^31 and
  // (C * F + C) * 8 < 2^31.
  constexpr int OOB = 0x7ff00000;
  const auto wR = __builtin_amdgcn_make_buffer_rsrc((void*)coef, (short)0, (C * F + C) * 8,
                                                    0x00020000);
  // pieces covering every index the B reads touch: (MK - 1) C + CP doubles
  const int wpieces = (((MK - 1) * C + CP) * 8 + 1023) / 1024;
  auto loadW = [&](int ch) {      // chunk ch's 16 x C run of coef into buffer ch & 1
    if constexpr ((CYC_MLR_PROBE & 4) != 0) return;
    double* dst = Ws[ch & 1];
    const int base = ch * MK * C * 8;
    for (int q = wave; q < wpieces; q += MT / 64)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wR, (__attribute__((address_space(3))) void*)(dst + q * 128), 16, base + q * 1024 +
          lane * 16, 0, 0, 0);
  };
  auto loadX = [&](int64_t r0, int ch, double (&x)[2][4]) {
    if constexpr ((CYC_MLR_PROBE & 1) != 0) {
      if (ch > 0) return;
    }
    const int f0 = ch * MK + 4 * g;
    const int64_t nr = min<int64_t>(MR, n - r0);
    const auto xR = __builtin_amdgcn_make_buffer_rsrc((void*)(X + r0 * F), (short)0,
                                                      (int)(nr * F * 8), 0x00020000);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int off = ((wave * 32 + t * 16 + (lane & 15)) * F + f0) * 8;
      if (f0 + 3 < F) {
        // nontemporal (aux 2): X streams through once per evaluation pass
        const v4i32 lo = __builtin_amdgcn_raw_buffer_load_b128(xR, off, 0, 2);
        const v4i32 hi = __builtin_amdgcn_raw_buffer_load_b128(xR, off + 16, 0, 2);
        x[t][0] = __builtin_bit_cast(double, (v2i32){lo[0], lo[1]});
        x[t][1] = __builtin_bit_cast(double, (v2i32){lo[2], lo[3]});
        x[t][2] = __builtin_bit_cast(double, (v2i32){hi[0], hi[1]});
        x[t][3] = __builtin_bit_cast(double, (v2i32){hi[2], hi[3]});
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[t][j] = __builtin_bit_cast(
              double, __builtin_amdgcn_raw_buffer_load_b64(xR, f0 + j < F ? off + 8 * j : OOB, 0,
                                                           0));
      }
    }
  };
  cyc_double4 acc[2][CT];
  // labL / wL: lane l holds label and weight of row 32 wave + (l & 31)
  auto epilogue = [&](int64_t r0, double labL, double wL) {
    if constexpr ((CYC_MLR_PROBE & 2) != 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) ms[ct] += acc[t][ct][0];
      wsum += lane < 32 ? 1.0 : 0.0;   // a nonzero weight for the host's check
      return;
    }
    // Epilogue: lane holds rows 32 wave + 16 t + (lane>>4) + 4r, classes
    // 16 ct + (lane & 15).  Branch-free (selects, DPP row reductions, the
    // multiplier stores through a per-tile buffer descriptor that drops rows
    // past n), so the wave never splits; the only branch is the wave-uniform
    // one into the +inf margin case.  Each row's label probability is parked
    // in LDS and the tile's 32 logs per wave run once, one row per lane.
    // l15: the lane's class within a tile, opaque to the optimizer: values derived
    // from it are recomputed per tile instead of hoisted out of the tile loop
    // into registers (which spilled)
    int l15 = lane & 15;
    asm volatile("" : "+v"(l15));
    const int64_t nr = min<int64_t>(MR, n - r0);
    const auto mR = __builtin_amdgcn_make_buffer_rsrc((void*)(mult + r0 * CP), (short)0,
                                                      (int)(nr * CP * 8), 0x00020000);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wave * 32 + t * 16 + (lane >> 4) + 4 * r;   // row within the tile
        const bool rowok = r0 + rl < n;
        double m[CT];
        // the row's max by fmax, +inf included (the reference leaves +inf
        // out of its max; a row holding one takes the branch below)
        double mx = -1.7976931348623157e308;  // Double.MinValue (Utils.scala:113)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int c = ct * 16 + l15;
          m[ct] = acc[t][ct][r] + offS[c];  // 1.0*temp + 1.0*offset (netlib dgemm)
          mx = fmax(mx, (ct < CT - 1 || c < C) ? m[ct] : mx);
        }
        mx = fmax(mx, dpp_f64<0xB1>(mx));   // quad_perm [1,0,3,2]
        mx = fmax(mx, dpp_f64<0x4E>(mx));   // quad_perm [2,3,0,1]
        mx = fmax(mx, dpp_f64<0x141>(mx));  // row_half_mirror
        mx = fmax(mx, dpp_f64<0x140>(mx));  // row_mirror
        // the probabilities replace the margins in place (p = m).  INF: the
        // wave holds a +inf margin (a wave-uniform branch, never taken on
        // finite margins): the max over the other classes, and for a row
        // holding one, probability 1 for the first such class and 0 * m for
        // the rest.
        auto softmax = [&](auto infTag) {
          constexpr bool INF = decltype(infTag)::value;
          int infc = 1 << 30;
          if constexpr (INF) {
            mx = -1.7976931348623157e308;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
              const int c = ct * 16 + l15;
              const bool valid = ct < CT - 1 || c < C;
              if (valid && m[ct] == __builtin_inf()) infc = min(infc, c);
              else if (valid && m[ct] > mx) mx = m[ct];
            }
#pragma unroll
            for (int k = 1; k < 16; k <<= 1) {
              mx = fmax(mx, __shfl_xor(mx, k));
              infc = min(infc, __shfl_xor(infc, k));
            }
          }
          const bool rowInf = INF && infc < (1 << 30);
          double sum = 0.0;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) {
            const int c = ct * 16 + l15;
            const double e = (CYC_MLR_PROBE & 16) ? (m[ct] - mx) : exp_neg(m[ct] - mx, expT);
            const double pe = (ct < CT - 1 || c < C) ? e : 0.0;
            m[ct] = rowInf ? ((c == infc) ? 1.0 : 0.0 * m[ct]) : pe;
            sum += m[ct];
          }
          // butterfly sums in which both lanes of a pair add the same two
          // values: every lane of the row ends with the same bits
          sum += dpp_f64<0xB1>(sum);
          sum += dpp_f64<0x4E>(sum);
          sum += dpp_f64<0x141>(sum);
          sum += dpp_f64<0x140>(sum);
          const double inv = 1.0 / sum;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) m[ct] = rowInf ? m[ct] : inv * m[ct];
        };
        if (__builtin_amdgcn_ballot_w64(mx == __builtin_inf()) != 0)
          softmax(std::true_type{});
        else
          softmax(std::false_type{});
        double (&p)[CT] = m;
        // unconditional shuffles: a shuffle under `rowok` made the compiler
        // wait vmcnt(0) on labL / wL at every row, draining the stores
        const int q = 16 * t + 4 * r + (lane >> 4);   // the row within the wave's 32
        const double wq = __shfl(wL, q), lq = __shfl(labL, q);
        const double w = (rowok && wq > 0) ? wq : 0.0;
        const int label = rowok ? (int)lq : 0;
        const int voff = rowok ? (rl * CP + l15) * 8 : OOB;   // rows past n: dropped
        double pl = 0.0;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) pl = (ct == (label >> 4)) ? p[ct] : pl;
        if ((lane & 15) == (label & 15)) plS[wave * 32 + q] = pl;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int c = ct * 16 + l15;
          // w p - w at the label (w * p is p at w = 1); 0 * p at w <= 0
          double mu = w * p[ct] - (c == label ? w : 0.0);
          mu = (ct < CT - 1 || c < C) && rowok ? mu : 0.0;
          if constexpr ((CYC_MLR_PROBE & 8) == 0)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i32, mu), mR,
                                                  voff + ct * 128, 0, 2);   // nontemporal
          ms[ct] += mu;
        }
        // one row group at a time: interleaving them spills
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the loss: row 32 wave + (lane & 31) on lanes 0..31
    const double pl = plS[wave * 32 + (lane & 31)];
    const double wr = (lane < 32 && r0 + wave * 32 + lane < n) ? wL : 0.0;
    wsum += wr;
    loss -= (wr > 0) ? wr * log(pl) : 0.0;
  };
  double xa[2][4], xb[2][4];
  bool pre = false;   // chunk 0 of this tile already in flight (xa, Ws[0])
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t r0 = tile * MR;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[t][ct] = cyc_double4{0.0, 0.0, 0.0, 0.0};
    if (!pre) {
      __syncthreads();   // the previous tile's last W buffer is free
      loadW(0);
    }
    loadX(r0, 0, xa);
    // chunk ch: wait for its loads, barrier (its W visible everywhere, every
    // wave past chunk ch - 1), issue chunk ch + 1's loads, multiply
    auto step = [&](int ch, double (&xc)[2][4], double (&xn)[2][4]) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (ch + 1 < nch) {
        loadX(r0, ch + 1, xn);
        loadW(ch + 1);
      }
      const double* W = Ws[ch & 1];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const double b = W[(4 * g + kk) * C + ct * 16 + (lane & 15)];
          acc[0][ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(xc[0][kk], b, acc[0][ct], 0, 0, 0);
          acc[1][ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(xc[1][kk], b, acc[1][ct], 0, 0, 0);
        }
      }
    };
    for (int ch = 0; ch < nch; ch += 2) {
      step(ch, xa, xb);
      if (ch + 1 < nch) step(ch + 1, xb, xa);
    }
    // the next tile's W chunk 0 goes out before this tile's epilogue (the X
    // registers stay free for it: prefetching X too spills at CT = 7): with
    // an even chunk count the last chunk read Ws[1], and every wave is past
    // chunk nch - 2 (Ws[0]) since the last barrier
    const int64_t next = tile + gridDim.x;
    pre = (nch % 2) == 0 && next < tiles;
    // the tile's labels and weights, loaded (unconditionally, from a
    // clamped row) before the W DMA and the stores of the epilogue
    const int64_t lr = min<int64_t>(r0 + wave * 32 + (lane & 31), n - 1);
    const double labL = labels[lr];
    const double wL = weights ? weights[lr] : 1.0;
    if (pre) loadW(0);
    epilogue(r0, labL, wL);
  }
  // per-wave partials: loss/wsum over the lanes (one row of each tile per
  // lane 0..31), multSum per class summed over the 4 row groups of the wave.
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    loss += __shfl_xor(loss, k);
    wsum += __shfl_xor(wsum, k);
  }
#pragma unroll
  for (int k = 16; k < 64; k <<= 1) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) ms[ct] += __shfl_xor(ms[ct], k);
  }
  const int64_t gw = (int64_t)blockIdx.x * (MT / 64) + wave;
  if (lane == 0) {
    slabS[gw * 2 + 0] = loss;
    slabS[gw * 2 + 1] = wsum;
  }
  if (lane < 16) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) slabMS[gw * CP + ct * 16 + lane] = ms[ct];
  }
}

constexpr int GR = 32;    // rows per chunk in the gradient GEMM
constexpr int GF = 256;   // features per workgroup

// grad^T (CP x GF per workgroup) = mult^T X over one split of rows, on
// v_mfma_f64_16x16x4f64 (8 waves x 32 features x CP classes).  Per 32-row
// chunk: the multipliers (32 x CP, contiguous) are DMA'd into one of two LDS
// buffers (buffer_load ... lds, 1 KiB pieces over the waves), X goes from
// HBM straight into registers in the MFMA B layout (lane: feature l & 15 of
// its 16-feature tile, row 4 kk + (l >> 4) of k-step kk; 128 contiguous
// bytes per row), both one chunk ahead; one barrier per chunk.
// T4 (C mod 16 in 1..4): the last class tile on v_mfma_f64_4x4x4f64, a
// quarter of the 16x16x4 cycles: 4 blocks of 4 x 4 x 4, lane 16k + 4b + i
// holding A(i, k), lane 16k + 4b + j B(k, j) of block b and lane 16i + 4b + j
// the result (measured on gfx950: tools/probe/mfma_f64_4x4.hip).  Here A =
// the 4 classes' multipliers of row k (the same for every block), B = the
// 16x16x4 X operand (block b: features 4b .. 4b + 3), so the result is class
// l >> 4, feature l & 15.
template <int CT, bool T4>
__global__ __launch_bounds__(512) void k_mlr_grad(const double* __restrict__ mult,
                                                  const double* __restrict__ X, int64_t n, int F,
                                                  int64_t rowsPerSplit, int ftiles, int splits,
                                                  double* __restrict__ slab) {
  constexpr int CP = CT * 16;
  constexpr int MB = GR * CP;                       // doubles per multiplier chunk
  constexpr int MPIECES = (MB * 8 + 1023) / 1024;
  __shared__ __attribute__((aligned(16))) double Ms[2][MPIECES * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1-D grid: block b runs on XCD b % 8; the ftiles workgroups of a split
  // share that XCD (consecutive b / 8), so the split's multipliers come from
  // HBM once and from that XCD's L2 for the other feature tiles
  const int xq = (int)blockIdx.x >> 3;
  const int ft = xq % ftiles;
  const int sp = (xq / ftiles) * 8 + ((int)blockIdx.x & 7);
  if (sp >= splits) return;   // splits padded to a multiple of 8
  const int F0 = ft * GF;
  const int64_t r0 = (int64_t)sp * rowsPerSplit;
  const int64_t r1 = min<int64_t>(n, r0 + rowsPerSplit);
  cyc_double4 acc[CT][2];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) acc[ct][0] = acc[ct][1] = cyc_double4{0.0, 0.0, 0.0, 0.0};
  double acc4[2] = {0.0, 0.0};
  // Buffer descriptors over this split's rows: 32-bit offsets, rows past the
  // split and features past F read as zero.  Host: rowsPerSplit * max(F, CP)
  // * 8 < 2^31.
  constexpr int OOB = 0x7ff00000;
  const int64_t nr = r1 > r0 ? r1 - r0 : 0;
  const auto mR = __builtin_amdgcn_make_buffer_rsrc((void*)(mult + r0 * CP), (short)0,
                                                    (int)(nr * CP * 8), 0x00020000);
  const auto xR = __builtin_amdgcn_make_buffer_rsrc((void*)(X + r0 * F), (short)0,
                                                    (int)(nr * F * 8), 0x00020000);
  const int g = lane >> 4;
  const int fcol = F0 + wave * 32 + (lane & 15);
  auto loadM = [&](int64_t rb, int buf) {
    const int base = (int)(rb - r0) * CP * 8;
    for (int q = wave; q < MPIECES; q += 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          mR, (__attribute__((address_space(3))) void*)(&Ms[buf][q * 128]), 16,
          base + q * 1024 + lane * 16, 0, 0, 0);
  };
  auto loadX = [&](int64_t rb, double (&x)[GR / 4][2]) {
    const int rowOff = (int)(rb - r0);
#pragma unroll
    for (int kk = 0; kk < GR / 4; ++kk)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int f = fcol + 16 * q;
        const int off = f < F ? ((rowOff + 4 * kk + g) * F + f) * 8 : OOB;
        x[kk][q] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xR, off, 0, 2));
      }
  };
  auto step = [&](int64_t rb, int buf, double (&xc)[GR / 4][2], double (&xn)[GR / 4][2]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // chunk rb's multipliers visible; every wave past the previous chunk
    if (rb + GR < r1) {
      loadX(rb + GR, xn);
      loadM(rb + GR, buf ^ 1);
    }
    const double* M = Ms[buf];
#pragma unroll
    for (int kk = 0; kk < GR / 4; ++kk) {
#pragma unroll
      for (int ct = 0; ct < (T4 ? CT - 1 : CT); ++ct) {
        const double a = M[(4 * kk + g) * CP + ct * 16 + (lane & 15)];
        acc[ct][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, xc[kk][0], acc[ct][0], 0, 0, 0);
        acc[ct][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, xc[kk][1], acc[ct][1], 0, 0, 0);
      }
      if constexpr (T4) {
        const double a = M[(4 * kk + g) * CP + (CT - 1) * 16 + (lane & 3)];
        acc4[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, xc[kk][0], acc4[0], 0, 0, 0);
        acc4[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, xc[kk][1], acc4[1], 0, 0, 0);
      }
    }
  };
  if (r0 < r1) {
    double xa[GR / 4][2], xb[GR / 4][2];
    loadX(r0, xa);
    loadM(r0, 0);
    for (int64_t rb = r0; rb < r1; rb += 2 * GR) {
      step(rb, 0, xa, xb);
      if (rb + GR < r1) step(rb + GR, 1, xb, xa);
    }
  }
  // slab[split][ftile][c][f_local]
  double* out = slab + ((size_t)sp * ftiles + ft) * CP * GF;
#pragma unroll
  for (int ct = 0; ct < (T4 ? CT - 1 : CT); ++ct)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = ct * 16 + (lane >> 4) + 4 * r;
        const int fl = wave * 32 + q * 16 + (lane & 15);
        out[(size_t)c * GF + fl] = acc[ct][q][r];
      }
  if constexpr (T4) {   // classes (CT - 1) 16 + 0..3; the fold reads only c < C
#pragma unroll
    for (int q = 0; q < 2; ++q)
      out[(size_t)((CT - 1) * 16 + (lane >> 4)) * GF + wave * 32 + q * 16 + (lane & 15)] = acc4[q];
  }
}

// grad[f*C + c] += sum_s slab (fixed order); the dger fitWithMean correction
// (:180-181) and the intercept daxpy (:184-185).  ms[CP] = total multSum.
__global__ void k_mlr_fold(const double* __restrict__ slab, int splits, int ftiles, int CP, int F,
                           int C, const double* __restrict__ ms, int fitIntercept,
                           int fitWithMean, const double* __restrict__ sm,
                           double* __restrict__ grad) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // c * F + f
  if (e < (int64_t)C * F) {
    const int c = (int)(e / F), f = (int)(e % F);
    const int ft = f / GF, fl = f % GF;
    double s = 0.0;
    for (int sp = 0; sp < splits; ++sp)
      s += slab[(((size_t)sp * ftiles + ft) * CP + c) * GF + fl];
    double g = 1.0 * s + 1.0 * grad[(int64_t)f * C + c];
    if (fitIntercept && fitWithMean && sm[f] != 0.0) g = g + ms[c] * (-1.0 * sm[f]);
    grad[(int64_t)f * C + c] = g;
  }
  if (fitIntercept && e < C) grad[(int64_t)C * F + e] = grad[(int64_t)C * F + e] + 1.0 * ms[e];
}

// Fold per-wave class sums: out[c] = sum_w slabMS[w][c].  One 256-thread
// workgroup per column: thread t sums rows t, t+256, ... in order, then a
// fixed LDS tree -- deterministic, and no 2048-long dependent chain.
__global__ __launch_bounds__(256) void k_fold_columns(const double* __restrict__ slab,
                                                      int64_t rows, int width,
                                                      double* __restrict__ out) {
  __shared__ double sh[256];
  const int c = blockIdx.x, t = threadIdx.x;
  double s = 0.0;
  for (int64_t w = t; w < rows; w += 256) s += slab[w * width + c];
  sh[t] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) sh[t] += sh[t + h];
    __syncthreads();
  }
  if (t == 0) out[c] = sh[0];
}

__global__ void k_add_scalars(const double* __restrict__ s2, double* __restrict__ lossSum,
                              double* __restrict__ weightSum) {
  *lossSum += s2[0];
  *weightSum += s2[1];
}

// ----------------------------------------------------- multinomial, CSR rows
// margins (:112-122 with the sparse-A gemm of ml/linalg/BLAS.scala:430-536:
// per row, t = sum over its nonzeros in order of value * linear(c, col), then
// C(i, c) = 1.0 * C(i, c) + t * 1.0 over the offset), Utils.softmax, loss and
// multipliers (:129-142) as in k_mlr_margins.  One wave per row, class
// c = lane + 64 q on its lane (CQ = classes per lane); mult is n x C.
// Per-wave partials: slabS[w][2] = (loss, weight), slabMS[w][C] = multSum.
template <int CQ>
__global__ __launch_bounds__(256) void k_mlr_csr_margins(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const double* __restrict__ vals, const double* __restrict__ labels,
    const double* __restrict__ weights, int64_t n, int C, const double* __restrict__ coef,
    const double* __restrict__ offset, double* __restrict__ mult, double* __restrict__ slabS,
    double* __restrict__ slabMS) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  double offc[CQ], ms[CQ];
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
    const int c = lane + 64 * q;
    offc[q] = (offset && c < C) ? offset[c] : 0.0;
    ms[q] = 0.0;
  }
  double loss = 0.0, wsum = 0.0;
  for (int64_t r = gw; r < n; r += nw) {
    double t[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) t[q] = 0.0;
    const int64_t p1 = rowptr[r + 1];
    for (int64_t p = rowptr[r]; p < p1; ++p) {
      const double v = vals[p];
      const double* lin = coef + (int64_t)colidx[p] * C;
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int c = lane + 64 * q;
        if (c < C) t[q] = t[q] + v * lin[c];
      }
    }
    double m[CQ];
    double mx = -1.7976931348623157e308;   // Double.MinValue (Utils.scala:113)
    int infc = 1 << 30;
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
      const int c = lane + 64 * q;
      m[q] = 1.0 * offc[q] + t[q] * 1.0;
      if (c < C) {
        if (m[q] == __builtin_inf()) infc = min(infc, c);
        else if (m[q] > mx) mx = m[q];
      }
    }
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      mx = fmax(mx, __shfl_xor(mx, k));
      infc = min(infc, __shfl_xor(infc, k));
    }
    double pr[CQ];
    if (infc < (1 << 30)) {
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int c = lane + 64 * q;
        pr[q] = (c == infc) ? 1.0 : 0.0 * m[q];
      }
    } else {
      double sum = 0.0;
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int c = lane + 64 * q;
        pr[q] = (c < C) ? exp(m[q] - mx) : 0.0;
        sum += pr[q];
      }
      sum = wave_sum_bcast(sum);
      const double inv = 1.0 / sum;
#pragma unroll
      for (int q = 0; q < CQ; ++q) pr[q] = inv * pr[q];
    }
    const double w = weights ? weights[r] : 1.0;
    const int label = (int)labels[r];
    double pl = 0.0;
#pragma unroll
    for (int q = 0; q < CQ; ++q)
      if (q == (label >> 6)) pl = pr[q];
    pl = __shfl(pl, label & 63);
    wsum += w;
    if (w > 0) loss -= w * log(pl);
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
      const int c = lane + 64 * q;
      double mu;
      if (w > 0) {
        mu = (w != 1.0) ? w * pr[q] : pr[q];
        if (c == label) mu -= w;
      } else {
        mu = 0.0 * pr[q];
      }
      if (c < C) {
        mult[r * C + c] = mu;
        ms[q] += mu;
      }
    }
  }
  if (lane == 0) {
    slabS[gw * 2 + 0] = loss;
    slabS[gw * 2 + 1] = wsum;
  }
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
    const int c = lane + 64 * q;
    if (c < C) slabMS[gw * C + c] = ms[q];
  }
}

// gradient over the row-blocked CSC copy (:156-162, linearGradSumMat =
// sm^T x mat): one wave per feature f, classes on lanes, blocks in order and
// each block's rows in order; then gradientSumArray(f C + c) += v and the
// fitWithMean dger correction (:175-182) with the total multiplier sums ms.
template <int CQ>
__global__ __launch_bounds__(256) void k_mlr_csc_grad(
    const int64_t* __restrict__ colptr, const int32_t* __restrict__ rowidx,
    const double* __restrict__ cv, int64_t nb, int F, int C, const double* __restrict__ mult,
    const double* __restrict__ ms, int fitIntercept, int fitWithMean,
    const double* __restrict__ sm, double* __restrict__ grad) {
  const int lane = threadIdx.x & 63;
  const int64_t f = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (f >= F) return;
  double tot[CQ];
#pragma unroll
  for (int q = 0; q < CQ; ++q) tot[q] = 0.0;
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t e = b * F + f;
    double sb[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) sb[q] = 0.0;
    const int64_t k1 = colptr[e + 1];
    for (int64_t k = colptr[e]; k < k1; ++k) {
      const double v = cv[k];
      const double* mrow = mult + (int64_t)rowidx[k] * C;
#pragma unroll
      for (int q = 0; q < CQ; ++q) {
        const int c = lane + 64 * q;
        if (c < C) sb[q] = sb[q] + v * mrow[c];
      }
    }
#pragma unroll
    for (int q = 0; q < CQ; ++q) tot[q] = tot[q] + sb[q];
  }
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
    const int c = lane + 64 * q;
    if (c >= C) continue;
    double g = grad[f * C + c] + tot[q];
    if (fitIntercept && fitWithMean && sm[f] != 0.0) g = g + ms[c] * (-1.0 * sm[f]);
    grad[f * C + c] = g;
  }
}

// intercept gradient (:184-185): grad[C F + c] += 1.0 * multSum[c]
__global__ void k_mlr_icpt(int F, int C, const double* __restrict__ ms, double* __restrict__ grad) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) grad[(int64_t)C * F + c] = grad[(int64_t)C * F + c] + 1.0 * ms[c];
}

}  // namespace

struct cyc_logistic_plan_s {
  int F = 0, C = 1, fitIntercept = 0, fitWithMean = 0;
  int loss = 0;   // binary plans: 0 logistic, 1 hinge (LinearSVC), 2 least squares, 3 Huber,
                  // 4 AFT survival
  double labelStd = 1.0, labelMean = 0.0;   // least squares
  double epsilon = 1.35;                     // Huber
  cyc::DeviceBuffer effCoef;
  std::mutex mu;
  cyc::DeviceBuffer slabG, slabS, slabMS, gradAcc, scal, offset, multBuf, gslab, msTot;
  cyc::DeviceBuffer rowMult;
};

namespace {

int check_common(cyc_logistic_plan p, const double* coef, const double* sm) {
  CYC_REQUIRE(p != nullptr && coef != nullptr, "plan and coefficients must not be null");
  if (p->fitWithMean) {
    CYC_REQUIRE(p->fitIntercept, "for training without intercept, should not center the vectors");
    CYC_REQUIRE(sm != nullptr, "scaled means is required when center the vectors");
  }
  return CYC_OK;
}

template <int FPL>
void launch_bin_dense(dim3 g, hipStream_t st, const double* X, const double* labels,
                      const double* weights, int64_t n, int F, const double* coef, int fi,
                      int kind, double offset, double lscale, double sigma, double eps,
                      int64_t rpw, double* sg, double* ss) {
  hipLaunchKernelGGL(k_binlog_dense<FPL>, g, dim3(256), 0, st, X, labels, weights, n, F, coef, fi,
                     kind, offset, lscale, sigma, eps, rpw, sg, ss);
}

}  // namespace

extern "C" {

int cyc_logistic_plan_create(int32_t numFeatures, int32_t numClasses, int fitIntercept,
                             int fitWithMean, cyc_logistic_plan* plan) {
  CYC_REQUIRE(plan != nullptr, "plan must not be null");
  CYC_REQUIRE(numFeatures > 0, "numFeatures must be positive");
  CYC_REQUIRE(numClasses >= 1, "numClasses must be positive");
  if (fitWithMean)
    CYC_REQUIRE(fitIntercept, "for training without intercept, should not center the vectors");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  auto* p = new cyc_logistic_plan_s();
  p->F = numFeatures;
  p->C = numClasses;
  p->fitIntercept = fitIntercept != 0;
  p->fitWithMean = fitWithMean != 0;
  *plan = p;
  return CYC_OK;
}

int cyc_logistic_plan_destroy(cyc_logistic_plan plan) {
  delete plan;
  return CYC_OK;
}

namespace {
// The margin offset every row starts from (see k_binlog_offset).  The
// original coefficients go in (least squares: not the effective ones).
int binary_offset(cyc_logistic_plan p, const double* coef, const double* scaledMean,
                  hipStream_t st, double* offset) {
  *offset = 0.0;
  if (!p->fitIntercept) return CYC_OK;
  if (p->fitWithMean || p->loss == 2) {
    // marginOffset = intercept - dot(coef, scaledMean) (:62-70); least
    // squares: labelMean / labelStd - dot (LeastSquaresBlockAggregator :59-66)
    if (int rc = p->offset.reserve(sizeof(double) * (2 + kOffParts))) return rc;
    double* part = (double*)p->offset.ptr + 2;
    hipLaunchKernelGGL(k_binlog_offset_part, dim3(kOffParts), dim3(256), 0, st, coef, scaledMean,
                       p->F, part);
    CYC_LAUNCH_CHECK("k_binlog_offset_part");
    hipLaunchKernelGGL(k_binlog_offset, dim3(1), dim3(64), 0, st, (const double*)part, coef, p->F,
                       p->loss == 2 ? 1 : 0, p->labelMean / p->labelStd, (double*)p->offset.ptr);
    CYC_LAUNCH_CHECK("k_binlog_offset");
    CYC_HIP(hipMemcpyAsync(offset, p->offset.ptr, sizeof(double), hipMemcpyDeviceToHost, st));
  } else {
    CYC_HIP(hipMemcpyAsync(offset, coef + p->F, sizeof(double), hipMemcpyDeviceToHost, st));
  }
  CYC_HIP(hipStreamSynchronize(st));
  return CYC_OK;
}

// The same offset left in HBM: *offDev points at it (nullptr without an
// intercept: offset 0), no host copy and no stream sync.
int binary_offset_dev(cyc_logistic_plan p, const double* coef, const double* scaledMean,
                      hipStream_t st, const double** offDev) {
  *offDev = nullptr;
  if (!p->fitIntercept) return CYC_OK;
  if (p->fitWithMean || p->loss == 2) {
    if (int rc = p->offset.reserve(sizeof(double) * (2 + kOffParts))) return rc;
    double* part = (double*)p->offset.ptr + 2;
    hipLaunchKernelGGL(k_binlog_offset_part, dim3(kOffParts), dim3(256), 0, st, coef, scaledMean,
                       p->F, part);
    CYC_LAUNCH_CHECK("k_binlog_offset_part");
    hipLaunchKernelGGL(k_binlog_offset, dim3(1), dim3(64), 0, st, (const double*)part, coef, p->F,
                       p->loss == 2 ? 1 : 0, p->labelMean / p->labelStd, (double*)p->offset.ptr);
    CYC_LAUNCH_CHECK("k_binlog_offset");
    *offDev = (const double*)p->offset.ptr;
  } else {
    *offDev = coef + p->F;
  }
  return CYC_OK;
}

// kcoef: the coefficients the margins use when they differ from coef (least
// squares' effectiveCoef); coef feeds the offset.
int binary_add_dense(cyc_logistic_plan p, const double* X, const double* labels,
                     const double* weights, int64_t n, const double* coef,
                     const double* scaledMean, double* grad, double* lossSum, double* weightSum,
                     void* stream, const double* kcoef = nullptr) {
  int rc = check_common(p, coef, scaledMean);
  if (rc) return rc;
  CYC_REQUIRE(n >= 0, "n >= 0");
  if (n == 0) return CYC_OK;
  const int F = p->F;
  if (F > 64 * 32) {
    cyc::set_error("dense binary aggregator supports numFeatures <= 2048 (use CSR blocks)");
    return CYC_ERR_UNSUPPORTED;
  }
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  const int64_t waves = std::min<int64_t>(4096, n);
  const int64_t rpw = (n + waves - 1) / waves;
  const int64_t nw = (n + rpw - 1) / rpw;
  const int64_t blocks = (nw + 3) / 4;
  const int64_t wtot = blocks * 4;
  if ((rc = p->slabG.reserve(sizeof(double) * (size_t)wtot * F)) ||
      (rc = p->slabS.reserve(sizeof(double) * (size_t)wtot * 4)) ||
      (rc = p->scal.reserve(sizeof(double) * 4)) || (rc = p->offset.reserve(sizeof(double) * 2)))
    return rc;
  double offset = 0.0;
  if ((rc = binary_offset(p, coef, scaledMean, st, &offset))) return rc;
  const double* kc = kcoef ? kcoef : coef;
  const double lscale = -1.0 / p->labelStd;
  const int foldIcpt = p->loss == 2 ? 0 : p->fitIntercept;
  // Huber: sigma = coefficientsArray.last (:97), its gradient entry last
  // AFT: sigma = math.exp(coefficientsArray(dim - 1)) (:91), dim = F + 2
  double sigma = 0.0;
  const int sigIdx = p->loss == 3 ? F + (p->fitIntercept ? 1 : 0) : p->loss == 4 ? F + 1 : -1;
  if (sigIdx >= 0) {
    CYC_HIP(hipMemcpyAsync(&sigma, coef + sigIdx, sizeof(double), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipStreamSynchronize(st));
    if (p->loss == 4) sigma = std::exp(sigma);
  }
  const double eps = p->epsilon;
  // waves past the last row still write (zero) partials, so the fold reads all
  dim3 grid((unsigned)blocks);
  const int fpl = (F + 63) / 64;
  double* sg = (double*)p->slabG.ptr;
  double* ss = (double*)p->slabS.ptr;
  {
  cyc::KernelTimer timer("k_binlog_dense", st);
  if (fpl <= 1) launch_bin_dense<1>(grid, st, X, labels, weights, n, F, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps, rpw, sg, ss);
  else if (fpl <= 2) launch_bin_dense<2>(grid, st, X, labels, weights, n, F, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps, rpw, sg, ss);
  else if (fpl <= 4) launch_bin_dense<4>(grid, st, X, labels, weights, n, F, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps, rpw, sg, ss);
  else if (fpl <= 8) launch_bin_dense<8>(grid, st, X, labels, weights, n, F, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps, rpw, sg, ss);
  else if (fpl <= 16) launch_bin_dense<16>(grid, st, X, labels, weights, n, F, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps, rpw, sg, ss);
  else launch_bin_dense<32>(grid, st, X, labels, weights, n, F, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps, rpw, sg, ss);
  CYC_LAUNCH_CHECK("k_binlog_dense");
  }
  hipLaunchKernelGGL(k_fold_scalars, dim3(1), dim3(256), 0, st, ss, wtot, 4, (double*)p->scal.ptr);
  CYC_LAUNCH_CHECK("k_fold_scalars");
  hipLaunchKernelGGL(k_binlog_fold, dim3((F + 255) / 256), dim3(256), 0, st, sg, wtot, nullptr,
                     F, (const double*)p->scal.ptr, foldIcpt, p->fitWithMean, sigIdx,
                     scaledMean, grad, lossSum, weightSum);
  CYC_LAUNCH_CHECK("k_binlog_fold");
  return CYC_OK;
}

int binary_add_csr(cyc_logistic_plan p, const int64_t* rowptr, const int32_t* colidx,
                   const double* vals, const double* labels, const double* weights, int64_t n,
                   const double* coef, const double* scaledMean, double* grad, double* lossSum,
                   double* weightSum, cyc_csc csc, void* stream,
                   const double* kcoef = nullptr) {
  int rc = check_common(p, coef, scaledMean);
  if (rc) return rc;
  CYC_REQUIRE(n >= 0, "n >= 0");
  if (n == 0) return CYC_OK;
  const int F = p->F;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  const int64_t waves = csc ? std::min<int64_t>(8192, (n + 63) / 64) : std::min<int64_t>(16384, n);
  const int64_t rpw = (n + waves - 1) / waves;
  const int64_t nw = csc ? waves : (n + rpw - 1) / rpw;
  const int64_t blocks = (nw + 3) / 4;
  const int64_t wtot = blocks * 4;
  if ((rc = p->gradAcc.reserve(sizeof(double) * (size_t)F)) ||
      (rc = p->slabS.reserve(sizeof(double) * (size_t)wtot * 4)) ||
      (rc = p->scal.reserve(sizeof(double) * 4)) || (rc = p->offset.reserve(sizeof(double) * 2)))
    return rc;
  double offset = 0.0;
  if ((rc = binary_offset(p, coef, scaledMean, st, &offset))) return rc;
  const double* kc = kcoef ? kcoef : coef;
  const double lscale = -1.0 / p->labelStd;
  const int foldIcpt = p->loss == 2 ? 0 : p->fitIntercept;
  // Huber: sigma = coefficientsArray.last (:97), its gradient entry last
  // AFT: sigma = math.exp(coefficientsArray(dim - 1)) (:91), dim = F + 2
  double sigma = 0.0;
  const int sigIdx = p->loss == 3 ? F + (p->fitIntercept ? 1 : 0) : p->loss == 4 ? F + 1 : -1;
  if (sigIdx >= 0) {
    CYC_HIP(hipMemcpyAsync(&sigma, coef + sigIdx, sizeof(double), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipStreamSynchronize(st));
    if (p->loss == 4) sigma = std::exp(sigma);
  }
  const double eps = p->epsilon;
  const int64_t* colptr = nullptr;
  const int32_t* rowidx = nullptr;
  const double* cvals = nullptr;
  if (csc) {
    CYC_REQUIRE(cyc_csc_rows(csc) == n && cyc_csc_features(csc) == F,
                "the CSC copy does not match the CSR rows (cyc_csc_build_dev of these rows)");
    cyc_csc_arrays(csc, &colptr, &rowidx, &cvals);
  }
  if (csc) {
    // Deterministic two-pass path: CSR margins -> mult, then the row-blocked
    // CSC's column sums, one row block at a time.  (The row-block x
    // column-tile layout, cyc_binary_add_tiles_dev, is the fast path for
    // large sparse shards.)
    if ((rc = p->rowMult.reserve(sizeof(double) * (size_t)n))) return rc;
    {
      cyc::KernelTimer timer("k_binlog_csr", st);
      hipLaunchKernelGGL(k_binlog_csr_mult8, dim3((unsigned)blocks), dim3(256), 0, st, rowptr,
                         colidx, vals, labels, weights, n, kc, p->fitIntercept, p->loss, offset,
                         lscale, sigma, eps, (double*)p->rowMult.ptr, (double*)p->slabS.ptr);
      CYC_LAUNCH_CHECK("k_binlog_csr_mult8");
    }
    int64_t rpb = 0, nb = 0;
    cyc_csc_blocks(csc, &rpb, &nb);
    // 32 lanes per group of 4 columns (round 1: 8 / 16 / 64 lanes and 2 / 8
    // columns per group measured slower or flat)
    const unsigned cgrid = (unsigned)((((int64_t)F + 3) / 4 * 32 + 255) / 256);
    cyc::KernelTimer timer("k_binlog_csc_grad", st);
    for (int64_t b = 0; b < nb; ++b) {
      hipLaunchKernelGGL(k_binlog_csc_grad_blk, dim3(cgrid), dim3(256), 0, st,
                         colptr + b * F, rowidx, cvals, (const double*)p->rowMult.ptr, F,
                         b == 0 ? 1 : 0, (double*)p->gradAcc.ptr);
    }
    CYC_LAUNCH_CHECK("k_binlog_csc_grad_blk");
  } else {
    CYC_HIP(hipMemsetAsync(p->gradAcc.ptr, 0, sizeof(double) * (size_t)F, st));
    cyc::KernelTimer timer("k_binlog_csr", st);
    hipLaunchKernelGGL(k_binlog_csr, dim3((unsigned)blocks), dim3(256), 0, st, rowptr, colidx,
                       vals, labels, weights, n, kc, p->fitIntercept, p->loss, offset, lscale, sigma, eps,
                       rpw,
                       (double*)p->gradAcc.ptr, (double*)p->slabS.ptr);
    CYC_LAUNCH_CHECK("k_binlog_csr");
  }
  hipLaunchKernelGGL(k_fold_scalars, dim3(1), dim3(256), 0, st, (const double*)p->slabS.ptr, wtot,
                     4, (double*)p->scal.ptr);
  CYC_LAUNCH_CHECK("k_fold_scalars");
  hipLaunchKernelGGL(k_binlog_fold, dim3((F + 255) / 256), dim3(256), 0, st, nullptr, 0,
                     (const double*)p->gradAcc.ptr, F, (const double*)p->scal.ptr,
                     foldIcpt, p->fitWithMean, sigIdx, scaledMean, grad, lossSum, weightSum);
  CYC_LAUNCH_CHECK("k_binlog_fold");
  return CYC_OK;
}

}  // namespace

namespace {
int ls_prepare(cyc_logistic_plan p, const double* coef, const double* inverseStd,
               const double* scaledMean, hipStream_t st, const double** eff) {
  CYC_REQUIRE(p != nullptr && p->loss == 2,
              "the plan is not a least squares plan (cyc_least_squares_plan_create)");
  CYC_REQUIRE(coef != nullptr && inverseStd != nullptr, "coef and inverseStd must not be null");
  CYC_REQUIRE(!p->fitIntercept || scaledMean != nullptr,
              "scaled means is required when fitting an intercept");
  int rc;
  if ((rc = p->effCoef.reserve(sizeof(double) * (size_t)p->F))) return rc;
  hipLaunchKernelGGL(k_effective_coef, dim3((p->F + 255) / 256), dim3(256), 0, st, coef,
                     inverseStd, p->F, (double*)p->effCoef.ptr);
  CYC_LAUNCH_CHECK("k_effective_coef");
  *eff = (const double*)p->effCoef.ptr;
  return CYC_OK;
}
}  // namespace

int cyc_binary_add_tiles_dev(cyc_logistic_plan p, cyc_tiles tiles, const double* labels,
                             const double* weights, const double* coef, const double* inverseStd,
                             const double* scaledMean, double* grad, double* lossSum,
                             double* weightSum, void* stream) {
  int rc = check_common(p, coef, scaledMean);
  if (rc) return rc;
  CYC_REQUIRE(tiles != nullptr, "tiles must not be null");
  cyc::TilesView v;
  if ((rc = cyc::tiles_view(tiles, &v))) return rc;
  const int F = p->F;
  CYC_REQUIRE(v.F == F, "Dimensions mismatch when adding new instance. Expecting " +
                            std::to_string(F) + " but got " + std::to_string(v.F) + ".");
  const int64_t n = v.n;
  if (n == 0) return CYC_OK;
  CYC_REQUIRE(labels != nullptr, "labels must not be null");
  hipStream_t st = cyc::as_stream(stream);
  const double* kc = coef;
  if (p->loss == 2) {      // LeastSquaresBlockAggregator.effectiveCoef (:48-55)
    if ((rc = ls_prepare(p, coef, inverseStd, scaledMean, st, &kc))) return rc;
  }
  std::lock_guard<std::mutex> g(p->mu);
  const int R = cyc::tiles_ranges(v);
  const int64_t wgMax = cyc::tiles_rows_blocks(n);
  if ((rc = p->rowMult.reserve(sizeof(double) * (size_t)n)) ||
      (rc = p->slabG.reserve(sizeof(double) * (size_t)R * F)) ||
      (rc = p->slabS.reserve(sizeof(double) * (size_t)wgMax * 4)) ||
      (rc = p->scal.reserve(sizeof(double) * 4)) || (rc = p->offset.reserve(sizeof(double) * 2)))
    return rc;
  // the margin offset stays in HBM for k_tiles_rows: no host round trip
  // (and no stream sync) before the margin pass
  const double* offDev = nullptr;
  if ((rc = binary_offset_dev(p, coef, scaledMean, st, &offDev))) return rc;
  const double lscale = -1.0 / p->labelStd;
  const int foldIcpt = p->loss == 2 ? 0 : p->fitIntercept;
  double sigma = 0.0;
  const int sigIdx = p->loss == 3 ? F + (p->fitIntercept ? 1 : 0) : p->loss == 4 ? F + 1 : -1;
  if (sigIdx >= 0) {
    CYC_HIP(hipMemcpyAsync(&sigma, coef + sigIdx, sizeof(double), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipStreamSynchronize(st));
    if (p->loss == 4) sigma = std::exp(sigma);
  }
  int64_t wgs = 0;
  {
    cyc::KernelTimer timer("k_tiles_margin", st);
    if ((rc = cyc::tiles_margin(v, kc, (double*)p->rowMult.ptr, st))) return rc;
  }
  {
    cyc::KernelTimer timer("k_tiles_rows", st);
    if ((rc = cyc::tiles_rows(n, labels, weights, p->fitIntercept, p->loss, 0.0, offDev, lscale,
                              sigma, p->epsilon, (double*)p->rowMult.ptr, (double*)p->slabS.ptr,
                              &wgs, st)))
      return rc;
  }
  int ranges = 0;
  {
    cyc::KernelTimer timer("k_tiles_grad", st);
    if ((rc = cyc::tiles_grad(v, (const double*)p->rowMult.ptr, (double*)p->slabG.ptr, &ranges,
                              st)))
      return rc;
  }
  hipLaunchKernelGGL(k_fold_scalars, dim3(1), dim3(256), 0, st, (const double*)p->slabS.ptr, wgs,
                     4, (double*)p->scal.ptr);
  CYC_LAUNCH_CHECK("k_fold_scalars");
  hipLaunchKernelGGL(k_binlog_fold, dim3((F + 255) / 256), dim3(256), 0, st,
                     (const double*)p->slabG.ptr, (int64_t)ranges, nullptr, F,
                     (const double*)p->scal.ptr, foldIcpt, p->fitWithMean, sigIdx, scaledMean, grad,
                     lossSum, weightSum);
  CYC_LAUNCH_CHECK("k_binlog_fold");
  return CYC_OK;
}

int cyc_binary_logistic_add_dense_dev(cyc_logistic_plan p, const double* X, const double* labels,
                                      const double* weights, int64_t n, const double* coef,
                                      const double* scaledMean, double* grad, double* lossSum,
                                      double* weightSum, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 0, "the plan is not a binary logistic plan");
  return binary_add_dense(p, X, labels, weights, n, coef, scaledMean, grad, lossSum, weightSum,
                          stream);
}

int cyc_binary_logistic_add_csr_dev(cyc_logistic_plan p, const int64_t* rowptr,
                                    const int32_t* colidx, const double* vals,
                                    const double* labels, const double* weights, int64_t n,
                                    const double* coef, const double* scaledMean, double* grad,
                                    double* lossSum, double* weightSum, cyc_csc csc,
                                    void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 0, "the plan is not a binary logistic plan");
  return binary_add_csr(p, rowptr, colidx, vals, labels, weights, n, coef, scaledMean, grad,
                        lossSum, weightSum, csc, stream);
}

int cyc_hinge_plan_create(int32_t numFeatures, int fitIntercept, cyc_logistic_plan* plan) {
  // HingeBlockAggregator centers whenever it fits an intercept (:62-72, :133-141)
  int rc = cyc_logistic_plan_create(numFeatures, 1, fitIntercept, fitIntercept, plan);
  if (rc == CYC_OK) (*plan)->loss = 1;
  return rc;
}

int cyc_hinge_add_dense_dev(cyc_logistic_plan p, const double* X, const double* labels,
                            const double* weights, int64_t n, const double* coef,
                            const double* scaledMean, double* grad, double* lossSum,
                            double* weightSum, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 1, "the plan is not a hinge plan (cyc_hinge_plan_create)");
  return binary_add_dense(p, X, labels, weights, n, coef, scaledMean, grad, lossSum, weightSum,
                          stream);
}

int cyc_hinge_add_csr_dev(cyc_logistic_plan p, const int64_t* rowptr, const int32_t* colidx,
                          const double* vals, const double* labels, const double* weights,
                          int64_t n, const double* coef, const double* scaledMean, double* grad,
                          double* lossSum, double* weightSum, cyc_csc csc, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 1, "the plan is not a hinge plan (cyc_hinge_plan_create)");
  return binary_add_csr(p, rowptr, colidx, vals, labels, weights, n, coef, scaledMean, grad,
                        lossSum, weightSum, csc, stream);
}

int cyc_huber_plan_create(int32_t numFeatures, int fitIntercept, double epsilon,
                          cyc_logistic_plan* plan) {
  CYC_REQUIRE(epsilon > 1.0, "epsilon must be > 1.0");
  // centers whenever it fits an intercept (marginOffset :66-71, daxpy :131-134)
  int rc = cyc_logistic_plan_create(numFeatures, 1, fitIntercept, fitIntercept, plan);
  if (rc == CYC_OK) {
    (*plan)->loss = 3;
    (*plan)->epsilon = epsilon;
  }
  return rc;
}

int cyc_huber_add_dense_dev(cyc_logistic_plan p, const double* X, const double* labels,
                            const double* weights, int64_t n, const double* coef,
                            const double* scaledMean, double* grad, double* lossSum,
                            double* weightSum, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 3, "the plan is not a Huber plan (cyc_huber_plan_create)");
  return binary_add_dense(p, X, labels, weights, n, coef, scaledMean, grad, lossSum, weightSum,
                          stream);
}

int cyc_huber_add_csr_dev(cyc_logistic_plan p, const int64_t* rowptr, const int32_t* colidx,
                          const double* vals, const double* labels, const double* weights,
                          int64_t n, const double* coef, const double* scaledMean, double* grad,
                          double* lossSum, double* weightSum, cyc_csc csc, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 3, "the plan is not a Huber plan (cyc_huber_plan_create)");
  return binary_add_csr(p, rowptr, colidx, vals, labels, weights, n, coef, scaledMean, grad,
                        lossSum, weightSum, csc, stream);
}

int cyc_aft_plan_create(int32_t numFeatures, int fitIntercept, cyc_logistic_plan* plan) {
  // centers whenever it fits an intercept (marginOffset :52-58, daxpy :118-121)
  int rc = cyc_logistic_plan_create(numFeatures, 1, fitIntercept, fitIntercept, plan);
  if (rc == CYC_OK) (*plan)->loss = 4;
  return rc;
}

int cyc_aft_add_dense_dev(cyc_logistic_plan p, const double* X, const double* labels,
                          const double* censors, int64_t n, const double* coef,
                          const double* scaledMean, double* grad, double* lossSum,
                          double* weightSum, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 4, "the plan is not an AFT plan (cyc_aft_plan_create)");
  return binary_add_dense(p, X, labels, censors, n, coef, scaledMean, grad, lossSum, weightSum,
                          stream);
}

int cyc_aft_add_csr_dev(cyc_logistic_plan p, const int64_t* rowptr, const int32_t* colidx,
                        const double* vals, const double* labels, const double* censors,
                        int64_t n, const double* coef, const double* scaledMean, double* grad,
                        double* lossSum, double* weightSum, cyc_csc csc, void* stream) {
  CYC_REQUIRE(p == nullptr || p->loss == 4, "the plan is not an AFT plan (cyc_aft_plan_create)");
  return binary_add_csr(p, rowptr, colidx, vals, labels, censors, n, coef, scaledMean, grad,
                        lossSum, weightSum, csc, stream);
}

int cyc_least_squares_plan_create(int32_t numFeatures, int fitIntercept, double labelStd,
                                  double labelMean, cyc_logistic_plan* plan) {
  CYC_REQUIRE(labelStd > 0.0, "LeastSquaresBlockAggregator requires the label standard "
                              "deviation to be positive.");
  int rc = cyc_logistic_plan_create(numFeatures, 1, fitIntercept, 0, plan);
  if (rc == CYC_OK) {
    (*plan)->loss = 2;
    (*plan)->labelStd = labelStd;
    (*plan)->labelMean = labelMean;
  }
  return rc;
}


int cyc_least_squares_add_dense_dev(cyc_logistic_plan p, const double* X, const double* labels,
                                    const double* weights, int64_t n, const double* coef,
                                    const double* inverseStd, const double* scaledMean,
                                    double* grad, double* lossSum, double* weightSum,
                                    void* stream) {
  const double* eff = nullptr;
  hipStream_t st = cyc::as_stream(stream);
  if (int rc = ls_prepare(p, coef, inverseStd, scaledMean, st, &eff)) return rc;
  if (n <= 0) return n < 0 ? (cyc::set_error("n >= 0"), CYC_ERR_INVALID_ARG) : CYC_OK;
  // the offset needs the original coefficients: computed first, from coef
  return binary_add_dense(p, X, labels, weights, n, coef, scaledMean, grad, lossSum, weightSum,
                          stream, eff);
}

int cyc_least_squares_add_csr_dev(cyc_logistic_plan p, const int64_t* rowptr,
                                  const int32_t* colidx, const double* vals, const double* labels,
                                  const double* weights, int64_t n, const double* coef,
                                  const double* inverseStd, const double* scaledMean,
                                  double* grad, double* lossSum, double* weightSum, cyc_csc csc,
                                  void* stream) {
  const double* eff = nullptr;
  hipStream_t st = cyc::as_stream(stream);
  if (int rc = ls_prepare(p, coef, inverseStd, scaledMean, st, &eff)) return rc;
  if (n <= 0) return n < 0 ? (cyc::set_error("n >= 0"), CYC_ERR_INVALID_ARG) : CYC_OK;
  return binary_add_csr(p, rowptr, colidx, vals, labels, weights, n, coef, scaledMean, grad,
                        lossSum, weightSum, csc, stream, eff);
}

int cyc_multinomial_logistic_add_dense_dev(cyc_logistic_plan p, const double* X,
                                           const double* labels, const double* weights,
                                           int64_t n, const double* coef,
                                           const double* scaledMean, double* grad,
                                           double* lossSum, double* weightSum, void* stream) {
  int rc = check_common(p, coef, scaledMean);
  if (rc) return rc;
  CYC_REQUIRE(n >= 0, "n >= 0");
  if (n == 0) return CYC_OK;
  const int F = p->F, C = p->C;
  if (C > 128) {
    cyc::set_error("multinomial aggregator supports numClasses <= 128");
    return CYC_ERR_UNSUPPORTED;
  }
  if (((int64_t)C * F + C) * 8 >= INT32_MAX || (int64_t)MR * F * 8 >= INT32_MAX) {
    cyc::set_error("dense multinomial aggregator supports numClasses * numFeatures < 2^28 "
                   "and numFeatures < 2^20");
    return CYC_ERR_UNSUPPORTED;
  }
  const int CT = (C + 15) / 16, CP = CT * 16;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  // Rows are processed in chunks of up to 8M so the multiplier matrix stays
  // bounded (8M x CP doubles: 7.3 GB at C = 100); a whole 6.25M-row shard of
  // the 8-GPU config is one launch (no second partial round of tiles).
  const int64_t chunk = std::min<int64_t>(n, 8 << 20);
  // k_mlr_grad: the last class tile on the 4x4x4 form when it holds 1..4
  // classes (2.6 % faster at C = 100)
  const bool t4 = C % 16 != 0 && C % 16 <= 4;
  // persistent: one 8-wave workgroup per CU (CYC_MLR_NW = 4: two 4-wave ones)
  constexpr int mnw = CYC_MLR_NW, mrows = 32 * mnw;
  const int mblocks = 256 * 8 / mnw;
  const int64_t mwaves = (int64_t)mblocks * mnw;
  const int ftiles = (F + GF - 1) / GF;
  if ((rc = p->multBuf.reserve(sizeof(double) * (size_t)chunk * CP)) ||
      (rc = p->slabS.reserve(sizeof(double) * (size_t)mwaves * 2)) ||
      (rc = p->slabMS.reserve(sizeof(double) * (size_t)mwaves * CP)) ||
      (rc = p->scal.reserve(sizeof(double) * 4)) ||
      (rc = p->msTot.reserve(sizeof(double) * CP)) ||
      (rc = p->offset.reserve(sizeof(double) * (size_t)C)))
    return rc;
  const double* off = nullptr;
  if (p->fitIntercept) {
    if (p->fitWithMean) {
      hipLaunchKernelGGL(k_mlr_offset, dim3((C + 63) / 64), dim3(64), 0, st, coef, scaledMean, F,
                         C, (double*)p->offset.ptr);
      CYC_LAUNCH_CHECK("k_mlr_offset");
      off = (const double*)p->offset.ptr;
    } else {
      off = coef + (int64_t)C * F;
    }
  }
  for (int64_t c0 = 0; c0 < n; c0 += chunk) {
    const int64_t m = std::min(chunk, n - c0);
    const double* Xc = X + c0 * F;
    const double* lc = labels + c0;
    const double* wc = weights ? weights + c0 : nullptr;
    const int64_t tiles = (m + mrows - 1) / mrows;
    const unsigned mb = (unsigned)std::min<int64_t>(mblocks, tiles);
    CYC_HIP(hipMemsetAsync(p->slabS.ptr, 0, sizeof(double) * (size_t)mwaves * 2, st));
    CYC_HIP(hipMemsetAsync(p->slabMS.ptr, 0, sizeof(double) * (size_t)mwaves * CP, st));
#define CYC_MLR_M(CTV)                                                                        \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mlr_margins<CTV, mnw, CYC_MLR_DEPHASE>), dim3(mb), dim3(64 * mnw), 0, st, Xc, lc, wc, m, F, C, coef, \
                     off, (double*)p->multBuf.ptr, (double*)p->slabS.ptr, (double*)p->slabMS.ptr)
    {
    cyc::KernelTimer tm("k_mlr_margins", st);
    switch (CT) {
      case 1: CYC_MLR_M(1); break;
      case 2: CYC_MLR_M(2); break;
      case 3: CYC_MLR_M(3); break;
      case 4: CYC_MLR_M(4); break;
      case 5: CYC_MLR_M(5); break;
      case 6: CYC_MLR_M(6); break;
      case 7: CYC_MLR_M(7); break;
      default: CYC_MLR_M(8); break;
    }
#undef CYC_MLR_M
    CYC_LAUNCH_CHECK("k_mlr_margins");
    }
    // split-K over rows for the gradient GEMM: ~1024 workgroups (4 rounds of
    // one per CU; fewer splits keep the k_mlr_fold read of the partials small)
    int64_t splits = std::max<int64_t>(1, 1024 / ftiles);
    splits = std::min<int64_t>(splits, std::max<int64_t>(1, m / 64));
    int64_t rps = cyc::round_up((m + splits - 1) / splits, GR);
    // k_mlr_grad's buffer descriptors span one split: keep it under 2^31 bytes
    const int64_t maxRps = ((int64_t)INT32_MAX / 8 / std::max(F, CP)) / GR * GR - GR;
    if (rps > maxRps) rps = std::max<int64_t>(GR, maxRps);
    splits = (m + rps - 1) / rps;
    if ((rc = p->gslab.reserve(sizeof(double) * (size_t)splits * ftiles * CP * GF))) return rc;
    const unsigned gblocks = (unsigned)(ftiles * cyc::round_up(splits, (int64_t)8));
#define CYC_MLR_G(CTV)                                                                         \
  if (t4) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mlr_grad<CTV, true>), dim3(gblocks), dim3(512), 0, st, \
                     (const double*)p->multBuf.ptr, Xc, m, F, rps, ftiles, (int)splits, (double*)p->gslab.ptr); \
  else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mlr_grad<CTV, false>), dim3(gblocks), dim3(512), 0, st, \
                     (const double*)p->multBuf.ptr, Xc, m, F, rps, ftiles, (int)splits, (double*)p->gslab.ptr)
    {
    cyc::KernelTimer tg("k_mlr_grad", st);
    switch (CT) {
      case 1: CYC_MLR_G(1); break;
      case 2: CYC_MLR_G(2); break;
      case 3: CYC_MLR_G(3); break;
      case 4: CYC_MLR_G(4); break;
      case 5: CYC_MLR_G(5); break;
      case 6: CYC_MLR_G(6); break;
      case 7: CYC_MLR_G(7); break;
      default: CYC_MLR_G(8); break;
    }
#undef CYC_MLR_G
    CYC_LAUNCH_CHECK("k_mlr_grad");
    }
    hipLaunchKernelGGL(k_fold_columns, dim3(CP), dim3(256), 0, st,
                       (const double*)p->slabMS.ptr, mwaves, CP, (double*)p->msTot.ptr);
    CYC_LAUNCH_CHECK("k_fold_columns");
    hipLaunchKernelGGL(k_fold_scalars, dim3(1), dim3(256), 0, st, (const double*)p->slabS.ptr,
                       mwaves, 2, (double*)p->scal.ptr);
    CYC_LAUNCH_CHECK("k_fold_scalars");
    const int64_t tot = std::max<int64_t>((int64_t)C * F, C);
    hipLaunchKernelGGL(k_mlr_fold, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                       (const double*)p->gslab.ptr, (int)splits, ftiles, CP, F, C,
                       (const double*)p->msTot.ptr, p->fitIntercept, p->fitWithMean, scaledMean,
                       grad);
    CYC_LAUNCH_CHECK("k_mlr_fold");
    hipLaunchKernelGGL(k_add_scalars, dim3(1), dim3(1), 0, st, (const double*)p->scal.ptr,
                       lossSum, weightSum);
    CYC_LAUNCH_CHECK("k_add_scalars");
  }
  return CYC_OK;
}


int cyc_multinomial_logistic_add_csr_dev(cyc_logistic_plan p, const int64_t* rowptr,
                                         const int32_t* colidx, const double* vals,
                                         const double* labels, const double* weights, int64_t n,
                                         const double* coef, const double* scaledMean,
                                         double* grad, double* lossSum, double* weightSum,
                                         cyc_csc csc, void* stream) {
  int rc = check_common(p, coef, scaledMean);
  if (rc) return rc;
  CYC_REQUIRE(n >= 0, "n >= 0");
  if (n == 0) return CYC_OK;
  const int F = p->F, C = p->C;
  CYC_REQUIRE(csc != nullptr && cyc_csc_rows(csc) == n && cyc_csc_features(csc) == F,
              "a CSC copy of these rows is required (cyc_csc_build_dev)");
  if (C > 1024) {
    cyc::set_error("multinomial CSR aggregator supports numClasses <= 1024");
    return CYC_ERR_UNSUPPORTED;
  }
  const int cq = (C + 63) / 64;
  std::lock_guard<std::mutex> g(p->mu);
  hipStream_t st = cyc::as_stream(stream);
  const int64_t waves = std::min<int64_t>(n, 8192);
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  const int64_t wtot = (int64_t)blocks * 4;
  if ((rc = p->multBuf.reserve(sizeof(double) * (size_t)n * C)) ||
      (rc = p->slabS.reserve(sizeof(double) * (size_t)wtot * 2)) ||
      (rc = p->slabMS.reserve(sizeof(double) * (size_t)wtot * C)) ||
      (rc = p->scal.reserve(sizeof(double) * 4)) ||
      (rc = p->msTot.reserve(sizeof(double) * (size_t)C)) ||
      (rc = p->offset.reserve(sizeof(double) * (size_t)C)))
    return rc;
  const double* off = nullptr;
  if (p->fitIntercept) {
    if (p->fitWithMean) {
      hipLaunchKernelGGL(k_mlr_offset, dim3((C + 63) / 64), dim3(64), 0, st, coef, scaledMean, F,
                         C, (double*)p->offset.ptr);
      CYC_LAUNCH_CHECK("k_mlr_offset");
      off = (const double*)p->offset.ptr;
    } else {
      off = coef + (int64_t)C * F;
    }
  }
  CYC_HIP(hipMemsetAsync(p->slabS.ptr, 0, sizeof(double) * (size_t)wtot * 2, st));
  CYC_HIP(hipMemsetAsync(p->slabMS.ptr, 0, sizeof(double) * (size_t)wtot * C, st));
  double* mult = (double*)p->multBuf.ptr;
#define CYC_MLRC_M(Q)                                                                          \
  hipLaunchKernelGGL(k_mlr_csr_margins<Q>, dim3(blocks), dim3(256), 0, st, rowptr, colidx, vals, \
                     labels, weights, n, C, coef, off, mult, (double*)p->slabS.ptr,             \
                     (double*)p->slabMS.ptr)
  {
    cyc::KernelTimer tm("k_mlr_csr_margins", st);
    if (cq <= 1) CYC_MLRC_M(1);
    else if (cq <= 2) CYC_MLRC_M(2);
    else if (cq <= 4) CYC_MLRC_M(4);
    else if (cq <= 8) CYC_MLRC_M(8);
    else CYC_MLRC_M(16);
    CYC_LAUNCH_CHECK("k_mlr_csr_margins");
  }
#undef CYC_MLRC_M
  hipLaunchKernelGGL(k_fold_columns, dim3(C), dim3(256), 0, st,
                     (const double*)p->slabMS.ptr, wtot, C, (double*)p->msTot.ptr);
  CYC_LAUNCH_CHECK("k_fold_columns");
  hipLaunchKernelGGL(k_fold_scalars, dim3(1), dim3(256), 0, st, (const double*)p->slabS.ptr, wtot,
                     2, (double*)p->scal.ptr);
  CYC_LAUNCH_CHECK("k_fold_scalars");
  int64_t R = 0, nb = 0;
  if ((rc = cyc_csc_blocks(csc, &R, &nb))) return rc;
  const int64_t* colptr;
  const int32_t* rowidx;
  const double* cv;
  if ((rc = cyc_csc_arrays(csc, &colptr, &rowidx, &cv))) return rc;
  const unsigned gblocks = (unsigned)(((int64_t)F + 3) / 4);
#define CYC_MLRC_G(Q)                                                                          \
  hipLaunchKernelGGL(k_mlr_csc_grad<Q>, dim3(gblocks), dim3(256), 0, st, colptr, rowidx, cv, nb, \
                     F, C, (const double*)mult, (const double*)p->msTot.ptr, p->fitIntercept,   \
                     p->fitWithMean, scaledMean, grad)
  {
    cyc::KernelTimer tg("k_mlr_csc_grad", st);
    if (cq <= 1) CYC_MLRC_G(1);
    else if (cq <= 2) CYC_MLRC_G(2);
    else if (cq <= 4) CYC_MLRC_G(4);
    else if (cq <= 8) CYC_MLRC_G(8);
    else CYC_MLRC_G(16);
    CYC_LAUNCH_CHECK("k_mlr_csc_grad");
  }
#undef CYC_MLRC_G
  if (p->fitIntercept) {
    hipLaunchKernelGGL(k_mlr_icpt, dim3((C + 255) / 256), dim3(256), 0, st, F, C,
                       (const double*)p->msTot.ptr, grad);
    CYC_LAUNCH_CHECK("k_mlr_icpt");
  }
  hipLaunchKernelGGL(k_add_scalars, dim3(1), dim3(1), 0, st, (const double*)p->scal.ptr, lossSum,
                     weightSum);
  CYC_LAUNCH_CHECK("k_add_scalars");
  return CYC_OK;
}

int cyc_softmax_exp_dev(const double* x, int64_t n, double* out, void* stream) {
  CYC_REQUIRE(n >= 0 && (n == 0 || (x && out)), "n >= 0 and non-null buffers");
  if (n == 0) return CYC_OK;
  const int64_t grid = std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_softmax_exp, dim3((unsigned)grid), dim3(256), 0, cyc::as_stream(stream), x,
                     n, out);
  CYC_LAUNCH_CHECK("k_softmax_exp");
  return CYC_OK;
}

}  // extern "C"
