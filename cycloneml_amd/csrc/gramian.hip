// gramian.hip -- RowMatrix Gramian / dense covariance on gfx950 (MI355X).
//
// Replaces the per-row BLAS.spr seqOp of RowMatrix.computeGramianMatrix
// (mllib/linalg/distributed/RowMatrix.scala:130-161) and of
// computeDenseVectorCovariance (:163-220), plus triuToFull (:845-867).
//
// U (packed upper, column-major: U[j(j+1)/2 + i], i <= j) += sum_r x_r x_r^T
// is a syrk with a huge contraction dimension (rows).  Layout / schedule:
//   - output split in 128 x 128 tiles, only the upper block triangle;
//   - rows split in S contiguous ranges (split-K) so that tiles x S >> 256
//     CUs; each workgroup accumulates its tile over its range with
//     v_mfma_f64_16x16x4f64 (4 waves, 64 x 64 per wave = 16 accumulators);
//   - 16-row chunks of the two 128-column panels are staged through LDS
//     (row stride 144 doubles: the two 16-lane halves of a ds_read_b64 hit
//     disjoint banks), the next chunk prefetched into registers;
//   - the covariance variant subtracts the mean while staging, which is the
//     reference's na(index) = ta(index) - means(index) bit for bit;
//   - partial tiles go to slabs, a second kernel folds the S slabs in fixed
//     order into U (deterministic, no atomics).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include <cstdlib>
#include <string>
#include <type_traits>

#include "common.hpp"

// 1: the plain k_gram_dma's blocks grouped by row split per XCD (an A/B
// switch; the covariance form keeps the 2-D grid: grouped, it measured
// 625.7 vs 586.0 ms at 30M x 1024 for a 6 % smaller FETCH_SIZE)
#ifndef CYC_GRAM_SKIPLOW
#define CYC_GRAM_SKIPLOW 1   // k_gram_dma covariance: diagonal tiles skip lower MFMAs
#endif
#ifndef CYC_GRAM_XCDMAP
#define CYC_GRAM_XCDMAP 1
#endif

namespace {

constexpr int TILE = 128;
constexpr int KC = 16;             // rows per LDS chunk
constexpr int LDSW = TILE + 16;    // LDS row stride (doubles)
constexpr int GT = 256;            // threads per workgroup

__global__ __launch_bounds__(GT, 2) void k_gram_tiles(
    const double* __restrict__ X, int64_t nrows, int p, const double* __restrict__ mean,
    int tilesPerSide, int64_t rowsPerSplit, double* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) double Ai[KC * LDSW];
  __shared__ __attribute__((aligned(16))) double Aj[KC * LDSW];
  // blockIdx.x -> (tile pair ti <= tj), blockIdx.y -> row split
  int t = blockIdx.x, ti = 0;
  while (t >= tilesPerSide - ti) { t -= tilesPerSide - ti; ++ti; }
  const int tj = ti + t;
  const int I0 = ti * TILE, J0 = tj * TILE;
  const int64_t r0 = (int64_t)blockIdx.y * rowsPerSplit;
  const int64_t r1 = min<int64_t>(nrows, r0 + rowsPerSplit);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wy = wave >> 1, wx = wave & 1;

  cyc_double4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = cyc_double4{0.0, 0.0, 0.0, 0.0};

  // Staging map: KC rows x 128 cols per panel = 2048 doubles; 256 threads x 8.
  // thread -> row sr = tid >> 4, cols sc..sc+7 (sc = (tid & 15) * 8)
  const int sr = tid >> 4, sc = (tid & 15) * 8;
  double ri[8], rj[8];
  auto load_panel = [&](const double* rowp, int c0, double* dst) {
    if ((p & 1) == 0 && c0 + 8 <= p) {
      // 64 contiguous bytes per thread: 4 x 16-byte loads
      const double2* v = reinterpret_cast<const double2*>(rowp + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        double2 t2 = v[e];
        dst[2 * e] = t2.x;
        dst[2 * e + 1] = t2.y;
      }
      if (mean) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = dsub(dst[e], mean[c0 + e]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        double v = 0.0;
        if (c < p) {
          v = rowp[c];
          if (mean) v = dsub(v, mean[c]);
        }
        dst[e] = v;
      }
    }
  };
  auto load = [&](int64_t rb) {
    const int64_t r = rb + sr;
    if (r < r1) {
      const double* rowp = X + r * p;
      load_panel(rowp, I0 + sc, ri);
      load_panel(rowp, J0 + sc, rj);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) ri[e] = rj[e] = 0.0;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      Ai[sr * LDSW + sc + e] = ri[e];
      Aj[sr * LDSW + sc + e] = rj[e];
    }
  };

  if (r0 < r1) load(r0);
  for (int64_t rb = r0; rb < r1; rb += KC) {
    __syncthreads();
    store();
    __syncthreads();
    if (rb + KC < r1) load(rb + KC);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      double a[4], b[4];
      const int krow = kk + (lane >> 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = Ai[krow * LDSW + wy * 64 + q * 16 + (lane & 15)];
        b[q] = Aj[krow * LDSW + wx * 64 + q * 16 + (lane & 15)];
      }
#pragma unroll
      for (int qa = 0; qa < 4; ++qa)
#pragma unroll
        for (int qb = 0; qb < 4; ++qb)
          acc[qa][qb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[qa], b[qb], acc[qa][qb], 0, 0, 0);
    }
  }

  // slab layout: [split][tilepair][i (128)][j (128)]
  const int pairs = tilesPerSide * (tilesPerSide + 1) / 2;
  double* out = slab + ((size_t)blockIdx.y * pairs + blockIdx.x) * TILE * TILE;
#pragma unroll
  for (int qa = 0; qa < 4; ++qa)
#pragma unroll
    for (int qb = 0; qb < 4; ++qb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = wy * 64 + qa * 16 + (lane >> 4) + 4 * r;
        const int j = wx * 64 + qb * 16 + (lane & 15);
        out[i * TILE + j] = acc[qa][qb][r];
      }
}

// The same tiles with the panels DMA'd from HBM straight into LDS
// (buffer_load ... lds, one 1 KiB row of a panel per wave instruction: no
// staging registers, no ds_write) into NB = 2 chunk buffers: the next
// chunk's DMAs fly during this one's MFMAs, one barrier per chunk.  At
// 30M x 1024 on one box: 8-row chunks with three workgroups per CU (166
// VGPRs, 36 KB of LDS) 498.0 ms; 16-row chunks, two per CU 515.0; 8-row
// chunks in three buffers, two per CU 525.8; 16-row chunks in three
// buffers, one per CU 574.4; the staged k_gram_tiles 542.5.  A chunk's rows past
// the split's end read as zero (buffer range); columns past p of the last
// panel read the next row's values, which only reach tile entries the fold
// discards.  MEAN: the mean is subtracted as the operands leave LDS (the
// same dsub as the staged kernel).  Rows past the split's end are DMA'd
// from the mean vector, so they centre to exact zeros (as SPARK-26158's
// accuracy case needs: a correction after the loop, missing rows x mean_i
// mean_j, cancels catastrophically there) with no select in the loop
// (zeroing them per operand cost two selects per operand and k-step; a
// second, select-free copy of the loop body for the full chunks spilled).
// The 8-row, three-per-CU form spills in the MEAN case (564 B), and the
// means read from LDS instead of registers measured 611.7 vs 567.7 ms at
// 30M x 1024.
// Needs p even (16-byte rows of a panel); odd p takes k_gram_tiles.
// MEAN 2 (CYC_COV_KERNEL=lds, a measurement switch): each wave centres the
// rows it DMA'd once, in LDS, between its DMA's landing and the chunk's
// barrier (x - mean by the same dsub, so the same bits), and the MFMAs read
// centred operands -- half the subtractions of MEAN 1 (each panel element
// is read by two waves), no mean registers in the loop (168 VGPRs), so it
// runs the plain form's 8-row chunks at three workgroups per CU with the
// XCD grouping.  Measured slower: 555.2 vs 548.4 ms at 30M x 1024 (29
// Gramian tests green with it); the centring pass doubles the chunk's LDS
// traffic and sits between the DMA wait and the barrier.
// SUMS (plain form only): the column sums ride the syrk.  On a diagonal
// tile the wave of rows 64..127 x columns 0..63 computes entries the fold
// discards (below the diagonal); in the SUMS form it runs 8 MFMAs per k-step
// instead of 16, each with one operand the constant 1.0: acc[q][q] += 1 x
// B[q] (the column sums of panel columns q*16 .. q*16+15, every output row
// the same) and acc[q][q+1 mod 4] += A[q] x 1 (columns 64 + q*16 ..), and
// writes the tile's 128 sums to sumsSlab[split][tile][128]
// (k_gram_sums_fold).  The other waves run the plain loop.  (Adding the
// rows with VALU from LDS on the diagonal workgroups cost 35-50 ms of 489:
// the reads either waited out the DMA prefetch or stalled the wave.)
template <int MEAN, int KCH = 8, int NB = 2, int OCC = 3,
          bool XCDMAP = MEAN != 1 && CYC_GRAM_XCDMAP, bool SUMS = false>
__global__ __launch_bounds__(GT, OCC) void k_gram_dma(
    const double* __restrict__ X, int64_t nrows, int p, const double* __restrict__ mean,
    int tilesPerSide, int64_t rowsPerSplit, int splits, double* __restrict__ slab,
    double* __restrict__ sumsSlab) {
  static_assert(!SUMS || MEAN == 0, "column sums ride the plain form only");
  __shared__ __attribute__((aligned(16))) double lds[NB * 2 * KCH * LDSW];   // the chunk panels
  auto Pn = [&](int b, int pn) { return lds + (b * 2 + pn) * KCH * LDSW; };
  constexpr int DPW = KCH / 2;   // DMAs per wave per chunk
  // a 1-D grid dealt round-robin over the 8 XCDs (blocks b and b + 8 share
  // one): block b -> XCD slot b % 8, k = b / 8; the XCD's k-th block takes
  // tile pair k % pairs of split 8 (k / pairs) + b % 8, so all tile pairs
  // of a split run on one XCD, started together, and the panels they share
  // can be L2 hits there (splits padded to a multiple of 8: the padding
  // blocks leave at once)
  const int pairs = tilesPerSide * (tilesPerSide + 1) / 2;
  int pair, split;
  if constexpr (XCDMAP) {
    const int kq = blockIdx.x >> 3;
    pair = kq % pairs;
    split = (kq / pairs) * 8 + (blockIdx.x & 7);
    if (split >= splits) return;
  } else {
    pair = blockIdx.x;
    split = blockIdx.y;
  }
  int t = pair, ti = 0;
  while (t >= tilesPerSide - ti) { t -= tilesPerSide - ti; ++ti; }
  const int tj = ti + t;
  const int I0 = ti * TILE, J0 = tj * TILE;
  const int64_t r0 = (int64_t)split * rowsPerSplit;
  const int64_t r1 = min<int64_t>(nrows, r0 + rowsPerSplit);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wy = wave >> 1, wx = wave & 1;

  cyc_double4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = cyc_double4{0.0, 0.0, 0.0, 0.0};
  double mI[4], mJ[4];
  if constexpr (MEAN == 1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ci = I0 + wy * 64 + q * 16 + (lane & 15), cj = J0 + wx * 64 + q * 16 + (lane & 15);
      mI[q] = ci < p ? mean[ci] : 0.0;
      mJ[q] = cj < p ? mean[cj] : 0.0;
    }
  }
  // chunk rb into buffer b: wave w DMAs rows KCH/4 w .. of both panels.
  // MEAN: a row past the split's end is the mean itself (its panel columns
  // DMA'd from the mean vector), which the subtraction below turns into
  // exact zeros -- no masking in the loop (the row index is wave-uniform,
  // so the choice is a scalar one)
  auto issue = [&](int64_t rb, int b) {
    const int64_t nr = max<int64_t>(0, min<int64_t>(KCH, r1 - rb));
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (nr ? rb : 0) * p), (short)0,
                                                      (int)(nr * p * 8), 0x00020000);
    const auto rm = __builtin_amdgcn_make_buffer_rsrc((void*)(MEAN ? mean : X), (short)0,
                                                      MEAN ? p * 8 : 0, 0x00020000);
#pragma unroll
    for (int u = 0; u < KCH / 4; ++u) {
      const int rr = wave * (KCH / 4) + u;
      const bool pad = MEAN != 0 && rr >= nr;
#pragma unroll
      for (int pn = 0; pn < 2; ++pn)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            pad ? rm : rs, (__attribute__((address_space(3))) void*)(Pn(b, pn) + rr * LDSW), 16,
            ((pad ? 0 : rr * p) + (pn ? J0 : I0)) * 8 + lane * 16, 0, 0, 0);
    }
  };
  // Covariance form: on a diagonal tile the wave of rows 64..127 x columns
  // 0..63 covers only entries the fold discards (below the diagonal): it
  // skips its MFMAs and leaves the pipe to the other workgroup's waves on
  // its SIMD (it still DMAs its rows and meets every barrier); with
  // SKIPLOW 2 the two diagonal waves also skip their 16x16 blocks below the
  // diagonal.  (The plain form, three workgroups per CU, measured slower
  // with it: 507.7 vs 488.6 ms.)
  const bool idle = CYC_GRAM_SKIPLOW && MEAN == 1 && ti == tj && wy > wx;
  const bool tri = CYC_GRAM_SKIPLOW >= 2 && MEAN == 1 && ti == tj && wy == wx;
  const bool sumsWave = SUMS && ti == tj && wy > wx && sumsSlab;   // wave-uniform
  auto compute = [&](int b, auto asSums) {
    if (idle) return;
    const double* Ai = Pn(b, 0);
    const double* Aj = Pn(b, 1);
#pragma unroll
    for (int kk = 0; kk < KCH; kk += 4) {
      double a[4], bb[4];
      const int krow = kk + (lane >> 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = Ai[krow * LDSW + wy * 64 + q * 16 + (lane & 15)];
        bb[q] = Aj[krow * LDSW + wx * 64 + q * 16 + (lane & 15)];
      }
      if constexpr (MEAN == 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a[q] = dsub(a[q], mI[q]);
          bb[q] = dsub(bb[q], mJ[q]);
        }
      }
      if constexpr (decltype(asSums)::value) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, bb[q], acc[q][q], 0, 0, 0);
          acc[q][(q + 1) & 3] =
              __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], 1.0, acc[q][(q + 1) & 3], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int qa = 0; qa < 4; ++qa)
#pragma unroll
          for (int qb = 0; qb < 4; ++qb)
            if (qa <= qb || !tri)
              acc[qa][qb] =
                  __builtin_amdgcn_mfma_f64_16x16x4f64(a[qa], bb[qb], acc[qa][qb], 0, 0, 0);
      }
    }
  };
  // NB - 1 chunks ahead; past the end the DMAs fetch nothing (empty
  // range), so every wave always has (NB - 2) DPW newer DMAs to leave in
  // flight at the counted wait
  // MEAN 2: the means of the two columns this lane DMAs in each panel
  double cm[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  if constexpr (MEAN == 2) {
#pragma unroll
    for (int pn = 0; pn < 2; ++pn)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int c = (pn ? J0 : I0) + lane * 2 + e;
        cm[pn][e] = c < p ? mean[c] : 0.0;
      }
  }
  auto centre = [&](int b) {   // this wave's DMA'd rows of chunk buffer b
#pragma unroll
    for (int u = 0; u < KCH / 4; ++u) {
      const int rr = wave * (KCH / 4) + u;
#pragma unroll
      for (int pn = 0; pn < 2; ++pn) {
        double2* q = reinterpret_cast<double2*>(Pn(b, pn) + rr * LDSW) + lane;
        double2 x = *q;
        x.x = dsub(x.x, cm[pn][0]);
        x.y = dsub(x.y, cm[pn][1]);
        *q = x;
      }
    }
  };
  // the loop as one straight block per form (a branch inside it splits the
  // block); the sums wave meets the same barriers the same number of times
  auto mainLoop = [&](auto asSums) {
#pragma unroll
    for (int c = 0; c < NB - 1; ++c) issue(r0 + c * KCH, c);
    int b = 0;
    for (int64_t rb = r0; rb < r1; rb += KCH) {
      if constexpr (NB == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 2) * DPW) : "memory");
      if constexpr (MEAN == 2) centre(b);
      __syncthreads();   // chunk rb landed (centred) everywhere; every wave is past rb - KCH
      issue(rb + (NB - 1) * KCH, b == 0 ? NB - 1 : b - 1);
      compute(b, asSums);
      b = b == NB - 1 ? 0 : b + 1;
    }
  };
  if (sumsWave) mainLoop(std::true_type{});
  else mainLoop(std::false_type{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (sumsWave) {
    // acc[q][q]: column q*16 + (lane & 15), the same in every row r;
    // acc[q][q+1]: column 64 + q*16 + (lane >> 4) + 4r, the same in every lane & 15
    double* ts = sumsSlab + ((size_t)split * tilesPerSide + ti) * TILE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (lane < 16) ts[q * 16 + lane] = acc[q][q][0];
      if ((lane & 15) == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[64 + q * 16 + (lane >> 4) + 4 * r] = acc[q][(q + 1) & 3][r];
    }
  }

  double* out = slab + ((size_t)split * pairs + pair) * TILE * TILE;
#pragma unroll
  for (int qa = 0; qa < 4; ++qa)
#pragma unroll
    for (int qb = 0; qb < 4; ++qb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = wy * 64 + qa * 16 + (lane >> 4) + 4 * r;
        const int j = wx * 64 + qb * 16 + (lane & 15);
        out[i * TILE + j] = acc[qa][qb][r];
      }
}

// U[iut(I0+i, J0+j)] += sum over splits (fixed order), upper triangle only.
__global__ void k_gram_fold(const double* __restrict__ slab, int splits, int tilesPerSide, int p,
                            double* __restrict__ U) {
  const int pair = blockIdx.y;
  int t = pair, ti = 0;
  while (t >= tilesPerSide - ti) { t -= tilesPerSide - ti; ++ti; }
  const int tj = ti + t;
  const int pairs = tilesPerSide * (tilesPerSide + 1) / 2;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;   // i * 128 + j
  if (e >= TILE * TILE) return;
  const int i = e / TILE, j = e % TILE;
  const int gi = ti * TILE + i, gj = tj * TILE + j;
  if (gi >= p || gj >= p || gi > gj) return;
  double s = 0.0;
  for (int sp = 0; sp < splits; ++sp) s = dadd(s, slab[((size_t)sp * pairs + pair) * TILE * TILE + e]);
  const int64_t idx = (int64_t)gj * (gj + 1) / 2 + gi;
  U[idx] = dadd(U[idx], s);
}

// sums[c] += the column sums of k_gram_dma<..., SUMS>, over splits in order.
__global__ void k_gram_sums_fold(const double* __restrict__ part, int splits, int tilesPerSide,
                                 int p, double* __restrict__ sums) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p) return;
  double s = 0.0;
  for (int sp = 0; sp < splits; ++sp) s = dadd(s, part[(size_t)sp * tilesPerSide * TILE + c]);
  sums[c] = dadd(sums[c], s);
}

// RowMatrix.triuToFull (:845-867): column-major full matrix from packed upper.
__global__ void k_triu_to_full(int n, const double* __restrict__ U, double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int col = (int)(e / n), row = (int)(e % n);
  G[e] = U[iut(row, col)];
}

// computeDenseVectorCovariance (:203-217): M(i,j) / (m - 1.0), symmetric.
__global__ void k_cov_finalize(int n, const double* __restrict__ U, double m1,
                               double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int col = (int)(e / n), row = (int)(e % n);
  G[e] = U[iut(row, col)] / m1;
}

// Column sums over a row range per thread (coalesced across the columns of a
// row), one partial per (split, column); folded in split order.  Feeds the
// mean of Statistics.colStats (mllib/stat/Statistics.scala:57) used by
// RowMatrix.computeCovariance (:452-467).
// SQ: the sums of squares beside them (the same rows, same order; the sums
// are the same bits either way), in the second half of the partials.
template <bool SQ>
__global__ void k_col_partial(const double* __restrict__ X, int64_t nrows, int p,
                              int64_t rowsPerSplit, double* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p) return;
  const int64_t r0 = (int64_t)blockIdx.y * rowsPerSplit;
  const int64_t r1 = min<int64_t>(nrows, r0 + rowsPerSplit);
  double s = 0.0, q = 0.0;
  // nontemporal: the rows stream through once
  for (int64_t r = r0; r < r1; ++r) {
    const double x = __builtin_nontemporal_load(&X[r * p + c]);
    s = dadd(s, x);
    if constexpr (SQ) q = dadd(q, dmul(x, x));
  }
  part[(int64_t)blockIdx.y * p + c] = s;
  if constexpr (SQ) part[((int64_t)gridDim.y + blockIdx.y) * p + c] = q;
}

__global__ void k_col_fold(const double* __restrict__ part, int splits, int p,
                           double* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p) return;
  double s = 0.0;
  for (int sp = 0; sp < splits; ++sp) s = dadd(s, part[(int64_t)sp * p + c]);
  out[c] = dadd(out[c], s);
}


// CSR rows [r0, r0 + rows) scattered into a zeroed dense row-major chunk
// (one wave per row): the sparse rows of a RowMatrix reach the same syrk.
// For a nonzero x_j the sparse spr branch (mllib/linalg/BLAS.scala:269-298)
// adds (alpha x_j) x_i exactly as dspr does, so the densified rows give the
// reference's per-row products.
__global__ __launch_bounds__(256) void k_csr_densify(const int64_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ colidx,
                                                     const double* __restrict__ vals, int64_t r0,
                                                     int64_t rows, int p,
                                                     double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  double* o = out + r * p;
  const int64_t a = rowptr[r0 + r], b = rowptr[r0 + r + 1];
  for (int64_t k = a + lane; k < b; k += 64) o[colidx[k]] = vals[k];
}

// RowMatrix.isSparseMatrix (:439-441): rows with sparsity() < 0.5, where
// sparsity = 1.0 - numNonzeros / size (mllib Vector.sparsity); the matrix is
// sparse iff the count is 0.
// CSR rows: a thread per row over its stored values.
__global__ __launch_bounds__(256) void k_dense_rows_csr(const int64_t* __restrict__ rowptr,
                                                        const double* __restrict__ vals, int64_t n,
                                                        int p, unsigned long long* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool dense = false;
  if (i < n) {
    int64_t nz = 0;
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) nz += vals[k] != 0.0;
    dense = 1.0 - (double)nz / (double)p < 0.5;
  }
  const unsigned long long m = __ballot(dense);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(cnt, (unsigned long long)__popcll(m));
}

// Dense rows: a wave per row, the lanes across its columns (coalesced), the
// row's nonzeros counted by ballots; grid-stride over the rows.
__global__ __launch_bounds__(256) void k_dense_rows(const double* __restrict__ X, int64_t n, int p,
                                                    unsigned long long* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long mine = 0;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += waves) {
    const double* row = X + i * p;
    int64_t nz = 0;
    for (int j = 0; j < p; j += 64) {
      const bool on = j + lane < p && row[j + lane] != 0.0;
      nz += __popcll(__ballot(on));
    }
    mine += 1.0 - (double)nz / (double)p < 0.5 ? 1 : 0;
  }
  if (lane == 0 && mine) atomicAdd(cnt, mine);
}

// computeSparseVectorCovariance (:222-246) from the packed Gramian:
// alpha = m / m1 * mean(i); G(i, j) = G(i, j) / m1 - alpha * mean(j) for
// i <= j, mirrored.
__global__ void k_sparse_cov_finalize(int n, const double* __restrict__ U, double m,
                                      const double* __restrict__ mean, double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int col = (int)(e / n), row = (int)(e % n);
  const int i = min(row, col), j = max(row, col);
  const double m1 = m - 1.0;
  const double alpha = m / m1 * mean[i];
  G[e] = U[iut(i, j)] / m1 - alpha * mean[j];
}

}  // namespace

struct cyc_gramian_plan_s {
  int p = 0;
  std::mutex mu;
  cyc::DeviceBuffer slab;
  cyc::DeviceBuffer chunk;   // densified CSR rows
  cyc::DeviceBuffer sumSlab;  // k_gram_dma<..., SUMS> column-sum partials
};

namespace {

int accumulate_locked(cyc_gramian_plan plan, const double* X, int64_t nrows, const double* mean,
                      double* U, double* sums, hipStream_t st);
int col_sums_locked(cyc_gramian_plan plan, const double* X, int64_t nrows, double* sums,
                    double* sumsq, hipStream_t st);

// CSR rows in chunks of about 1 GiB of dense rows: densify, then `dense`.
template <class F>
int over_csr_chunks(cyc_gramian_plan plan, const int64_t* rowptr, const int32_t* colidx,
                    const double* vals, int64_t nrows, hipStream_t st, F dense) {
  const int p = plan->p;
  const int64_t R = std::max<int64_t>(256, ((int64_t)1 << 30) / (8 * (int64_t)p)) / 256 * 256;
  const int64_t rows = std::min<int64_t>(R, nrows);
  if (int rc = plan->chunk.reserve(sizeof(double) * (size_t)rows * p)) return rc;
  double* buf = (double*)plan->chunk.ptr;
  for (int64_t r0 = 0; r0 < nrows; r0 += R) {
    const int64_t nr = std::min<int64_t>(R, nrows - r0);
    CYC_HIP(hipMemsetAsync(buf, 0, sizeof(double) * (size_t)nr * p, st));
    hipLaunchKernelGGL(k_csr_densify, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, st, rowptr,
                       colidx, vals, r0, nr, p, buf);
    CYC_LAUNCH_CHECK("k_csr_densify");
    if (int rc = dense((const double*)buf, nr)) return rc;
  }
  return CYC_OK;
}

}  // namespace

extern "C" {

int cyc_gramian_plan_create(int32_t ncols, cyc_gramian_plan* plan) {
  CYC_REQUIRE(plan != nullptr, "plan must not be null");
  if (ncols > 65535)
    CYC_REQUIRE(false, "Argument with more than 65535 cols: " + std::to_string(ncols));
  CYC_REQUIRE(ncols > 0, "ncols must be positive");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  auto* p = new cyc_gramian_plan_s();
  p->p = ncols;
  *plan = p;
  return CYC_OK;
}

int cyc_gramian_plan_destroy(cyc_gramian_plan plan) {
  delete plan;
  return CYC_OK;
}

int cyc_gramian_accumulate_dev(cyc_gramian_plan plan, const double* X, int64_t nrows,
                               const double* mean, double* U, void* stream) {
  CYC_REQUIRE(plan != nullptr && U != nullptr, "plan and U must not be null");
  CYC_REQUIRE(nrows >= 0, "nrows >= 0");
  if (nrows == 0) return CYC_OK;
  std::lock_guard<std::mutex> g(plan->mu);
  return accumulate_locked(plan, X, nrows, mean, U, nullptr, cyc::as_stream(stream));
}

int cyc_gramian_accumulate_sums_dev(cyc_gramian_plan plan, const double* X, int64_t nrows,
                                    double* U, double* sums, void* stream) {
  CYC_REQUIRE(plan != nullptr && U != nullptr && sums != nullptr,
              "plan, U and sums must not be null");
  CYC_REQUIRE(nrows >= 0, "nrows >= 0");
  if (nrows == 0) return CYC_OK;
  std::lock_guard<std::mutex> g(plan->mu);
  return accumulate_locked(plan, X, nrows, nullptr, U, sums, cyc::as_stream(stream));
}

int cyc_gramian_accumulate_csr_dev(cyc_gramian_plan plan, const int64_t* rowptr,
                                   const int32_t* colidx, const double* vals, int64_t nrows,
                                   const double* mean, double* U, void* stream) {
  CYC_REQUIRE(plan != nullptr && U != nullptr, "plan and U must not be null");
  CYC_REQUIRE(nrows >= 0, "nrows >= 0");
  if (nrows == 0) return CYC_OK;
  CYC_REQUIRE(rowptr && colidx && vals, "non-null CSR arrays");
  hipStream_t st = cyc::as_stream(stream);
  if (int rc = cyc::check_csr_indices(rowptr, colidx, nrows, plan->p, st)) return rc;
  std::lock_guard<std::mutex> g(plan->mu);
  return over_csr_chunks(plan, rowptr, colidx, vals, nrows, st, [&](const double* D, int64_t nr) {
    return accumulate_locked(plan, D, nr, mean, U, nullptr, st);
  });
}

int cyc_col_moments_dev(cyc_gramian_plan plan, const double* X, int64_t nrows, double* sums,
                        double* sumsq, void* stream) {
  CYC_REQUIRE(plan != nullptr && sums != nullptr, "plan and sums must not be null");
  CYC_REQUIRE(nrows >= 0, "nrows >= 0");
  if (nrows == 0) return CYC_OK;
  std::lock_guard<std::mutex> g(plan->mu);
  return col_sums_locked(plan, X, nrows, sums, sumsq, cyc::as_stream(stream));
}

int cyc_col_sums_dev(cyc_gramian_plan plan, const double* X, int64_t nrows, double* sums,
                     void* stream) {
  return cyc_col_moments_dev(plan, X, nrows, sums, nullptr, stream);
}

int cyc_col_moments_csr_dev(cyc_gramian_plan plan, const int64_t* rowptr, const int32_t* colidx,
                            const double* vals, int64_t nrows, double* sums, double* sumsq,
                            void* stream) {
  CYC_REQUIRE(plan != nullptr && sums != nullptr, "plan and sums must not be null");
  CYC_REQUIRE(nrows >= 0, "nrows >= 0");
  if (nrows == 0) return CYC_OK;
  CYC_REQUIRE(rowptr && colidx && vals, "non-null CSR arrays");
  hipStream_t st = cyc::as_stream(stream);
  if (int rc = cyc::check_csr_indices(rowptr, colidx, nrows, plan->p, st)) return rc;
  std::lock_guard<std::mutex> g(plan->mu);
  return over_csr_chunks(plan, rowptr, colidx, vals, nrows, st, [&](const double* D, int64_t nr) {
    return col_sums_locked(plan, D, nr, sums, sumsq, st);
  });
}

int cyc_col_sums_csr_dev(cyc_gramian_plan plan, const int64_t* rowptr, const int32_t* colidx,
                         const double* vals, int64_t nrows, double* sums, void* stream) {
  return cyc_col_moments_csr_dev(plan, rowptr, colidx, vals, nrows, sums, nullptr, stream);
}

int cyc_rowmatrix_dense_rows_dev(const double* X, const int64_t* rowptr, const double* vals,
                                 int64_t nrows, int32_t ncols, int64_t* count, void* stream) {
  CYC_REQUIRE(nrows >= 0 && ncols > 0 && count, "nrows >= 0, ncols > 0, non-null count");
  CYC_REQUIRE(nrows == 0 || (X != nullptr) != (rowptr != nullptr && vals != nullptr),
              "exactly one of the dense rows or the CSR (rowptr, values)");
  hipStream_t st = cyc::as_stream(stream);
  CYC_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), st));
  if (nrows == 0) return CYC_OK;
  if (X) {
    const int64_t grid = std::min<int64_t>((nrows + 3) / 4, 16 * (int64_t)cyc::device_cus());
    hipLaunchKernelGGL(k_dense_rows, dim3((unsigned)grid), dim3(256), 0, st, X, nrows, (int)ncols,
                       (unsigned long long*)count);
  } else {
    hipLaunchKernelGGL(k_dense_rows_csr, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, st,
                       rowptr, vals, nrows, (int)ncols, (unsigned long long*)count);
  }
  CYC_LAUNCH_CHECK("k_dense_rows");
  return CYC_OK;
}

int cyc_sparse_covariance_finalize_dev(int32_t n, const double* U, int64_t m, const double* mean,
                                       double* G, void* stream) {
  CYC_REQUIRE(m > 1, "RowMatrix.computeCovariance called on matrix with only " +
                         std::to_string(m) + " rows.  Cannot compute the covariance of a "
                         "RowMatrix with <= 1 row.");
  CYC_REQUIRE(n > 0 && U && G && mean, "n > 0 and non-null buffers");
  const int64_t tot = (int64_t)n * n;
  hipLaunchKernelGGL(k_sparse_cov_finalize, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     cyc::as_stream(stream), n, U, (double)m, mean, G);
  CYC_LAUNCH_CHECK("k_sparse_cov_finalize");
  return CYC_OK;
}

int cyc_triu_to_full_dev(int32_t n, const double* U, double* G, void* stream) {
  CYC_REQUIRE(n > 0 && U && G, "n > 0 and non-null buffers");
  const int64_t tot = (int64_t)n * n;
  hipLaunchKernelGGL(k_triu_to_full, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     cyc::as_stream(stream), n, U, G);
  CYC_LAUNCH_CHECK("k_triu_to_full");
  return CYC_OK;
}

int cyc_covariance_finalize_dev(int32_t n, const double* U, int64_t m, double* G, void* stream) {
  CYC_REQUIRE(m > 1, "RowMatrix.computeCovariance called on matrix with only " +
                         std::to_string(m) + " rows.  Cannot compute the covariance of a "
                         "RowMatrix with <= 1 row.");
  CYC_REQUIRE(n > 0 && U && G, "n > 0 and non-null buffers");
  const int64_t tot = (int64_t)n * n;
  hipLaunchKernelGGL(k_cov_finalize, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     cyc::as_stream(stream), n, U, (double)m - 1.0, G);
  CYC_LAUNCH_CHECK("k_cov_finalize");
  return CYC_OK;
}

}  // extern "C"

namespace {

int accumulate_locked(cyc_gramian_plan plan, const double* X, int64_t nrows, const double* mean,
                      double* U, double* sums, hipStream_t st) {
  const int p = plan->p;
  const int tps = (p + TILE - 1) / TILE;
  const int pairs = tps * (tps + 1) / 2;
  // split-K: at least 4 rounds of workgroups (2 per CU) and at least 64 rows
  // per split, with the split count whose last round is fullest (36 tile
  // pairs x 57 splits = 2052 workgroups ran 5 rounds, the 5th holding 4;
  // 36 x 71 = 2556 fill 4.99 rounds).
  // k_gram_dma for even p; CYC_GRAMIAN_KERNEL=tiles selects the staged
  // k_gram_tiles (a measurement switch)
  const char* gk = std::getenv("CYC_GRAMIAN_KERNEL");
  const bool dma = (p % 2) == 0 && !(gk && std::string(gk) == "tiles");
  // the covariance: the mean subtracted from every MFMA operand (MEAN 1), or
  // CYC_COV_KERNEL=lds for the chunks centred in LDS (MEAN 2; a measurement
  // switch)
  const char* ck = std::getenv("CYC_COV_KERNEL");
  const bool operand = mean && !(ck && std::string(ck) == "lds");
  // workgroups per CU: three for k_gram_dma's 8-row forms, two for the
  // 16-row MEAN 1 form (the mean operands spill at three) and k_gram_tiles
  const int64_t slots = (dma && !operand ? 3 : 2) * (int64_t)cyc::device_cus();
  const int64_t lo = std::max<int64_t>(1, (4 * slots + pairs - 1) / pairs);
  int64_t splits = cyc::balanced_splits(pairs, lo, 2 * lo, slots);
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, nrows / 64));
  int64_t rps = cyc::round_up((nrows + splits - 1) / splits, KC);
  splits = (nrows + rps - 1) / rps;
  int rc = plan->slab.reserve(sizeof(double) * (size_t)splits * pairs * TILE * TILE);
  if (rc) return rc;
  // the column sums ride the plain k_gram_dma; other forms add a pass
  const bool fusedSums = sums && dma && !mean;
  if (fusedSums) {
    rc = plan->sumSlab.reserve(sizeof(double) * (size_t)splits * tps * TILE);
    if (rc) return rc;
  }
  {
  // timed under the name of the kernel that runs (rocprofv3 lists the
  // covariance instances as k_gram_dma too)
  cyc::KernelTimer timer(!dma ? "k_gram_tiles" : mean ? "k_gram_dma_cov" : "k_gram_dma", st);
  const dim3 grid(pairs, (unsigned)splits);
  // the plain k_gram_dma: one dimension, splits padded to a multiple of 8
  // (XCDMAP)
  const dim3 gridD = CYC_GRAM_XCDMAP ? dim3((unsigned)(pairs * ((splits + 7) / 8) * 8)) : grid;
  double* slab = (double*)plan->slab.ptr;
  double* sumSlab = (double*)plan->sumSlab.ptr;
  if (dma && operand)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gram_dma<1, 16, 2, 2>), grid, dim3(GT), 0, st, X,
                       nrows, p, mean, tps, rps, (int)splits, slab, nullptr);
  else if (dma && mean)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gram_dma<2>), gridD, dim3(GT), 0, st, X, nrows, p,
                       mean, tps, rps, (int)splits, slab, nullptr);
  else if (fusedSums)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gram_dma<0, 8, 2, 3, CYC_GRAM_XCDMAP, true>), gridD,
                       dim3(GT), 0, st, X, nrows, p, mean, tps, rps, (int)splits, slab, sumSlab);
  else if (dma)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gram_dma<0>), gridD, dim3(GT), 0, st, X, nrows, p,
                       mean, tps, rps, (int)splits, slab, nullptr);
  else
    hipLaunchKernelGGL(k_gram_tiles, grid, dim3(GT), 0, st, X, nrows, p, mean, tps, rps, slab);
  CYC_LAUNCH_CHECK("k_gram_dma / k_gram_tiles");
  }
  hipLaunchKernelGGL(k_gram_fold, dim3(TILE * TILE / 256, pairs), dim3(256), 0, st,
                     (const double*)plan->slab.ptr, (int)splits, tps, p, U);
  CYC_LAUNCH_CHECK("k_gram_fold");
  if (fusedSums) {
    hipLaunchKernelGGL(k_gram_sums_fold, dim3((p + 255) / 256), dim3(256), 0, st,
                       (const double*)plan->sumSlab.ptr, (int)splits, tps, p, sums);
    CYC_LAUNCH_CHECK("k_gram_sums_fold");
  } else if (sums) {
    return col_sums_locked(plan, X, nrows, sums, nullptr, st);
  }
  return CYC_OK;
}

int col_sums_locked(cyc_gramian_plan plan, const double* X, int64_t nrows, double* sums,
                    double* sumsq, hipStream_t st) {
  const int p = plan->p;
  const int ctiles = (p + 255) / 256;
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(4096 / ctiles, nrows / 256));
  const int64_t rps = (nrows + splits - 1) / splits;
  splits = (nrows + rps - 1) / rps;
  int rc = plan->slab.reserve(sizeof(double) * (size_t)splits * p * (sumsq ? 2 : 1));
  if (rc) return rc;
  double* part = (double*)plan->slab.ptr;
  cyc::KernelTimer timer("k_col_sums", st);
  if (sumsq)
    hipLaunchKernelGGL(k_col_partial<true>, dim3(ctiles, (unsigned)splits), dim3(256), 0, st, X,
                       nrows, p, rps, part);
  else
    hipLaunchKernelGGL(k_col_partial<false>, dim3(ctiles, (unsigned)splits), dim3(256), 0, st, X,
                       nrows, p, rps, part);
  CYC_LAUNCH_CHECK("k_col_partial");
  hipLaunchKernelGGL(k_col_fold, dim3(ctiles), dim3(256), 0, st, (const double*)part,
                     (int)splits, p, sums);
  CYC_LAUNCH_CHECK("k_col_fold");
  if (sumsq) {
    hipLaunchKernelGGL(k_col_fold, dim3(ctiles), dim3(256), 0, st,
                       (const double*)part + splits * p, (int)splits, p, sumsq);
    CYC_LAUNCH_CHECK("k_col_fold");
  }
  return CYC_OK;
}

}  // namespace
