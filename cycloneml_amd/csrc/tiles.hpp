// tiles.hpp -- internal interface of the row-block x column-tile layout
// (tiles.hip) for the binary block aggregators (logistic.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace cyc {

constexpr int kTileRows = 2048;               // rows per row block (R)
constexpr int kTileCols = 2048;               // columns per column chunk (W, at most)
constexpr int kTileWaves = 8;                 // waves per workgroup
constexpr int kTileSuperRows = kTileWaves * kTileRows;   // rows of one margin workgroup step
constexpr int kTileSuperCols = kTileWaves * kTileCols;   // columns of one gradient workgroup

// What the kernels need to walk a built layout.  Segment s = rb * T + c
// (row block rb, column chunk c) spans nonzeros [segStart[s], segStart[s+1])
// in CSR order; idx packs (row in block << 16 | column in chunk) -- or, for
// the compact format, 16 bits: the column and the row's step (tiles.hip) --
// and vals the fp64 values.
struct TilesView {
  int64_t n = 0;         // rows
  int F = 0;             // numFeatures
  int T = 1;             // column chunks
  int Wt = 1;            // columns per chunk (the last chunk may be shorter)
  int64_t nRB = 0;       // row blocks
  int64_t maxSeg = 0;    // entries of the longest segment
  bool compact = false;  // 16-bit compact entries (idx is then uint16_t[])
  const int64_t* segStart = nullptr;
  const uint32_t* idx = nullptr;
  const double* vals = nullptr;
};

int tiles_view(cyc_tiles t, TilesView* v);

// Margin pass: dots[r] = row r's dot with coef over its nonzeros, in
// column order.
int tiles_margin(const TilesView& v, const double* coef, double* dots, hipStream_t st);

// The rows' epilogue after it: dm[r] (the dot) becomes the per-row
// multiplier of aggregator `kind` (binary_rows.hpp) from margin =
// row_margin(offset + dot); per-workgroup (loss, weight, multiplierSum,
// sigmaGradSum) partials to slabS[wg * 4 + k], the workgroup count through
// *wgs (at most tiles_rows_blocks(n)).
int64_t tiles_rows_blocks(int64_t n);
// offsetDev: the offset in HBM (read by the kernel), else `offset`
int tiles_rows(int64_t n, const double* labels, const double* weights, int fitIntercept,
               int kind, double offset, const double* offsetDev, double lscale, double sigma,
               double eps, double* dm, double* slabS, int64_t* wgs, hipStream_t st);

// Gradient pass: slabG[range * F + f] = sum over the rows of row range
// `range` (row order) of vals * mult[row]; *ranges receives the range count.
// slabG needs tiles_ranges(v) * F doubles.
int tiles_ranges(const TilesView& v);
int tiles_grad(const TilesView& v, const double* mult, double* slabG, int* ranges,
               hipStream_t st);

}  // namespace cyc
