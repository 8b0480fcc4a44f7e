// tiles.hip -- the row-block x column-tile layout of a sparse (CSR) shard for
// the binary block aggregators: BinaryLogisticBlockAggregator.add
// (ml/optim/aggregator/BinaryLogisticBlockAggregator.scala:81-145) and the
// Hinge / LeastSquares / Huber / AFT aggregators of the same shape.
//
// Why a layout of its own.  An aggregator add runs two sparse gemv
// (BinaryLogisticBlockAggregator.scala:97 and :130; ml/linalg/BLAS.scala:
// 764-805): margins gather one fp64 coefficient per nonzero, the gradient
// gathers one fp64 multiplier per nonzero.  At F = 1M with 64 random columns
// per row those gathers are L2 requests, and round 1 measured both passes
// bound by that request rate (~146 G gathers/s), not by HBM.  Here the shard
// is cut into row blocks of R = 8192 rows and column tiles of W = 8192
// columns; a (row block, column tile) segment stores its nonzeros with the
// row inside the block and the column inside the tile packed into 32 bits,
// so both gathers become LDS reads:
//   margin pass    one workgroup per row block holds the block's 8192 partial
//                  dots in LDS and streams the coefficient tiles through LDS
//                  (all workgroups sweep the same tiles: L2 hits);
//   gradient pass  one workgroup per column tile (and row range) holds the
//                  tile's 8192 gradient sums in LDS and streams the
//                  multiplier slices through LDS.
// Either pass reads 12 B per nonzero (value + packed ids) and nothing else
// per nonzero.  Every segment is cut into 8 x 8 sub-segments (row range i x
// column range j, an eighth of each); wave i owns the rows of range i in the
// margin pass and wave j the columns of range j in the gradient pass, so each
// LDS sum has exactly one writer wave and its adds land in a fixed order:
// a row's dot in column order from 0.0 (the reference's CSR row loop,
// BLAS.scala:777-789, bit for bit), a column's gradient sum in row order
// within a row range (the transposed loop :790-804).
//
// Built once per dataset (like InstanceBlock.blokifyWithMaxMemUsage +
// persist, ml/feature/Instance.scala:146-187, LogisticRegression.scala:
// 967-970) by appending CSR row blocks: per chunk a stable radix sort of the
// nonzeros by (row block, tile, row range, column range) keeps each
// sub-segment in CSR order.  The CSR input can be freed after the append, so
// the layout is the only copy of the shard in HBM (12 B per nonzero + 0.5 %
// of segment offsets): a 200M x 1M, 64-per-row shard takes 157 GB.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "binary_rows.hpp"
#include "common.hpp"
#include "tiles.hpp"

struct cyc_tiles_s {
  int F = 0, T = 1, Wt = 1, WS = 1;
  int64_t capRows = 0, capNnz = 0, n = 0, nnz = 0;
  bool sealed = false;    // ends with a partial row block: no further appends
  std::mutex mu;
  cyc::DeviceBuffer segStart, subRel, idx, vals;
};

namespace {

using cyc::kTileCols;
using cyc::kTileRowRange;
using cyc::kTileRows;
using cyc::kTileSub;
using cyc::kTileWaves;

constexpr int kTPB = 512;                      // threads per workgroup (8 waves)
constexpr int kCPT = kTileCols / kTPB;         // coefficient / gradient entries per thread
constexpr int kRPT = kTileRows / kTPB;         // rows per thread
constexpr int kCap = 10;                       // nonzeros per lane prefetched per run

// ----------------------------------------------------------------- build

// Per nonzero of rows [0, rows) of a chunk: its sub-segment key
// ((rb * T + t) * 8 + i) * 8 + j and its packed ids.  Wave per row.
__global__ void k_tile_keys(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
                            int64_t rows, int64_t q0, int T, int Wt, int WS,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ packed) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < rows; r += stride) {
    const int64_t rbl = r / kTileRows;
    const uint32_t rin = (uint32_t)(r % kTileRows);
    const uint32_t i = rin / kTileRowRange;
    const int64_t p1 = rowptr[r + 1] - q0;
    for (int64_t p = rowptr[r] - q0 + lane; p < p1; p += 64) {
      const int c = colidx[p];
      const int t = c / Wt, cin = c - t * Wt;
      const uint32_t j = (uint32_t)(cin / WS);
      keys[p] = ((uint32_t)(rbl * T + t) * kTileWaves + i) * kTileWaves + j;
      packed[p] = (rin << 16) | (uint32_t)cin;
    }
  }
}

__global__ void k_tile_gather(const uint32_t* __restrict__ perm, int64_t cnt,
                              const uint32_t* __restrict__ packed, const double* __restrict__ vals,
                              uint32_t* __restrict__ outIdx, double* __restrict__ outVals) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < cnt;
       q += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t p = perm[q];
    outIdx[q] = packed[p];
    outVals[q] = vals[p];
  }
}

// starts[key] = first sorted position with key' >= key, key in [0, nkeys]
__global__ void k_tile_starts(const uint32_t* __restrict__ keys, int64_t cnt, int64_t nkeys,
                              int64_t* __restrict__ starts) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= cnt;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prev = q == 0 ? -1 : (int64_t)keys[q - 1];
    const int64_t cur = q == cnt ? nkeys : (int64_t)keys[q];
    for (int64_t k = prev + 1; k <= cur; ++k) starts[k] = q;
  }
}

// segment starts (absolute) and sub-segment offsets (relative) of the chunk
__global__ void k_tile_offsets(const int64_t* __restrict__ starts, int64_t nkeys, int64_t seg0,
                               int64_t base, int64_t* __restrict__ segStart,
                               uint32_t* __restrict__ subRel) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = k / kTileSub;
    const int64_t s0 = starts[s * kTileSub];
    if (k % kTileSub == 0) segStart[seg0 + s] = base + s0;
    subRel[(seg0 + s) * kTileSub + k % kTileSub] = (uint32_t)(starts[k] - s0);
  }
}

__global__ void k_set_i64(int64_t* p, int64_t v) { *p = v; }

// ----------------------------------------------------------------- passes

__device__ __forceinline__ void lds_add(double* p, double x) {
  __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// buffer resource over [p, p + bytes): lanes past the end read 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                           (int)std::min<int64_t>(bytes, 0x7fffffff), 0x00020000);
}

// Margin pass, persistent over (row block, column tile) steps: this
// workgroup's row blocks rb = blockIdx.x + i * gridDim.x, each swept over the
// T column tiles, as one flat sequence of steps g.  Per step: the
// coefficient tile goes registers -> LDS (the next step's tile is loaded
// meanwhile, an L2 hit), and each wave walks its row range's sub-segments
// (one contiguous run); the runs of the next TWO steps are in flight in
// registers (~100 KB per CU), across row-block boundaries too.
// The layout's arrays come as separate __restrict__ arguments: the
// per-step segment offsets are uniform, and only restrict-qualified
// read-only pointers let the compiler fetch them with scalar loads (counted
// by lgkmcnt), so reading them never waits on the runs in flight (vmcnt).
struct TileDims {
  int64_t n, nRB;
  int F, T, Wt;
};

__global__ __launch_bounds__(kTPB) void k_tiles_margin(
    TileDims v, const int64_t* __restrict__ segStart, const uint32_t* __restrict__ subRel,
    const uint32_t* __restrict__ vidx, const double* __restrict__ vvals,
    const double* __restrict__ labels, const double* __restrict__ weights,
    const double* __restrict__ coef, int fitIntercept, int kind, double offset, double lscale,
    double sigma, double eps, double* __restrict__ mult, double* __restrict__ slabS) {
  // dots[kTileRows + lane]: a per-lane sink for masked lanes (no branches,
  // no shared address among them)
  __shared__ double dots[kTileRows + 64];
  __shared__ double cf[kTileCols];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = v.T;
  const uint32_t sink = (uint32_t)(kTileRows + lane) << 16;
  // steps per row block padded to a multiple of 3 (the unroll of the run
  // buffers); the padding steps have empty runs and fetch nothing
  const int Tp = (T + 2) / 3 * 3;
  const int64_t myRB = v.nRB > blockIdx.x ? (v.nRB - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const int64_t G = myRB * Tp;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};     // loss, weight, multiplierSum, sigmaGradSum
  double creg[kCPT];
  uint32_t iA[kCap], iB[kCap], iC[kCap];
  double vA[kCap], vB[kCap], vC[kCap];
  int64_t sA = 0, lA = 0, sB = 0, lB = 0, sC = 0, lC = 0;

  auto rb_of = [&](int64_t g) { return (int64_t)blockIdx.x + (g / Tp) * gridDim.x; };
  auto run_of = [&](int64_t g, int64_t& s0, int64_t& len) {
    if (g >= G || g % Tp >= T) {   // past the end, or a padding step: an empty run
      s0 = 0;
      len = 0;
      return;
    }
    const int64_t seg = rb_of(g) * T + g % Tp;
    const int64_t base = segStart[seg];
    const uint32_t* sr = subRel + seg * kTileSub;
    const uint32_t a = sr[wave * kTileWaves];
    const uint32_t b = wave == kTileWaves - 1 ? (uint32_t)(segStart[seg + 1] - base)
                                              : sr[(wave + 1) * kTileWaves];
    s0 = base + a;
    len = (int64_t)b - (int64_t)a;
  };
  auto load_run = [&](int64_t s0, int64_t len, uint32_t (&ix)[kCap], double (&vx)[kCap]) {
    const auto ri = rsrc(vidx + s0, len * 4);
    const auto rv = rsrc(vvals + s0, len * 8);
    // lane part in the VGPR offset, chunk part in the scalar offset: one
    // offset register for all kCap loads
#pragma unroll
    for (int j = 0; j < kCap; ++j) {
      ix[j] = __builtin_amdgcn_raw_buffer_load_b32(ri, lane * 4, j * 256, 2);
      vx[j] = __builtin_bit_cast(double,
                                 __builtin_amdgcn_raw_buffer_load_b64(rv, lane * 8, j * 512, 2));
    }
  };
  auto load_coef = [&](int64_t g) {
    const int t = (int)(g % Tp);
    const int64_t c0 = t < T ? (int64_t)t * v.Wt : 0;
    const int wl = (g < G && t < T) ? (int)std::min<int64_t>(v.Wt, v.F - c0) : 0;
    const auto rc = rsrc(coef + c0, (int64_t)wl * 8);
#pragma unroll
    for (int i = 0; i < kCPT; ++i)
      creg[i] = __builtin_bit_cast(
          double, __builtin_amdgcn_raw_buffer_load_b64(rc, tid * 8, i * kTPB * 8, 0));
  };
  // branch-free: all gathers issue together, masked lanes add 0 to their sink
  auto consume = [&](int64_t len, const uint32_t (&ix)[kCap], const double (&vx)[kCap]) {
    double c[kCap];
#pragma unroll
    for (int j = 0; j < kCap; ++j) c[j] = cf[(j * 64 + lane < len ? ix[j] : sink) & 0xffff];
#pragma unroll
    for (int j = 0; j < kCap; ++j) {
      const bool on = j * 64 + lane < len;
      lds_add(&dots[(on ? ix[j] : sink) >> 16], on ? vx[j] * c[j] : 0.0);
    }
  };
  // One step g: coefficient tile to LDS, the loads of step g + 1's tile and
  // step g + 2's run issued (unconditionally: past the end they fetch
  // nothing, so the waits for the current run stay counted), the current
  // run into the row sums, the epilogue after a row block's last tile.  The
  // three run buffers rotate by unrolling (never by copying a register that
  // a load is still filling).
  auto step = [&](int64_t g, int64_t sc, int64_t lc, uint32_t (&ic)[kCap], double (&vc)[kCap],
                  int64_t& sn, int64_t& ln, uint32_t (&in)[kCap], double (&vn)[kCap]) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kCPT; ++i) cf[tid + kTPB * i] = creg[i];
    load_coef(g + 1);
    run_of(g + 2, sn, ln);
    load_run(sn, ln, in, vn);
    __syncthreads();
    consume(lc, ic, vc);
    for (int64_t b = kCap * 64; b < lc; b += kCap * 64) {   // rare: a long run
      load_run(sc + b, lc - b, ic, vc);
      consume(lc - b, ic, vc);
    }
  };

  load_coef(0);
  run_of(0, sA, lA);
  load_run(sA, lA, iA, vA);
  run_of(1, sB, lB);
  load_run(sB, lB, iB, vB);
  for (int64_t g0 = 0; g0 < G; g0 += Tp) {      // one row block per pass
#pragma unroll
    for (int i = 0; i < kRPT; ++i) dots[tid + kTPB * i] = 0.0;
    for (int64_t g = g0; g < g0 + Tp; g += 3) {
      step(g, sA, lA, iA, vA, sC, lC, iC, vC);
      step(g + 1, sB, lB, iB, vB, sA, lA, iA, vA);
      step(g + 2, sC, lC, iC, vC, sB, lB, iB, vB);
    }
    __syncthreads();
    // epilogue (BinaryLogisticBlockAggregator.scala:104-122 and siblings)
    const int64_t rb = rb_of(g0);
    for (int i = 0; i < kRPT; ++i) {
      const int rl = tid + kTPB * i;
      const int64_t r = rb * kTileRows + rl;
      if (r < v.n) {
        const double label = labels[r];
        const double margin = cyc::row_margin(kind, fitIntercept, offset, lscale, label, dots[rl]);
        const double w = weights ? weights[r] : 1.0;
        const double m = cyc::bin_row(kind, margin, w, label, acc[0], acc[1], acc[3], sigma, eps);
        acc[2] += m;
        mult[r] = m;
      }
    }
  }
  // workgroup partials: fixed shuffle tree per wave, then waves in order
  __shared__ double red[kTileWaves][4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc[k] += __shfl_xor(acc[k], m);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wave][k] = acc[k];
  }
  __syncthreads();
  if (tid < 4) {
    double s = 0.0;
    for (int w = 0; w < kTileWaves; ++w) s += red[w][tid];
    slabS[(int64_t)blockIdx.x * 4 + tid] = s;
  }
}

// Gradient pass: workgroup (tile t, row range) over its row blocks.  Per row
// block: the multiplier slice goes registers -> LDS (the next one loaded
// while this one is used); wave j walks the 8 sub-segments (i, j) of the
// segment as one virtual run -- lane position p lies in piece k when
// cum[k] <= p < cum[k + 1] -- with the next row block's run in flight.
struct GradRun {
  int64_t base;                     // segment start (absolute)
  uint32_t rel[kTileWaves];         // piece k's start, relative to base
  uint32_t cum[kTileWaves + 1];     // prefix lengths
};

__global__ __launch_bounds__(kTPB) void k_tiles_grad(
    TileDims v, const int64_t* __restrict__ segStart, const uint32_t* __restrict__ subRel,
    const uint32_t* __restrict__ vidx, const double* __restrict__ vvals,
    const double* __restrict__ mult, int ranges, double* __restrict__ slabG) {
  __shared__ double gt[kTileCols + 64];     // + a per-lane sink for masked lanes
  __shared__ double mv[kTileRows];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t sink = (uint32_t)(kTileCols + lane);
  const int range = blockIdx.x % ranges, t = blockIdx.x / ranges;
  const int64_t rbA = v.nRB * range / ranges, rbB = v.nRB * (range + 1) / ranges;
  const int64_t c0 = (int64_t)t * v.Wt;
  const int wl = (int)std::min<int64_t>(v.Wt, v.F - c0);
  double mreg[kRPT];
  uint32_t iA[kCap], iB[kCap], iC[kCap];
  double vA[kCap], vB[kCap], vC[kCap];
  GradRun rA, rB, rC;

  auto run_of = [&](int64_t rb, GradRun& r) {
    if (rb >= rbB) {     // past the range: an empty run (its loads read element 0)
      r.base = 0;
#pragma unroll
      for (int k = 0; k < kTileWaves; ++k) r.rel[k] = 0, r.cum[k] = 0;
      r.cum[kTileWaves] = 0;
      return;
    }
    const int64_t seg = rb * v.T + t;
    r.base = segStart[seg];
    const uint32_t segLen = (uint32_t)(segStart[seg + 1] - r.base);
    const uint32_t* sr = subRel + seg * kTileSub;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < kTileWaves; ++k) {
      const int e = k * kTileWaves + wave;
      const uint32_t a = sr[e];
      const uint32_t b = e + 1 < kTileSub ? sr[e + 1] : segLen;
      r.rel[k] = a;
      r.cum[k] = acc;
      acc += b - a;
    }
    r.cum[kTileWaves] = acc;
  };
  // element of virtual position p (p < cum[8]): p + rel[k] - cum[k] for the
  // piece k holding p, as p + rel[0] plus the (uniform, modulo 2^32) steps
  // of the pieces it has passed -- a compare, a select and an add per piece
  // (the steps are scalar work, once per run)
  auto elem = [&](const GradRun& r, const uint32_t (&step)[kTileWaves], uint32_t p) {
    uint32_t s = r.rel[0] + p;
#pragma unroll
    for (int kk = 1; kk < kTileWaves; ++kk) s += p >= r.cum[kk] ? step[kk] : 0u;
    return r.base + s;
  };
  auto load_run = [&](const GradRun& r, uint32_t p0, uint32_t (&ix)[kCap], double (&vx)[kCap]) {
    uint32_t step[kTileWaves];
    step[0] = 0;
#pragma unroll
    for (int k = 1; k < kTileWaves; ++k)
      step[k] = (r.rel[k] - r.cum[k]) - (r.rel[k - 1] - r.cum[k - 1]);
#pragma unroll
    for (int j = 0; j < kCap; ++j) {
      const uint32_t p = p0 + j * 64 + lane;
      const int64_t s = p < r.cum[kTileWaves] ? elem(r, step, p) : 0;   // masked lanes: element 0
      ix[j] = __builtin_nontemporal_load(vidx + s);
      vx[j] = __builtin_nontemporal_load(vvals + s);
    }
  };
  auto load_mult = [&](int64_t rb) {
    const int64_t r0 = rb * kTileRows;
    const auto rm = rsrc(mult + (rb < rbB ? r0 : 0),
                         rb < rbB ? std::min<int64_t>(kTileRows, v.n - r0) * 8 : 0);
#pragma unroll
    for (int i = 0; i < kRPT; ++i)
      mreg[i] = __builtin_bit_cast(
          double, __builtin_amdgcn_raw_buffer_load_b64(rm, tid * 8, i * kTPB * 8, 0));
  };
  auto consume = [&](int64_t rem, const uint32_t (&ix)[kCap], const double (&vx)[kCap]) {
    double m[kCap];
#pragma unroll
    for (int j = 0; j < kCap; ++j) m[j] = mv[(j * 64 + lane < rem ? ix[j] : 0u) >> 16];
#pragma unroll
    for (int j = 0; j < kCap; ++j) {
      const bool on = j * 64 + lane < rem;
      lds_add(&gt[on ? (ix[j] & 0xffff) : sink], on ? vx[j] * m[j] : 0.0);
    }
  };

#pragma unroll
  for (int i = 0; i < kCPT; ++i) gt[tid + kTPB * i] = 0.0;
  // one row block: multiplier slice to LDS, the next slice and the run two
  // row blocks ahead issued (unconditionally), the current run into the
  // column sums; run buffers rotate by unrolling
  auto step = [&](int64_t rb, const GradRun& rc, uint32_t (&ic)[kCap], double (&vc)[kCap],
                  GradRun& rn, uint32_t (&in)[kCap], double (&vn)[kCap]) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRPT; ++i) mv[tid + kTPB * i] = mreg[i];
    load_mult(rb + 1);
    run_of(rb + 2, rn);
    load_run(rn, 0, in, vn);
    __syncthreads();
    const uint32_t len = rc.cum[kTileWaves];
    consume(len, ic, vc);
    for (uint32_t b = kCap * 64; b < len; b += kCap * 64) {   // rare: a long run
      load_run(rc, b, ic, vc);
      consume(len - b, ic, vc);
    }
  };

  load_mult(rbA);
  run_of(rbA, rA);
  load_run(rA, 0, iA, vA);
  run_of(rbA + 1, rB);
  load_run(rB, 0, iB, vB);
  int64_t rb = rbA;
  for (; rb + 3 <= rbB; rb += 3) {
    step(rb, rA, iA, vA, rC, iC, vC);
    step(rb + 1, rB, iB, vB, rA, iA, vA);
    step(rb + 2, rC, iC, vC, rB, iB, vB);
  }
  if (rb < rbB) step(rb, rA, iA, vA, rC, iC, vC);
  if (rb + 1 < rbB) step(rb + 1, rB, iB, vB, rA, iA, vA);
  __syncthreads();
  double* out = slabG + (int64_t)range * v.F + c0;
#pragma unroll
  for (int i = 0; i < kCPT; ++i) {
    const int e = tid + kTPB * i;
    if (e < wl) out[e] = gt[e];
  }
}

}  // namespace

namespace cyc {

int tiles_view(cyc_tiles t, TilesView* v) {
  CYC_REQUIRE(t != nullptr && v != nullptr, "tiles must not be null");
  v->n = t->n;
  v->F = t->F;
  v->T = t->T;
  v->Wt = t->Wt;
  v->WS = t->WS;
  v->nRB = (t->n + kTileRows - 1) / kTileRows;
  v->segStart = (const int64_t*)t->segStart.ptr;
  v->subRel = (const uint32_t*)t->subRel.ptr;
  v->idx = (const uint32_t*)t->idx.ptr;
  v->vals = (const double*)t->vals.ptr;
  return CYC_OK;
}

int tiles_margin(const TilesView& v, const double* labels, const double* weights,
                 const double* coef, int fitIntercept, int kind, double offset, double lscale,
                 double sigma, double eps, double* mult, double* slabS, int64_t* wgs,
                 hipStream_t st) {
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(v.nRB, device_cus()));
  *wgs = grid;
  const TileDims d{v.n, v.nRB, v.F, v.T, v.Wt};
  hipLaunchKernelGGL(k_tiles_margin, dim3((unsigned)grid), dim3(kTPB), 0, st, d, v.segStart,
                     v.subRel, v.idx, v.vals, labels, weights, coef, fitIntercept, kind, offset,
                     lscale, sigma, eps, mult, slabS);
  CYC_LAUNCH_CHECK("k_tiles_margin");
  return CYC_OK;
}

int tiles_ranges(const TilesView& v) {
  const int64_t cus = device_cus();
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(v.nRB, 1),
                                                     cus / std::max(v.T, 1)));
}

int tiles_grad(const TilesView& v, const double* mult, double* slabG, int* ranges,
               hipStream_t st) {
  const int R = tiles_ranges(v);
  *ranges = R;
  const TileDims d{v.n, v.nRB, v.F, v.T, v.Wt};
  hipLaunchKernelGGL(k_tiles_grad, dim3((unsigned)((int64_t)v.T * R)), dim3(kTPB), 0, st, d,
                     v.segStart, v.subRel, v.idx, v.vals, mult, R, slabG);
  CYC_LAUNCH_CHECK("k_tiles_grad");
  return CYC_OK;
}

}  // namespace cyc

extern "C" {

int cyc_tiles_create(int32_t numFeatures, int64_t capacity_rows, int64_t capacity_nnz,
                     cyc_tiles* out) {
  CYC_REQUIRE(out != nullptr, "out must not be null");
  CYC_REQUIRE(numFeatures > 0, "numFeatures must be positive");
  CYC_REQUIRE(capacity_rows >= 0 && capacity_nnz >= 0, "capacities must be nonnegative");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  auto* t = new cyc_tiles_s();
  t->F = numFeatures;
  t->Wt = std::min(numFeatures, kTileCols);
  t->T = (numFeatures + t->Wt - 1) / t->Wt;
  t->WS = (t->Wt + kTileWaves - 1) / kTileWaves;
  t->capRows = capacity_rows;
  t->capNnz = capacity_nnz;
  const int64_t segs = (capacity_rows + kTileRows - 1) / kTileRows * t->T;
  int rc;
  if ((rc = t->segStart.reserve(sizeof(int64_t) * (size_t)(segs + 1))) ||
      (rc = t->subRel.reserve(sizeof(uint32_t) * (size_t)std::max<int64_t>(segs * kTileSub, 1))) ||
      (rc = t->idx.reserve(sizeof(uint32_t) * (size_t)std::max<int64_t>(capacity_nnz, 1))) ||
      (rc = t->vals.reserve(sizeof(double) * (size_t)std::max<int64_t>(capacity_nnz, 1)))) {
    delete t;
    return rc;
  }
  CYC_HIP(hipMemset(t->segStart.ptr, 0, sizeof(int64_t)));
  *out = t;
  return CYC_OK;
}

int cyc_tiles_destroy(cyc_tiles t) {
  delete t;
  return CYC_OK;
}

int64_t cyc_tiles_rows(cyc_tiles t) { return t ? t->n : -1; }
int64_t cyc_tiles_nnz(cyc_tiles t) { return t ? t->nnz : -1; }
int32_t cyc_tiles_features(cyc_tiles t) { return t ? t->F : -1; }
int32_t cyc_tiles_row_block(void) { return kTileRows; }

int64_t cyc_tiles_bytes(cyc_tiles t) {
  return t ? (int64_t)(t->segStart.bytes + t->subRel.bytes + t->idx.bytes + t->vals.bytes) : 0;
}

int cyc_tiles_append_dev(cyc_tiles t, const int64_t* rowptr, const int32_t* colidx,
                         const double* vals, int64_t rows, void* stream) {
  CYC_REQUIRE(t != nullptr, "tiles must not be null");
  CYC_REQUIRE(rows >= 0, "rows must be nonnegative");
  if (rows == 0) return CYC_OK;
  CYC_REQUIRE(rowptr != nullptr, "rowptr must not be null");
  std::lock_guard<std::mutex> g(t->mu);
  CYC_REQUIRE(!t->sealed, "the layout ends with a partial row block: append whole row blocks of "
                          "cyc_tiles_row_block() rows, except the last append");
  CYC_REQUIRE(t->n + rows <= t->capRows, "appending " + std::to_string(rows) + " rows exceeds "
                                         "the capacity of " + std::to_string(t->capRows) + " rows");
  hipStream_t st = cyc::as_stream(stream);
  int64_t ends[2];
  CYC_HIP(hipMemcpyAsync(&ends[0], rowptr, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipMemcpyAsync(&ends[1], rowptr + rows, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  const int64_t q0 = ends[0], chunkNnz = ends[1] - ends[0];
  CYC_REQUIRE(chunkNnz >= 0, "rowptr must be nondecreasing");
  CYC_REQUIRE(t->nnz + chunkNnz <= t->capNnz,
              "appending " + std::to_string(chunkNnz) + " nonzeros exceeds the capacity of " +
                  std::to_string(t->capNnz));
  CYC_REQUIRE(chunkNnz == 0 || (colidx != nullptr && vals != nullptr),
              "colidx and values must not be null");
  if (int rc = cyc::check_csr_indices(rowptr, colidx, rows, t->F, st)) return rc;
  const int T = t->T;
  // sub-chunks of at most 128 row blocks: bounded scratch, 32-bit sort keys
  const int64_t chRows = (int64_t)128 * kTileRows;
  const int64_t rb0 = t->n / kTileRows;
  cyc::DeviceBuffer keys, packed, keysOut, perm, starts, tmp;
  for (int64_t a = 0; a < rows; a += chRows) {
    const int64_t b = std::min(rows, a + chRows);
    int64_t qa = 0, qb = 0;
    CYC_HIP(hipMemcpyAsync(&qa, rowptr + a, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipMemcpyAsync(&qb, rowptr + b, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipStreamSynchronize(st));
    const int64_t cnt = qb - qa;
    const int64_t nrb = (b - a + kTileRows - 1) / kTileRows;
    const int64_t nkeys = nrb * T * kTileSub;
    const int64_t seg0 = (rb0 + a / kTileRows) * T;
    CYC_REQUIRE(cnt < ((int64_t)1 << 32), "a chunk of 128 row blocks holds 2^32 nonzeros or more");
    int rc;
    if ((rc = starts.reserve(sizeof(int64_t) * (size_t)(nkeys + 1)))) return rc;
    if (cnt > 0) {
      if ((rc = keys.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
          (rc = packed.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
          (rc = keysOut.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
          (rc = perm.reserve(sizeof(uint32_t) * (size_t)cnt)))
        return rc;
      hipLaunchKernelGGL(k_tile_keys, dim3(8192), dim3(256), 0, st, rowptr + a, colidx + (qa - q0),
                         b - a, qa, T, t->Wt, t->WS, (uint32_t*)keys.ptr, (uint32_t*)packed.ptr);
      CYC_LAUNCH_CHECK("k_tile_keys");
      unsigned endBit = 1;
      while (endBit < 32 && ((int64_t)1 << endBit) < nkeys) ++endBit;
      size_t tmpBytes = 0;
      rocprim::counting_iterator<uint32_t> pos(0);
      CYC_HIP(rocprim::radix_sort_pairs(nullptr, tmpBytes, (const uint32_t*)keys.ptr,
                                        (uint32_t*)nullptr, pos, (uint32_t*)nullptr, (size_t)cnt,
                                        0, endBit, st));
      if ((rc = tmp.reserve(tmpBytes))) return rc;
      CYC_HIP(rocprim::radix_sort_pairs(tmp.ptr, tmpBytes, (const uint32_t*)keys.ptr,
                                        (uint32_t*)keysOut.ptr, pos, (uint32_t*)perm.ptr,
                                        (size_t)cnt, 0, endBit, st));
      hipLaunchKernelGGL(k_tile_gather, dim3(8192), dim3(256), 0, st, (const uint32_t*)perm.ptr,
                         cnt, (const uint32_t*)packed.ptr, vals + (qa - q0),
                         (uint32_t*)t->idx.ptr + t->nnz, (double*)t->vals.ptr + t->nnz);
      CYC_LAUNCH_CHECK("k_tile_gather");
    }
    hipLaunchKernelGGL(k_tile_starts, dim3((unsigned)std::min<int64_t>((cnt + 256) / 256, 8192)),
                       dim3(256), 0, st, (const uint32_t*)keysOut.ptr, cnt, nkeys,
                       (int64_t*)starts.ptr);
    CYC_LAUNCH_CHECK("k_tile_starts");
    hipLaunchKernelGGL(k_tile_offsets,
                       dim3((unsigned)std::min<int64_t>((nkeys + 255) / 256, 8192)), dim3(256), 0,
                       st, (const int64_t*)starts.ptr, nkeys, seg0, t->nnz,
                       (int64_t*)t->segStart.ptr, (uint32_t*)t->subRel.ptr);
    CYC_LAUNCH_CHECK("k_tile_offsets");
    t->nnz += cnt;
    // scratch is reused by the next sub-chunk on this stream; freed on return
  }
  t->n += rows;
  if (t->n % kTileRows != 0) t->sealed = true;
  const int64_t segs = (t->n + kTileRows - 1) / kTileRows * T;
  hipLaunchKernelGGL(k_set_i64, dim3(1), dim3(1), 0, st, (int64_t*)t->segStart.ptr + segs, t->nnz);
  CYC_LAUNCH_CHECK("k_set_i64");
  CYC_HIP(hipStreamSynchronize(st));
  return CYC_OK;
}

}  // extern "C"
