// tiles.hip -- the row-block x column-chunk layout of a sparse (CSR) shard
// for the binary block aggregators: BinaryLogisticBlockAggregator.add
// (ml/optim/aggregator/BinaryLogisticBlockAggregator.scala:81-145) and the
// Hinge / LeastSquares / Huber / AFT aggregators of the same shape.
//
// Why a layout of its own.  An aggregator add runs two sparse gemv
// (BinaryLogisticBlockAggregator.scala:97 and :130; ml/linalg/BLAS.scala:
// 764-805): margins gather one fp64 coefficient per nonzero, the gradient
// gathers one fp64 multiplier per nonzero.  At F = 1M with 64 random columns
// per row those gathers are L2 requests, and round 1 measured both passes
// bound by that request rate (~146 G gathers/s), not by HBM.  Here the shard
// is cut into row blocks of R = 2048 rows and column chunks of W <= 2048
// columns; a (row block, column chunk) segment stores its nonzeros in CSR
// order with the row inside the block and the column inside the chunk
// packed into 32 bits, so both gathers become LDS reads:
//   margin pass    one workgroup per 8 row blocks (16384 rows): their partial
//                  dots in LDS (128 KB), the coefficient chunks streamed
//                  through LDS (16 KB each; all workgroups sweep the same
//                  chunks: L2 hits); wave i walks segment (8 sb + i, c), ONE
//                  contiguous run;
//   gradient pass  one workgroup per 8 column chunks (16384 columns) and row
//                  range: their gradient sums in LDS (128 KB), the multiplier
//                  slices streamed through LDS (16 KB each); wave j walks
//                  segment (rb, 8 st + j), ONE contiguous run.
// Either pass reads 12 B per nonzero (value + packed ids) from HBM and
// stages one 16 KB slice (L2) per 8 segments: 7.6 B per nonzero at F = 1M,
// 64 nonzeros per row (the 8192 x 8192 tiles of round 2 staged 15.3 B per
// nonzero, and their waves walked 8 sub-segments each).  Each LDS sum
// has exactly one writer wave and its adds land in a fixed order: a row's
// dot in column order from 0.0 (the reference's CSR row loop, BLAS.scala:
// 777-789, bit for bit: chunks in order, CSR order inside a segment), a
// column's gradient sum in row order within a row range (the transposed
// loop :790-804).
//
// Built once per dataset (like InstanceBlock.blokifyWithMaxMemUsage +
// persist, ml/feature/Instance.scala:146-187, LogisticRegression.scala:
// 967-970) by appending CSR row blocks: per chunk a stable radix sort of the
// nonzeros by segment keeps each segment in CSR order.  The CSR input can be
// freed after the append, so the layout is the only copy of the shard in
// HBM (12 B per nonzero + 8 B per segment): a 200M x 1M, 64-per-row shard
// takes 154 GB.
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
  int F = 0, T = 1, Wt = 1;
  int64_t capRows = 0, capNnz = 0, n = 0, nnz = 0;
  bool sealed = false;    // ends with a partial row block: no further appends
  int64_t maxSeg = 0;     // nonzeros of the longest segment (picks the pass instances)
  std::mutex mu;
  cyc::DeviceBuffer segStart, idx, vals, maxDev;
};

namespace {

using cyc::kTileCols;
using cyc::kTileRows;
using cyc::kTileSuperCols;
using cyc::kTileSuperRows;
using cyc::kTileWaves;

constexpr int kTPB = 64 * kTileWaves;          // threads per workgroup (8 waves)
constexpr int kCPT = kTileCols / kTPB;         // staged coefficients per thread
constexpr int kMPT = kTileRows / kTPB;         // staged multipliers per thread
constexpr int kDPT = kTileSuperRows / kTPB;    // dots per thread (margin)
constexpr int kGPT = kTileSuperCols / kTPB;    // gradient sums per thread

// columns per chunk: an eighth of F (so a gradient workgroup's 8 waves all
// have a chunk when F is small), a multiple of 64, at most kTileCols
int chunk_cols(int F) {
  const int w = (int)std::min<int64_t>(kTileCols, ((int64_t)F + 8 * 64 - 1) / (8 * 64) * 64);
  return std::max(w, 64);
}

// ----------------------------------------------------------------- build

// Per nonzero of rows [0, rows) of a chunk: its segment key rb * T + c and
// its packed ids.  Wave per row.
__global__ void k_tile_keys(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
                            int64_t rows, int64_t q0, int T, int Wt,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ packed) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < rows; r += stride) {
    const int64_t rbl = r / kTileRows;
    const uint32_t rin = (uint32_t)(r % kTileRows);
    const int64_t p1 = rowptr[r + 1] - q0;
    for (int64_t p = rowptr[r] - q0 + lane; p < p1; p += 64) {
      const int c = colidx[p];
      const int t = c / Wt, cin = c - t * Wt;
      keys[p] = (uint32_t)(rbl * T + t);
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

// segStart[seg0 + key] = base + first sorted position with key' >= key,
// key in [0, nkeys)
__global__ void k_tile_starts(const uint32_t* __restrict__ keys, int64_t cnt, int64_t nkeys,
                              int64_t seg0, int64_t base, int64_t* __restrict__ segStart) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= cnt;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prev = q == 0 ? -1 : (int64_t)keys[q - 1];
    const int64_t cur = q == cnt ? nkeys : (int64_t)keys[q];
    for (int64_t k = prev + 1; k <= cur && k < nkeys; ++k) segStart[seg0 + k] = base + q;
  }
}

__global__ void k_set_i64(int64_t* p, int64_t v) { *p = v; }

// *mx = max(*mx, longest segment of [s0, s1)) -- a wave max, then one
// atomic per wave
__global__ void k_seg_max(const int64_t* __restrict__ segStart, int64_t s0, int64_t s1,
                          unsigned long long* __restrict__ mx) {
  unsigned long long m = 0;
  for (int64_t q = s0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < s1;
       q += (int64_t)gridDim.x * blockDim.x)
    m = max(m, (unsigned long long)(segStart[q + 1] - segStart[q]));
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}

// ----------------------------------------------------------------- passes

// tools/probe/tiles_mall_probe.py times library builds with parts of both
// passes removed (results then meaningless): bits 1 = plain LDS stores in
// place of the LDS atomic adds, 2 = no LDS gathers of coefficients /
// multipliers, 4 = no per-step barrier, 8 = no staging of the chunk / slice,
// 16 = no run loads (synthetic ids and values), 32 = no segment offset
// loads (every run 256 long).  0 in the library.
#ifndef CYC_TILES_PROBE
#define CYC_TILES_PROBE 0
#endif

__device__ __forceinline__ void lds_add(double* p, double x) {
  if constexpr ((CYC_TILES_PROBE & 1) != 0) *p = x;
  else __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// s_waitcnt immediate for "at most n vector memory operations outstanding"
// (gfx9 encoding: vmcnt in bits 3:0 and 15:14; expcnt and lgkmcnt left at
// their maxima, i.e. not waited for)
constexpr int vm_wait(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

__device__ __forceinline__ void step_barrier() {
  if constexpr ((CYC_TILES_PROBE & 4) == 0) __syncthreads();
}

// buffer resource over [p, p + bytes): lanes past the end read 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                           (int)std::min<int64_t>(bytes, 0x7fffffff), 0x00020000);
}

struct TileDims {
  int64_t n, nRB;
  int F, T, Wt;
};

// One wave's run: a segment's nonzeros [s0, s0 + len).  The segment offsets
// come through __restrict__ read-only pointers, so the compiler fetches
// them with scalar loads (lgkmcnt): reading them never waits on the runs in
// flight (vmcnt).
struct Run {
  int64_t s0, len;
};

__device__ __forceinline__ Run seg_run(const int64_t* __restrict__ segStart, int64_t seg,
                                       bool on) {
  if (!on) return Run{0, 0};
  if constexpr ((CYC_TILES_PROBE & 32) != 0) return Run{0, 256};   // the first 256 nonzeros
  const int64_t a = segStart[seg];
  return Run{a, segStart[seg + 1] - a};
}

// the first KC x 64 nonzeros of a run from `from` on, lane-strided; lanes
// past the end read 0 (buffer range check)
template <int KC>
__device__ __forceinline__ void load_run(const uint32_t* __restrict__ vidx,
                                         const double* __restrict__ vvals, const Run& r,
                                         int64_t from, int lane, uint32_t (&ix)[KC],
                                         double (&vx)[KC]) {
  const int64_t len = r.len - from;
  if constexpr ((CYC_TILES_PROBE & 16) != 0) {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      ix[j] = ((uint32_t)(lane * 31 + j * 7) & 2047) << 16 | ((uint32_t)(lane * 29 + j) & 1023);
      vx[j] = 1.0 + j;
    }
    return;
  }
  const auto ri = rsrc(vidx + r.s0 + from, len > 0 ? len * 4 : 0);
  const auto rv = rsrc(vvals + r.s0 + from, len > 0 ? len * 8 : 0);
  // lane part in the VGPR offset, batch part in the immediate offset
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    ix[j] = __builtin_amdgcn_raw_buffer_load_b32(ri, lane * 4, j * 256, 2);
    vx[j] = __builtin_bit_cast(double,
                               __builtin_amdgcn_raw_buffer_load_b64(rv, lane * 8, j * 512, 2));
  }
}

// run buffers of the margin pass (the runs of the next NB - 1 steps in
// flight) and coefficient chunks in registers (CS = 2: a chunk is loaded two
// steps before it is staged; NB a multiple of CS)
#ifndef CYC_TILES_MARGIN_NB
#define CYC_TILES_MARGIN_NB 3
#endif
#ifndef CYC_TILES_MARGIN_CS
#define CYC_TILES_MARGIN_CS 1
#endif
// 1: the margin pass's coefficient chunks staged by LDS DMA (an A/B switch)
#ifndef CYC_TILES_MARGIN_DMA
#define CYC_TILES_MARGIN_DMA 1
#endif

// Margin pass, persistent over (super row block sb, column chunk c) steps:
// this workgroup's super blocks sb = blockIdx.x + i * gridDim.x (8 row blocks
// each), each swept over the T chunks, as one flat sequence of steps g.  Per
// step: the coefficient chunk goes registers -> LDS (the next CS steps'
// chunks are loaded meanwhile, L2 hits), and wave i walks segment
// (8 sb + i, c); the runs of the next NB - 1 steps are in flight in
// registers, across super block boundaries too.
// DMA: the coefficient chunks go HBM/L2 -> LDS by buffer_load ... lds (two
// 1 KiB pieces per wave, issued one step ahead), no staging registers or
// ds_writes; else through registers, CS steps ahead.
template <int NB, int CS, int KC, bool LONG, bool DMA>
__global__ __launch_bounds__(kTPB) void k_tiles_margin(
    TileDims v, const int64_t* __restrict__ segStart, const uint32_t* __restrict__ vidx,
    const double* __restrict__ vvals, const double* __restrict__ labels,
    const double* __restrict__ weights, const double* __restrict__ coef, int fitIntercept,
    int kind, double offset, double lscale, double sigma, double eps, double* __restrict__ mult,
    double* __restrict__ slabS) {
  static_assert(NB % CS == 0, "the chunk sets rotate within the unroll");
  // 160 KiB: the super block's dots and two coefficient chunk buffers (the
  // chunk of step s in cf[s & 1]); the final reduction reuses cf
  __shared__ double lds[kTileSuperRows + 2 * kTileCols];
  double* const dots = lds;
  double* const cf = lds + kTileSuperRows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = v.T;
  const int64_t nSB = (v.nRB + kTileWaves - 1) / kTileWaves;
  // steps per super block padded to a multiple of NB (the unroll of the run
  // buffers; with CS = 2, NB and so Tp are even, and a step's chunk set is
  // fixed by its place in the unroll); the padding steps have empty runs and
  // fetch nothing
  const int Tp = (T + NB - 1) / NB * NB;
  const int64_t mySB = nSB > blockIdx.x ? (nSB - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};     // loss, weight, multiplierSum, sigmaGradSum
  double creg[DMA ? 1 : CS][kCPT];          // chunk of step g in creg[g % CS]
  uint32_t ib[NB][KC];
  double vb[NB][KC];
  Run rr[NB];

  // a step is (k, c): this workgroup's k-th super block, chunk c < Tp; the
  // positions a few steps ahead by compare-and-wrap (no divisions)
  auto ahead = [&](int64_t k, int c, int by, int64_t& k2, int& c2) {
    c2 = c + by;
    k2 = k;
    if (c2 >= Tp) c2 -= Tp, k2 += 1;
  };
  auto run_of = [&](int64_t k, int c) {
    const int64_t rb = ((int64_t)blockIdx.x + k * gridDim.x) * kTileWaves + wave;
    return seg_run(segStart, rb * T + c, k < mySB && c < T && rb < v.nRB);
  };
  auto load_coef = [&](int64_t k, int c, double (&cr)[kCPT]) {
    const bool on = k < mySB && c < T;
    const int64_t c0 = on ? (int64_t)c * v.Wt : 0;
    const int wl = on ? (int)std::min<int64_t>(v.Wt, v.F - c0) : 0;
    const auto rc = rsrc(coef + c0, (int64_t)wl * 8);
#pragma unroll
    for (int i = 0; i < kCPT; ++i)
      cr[i] = __builtin_bit_cast(
          double, __builtin_amdgcn_raw_buffer_load_b64(rc, tid * 8, i * kTPB * 8, 0));
  };
  double* myDots = dots + wave * kTileRows;
  // waits for the whole run first, on every path: its values are used only
  // under the lanes' `< len` branches, and a path that skips one left the
  // compiler's wait analysis treating the registers as still loading at the
  // loop head, where it then drained every prefetched run (vmcnt(0)).  The
  // runs of the other NB - 2 steps and the staging loads of the steps since
  // -- (NB - 2) (2 KC + 4) operations -- stay in flight.
  // the chunk of step (k, c) into b by DMA: wave w's pieces 2w, 2w + 1
  auto dma_coef = [&](int64_t k, int c, double* b) {
    const bool on = k < mySB && c < T;
    const int64_t c0 = on ? (int64_t)c * v.Wt : 0;
    const int wl = on ? (int)std::min<int64_t>(v.Wt, v.F - c0) : 0;
    const auto rc = rsrc(coef + c0, (int64_t)wl * 8);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rc, (__attribute__((address_space(3))) void*)(b + (wave * 2 + i) * 128), 16,
          (wave * 2 + i) * 1024 + lane * 16, 0, 0, 0);
  };
  static_assert(!DMA || kTileCols * 8 == kTileWaves * 2 * 1024, "two 1 KiB pieces per wave");
  auto consume = [&](int64_t len, const double* cfp, const uint32_t (&ix)[KC],
                     const double (&vx)[KC]) {
    __builtin_amdgcn_s_waitcnt(vm_wait((NB - 2) * (2 * KC + (DMA ? 2 : 4))));
    double c[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j)   // lanes past the end read [0]
      c[j] = (CYC_TILES_PROBE & 2) ? vx[j] : cfp[ix[j] & 0xffff];
#pragma unroll
    for (int j = 0; j < KC; ++j)
      if (j * 64 + lane < len) lds_add(&myDots[ix[j] >> 16], vx[j] * c[j]);
  };
  // One step (k, c), ONE barrier: the current run into the row sums with
  // chunk s in cf[s & 1], the next chunk (in registers since CS steps ago)
  // into the other buffer -- every wave left it behind the last barrier --,
  // then the loads of the chunk CS + 1 steps and of the run NB - 1 steps
  // ahead issued (unconditionally: past the end they fetch nothing, so the
  // waits for the current run stay counted).  The run buffers and chunk sets
  // rotate by unrolling (never by copying a register that a load is still
  // filling).
  auto step = [&](int64_t k, int c, const Run& rc, uint32_t (&ic)[KC], double (&vc)[KC],
                  Run& rn, uint32_t (&in)[KC], double (&vn)[KC], double (&cs)[kCPT]) {
    const int par = (int)((k * Tp + c) & 1);
    const double* cur = cf + par * kTileCols;
    consume(rc.len, cur, ic, vc);
    // a run longer than KC x 64: only in the LONG instance (a layout with
    // such segments), in registers of its own -- any load in this loop's
    // body makes the compiler's wait analysis drain every prefetched run
    // at the loop head
    if constexpr (LONG) {
      for (int64_t b = KC * 64; b < rc.len; b += KC * 64) {
        uint32_t it[KC];
        double vt[KC];
        load_run(vidx, vvals, rc, b, lane, it, vt);
        consume(rc.len - b, cur, it, vt);
      }
    }
    double* nxt = cf + (par ^ 1) * kTileCols;
    int64_t k2;
    int c2;
    if constexpr (DMA) {
      // chunk of the next step into the buffer every wave left behind the
      // last barrier; landed (this wave's pieces) before the next barrier:
      // only this step's run loads are issued after it
      ahead(k, c, 1, k2, c2);
      dma_coef(k2, c2, nxt);
    } else if constexpr ((CYC_TILES_PROBE & 8) == 0) {
#pragma unroll
      for (int i = 0; i < kCPT; ++i) nxt[tid + kTPB * i] = cs[i];
      ahead(k, c, CS + 1, k2, c2);
      load_coef(k2, c2, cs);
    }
    ahead(k, c, NB - 1, k2, c2);
    rn = run_of(k2, c2);
    load_run(vidx, vvals, rn, 0, lane, in, vn);
    if constexpr (DMA) __builtin_amdgcn_s_waitcnt(vm_wait(2 * KC));
    step_barrier();
  };

  // prologue: chunk 0 into cf[0], chunks 1 .. CS in registers (DMA: chunk
  // 0 only, landed before the first barrier), runs of steps 0 .. NB - 2 in
  // flight
  if constexpr (DMA) {
    dma_coef(0, 0, cf);
    __builtin_amdgcn_s_waitcnt(vm_wait(0));
  } else {
    load_coef(0, 0, creg[0]);
#pragma unroll
    for (int i = 0; i < kCPT; ++i) cf[tid + kTPB * i] = creg[0][i];
#pragma unroll
    for (int s1 = 1; s1 <= CS; ++s1) {
      int64_t k1;
      int c1;
      ahead(0, 0, s1, k1, c1);
      load_coef(k1, c1, creg[s1 % CS]);
    }
  }
#pragma unroll
  for (int u = 0; u < NB - 1; ++u) {
    int64_t k1;
    int c1;
    ahead(0, 0, u, k1, c1);
    rr[u] = run_of(k1, c1);
    load_run(vidx, vvals, rr[u], 0, lane, ib[u], vb[u]);
  }
  // The binary logistic epilogue (kind 0: BinaryLogisticBlockAggregator.
  // scala:104-122) without branches, EB rows at a time with the next EB
  // rows' labels and weights loaded before this batch's multiplier stores
  // (vmcnt waits are in issue order: a load issued after a store waits for
  // it too).  log1pExp(x) (ml/impl/Utils.scala:91-97) as max(x, 0) +
  // log1p(exp(-|x|)): the same two branches, the same bits (0 + y == y for
  // the x <= 0 one).  Rows are visited in the plain loop's order, so the
  // sums are the same bits as well.
  auto logistic_epilogue = [&](int64_t r0) {
    constexpr int EB = 4;
    double lab[2][EB], wt[2][EB];
    auto ld = [&](int i0, double (&l)[EB], double (&w)[EB]) {
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int64_t rr = min<int64_t>(r0 + tid + (int64_t)kTPB * (i0 + u), v.n - 1);
        l[u] = __builtin_nontemporal_load(&labels[rr]);   // streamed once
        w[u] = weights ? __builtin_nontemporal_load(&weights[rr]) : 1.0;
      }
    };
    ld(0, lab[0], wt[0]);
#pragma unroll
    for (int i0 = 0; i0 < kDPT; i0 += EB) {
      const int cb = (i0 / EB) & 1;
      if (i0 + EB < kDPT) ld(i0 + EB, lab[cb ^ 1], wt[cb ^ 1]);
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int rl = tid + kTPB * (i0 + u);
        const int64_t r = r0 + rl;
        const double label = lab[cb][u], w = wt[cb][u];
        const double margin = fitIntercept ? offset + dots[rl] : dots[rl];
        const double x = -margin;
        const double lp = __builtin_fmax(x, 0.0) + log1p(exp(-__builtin_fabs(x)));
        const double term = label > 0 ? lp : lp + margin;
        const double mm = w * (1.0 / (1.0 + exp(-margin)) - label);
        if (r < v.n) {
          acc[1] += w;
          double m = 0.0;
          if (w > 0) {
            acc[0] += w * term;
            m = mm;
          }
          acc[2] += m;
          __builtin_nontemporal_store(m, &mult[r]);
        }
      }
    }
  };
  for (int64_t k = 0; k < mySB; ++k) {          // one super block per pass
#pragma unroll
    for (int i = 0; i < kDPT; ++i) dots[tid + kTPB * i] = 0.0;
    __syncthreads();                            // zeroed dots, chunk 0 in cf[0]
    for (int c = 0; c < Tp; c += NB) {
#pragma unroll
      for (int u = 0; u < NB; ++u)
        step(k, c + u, rr[u], ib[u], vb[u], rr[(u + NB - 1) % NB], ib[(u + NB - 1) % NB],
             vb[(u + NB - 1) % NB], creg[DMA ? 0 : (u + 1) % CS]);
    }
    // epilogue (BinaryLogisticBlockAggregator.scala:104-122 and siblings)
    const int64_t r0 = ((int64_t)blockIdx.x + k * gridDim.x) * kTileSuperRows;
    if (kind == 0) {
      logistic_epilogue(r0);
      __syncthreads();                          // dots read before the next zeroing
      continue;
    }
    for (int i = 0; i < kDPT; ++i) {
      const int rl = tid + kTPB * i;
      const int64_t r = r0 + rl;
      if (r < v.n) {
        const double label = labels[r];
        const double margin = cyc::row_margin(kind, fitIntercept, offset, lscale, label, dots[rl]);
        const double w = weights ? weights[r] : 1.0;
        const double m = cyc::bin_row(kind, margin, w, label, acc[0], acc[1], acc[3], sigma, eps);
        acc[2] += m;
        mult[r] = m;
      }
    }
    __syncthreads();                            // dots read before the next zeroing
  }
  // workgroup partials: fixed shuffle tree per wave, then waves in order
  double (*red)[4] = reinterpret_cast<double (*)[4]>(cf);
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

// run buffers of the gradient pass: the runs of the next NB - 1 row blocks
// are in flight while one is consumed; MS multiplier slices in registers
// (MS = 2: a slice is loaded two row blocks before it is staged; NB even)
#ifndef CYC_TILES_GRAD_NB
#define CYC_TILES_GRAD_NB 3
#endif
#ifndef CYC_TILES_GRAD_MS
#define CYC_TILES_GRAD_MS 1
#endif
// 1: the gradient pass's multiplier slices staged by LDS DMA (an A/B switch)
#ifndef CYC_TILES_GRAD_DMA
#define CYC_TILES_GRAD_DMA 1
#endif

// Gradient pass: workgroup (super chunk st = 8 column chunks, row range)
// over its row blocks.  Per row block: the multiplier slice goes registers
// -> LDS (the next ones loaded while this one is used); wave j walks segment
// (rb, 8 st + j) into its chunk's column sums, with the runs of the next
// NB - 1 row blocks in flight.
// DMA: the multiplier slices go to LDS by buffer_load ... lds, one row
// block ahead (as the margin pass's coefficient chunks).
template <int NB, int MS, int KC, bool LONG, bool DMA>
__global__ __launch_bounds__(kTPB) void k_tiles_grad(
    TileDims v, const int64_t* __restrict__ segStart, const uint32_t* __restrict__ vidx,
    const double* __restrict__ vvals, const double* __restrict__ mult, int ranges,
    double* __restrict__ slabG) {
  static_assert(MS == 1 || (MS == 2 && NB % 2 == 0), "two slice sets need an even unroll");
  // 160 KiB: the 8 chunks' column sums and two multiplier slice buffers
  // (row block rb's slice in mv[(rb - rbA) & 1])
  __shared__ double lds[kTileSuperCols + 2 * kTileRows];
  double* const gt = lds;
  double* const mv = lds + kTileSuperCols;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int range = blockIdx.x % ranges, st = blockIdx.x / ranges;
  const int64_t rbA = v.nRB * range / ranges, rbB = v.nRB * (range + 1) / ranges;
  const int c = st * kTileWaves + wave;                 // this wave's column chunk
  double mreg[DMA ? 1 : MS][kMPT];                      // slice r in mreg[(r - rbA) % MS]
  uint32_t ib[NB][KC];
  double vb[NB][KC];
  Run rr[NB];

  auto run_of = [&](int64_t rb) { return seg_run(segStart, rb * v.T + c, rb < rbB && c < v.T); };
  auto load_mult = [&](int64_t rb, double (&m)[kMPT]) {
    const int64_t r0 = rb * kTileRows;
    const auto rm = rsrc(mult + (rb < rbB ? r0 : 0),
                         rb < rbB ? std::min<int64_t>(kTileRows, v.n - r0) * 8 : 0);
#pragma unroll
    for (int i = 0; i < kMPT; ++i)
      m[i] = __builtin_bit_cast(
          double, __builtin_amdgcn_raw_buffer_load_b64(rm, tid * 8, i * kTPB * 8, 0));
  };
  // row block rb's slice into b by DMA: wave w's pieces 2w, 2w + 1
  auto dma_mult = [&](int64_t rb, double* b) {
    const int64_t r0 = rb * kTileRows;
    const auto rm = rsrc(mult + (rb < rbB ? r0 : 0),
                         rb < rbB ? std::min<int64_t>(kTileRows, v.n - r0) * 8 : 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rm, (__attribute__((address_space(3))) void*)(b + (wave * 2 + i) * 128), 16,
          (wave * 2 + i) * 1024 + lane * 16, 0, 0, 0);
  };
  static_assert(!DMA || kTileRows * 8 == kTileWaves * 2 * 1024, "two 1 KiB pieces per wave");
  double* myG = gt + wave * v.Wt;
  // waits for the whole run first, on every path (the margin pass's
  // consume says why)
  auto consume = [&](int64_t len, const double* mvp, const uint32_t (&ix)[KC],
                     const double (&vx)[KC]) {
    __builtin_amdgcn_s_waitcnt(vm_wait((NB - 2) * (2 * KC + (DMA ? 2 : 4 * MS))));
    double m[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j)   // lanes past the end read [0]
      m[j] = (CYC_TILES_PROBE & 2) ? vx[j] : mvp[ix[j] >> 16];
#pragma unroll
    for (int j = 0; j < KC; ++j)
      if (j * 64 + lane < len) lds_add(&myG[ix[j] & 0xffff], vx[j] * m[j]);
  };

#pragma unroll
  for (int i = 0; i < kGPT; ++i) gt[tid + kTPB * i] = 0.0;
  // one row block (the u-th of an unrolled group), ONE barrier: the current
  // run into the column sums with the slice in mv[par], the next slice (in
  // registers since MS steps ago) into the other buffer -- every wave left
  // it behind the last barrier --, then the slice MS + 1 row blocks ahead
  // and the run NB - 1 row blocks ahead issued (unconditionally, into the
  // registers just freed); run buffers and slice sets rotate by unrolling
  auto step = [&](int64_t rb, const Run& rc, uint32_t (&ic)[KC], double (&vc)[KC],
                  Run& rn, uint32_t (&in)[KC], double (&vn)[KC], double (&ms)[kMPT]) {
    const int par = (int)((rb - rbA) & 1);
    const double* cur = mv + par * kTileRows;
    consume(rc.len, cur, ic, vc);
    // a run longer than KC x 64: only in the LONG instance (a layout with
    // such segments), in registers of its own -- any load in this loop's
    // body makes the compiler's wait analysis drain every prefetched run
    // at the loop head
    if constexpr (LONG) {
      for (int64_t b = KC * 64; b < rc.len; b += KC * 64) {
        uint32_t it[KC];
        double vt[KC];
        load_run(vidx, vvals, rc, b, lane, it, vt);
        consume(rc.len - b, cur, it, vt);
      }
    }
    double* nxt = mv + (par ^ 1) * kTileRows;
    if constexpr (DMA) {
      dma_mult(rb + 1, nxt);   // landed before the barrier: only the run loads follow it
    } else if constexpr ((CYC_TILES_PROBE & 8) == 0) {
#pragma unroll
      for (int i = 0; i < kMPT; ++i) nxt[tid + kTPB * i] = ms[i];
      load_mult(rb + 1 + MS, ms);
    }
    rn = run_of(rb + NB - 1);
    load_run(vidx, vvals, rn, 0, lane, in, vn);
    if constexpr (DMA) __builtin_amdgcn_s_waitcnt(vm_wait(2 * KC));
    step_barrier();
  };

  // prologue: slice rbA into mv[0], slices rbA + 1 .. rbA + MS in
  // registers, runs rbA .. rbA + NB - 2 in flight
  if constexpr (DMA) {
    dma_mult(rbA, mv);
    __builtin_amdgcn_s_waitcnt(vm_wait(0));
  } else {
    load_mult(rbA, mreg[0]);
#pragma unroll
    for (int i = 0; i < kMPT; ++i) mv[tid + kTPB * i] = mreg[0][i];
#pragma unroll
    for (int s = 1; s <= MS; ++s) load_mult(rbA + s, mreg[s % MS]);
  }
#pragma unroll
  for (int u = 0; u < NB - 1; ++u) {
    rr[u] = run_of(rbA + u);
    load_run(vidx, vvals, rr[u], 0, lane, ib[u], vb[u]);
  }
  __syncthreads();                              // zeroed sums, slice rbA in mv[0]
  // whole groups of NB steps: the last group's steps past rbB have empty
  // runs and slices (no guard inside the unroll: a skipped step left the
  // compiler's wait analysis draining every prefetched run at the loop head)
  for (int64_t rb = rbA; rb < rbB; rb += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u)
      step(rb + u, rr[u], ib[u], vb[u], rr[(u + NB - 1) % NB], ib[(u + NB - 1) % NB],
           vb[(u + NB - 1) % NB], mreg[DMA ? 0 : (u + 1) % MS]);
  }
  __syncthreads();
  const int64_t col0 = (int64_t)st * kTileWaves * v.Wt;
  double* out = slabG + (int64_t)range * v.F + col0;
  const int64_t wl = std::min<int64_t>((int64_t)kTileWaves * v.Wt, v.F - col0);
#pragma unroll
  for (int i = 0; i < kGPT; ++i) {
    const int e = tid + kTPB * i;
    if (e < wl) out[e] = gt[e];
  }
}

// Five nonzeros per lane per run buffer: a layout whose longest segment has
// at most 320 takes the instance without the reload loop, any other the
// LONG one (config 5's 47.7M segments average 268, the longest ~360: LONG,
// whose common path waits the same; six per lane without the loop costs
// more load and LDS instructions per step for mostly idle lanes).
bool long_runs(int64_t maxSeg) { return maxSeg > 5 * 64; }

}  // namespace

namespace cyc {

int tiles_view(cyc_tiles t, TilesView* v) {
  CYC_REQUIRE(t != nullptr && v != nullptr, "tiles must not be null");
  v->n = t->n;
  v->F = t->F;
  v->T = t->T;
  v->Wt = t->Wt;
  v->nRB = (t->n + kTileRows - 1) / kTileRows;
  v->segStart = (const int64_t*)t->segStart.ptr;
  v->idx = (const uint32_t*)t->idx.ptr;
  v->vals = (const double*)t->vals.ptr;
  v->maxSeg = t->maxSeg;
  return CYC_OK;
}

int tiles_margin(const TilesView& v, const double* labels, const double* weights,
                 const double* coef, int fitIntercept, int kind, double offset, double lscale,
                 double sigma, double eps, double* mult, double* slabS, int64_t* wgs,
                 hipStream_t st) {
  const int64_t nSB = (v.nRB + kTileWaves - 1) / kTileWaves;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(nSB, device_cus()));
  *wgs = grid;
  const TileDims d{v.n, v.nRB, v.F, v.T, v.Wt};
#define CYC_TILES_MARGIN(KC, LONG, DMA)                                                         \
  hipLaunchKernelGGL(                                                                           \
      HIP_KERNEL_NAME(k_tiles_margin<CYC_TILES_MARGIN_NB, CYC_TILES_MARGIN_CS, KC, LONG, DMA>),  \
      dim3((unsigned)grid), dim3(kTPB), 0, st, d, v.segStart, v.idx, v.vals, labels, weights,   \
      coef, fitIntercept, kind, offset, lscale, sigma, eps, mult, slabS)
  // the DMA pieces are 16-byte loads: a coefficient vector that is not
  // 16-byte aligned takes the register-staged instance
  const bool dma = CYC_TILES_MARGIN_DMA && (reinterpret_cast<uintptr_t>(coef) & 15) == 0;
  if (long_runs(v.maxSeg)) {
    if (dma) CYC_TILES_MARGIN(5, true, true);
    else CYC_TILES_MARGIN(5, true, false);
  } else {
    if (dma) CYC_TILES_MARGIN(5, false, true);
    else CYC_TILES_MARGIN(5, false, false);
  }
#undef CYC_TILES_MARGIN
  CYC_LAUNCH_CHECK("k_tiles_margin");
  return CYC_OK;
}

int tiles_ranges(const TilesView& v) {
  const int64_t cus = device_cus();
  const int64_t sts = (v.T + kTileWaves - 1) / kTileWaves;
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(v.nRB, 1), cus / sts));
}

int tiles_grad(const TilesView& v, const double* mult, double* slabG, int* ranges,
               hipStream_t st) {
  const int R = tiles_ranges(v);
  *ranges = R;
  const int64_t sts = (v.T + kTileWaves - 1) / kTileWaves;
  const TileDims d{v.n, v.nRB, v.F, v.T, v.Wt};
#define CYC_TILES_GRAD(KC, LONG, DMA)                                                           \
  hipLaunchKernelGGL(                                                                           \
      HIP_KERNEL_NAME(k_tiles_grad<CYC_TILES_GRAD_NB, CYC_TILES_GRAD_MS, KC, LONG, DMA>),        \
      dim3((unsigned)(sts * R)), dim3(kTPB), 0, st, d, v.segStart, v.idx, v.vals, mult, R, slabG)
  const bool dma = CYC_TILES_GRAD_DMA && (reinterpret_cast<uintptr_t>(mult) & 15) == 0;
  if (long_runs(v.maxSeg)) {
    if (dma) CYC_TILES_GRAD(5, true, true);
    else CYC_TILES_GRAD(5, true, false);
  } else {
    if (dma) CYC_TILES_GRAD(5, false, true);
    else CYC_TILES_GRAD(5, false, false);
  }
#undef CYC_TILES_GRAD
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
  t->Wt = chunk_cols(numFeatures);
  t->T = (int)(((int64_t)numFeatures + t->Wt - 1) / t->Wt);
  t->capRows = capacity_rows;
  t->capNnz = capacity_nnz;
  const int64_t segs = (capacity_rows + kTileRows - 1) / kTileRows * t->T;
  int rc;
  if ((rc = t->segStart.reserve(sizeof(int64_t) * (size_t)(segs + 1))) ||
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
  return t ? (int64_t)(t->segStart.bytes + t->idx.bytes + t->vals.bytes) : 0;
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
  // sub-chunks of whole row blocks, at most 2^24 segment keys (bounded
  // scratch, 32-bit sort keys)
  const int64_t nrbSub = std::max<int64_t>(1, std::min<int64_t>(512, ((int64_t)1 << 24) / T));
  const int64_t chRows = nrbSub * kTileRows;
  const int64_t rb0 = t->n / kTileRows;
  cyc::DeviceBuffer keys, packed, keysOut, perm, tmp;
  for (int64_t a = 0; a < rows; a += chRows) {
    const int64_t b = std::min(rows, a + chRows);
    int64_t qa = 0, qb = 0;
    CYC_HIP(hipMemcpyAsync(&qa, rowptr + a, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipMemcpyAsync(&qb, rowptr + b, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CYC_HIP(hipStreamSynchronize(st));
    const int64_t cnt = qb - qa;
    const int64_t nrb = (b - a + kTileRows - 1) / kTileRows;
    const int64_t nkeys = nrb * T;
    const int64_t seg0 = (rb0 + a / kTileRows) * T;
    CYC_REQUIRE(cnt < ((int64_t)1 << 32), "a chunk of " + std::to_string(nrbSub) +
                                              " row blocks holds 2^32 nonzeros or more");
    int rc;
    if (cnt > 0) {
      if ((rc = keys.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
          (rc = packed.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
          (rc = keysOut.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
          (rc = perm.reserve(sizeof(uint32_t) * (size_t)cnt)))
        return rc;
      hipLaunchKernelGGL(k_tile_keys, dim3(8192), dim3(256), 0, st, rowptr + a, colidx + (qa - q0),
                         b - a, qa, T, t->Wt, (uint32_t*)keys.ptr, (uint32_t*)packed.ptr);
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
                       dim3(256), 0, st, (const uint32_t*)keysOut.ptr, cnt, nkeys, seg0, t->nnz,
                       (int64_t*)t->segStart.ptr);
    CYC_LAUNCH_CHECK("k_tile_starts");
    t->nnz += cnt;
    // scratch is reused by the next sub-chunk on this stream; freed on return
  }
  t->n += rows;
  if (t->n % kTileRows != 0) t->sealed = true;
  const int64_t segs = (t->n + kTileRows - 1) / kTileRows * T;
  hipLaunchKernelGGL(k_set_i64, dim3(1), dim3(1), 0, st, (int64_t*)t->segStart.ptr + segs, t->nnz);
  CYC_LAUNCH_CHECK("k_set_i64");
  if (int rc = t->maxDev.reserve(sizeof(unsigned long long))) return rc;
  CYC_HIP(hipMemsetAsync(t->maxDev.ptr, 0, sizeof(unsigned long long), st));
  const int64_t s0 = rb0 * T;
  hipLaunchKernelGGL(k_seg_max, dim3((unsigned)std::min<int64_t>((segs - s0 + 255) / 256, 4096)),
                     dim3(256), 0, st, (const int64_t*)t->segStart.ptr, s0, segs,
                     (unsigned long long*)t->maxDev.ptr);
  CYC_LAUNCH_CHECK("k_seg_max");
  unsigned long long mx = 0;
  CYC_HIP(hipMemcpyAsync(&mx, t->maxDev.ptr, sizeof(mx), hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  t->maxSeg = std::max<int64_t>(t->maxSeg, (int64_t)mx);
  return CYC_OK;
}

}  // extern "C"
