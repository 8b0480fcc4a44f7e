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
#include <cstdlib>
#include <mutex>
#include <string>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "binary_rows.hpp"
#include "common.hpp"
#include "tiles.hpp"

struct cyc_tiles_s {
  int F = 0, T = 1, Wt = 1;
  int64_t capRows = 0, capNnz = 0, n = 0, nnz = 0;
  // entry format: CYC_TILES_AUTO until the first append decides,
  // CYC_TILES_WIDE (32-bit packed ids) or CYC_TILES_COMPACT (16-bit ids:
  // column + row delta, with filler entries); entries = positions used
  int fmt = CYC_TILES_AUTO;
  bool autoFmt = false;   // fmt chosen by AUTO (compact may still go wide: demote_to_wide)
  int64_t capEntries = 0, entries = 0;
  bool sealed = false;    // ends with a partial row block: no further appends
  int64_t maxSeg = 0;     // entries of the longest segment (picks the pass instances)
  std::mutex mu;
  cyc::DeviceBuffer segStart, idx, vals, maxDev, scal;
};

namespace {

using cyc::kTileCols;
using cyc::kTileRows;
using cyc::kTileSuperCols;
using cyc::kTileSuperRows;
using cyc::kTileWaves;

constexpr int kTPB = 64 * kTileWaves;          // threads of the compute waves (8 waves)
constexpr int kGPT = kTileSuperCols / kTPB;    // gradient sums per thread

// columns per chunk: an eighth of F (so a gradient workgroup's 8 waves all
// have a chunk when F is small), a multiple of 64, at most kTileCols
// ... and at most kTileCols - 2 = 2046: column 2047 is the compact format's
// filler code, and 2046 keeps a chunk's coefficients 16-byte aligned
// (2046 x 8 = 16 x 1023) for the loader's DMA.
int chunk_cols(int F) {
  const int w = (int)std::min<int64_t>(kTileCols - 2, ((int64_t)F + 8 * 64 - 1) / (8 * 64) * 64);
  return std::max(w, 64);
}

// ----------------------------------------------------------------- build

// Fix the entry format and reserve the entry arrays: the wide format
// capNnz entries of 4 + 8 bytes; the compact one capNnz + capNnz / 16 +
// 65536 entries of 2 + 8 bytes (a 6.25 % allowance for filler entries; an
// append that would need more fails with a message naming the wide format).
int set_storage(cyc_tiles t, int fmt) {
  t->fmt = fmt;
  const int64_t cap = std::max<int64_t>(t->capNnz, 1);
  t->capEntries = fmt == CYC_TILES_COMPACT ? cap + cap / 16 + 65536 : cap;
  int rc;
  if ((rc = t->idx.reserve((fmt == CYC_TILES_COMPACT ? 2 : 4) * (size_t)t->capEntries)) ||
      (rc = t->vals.reserve(sizeof(double) * (size_t)t->capEntries)))
    return rc;
  return CYC_OK;
}

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

// The compact entry (CYC_TILES_COMPACT): 16 bits -- the row's low 5 bits
// (row in block mod 32) and the column in the chunk (11 bits; column 2047,
// never a chunk's since chunks hold at most 2046, marks a filler entry: no
// nonzero, value 0.0).  Entries of a segment are in CSR order, so rows never
// decrease; a row that is 32 or more past the previous entry's (row 0 for
// the first) gets fillers at every 31 rows in front of it, so each step is
// below 32 and a row's high part is the number of times the low part went
// down so far -- a ballot + mbcnt per wave instruction in the passes, no
// prefix sum.  10 bytes per entry instead of 12; at config 5's density
// (268 nonzeros per segment, rows ~7.6 apart) ~1 % of the entries are
// fillers.
constexpr uint32_t kStep = 31;          // filler spacing (largest step without one)
constexpr int kColBits = 11;
constexpr uint32_t kFillCol = (1u << kColBits) - 1;

// fillers in front of an entry whose row is d past the previous one
__device__ __forceinline__ uint32_t fillers(uint32_t d) { return d == 0 ? 0 : (d - 1) / kStep; }

__device__ __forceinline__ uint32_t prev_row(const uint32_t* __restrict__ keysOut,
                                             const uint32_t* __restrict__ perm,
                                             const uint32_t* __restrict__ packed, int64_t q) {
  return (q > 0 && keysOut[q - 1] == keysOut[q]) ? packed[perm[q - 1]] >> 16 : 0u;
}

// entries per sorted position q: the fillers its row step needs + itself
__global__ void k_tile_fill_counts(const uint32_t* __restrict__ keysOut,
                                   const uint32_t* __restrict__ perm,
                                   const uint32_t* __restrict__ packed, int64_t cnt,
                                   uint32_t* __restrict__ counts) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < cnt;
       q += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t row = packed[perm[q]] >> 16;
    counts[q] = 1 + fillers(row - prev_row(keysOut, perm, packed, q));
  }
}

__global__ void k_tile_total(const uint32_t* __restrict__ counts,
                             const unsigned long long* __restrict__ pos, int64_t cnt,
                             int64_t* __restrict__ out) {
  out[0] = cnt > 0 ? (int64_t)(pos[cnt - 1] + counts[cnt - 1]) : 0;
}

// position q's fillers and entry at pos[q] (sub-chunk relative)
__global__ void k_tile_compact(const uint32_t* __restrict__ keysOut,
                               const uint32_t* __restrict__ perm,
                               const uint32_t* __restrict__ packed,
                               const double* __restrict__ vals, int64_t cnt,
                               const unsigned long long* __restrict__ pos,
                               uint16_t* __restrict__ outIdx, double* __restrict__ outVals) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < cnt;
       q += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t p = perm[q], pk = packed[p];
    const uint32_t row = pk >> 16, prev = prev_row(keysOut, perm, packed, q);
    const uint32_t f = fillers(row - prev);
    const int64_t o = (int64_t)pos[q];
    for (uint32_t i = 0; i < f; ++i) {
      outIdx[o + i] = (uint16_t)((((prev + kStep * (i + 1)) & 31u) << kColBits) | kFillCol);
      outVals[o + i] = 0.0;
    }
    outIdx[o + f] = (uint16_t)(((row & 31u) << kColBits) | (pk & 0xffff));
    outVals[o + f] = vals[p];
  }
}

// segStart[seg0 + key] = base + the entry position of the first sorted
// position q with key' >= key (q itself for the wide format, pos[q] for the
// compact one, total past the end), key in [0, nkeys)
__global__ void k_tile_starts(const uint32_t* __restrict__ keys, int64_t cnt, int64_t nkeys,
                              int64_t seg0, int64_t base,
                              const unsigned long long* __restrict__ pos, int64_t total,
                              int64_t* __restrict__ segStart) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= cnt;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prev = q == 0 ? -1 : (int64_t)keys[q - 1];
    const int64_t cur = q == cnt ? nkeys : (int64_t)keys[q];
    const int64_t at = pos == nullptr ? q : (q == cnt ? total : (int64_t)pos[q]);
    for (int64_t k = prev + 1; k <= cur && k < nkeys; ++k) segStart[seg0 + k] = base + at;
  }
}

__global__ void k_set_i64(int64_t* p, int64_t v) { *p = v; }

// AUTO layouts demoted to WIDE (demote_to_wide): a thread per segment walks
// its compact entries in order.  Pass 1 counts the fillers; pass 2 writes
// the nonzeros as wide entries at segStart[s] - fillers before s, the row
// rebuilt from the low bits (its high part = the times the low part went
// down so far, k_tile_compact).
__global__ void k_seg_fillers(const int64_t* __restrict__ segStart, const uint16_t* __restrict__ idx,
                              int64_t segs, int64_t* __restrict__ fill) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < segs;
       s += (int64_t)gridDim.x * blockDim.x) {
    int64_t f = 0;
    for (int64_t q = segStart[s]; q < segStart[s + 1]; ++q) f += (idx[q] & kFillCol) == kFillCol;
    fill[s] = f;
  }
}

__global__ void k_seg_widen(const int64_t* __restrict__ segStart, const uint16_t* __restrict__ idx,
                            const double* __restrict__ vals, int64_t segs,
                            const int64_t* __restrict__ fillBefore, uint32_t* __restrict__ outIdx,
                            double* __restrict__ outVals) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < segs;
       s += (int64_t)gridDim.x * blockDim.x) {
    int64_t o = segStart[s] - fillBefore[s];
    uint32_t hi = 0, lowPrev = 0;
    for (int64_t q = segStart[s]; q < segStart[s + 1]; ++q) {
      const uint32_t e = idx[q], low = e >> kColBits, col = e & kFillCol;
      if (low < lowPrev) hi += 32;
      lowPrev = low;
      if (col == kFillCol) continue;
      outIdx[o] = ((hi + low) << 16) | col;
      outVals[o] = vals[q];
      ++o;
    }
  }
}

__global__ void k_seg_shift(int64_t* __restrict__ segStart, const int64_t* __restrict__ fillBefore,
                            int64_t segs) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= segs;
       s += (int64_t)gridDim.x * blockDim.x)
    segStart[s] -= fillBefore[s];
}

// An AUTO layout took COMPACT at its first append (dense enough rows) and an
// append now meets rows too sparse for the filler allowance: rewrite the
// first `segs` segments (everything committed) as WIDE entries in fresh
// arrays, then free the compact ones.  Needs both layouts' memory at once;
// on failure the layout is left as it was (still COMPACT).
int demote_to_wide(cyc_tiles t, int64_t segs, hipStream_t st) {
  cyc::DeviceBuffer fill, pre, tmp, idxW, valsW;
  int rc;
  const int64_t cap = std::max<int64_t>(t->capNnz, 1);
  if ((rc = fill.reserve(sizeof(int64_t) * (size_t)(segs + 1))) ||
      (rc = pre.reserve(sizeof(int64_t) * (size_t)(segs + 1))) ||
      (rc = idxW.reserve(sizeof(uint32_t) * (size_t)cap)) ||
      (rc = valsW.reserve(sizeof(double) * (size_t)cap)))
    return rc;
  CYC_HIP(hipMemsetAsync((int64_t*)fill.ptr + segs, 0, sizeof(int64_t), st));
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((segs + 255) / 256, 65536));
  hipLaunchKernelGGL(k_seg_fillers, dim3(grid), dim3(256), 0, st, (const int64_t*)t->segStart.ptr,
                     (const uint16_t*)t->idx.ptr, segs, (int64_t*)fill.ptr);
  CYC_LAUNCH_CHECK("k_seg_fillers");
  size_t bytes = 0;
  CYC_HIP(rocprim::exclusive_scan(nullptr, bytes, (const int64_t*)fill.ptr, (int64_t*)pre.ptr,
                                  (int64_t)0, (size_t)(segs + 1), rocprim::plus<int64_t>(), st));
  if ((rc = tmp.reserve(std::max<size_t>(bytes, 1)))) return rc;
  CYC_HIP(rocprim::exclusive_scan(tmp.ptr, bytes, (const int64_t*)fill.ptr, (int64_t*)pre.ptr,
                                  (int64_t)0, (size_t)(segs + 1), rocprim::plus<int64_t>(), st));
  hipLaunchKernelGGL(k_seg_widen, dim3(grid), dim3(256), 0, st, (const int64_t*)t->segStart.ptr,
                     (const uint16_t*)t->idx.ptr, (const double*)t->vals.ptr, segs,
                     (const int64_t*)pre.ptr, (uint32_t*)idxW.ptr, (double*)valsW.ptr);
  CYC_LAUNCH_CHECK("k_seg_widen");
  hipLaunchKernelGGL(k_seg_shift, dim3(grid), dim3(256), 0, st, (int64_t*)t->segStart.ptr,
                     (const int64_t*)pre.ptr, segs);
  CYC_LAUNCH_CHECK("k_seg_shift");
  int64_t fillers = 0;
  CYC_HIP(hipMemcpyAsync(&fillers, (const int64_t*)pre.ptr + segs, sizeof(int64_t),
                         hipMemcpyDeviceToHost, st));
  CYC_HIP(hipStreamSynchronize(st));
  std::swap(t->idx.ptr, idxW.ptr);
  std::swap(t->idx.bytes, idxW.bytes);
  std::swap(t->idx.device, idxW.device);
  std::swap(t->vals.ptr, valsW.ptr);
  std::swap(t->vals.bytes, valsW.bytes);
  std::swap(t->vals.device, valsW.device);
  t->fmt = CYC_TILES_WIDE;
  t->capEntries = cap;
  t->entries -= fillers;   // the old arrays are freed with idxW / valsW
  return CYC_OK;
}

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
// multipliers, 8 = no staging of the chunk / slice (the loader wave idles),
// 16 = no run loads (synthetic ids and values), 32 = no segment offset
// loads (every run 256 long), 64 = full-occupancy repeats (round 6's MALL
// residency probe: every CU busy however small the layout -- the margin
// pass on one workgroup per CU, each taking TileDims::reps super blocks
// modulo the layout's; the gradient pass walking its row range reps times --
// so a layout that fits the Infinity Cache is re-read by hundreds of steps
// per workgroup, the per-step time comparable with a streamed layout's;
// CYC_TILES_REPS sets reps).  0 in the library.
#ifndef CYC_TILES_PROBE
#define CYC_TILES_PROBE 0
#endif
constexpr bool kRepeatProbe = (CYC_TILES_PROBE & 64) != 0;

// LDS pointers are kept in address space 3 from the __shared__ array on
// (the cast of the array folds): derived through generic pointers, the
// compiler emitted an is-shared check for the DMA's LDS address that
// gfx950's instruction selection rejects (src_shared_base in a VALU compare)
using lds_f64 = __attribute__((address_space(3))) double;

__device__ __forceinline__ void lds_add(lds_f64* p, double x) {
  if constexpr ((CYC_TILES_PROBE & 1) != 0) *p = x;
  else __builtin_amdgcn_ds_atomic_fadd_f64(p, x);
}

// s_waitcnt immediate for "at most n vector memory operations outstanding"
// (gfx9 encoding: vmcnt in bits 3:0 and 15:14; expcnt and lgkmcnt left at
// their maxima, i.e. not waited for)
constexpr int vm_wait(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

// buffer resource over [p, p + bytes): lanes past the end read 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                           (int)std::min<int64_t>(bytes, 0x7fffffff), 0x00020000);
}

// A/B switches of the step's shape (tools/build_variant.sh), measured at
// 200M rows (config 5; the first value is kept):
//   MARGIN_SYNC / GRAD_SYNC  0 = a bare s_barrier per step, 1 = a full
//       __syncthreads (its fence waits for the step's LDS atomics and
//       offset loads first): margin 30.3 (0) / 32.0-32.3 (1) ms, gradient
//       27.0 (1) / 27.9 (0) ms;
//   SCHED 1 = scheduling barriers that pin the issue order (no gain);
//   LATE_LOADS 1 = the next run's loads issued after the current run's
//       LDS work; issued before it (0) both passes took 36 / 33.4 ms.
#ifndef CYC_TILES_MARGIN_SYNC
#define CYC_TILES_MARGIN_SYNC 0
#endif
#ifndef CYC_TILES_GRAD_SYNC
#define CYC_TILES_GRAD_SYNC 1
#endif
#ifndef CYC_TILES_SCHED
#define CYC_TILES_SCHED 0
#endif
#ifndef CYC_TILES_LATE_LOADS
#define CYC_TILES_LATE_LOADS 1
#endif
#define CYC_TILES_SCHED_BARRIER()                                \
  do {                                                           \
    if constexpr (CYC_TILES_SCHED) __builtin_amdgcn_sched_barrier(0); \
  } while (0)

// The per-step barrier (step_sync<0>: a bare s_barrier).  Within the step loops a barrier
// only has to order the compute waves' LDS READS of the step's slice (their
// values are consumed before it) before the loader's next DMA into that
// buffer, and the loader waits for its own DMA before it; the LDS atomics
// and the next step's offset loads may stay in flight across it (the
// __syncthreads fence would wait for both: lgkmcnt(0)).  A full
// __syncthreads follows each step loop before anything reads the sums.
template <int FULL>
__device__ __forceinline__ void step_sync() {
  if constexpr (FULL) __syncthreads();
  else __builtin_amdgcn_s_barrier();
}

struct TileDims {
  int64_t n, nRB;
  int F, T, Wt;
  int reps = 1;   // probe bit 64 only
};

// One wave's run: a segment's nonzeros [a, b), empty when !on.  The
// segment offsets come through __restrict__ read-only pointers, so the
// compiler fetches them with scalar loads (lgkmcnt): reading them never
// waits on the runs in flight (vmcnt).  The loads are unconditional (from
// segment 0 when off) and the length is formed only where it is used, a
// step later: a branch around them, or the subtraction beside them, put an
// s_waitcnt lgkmcnt(0) right behind every step's offset load.
struct Run {
  int64_t a, b;
  bool on;
  __device__ __forceinline__ int64_t len() const { return on ? b - a : 0; }
};

__device__ __forceinline__ Run seg_run(const int64_t* __restrict__ segStart, int64_t seg,
                                       bool on) {
  if constexpr ((CYC_TILES_PROBE & 32) != 0) return Run{0, 256, on};   // the first 256 nonzeros
  const int64_t q = on ? seg : 0;
  return Run{segStart[q], segStart[q + 1], on};
}

// the first KC x 64 entries of a run from `from` on, lane-strided; lanes
// past the end read 0 (buffer range check).  CPT: 16-bit compact ids
// (zero-extended), else the 32-bit packed ones.
template <int KC, bool CPT>
__device__ __forceinline__ void load_run(const uint32_t* __restrict__ vidx,
                                         const double* __restrict__ vvals, const Run& r,
                                         int64_t from, int lane, uint32_t (&ix)[KC],
                                         double (&vx)[KC]) {
  const int64_t len = r.len() - from;
  if constexpr ((CYC_TILES_PROBE & 16) != 0) {   // in-range ids of both formats
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      ix[j] = CPT ? ((uint32_t)(lane * 29 + j) & 1023)
                  : ((uint32_t)(lane * 31 + j * 7) & 2047) << 16 | ((uint32_t)(lane * 29 + j) & 1023);
      vx[j] = 1.0 + j;
    }
    return;
  }
  const auto rv = rsrc(vvals + r.a + from, len > 0 ? len * 8 : 0);
  if constexpr (CPT) {
    const auto rh = rsrc(reinterpret_cast<const uint16_t*>(vidx) + r.a + from,
                         len > 0 ? len * 2 : 0);
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      ix[j] = __builtin_amdgcn_raw_buffer_load_b16(rh, lane * 2, j * 128, 2);
      vx[j] = __builtin_bit_cast(double,
                                 __builtin_amdgcn_raw_buffer_load_b64(rv, lane * 8, j * 512, 2));
    }
    return;
  }
  const auto ri = rsrc(vidx + r.a + from, len > 0 ? len * 4 : 0);
  // lane part in the VGPR offset, batch part in the immediate offset
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    ix[j] = __builtin_amdgcn_raw_buffer_load_b32(ri, lane * 4, j * 256, 2);
    vx[j] = __builtin_bit_cast(double,
                               __builtin_amdgcn_raw_buffer_load_b64(rv, lane * 8, j * 512, 2));
  }
}

// The (row in block, column in chunk) of a slot's entries and whether each
// is a nonzero.  Compact: low = row mod 32; each lane compares its low with
// the previous entry's (the lane below, by DPP wave_shr:1; lane 0 the last
// entry of the slot before, `lowc`), a drop means the row passed a multiple
// of 32, and the row's high part is `highc` (the drops of the run's earlier
// slots) + the drops in the lanes up to this one (ballot + mbcnt).  Lanes
// past the run's end read 0; they only come after its last entry.
template <int KC, bool CPT>
__device__ __forceinline__ void decode(const uint32_t (&ix)[KC], uint32_t& highc,
                                       uint32_t& lowc, uint32_t (&row)[KC],
                                       uint32_t (&col)[KC], bool (&real)[KC]) {
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    if constexpr (CPT) {
      const uint32_t low = ix[j] >> kColBits;
      const uint32_t prev =
          (uint32_t)__builtin_amdgcn_update_dpp((int)lowc, (int)low, 0x138, 0xf, 0xf, false);
      const bool drop = low < prev;
      const uint64_t m = __ballot(drop);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      row[j] = ((highc + below + (drop ? 1u : 0u)) << 5) | low;
      highc += (uint32_t)__builtin_popcountll(m);
      lowc = (uint32_t)__builtin_amdgcn_readlane((int)low, 63);
      col[j] = ix[j] & kFillCol;
      real[j] = col[j] != kFillCol;
    } else {
      row[j] = ix[j] >> 16;
      col[j] = ix[j] & 0xffff;
      real[j] = true;
    }
  }
}

// Both passes run 8 compute waves and ONE loader wave per workgroup.  The
// loader stages the step's shared 16 KiB slice (the margin pass's
// coefficient chunk, the gradient pass's multiplier slice) into LDS one step
// ahead and waits for it itself; the compute waves only issue and wait for
// their own runs.  vmcnt counts a wave's vector-memory operations in issue
// order, so a compute wave that staged the slice itself had to wait, before
// each barrier, for the slice AND every run it had prefetched before it --
// its run prefetch was one step deep whatever its depth.  With the loader
// the runs of the next NB - 1 steps stay in flight across barriers.
constexpr int kLoaderWave = kTileWaves;
constexpr int kTPBL = 64 * (kTileWaves + 1);

// run buffers per compute wave: the runs of the next NB - 1 steps in flight
#ifndef CYC_TILES_NB
#define CYC_TILES_NB 6
#endif

// The loader wave's staging of one slice src[0, count) (count <= 2048
// doubles, lanes past it read 0) into the LDS buffer b by LDS DMA (16
// one-KiB wave-instructions, 16-byte pieces; 64 of 4-byte pieces when src
// is not 16-byte aligned), waited for by the loader alone before the step's
// barrier.  (Staging through the loader's registers two steps ahead, the
// slice written by ds_write, measured slower: 36.8 / 33.9 against 30.8 /
// 30.1 ms per margin / gradient pass at 200M rows.)
__device__ __forceinline__ int dma_slice(const double* src, int64_t count, lds_f64* b, int lane) {
  const auto rs = rsrc(src, count * 8);
  if constexpr ((CYC_TILES_PROBE & 8) != 0) return 0;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(b + i * 128), 16, i * 1024 + lane * 16, 0,
          0, 0);
    return 16;
  }
#pragma unroll
  for (int i = 0; i < 64; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(b + i * 32), 4, i * 256 + lane * 4, 0, 0, 0);
  return 64;
}
__device__ __forceinline__ void stage_slice(const double* src, int64_t count, lds_f64* b,
                                            int lane) {
  dma_slice(src, count, b, lane);
  __builtin_amdgcn_s_waitcnt(vm_wait(0));
}
static_assert(kTileCols == 16 * 128 && kTileRows == 16 * 128, "16 one-KiB pieces per slice");


// Margin pass, persistent over (super row block sb, column chunk c) steps:
// this workgroup's super blocks sb = blockIdx.x + i * gridDim.x (kMW = 7 row
// blocks each), each swept over the T chunks (padded to Tp, a multiple of
// NB), as one flat sequence of steps g = k * Tp + c.  Per step: compute wave
// i walks segment (7 sb + i, c) with chunk c in cf[g % 3] (ONE barrier), the
// runs of the next NB - 1 steps in flight across super block boundaries too;
// the loader wave DMAs the chunk of step g + 2 into cf[(g + 2) % 3] -- the
// buffer of step g - 1, free since the last barrier -- and waits only for
// the chunk of step g + 1, issued a step ago: a whole step for every DMA to
// land (with two buffers and 8 row blocks it had to land within the step it
// was issued in; the coefficients' 8 MB drift out of L2 and the Infinity
// Cache between two workgroups' uses).  7 row blocks of dots (112 KiB) + 3
// chunk buffers (48 KiB) fill the 160 KiB.  The super block's finished dots
// go to dotOut (the rows' epilogue is k_tiles_rows: in here each batch of
// rows waited on a fresh label load from HBM while the CU streamed nothing,
// ~2 ms of a 30 ms pass at 200M rows).
// chunk buffers of the margin pass: 2 (8 row blocks per super block, the
// DMA lands within the step it is issued in) or 3 (7 row blocks, each DMA a
// step of lead) -- an A/B switch: with the compact entries and branch-free
// adds, 25.7 (2) against 27.7 (3) ms per margin pass at 200M rows (9 % more
// steps with 7 row blocks; before those two changes 3 buffers had won)
#ifndef CYC_TILES_MARGIN_BUFS
#define CYC_TILES_MARGIN_BUFS 2
#endif
constexpr int kMBufs = CYC_TILES_MARGIN_BUFS;
constexpr int kMW = kMBufs == 3 ? 7 : 8;        // compute waves (row blocks) per margin workgroup
constexpr int kMTPB = 64 * (kMW + 1);          // + the loader wave
constexpr int kMRows = kMW * kTileRows;         // rows per margin super block

template <int NB, int KC, bool LONG, bool CPT>
__global__ __launch_bounds__(kMTPB) void k_tiles_margin(
    TileDims v, const int64_t* __restrict__ segStart, const uint32_t* __restrict__ vidx,
    const double* __restrict__ vvals, const double* __restrict__ coef,
    double* __restrict__ dotOut) {
  static_assert(NB >= 2, "at least one run in flight");
  static_assert(kMRows * 8 + kMBufs * kTileCols * 8 <= 160 * 1024, "LDS");
  __shared__ double lds[kMRows + kMBufs * kTileCols];
  lds_f64* const dots = (lds_f64*)lds;
  lds_f64* const cf = dots + kMRows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = v.T;
  const int64_t nSB = (v.nRB + kMW - 1) / kMW;
  const int Tp = (T + NB - 1) / NB * NB;
  const int64_t mySB = kRepeatProbe ? v.reps
                                    : nSB > blockIdx.x ? (nSB - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  // this workgroup's k-th super block (the probe: modulo the layout's)
  auto sbOf = [&](int64_t k) {
    const int64_t sb = (int64_t)blockIdx.x + k * gridDim.x;
    return kRepeatProbe ? sb % nSB : sb;
  };
  // buffer of flat step g: g % kMBufs (the flat step count fits 32 bits:
  // Tp * super blocks per workgroup is the launch's per-workgroup steps)
  auto bufOf = [&](int64_t k, int c) {
    return cf + ((uint32_t)(k * Tp + c) % (uint32_t)kMBufs) * kTileCols;
  };

  if (wave == kMW) {
    // the loader: the same barriers as the compute waves, in the same order
    auto chunk = [&](int64_t k, int c) {
      const bool on = k < mySB && c < T;
      const int64_t c0 = on ? (int64_t)c * v.Wt : 0;
      const int64_t wl = on ? std::min<int64_t>(v.Wt, v.F - c0) : 0;
      return dma_slice(coef + c0, wl, bufOf(k, c), lane);
    };
    auto next = [&](int64_t& k, int& c) {
      if (++c >= Tp) c = 0, ++k;
    };
    int64_t k2 = 0;
    int c2 = 0;
    chunk(k2, c2);                                // step 0
    next(k2, c2);
    if constexpr (kMBufs == 3) {
      const int n1 = chunk(k2, c2);               // step 1
      next(k2, c2);
      if (n1 == 16) __builtin_amdgcn_s_waitcnt(vm_wait(16));   // step 0's landed
      else __builtin_amdgcn_s_waitcnt(vm_wait(0));
    } else {
      __builtin_amdgcn_s_waitcnt(vm_wait(0));
    }
    for (int64_t k = 0; k < mySB; ++k) {
      __syncthreads();                            // dots zeroed, chunk (k, 0) in place
      for (int c = 0; c < Tp; ++c) {
        // the chunk kMBufs - 1 steps ahead (k2, c2) into the buffer the last
        // barrier freed; then the chunk of the next step landed (3 buffers:
        // issued a step ago, only the DMA just issued may stay in flight)
        const int n2 = chunk(k2, c2);
        next(k2, c2);
        if (kMBufs == 3 && n2 == 16) __builtin_amdgcn_s_waitcnt(vm_wait(16));
        else __builtin_amdgcn_s_waitcnt(vm_wait(0));
        step_sync<CYC_TILES_MARGIN_SYNC>();       // step (k, c)
      }
      __syncthreads();                            // the super block's dots complete
      __syncthreads();                            // dots stored
    }
    return;
  }

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
    const int64_t rb = sbOf(k) * kMW + wave;
    return seg_run(segStart, rb * T + c, k < mySB && c < T && rb < v.nRB);
  };
  lds_f64* const myDots = dots + wave * kTileRows;
  // waits for the whole run first, on every path: its values are used only
  // under the lanes' `< len` branches, and a path that skips one left the
  // compiler's wait analysis treating the registers as still loading at the
  // loop head, where it then drained every prefetched run (vmcnt(0)); the
  // runs of the next NB - 2 steps stay in flight
  // The adds are branch-free: a lane past the run's end or on a filler adds
  // +0.0 to the wave's own dot [lane] -- an exact no-op, since a sum that
  // starts at +0.0 is never -0.0 (x + +0.0 == x for every other x, NaN and
  // infinities included) -- so the compiler issues the step's gathers, ONE
  // wait, then every atomic (behind an exec-mask branch each atomic waited
  // lgkmcnt(0), i.e. for the atomic before it; one shared dummy address
  // serialised the masked lanes).
  auto consume = [&](int64_t len, lds_f64* cfp, const uint32_t (&ix)[KC],
                     const double (&vx)[KC], uint32_t& highc, uint32_t& lowc) {
    __builtin_amdgcn_s_waitcnt(vm_wait((NB - 2 + !CYC_TILES_LATE_LOADS) * 2 * KC));
    uint32_t row[KC], col[KC];
    bool real[KC];
    decode<KC, CPT>(ix, highc, lowc, row, col, real);
    double c[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j)   // lanes past the end read [0]
      c[j] = (CYC_TILES_PROBE & 2) ? vx[j] : cfp[col[j]];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const bool on = j * 64 + lane < len && real[j];
      lds_add(&myDots[on ? row[j] : (uint32_t)lane], on ? vx[j] * c[j] : 0.0);
    }
  };
  // One step (k, c), ONE barrier: the current run into the row sums with
  // chunk (k, c) in cf[g % 3], then the loads of the run NB - 1 steps ahead
  // (its offsets loaded a step ago), then the scalar loads of the offsets of
  // the run NB steps ahead (into this step's slot, its own offsets kept in
  // `cur`): issued after the step's LDS reads, since an SMEM load in flight
  // turns every lgkmcnt wait into lgkmcnt(0) (SMEM returns out of order),
  // and waited for by the next step's first use -- before, a scalar load
  // waited for in front of the run loads also drained the step's LDS
  // atomics.  The loads are issued unconditionally (past the end they fetch
  // nothing, so the waits stay counted); the run buffers rotate by
  // unrolling (never by copying a register that a load is still filling).
  auto step = [&](int64_t k, int c, Run& rc, uint32_t (&ic)[KC], double (&vc)[KC],
                  const Run& rn, uint32_t (&in)[KC], double (&vn)[KC]) {
    const Run cur = rc;
    lds_f64* buf = bufOf(k, c);
    if constexpr (!CYC_TILES_LATE_LOADS) {
      load_run<KC, CPT>(vidx, vvals, rn, 0, lane, in, vn);
      CYC_TILES_SCHED_BARRIER();                  // the loads issue first
    }
    uint32_t highc = 0, lowc = 0;               // the run's row before each slot
    consume(cur.len(), buf, ic, vc, highc, lowc);
    // a run longer than KC x 64: only in the LONG instance (a layout with
    // such segments), in registers of its own -- any load in this loop's
    // body makes the compiler's wait analysis drain every prefetched run
    // at the loop head
    if constexpr (LONG) {
      for (int64_t b = KC * 64; b < cur.len(); b += KC * 64) {
        uint32_t it[KC];
        double vt[KC];
        load_run<KC, CPT>(vidx, vvals, cur, b, lane, it, vt);
        consume(cur.len() - b, buf, it, vt, highc, lowc);
      }
    }
    if constexpr (CYC_TILES_LATE_LOADS) load_run<KC, CPT>(vidx, vvals, rn, 0, lane, in, vn);
    CYC_TILES_SCHED_BARRIER();
    int64_t k2;
    int c2;
    ahead(k, c, NB, k2, c2);
    rc = run_of(k2, c2);
    step_sync<CYC_TILES_MARGIN_SYNC>();
  };

  // prologue: the offsets of steps 0 .. NB - 1, the runs of steps
  // 0 .. NB - 2 in flight
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    int64_t k1;
    int c1;
    ahead(0, 0, u, k1, c1);
    rr[u] = run_of(k1, c1);
  }
#pragma unroll
  for (int u = 0; u < NB - 1; ++u) load_run<KC, CPT>(vidx, vvals, rr[u], 0, lane, ib[u], vb[u]);
  constexpr int kCT = 64 * kMW;                  // compute threads
  static_assert(kMRows % kCT == 0, "whole dots per thread");
  for (int64_t k = 0; k < mySB; ++k) {          // one super block per pass
#pragma unroll
    for (int i = 0; i < kMRows / kCT; ++i) dots[tid + kCT * i] = 0.0;
    __syncthreads();                            // zeroed dots, chunk (k, 0) in place
    for (int c = 0; c < Tp; c += NB) {
#pragma unroll
      for (int u = 0; u < NB; ++u)
        step(k, c + u, rr[u], ib[u], vb[u], rr[(u + NB - 1) % NB], ib[(u + NB - 1) % NB],
             vb[(u + NB - 1) % NB]);
    }
    __syncthreads();                            // every wave's atomics landed
    const int64_t r0 = sbOf(k) * kMRows;
#pragma unroll
    for (int i = 0; i < kMRows / kCT; ++i) {
      const int64_t r = r0 + tid + kCT * i;
      if (r < v.n) __builtin_nontemporal_store(dots[tid + kCT * i], &dotOut[r]);
    }
    __syncthreads();                            // dots read before the next zeroing
  }
}

// The rows' epilogue of the binary aggregators after the margin pass: per
// row r, margin = row_margin(offset + dot_r) and the aggregator kind's
// multiplier (binary_rows.hpp; kind 0 BinaryLogisticBlockAggregator.scala:
// 104-122 without branches: log1pExp(x) (ml/impl/Utils.scala:91-97) as
// max(x, 0) + log1p(exp(-|x|)), the same two branches and bits), written
// over the dot in dm; per-workgroup (loss, weight, multiplierSum,
// sigmaGradSum) partials to slabS[wg * 4 + k] -- each thread's rows in row
// order, a fixed shuffle tree per wave, the waves in order.  Streams 24 B
// per row (dot, label, multiplier; + 8 with weights).
#ifndef CYC_TILES_ROWS_U
#define CYC_TILES_ROWS_U 2
#endif
// LOG: the logistic instance alone (kind 0, the bench's and LogisticRegression's
// path): without the other kinds' code its registers stay low (more waves in
// flight for the stream)
template <bool LOG>
__global__ __launch_bounds__(256) void k_tiles_rows(
    int64_t n, const double* __restrict__ labels, const double* __restrict__ weights,
    int fitIntercept, int kind, double offsetH, const double* __restrict__ offsetD,
    double lscale, double sigma, double eps, double* __restrict__ dm,
    double* __restrict__ slabS) {
  // the margin offset from the device when given (no host round trip)
  const double offset = offsetD ? *offsetD : offsetH;
  __shared__ double red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};     // loss, weight, multiplierSum, sigmaGradSum
  const int64_t stride = (int64_t)gridDim.x * 256;
  // U rows per batch, two batches in registers: the next batch's loads are
  // in flight while this one's rows are computed (software-pipelined)
  constexpr int U = CYC_TILES_ROWS_U;
  struct Batch {
    double dot[U], lab[U], w[U];
  };
  auto ld = [&](int64_t r0, Batch& b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = min<int64_t>(r0 + u * stride, n - 1);
      b.dot[u] = __builtin_nontemporal_load(&dm[r]);
      b.lab[u] = __builtin_nontemporal_load(&labels[r]);
      b.w[u] = weights ? __builtin_nontemporal_load(&weights[r]) : 1.0;
    }
  };
  auto rows = [&](int64_t r0, const Batch& b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + u * stride;
      if (r >= n) break;
      double m;
      if constexpr (LOG) {
        const double margin = fitIntercept ? offset + b.dot[u] : b.dot[u];
        const double x = -margin;
        const double lp = __builtin_fmax(x, 0.0) + log1p(exp(-__builtin_fabs(x)));
        const double term = b.lab[u] > 0 ? lp : lp + margin;
        const double mm = b.w[u] * (1.0 / (1.0 + exp(-margin)) - b.lab[u]);
        acc[1] += b.w[u];
        m = 0.0;
        if (b.w[u] > 0) {
          acc[0] += b.w[u] * term;
          m = mm;
        }
      } else {
        const double margin =
            cyc::row_margin(kind, fitIntercept, offset, lscale, b.lab[u], b.dot[u]);
        m = cyc::bin_row(kind, margin, b.w[u], b.lab[u], acc[0], acc[1], acc[3], sigma, eps);
      }
      acc[2] += m;
      __builtin_nontemporal_store(m, &dm[r]);
    }
  };
  const int64_t first = (int64_t)blockIdx.x * 256 + tid;
  Batch ba, bb;
  if (first < n) ld(first, ba);
#pragma unroll 1
  for (int64_t r0 = first; r0 < n; r0 += 2 * U * stride) {
    const int64_t r1 = r0 + U * stride, r2 = r1 + U * stride;
    if (r1 < n) ld(r1, bb);
    rows(r0, ba);
    if (r2 < n) ld(r2, ba);
    if (r1 < n) rows(r1, bb);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc[k] += __shfl_xor(acc[k], m);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wave][k] = acc[k];
  }
  __syncthreads();
  if (tid < 4) slabS[(int64_t)blockIdx.x * 4 + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) +
                                                     red[3][tid];
}

// Gradient pass: workgroup (super chunk st = 8 column chunks, row range)
// over its row blocks.  Per row block: compute wave j walks segment
// (rb, 8 st + j) into its chunk's column sums with the multiplier slice of
// rb in mv[(rb - rbA) & 1] (ONE barrier), the runs of the next NB - 1 row
// blocks in flight; the loader stages the next row block's slice.  Block b
// is (st = b / R, range = b % R): the blocks of one XCD (b mod 8) walk the
// same row ranges together, so a row block's multiplier slice is read from
// the XCD's L2 by all but the first.  (A flat split of the sts * nRB units
// over exactly one workgroup per CU -- config 5's 62 super chunks x 4
// ranges leave 8 of 256 CUs idle -- took 29.7 against 24.6 ms: its
// workgroups on an XCD walked different rows and every slice came from
// HBM.)
template <int NB, int KC, bool LONG, bool CPT>
__global__ __launch_bounds__(kTPBL) void k_tiles_grad(
    TileDims v, const int64_t* __restrict__ segStart, const uint32_t* __restrict__ vidx,
    const double* __restrict__ vvals, const double* __restrict__ mult, int ranges,
    double* __restrict__ slabG) {
  static_assert(NB >= 2, "at least one run in flight");
  // 160 KiB: the 8 chunks' column sums and two multiplier slice buffers
  __shared__ double lds[kTileSuperCols + 2 * kTileRows];
  lds_f64* const gt = (lds_f64*)lds;
  lds_f64* const mv = gt + kTileSuperCols;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int range = blockIdx.x % ranges, st = blockIdx.x / ranges;
  const int64_t rbA = v.nRB * range / ranges, rbB = v.nRB * (range + 1) / ranges;
  // whole groups of NB steps: the last group's steps past rbB have empty
  // runs and slices (no guard inside the unroll: a skipped step left the
  // compiler's wait analysis draining every prefetched run at the loop head)
  const int64_t span = rbB - rbA;
  const int64_t steps = ((kRepeatProbe ? span * v.reps : span) + NB - 1) / NB * NB;
  // the probe's repeats: row block rb of the walk is rbA + (rb - rbA) % span
  auto wrap = [&](int64_t rb) {
    return kRepeatProbe && span > 0 ? rbA + (rb - rbA) % span : rb;
  };

  if (wave == kLoaderWave) {
    auto slice = [&](int64_t rbu) {
      const int64_t rb = wrap(rbu);
      const bool on = rb < rbB;
      const int64_t r0 = on ? rb * kTileRows : 0;
      stage_slice(mult + r0, on ? std::min<int64_t>(kTileRows, v.n - r0) : 0,
                  mv + ((rbu - rbA) & 1) * kTileRows, lane);
    };
    slice(rbA);
    __syncthreads();                              // sums zeroed, slice rbA in place
    for (int64_t s = 0; s < steps; ++s) {
      slice(rbA + s + 1);                         // into the buffer the last barrier freed
      step_sync<CYC_TILES_GRAD_SYNC>();           // step rbA + s
    }
    __syncthreads();                              // sums complete
    return;
  }

  const int c = st * kTileWaves + wave;           // this wave's column chunk
  uint32_t ib[NB][KC];
  double vb[NB][KC];
  Run rr[NB];
  auto run_of = [&](int64_t rbu) {
    const int64_t rb = wrap(rbu);
    return seg_run(segStart, rb * v.T + c, rb < rbB && c < v.T);
  };
  lds_f64* const myG = gt + wave * v.Wt;
  // waits for the whole run first, on every path (the margin pass's
  // consume says why); branch-free adds: a masked lane adds +0.0 to the
  // wave's sum [lane] (the margin pass's consume says why; a chunk holds at
  // least 64 columns)
  auto consume = [&](int64_t len, const lds_f64* mvp, const uint32_t (&ix)[KC],
                     const double (&vx)[KC], uint32_t& highc, uint32_t& lowc) {
    __builtin_amdgcn_s_waitcnt(vm_wait((NB - 2 + !CYC_TILES_LATE_LOADS) * 2 * KC));
    uint32_t row[KC], col[KC];
    bool real[KC];
    decode<KC, CPT>(ix, highc, lowc, row, col, real);
    double m[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j)   // lanes past the end read [0]
      m[j] = (CYC_TILES_PROBE & 2) ? vx[j] : mvp[row[j]];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const bool on = j * 64 + lane < len && real[j];
      lds_add(&myG[on ? col[j] : (uint32_t)lane], on ? vx[j] * m[j] : 0.0);
    }
  };

#pragma unroll
  for (int i = 0; i < kGPT; ++i) gt[tid + kTPB * i] = 0.0;
  // one row block (the u-th of an unrolled group), ONE barrier: the run
  // NB - 1 row blocks ahead issued (its offsets loaded a step ago), the
  // current run into the column sums with the slice in mv[(rb - rbA) & 1],
  // then the offsets of the run NB ahead loaded into this step's slot (the
  // margin pass's step says why in this order); the run buffers rotate by
  // unrolling
  auto step = [&](int64_t rb, Run& rc, uint32_t (&ic)[KC], double (&vc)[KC], const Run& rn,
                  uint32_t (&in)[KC], double (&vn)[KC]) {
    const Run cur = rc;
    const lds_f64* buf = mv + ((rb - rbA) & 1) * kTileRows;
    if constexpr (!CYC_TILES_LATE_LOADS) {
      load_run<KC, CPT>(vidx, vvals, rn, 0, lane, in, vn);
      CYC_TILES_SCHED_BARRIER();                  // the loads issue first
    }
    uint32_t highc = 0, lowc = 0;                 // the run's row before each slot
    consume(cur.len(), buf, ic, vc, highc, lowc);
    if constexpr (LONG) {
      for (int64_t b = KC * 64; b < cur.len(); b += KC * 64) {
        uint32_t it[KC];
        double vt[KC];
        load_run<KC, CPT>(vidx, vvals, cur, b, lane, it, vt);
        consume(cur.len() - b, buf, it, vt, highc, lowc);
      }
    }
    if constexpr (CYC_TILES_LATE_LOADS) load_run<KC, CPT>(vidx, vvals, rn, 0, lane, in, vn);
    CYC_TILES_SCHED_BARRIER();                    // after the LDS reads (the margin pass's step)
    rc = run_of(rb + NB);
    step_sync<CYC_TILES_GRAD_SYNC>();
  };

  // prologue: the offsets of row blocks rbA .. rbA + NB - 1, the runs of
  // rbA .. rbA + NB - 2 in flight
#pragma unroll
  for (int u = 0; u < NB; ++u) rr[u] = run_of(rbA + u);
#pragma unroll
  for (int u = 0; u < NB - 1; ++u) load_run<KC, CPT>(vidx, vvals, rr[u], 0, lane, ib[u], vb[u]);
  __syncthreads();                                // zeroed sums, slice rbA in place
  for (int64_t s = 0; s < steps; s += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u)
      step(rbA + s + u, rr[u], ib[u], vb[u], rr[(u + NB - 1) % NB], ib[(u + NB - 1) % NB],
           vb[(u + NB - 1) % NB]);
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

// probe bit 64's repeats (CYC_TILES_REPS, default 1)
int probe_reps() {
  if constexpr (!kRepeatProbe) return 1;
  const char* e = std::getenv("CYC_TILES_REPS");
  return e ? std::max(1, std::atoi(e)) : 1;
}

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
  v->compact = t->fmt == CYC_TILES_COMPACT;
  return CYC_OK;
}

int tiles_margin(const TilesView& v, const double* coef, double* dots, hipStream_t st) {
  const int64_t nSB = (v.nRB + kMW - 1) / kMW;
  const int64_t grid =
      kRepeatProbe ? device_cus() : std::max<int64_t>(1, std::min<int64_t>(nSB, device_cus()));
  const TileDims d{v.n, v.nRB, v.F, v.T, v.Wt, probe_reps()};
#define CYC_TILES_MARGIN(KC, LONG, CPT)                                                         \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_tiles_margin<CYC_TILES_NB, KC, LONG, CPT>),              \
                     dim3((unsigned)grid), dim3(kMTPB), 0, st, d, v.segStart, v.idx, v.vals,    \
                     coef, dots)
  if (v.compact) {
    if (long_runs(v.maxSeg)) CYC_TILES_MARGIN(5, true, true);
    else CYC_TILES_MARGIN(5, false, true);
  } else {
    if (long_runs(v.maxSeg)) CYC_TILES_MARGIN(5, true, false);
    else CYC_TILES_MARGIN(5, false, false);
  }
#undef CYC_TILES_MARGIN
  CYC_LAUNCH_CHECK("k_tiles_margin");
  return CYC_OK;
}

int64_t tiles_rows_blocks(int64_t n) {
  return std::max<int64_t>(1, std::min<int64_t>(8 * device_cus(), (n + 1023) / 1024));
}

int tiles_rows(int64_t n, const double* labels, const double* weights, int fitIntercept,
               int kind, double offset, const double* offsetDev, double lscale, double sigma,
               double eps, double* dm, double* slabS, int64_t* wgs, hipStream_t st) {
  const int64_t g = tiles_rows_blocks(n);
  *wgs = g;
  if (kind == 0)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_tiles_rows<true>), dim3((unsigned)g), dim3(256), 0, st, n,
                       labels, weights, fitIntercept, kind, offset, offsetDev, lscale, sigma, eps,
                       dm, slabS);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_tiles_rows<false>), dim3((unsigned)g), dim3(256), 0, st, n,
                       labels, weights, fitIntercept, kind, offset, offsetDev, lscale, sigma, eps,
                       dm, slabS);
  CYC_LAUNCH_CHECK("k_tiles_rows");
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
  const TileDims d{v.n, v.nRB, v.F, v.T, v.Wt, probe_reps()};
#define CYC_TILES_GRAD(KC, LONG, CPT)                                                           \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_tiles_grad<CYC_TILES_NB, KC, LONG, CPT>),                \
                     dim3((unsigned)(sts * R)), dim3(kTPBL), 0, st, d, v.segStart, v.idx, v.vals, \
                     mult, R, slabG)
  if (v.compact) {
    if (long_runs(v.maxSeg)) CYC_TILES_GRAD(5, true, true);
    else CYC_TILES_GRAD(5, false, true);
  } else {
    if (long_runs(v.maxSeg)) CYC_TILES_GRAD(5, true, false);
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
  // the entry arrays are reserved once the format is known (set_format, or
  // the first append that holds nonzeros)
  if (int rc = t->segStart.reserve(sizeof(int64_t) * (size_t)(segs + 1))) {
    delete t;
    return rc;
  }
  CYC_HIP(hipMemset(t->segStart.ptr, 0, sizeof(int64_t)));
  *out = t;
  return CYC_OK;
}

int cyc_tiles_set_format(cyc_tiles t, int32_t format) {
  CYC_REQUIRE(t != nullptr, "tiles must not be null");
  CYC_REQUIRE(format == CYC_TILES_AUTO || format == CYC_TILES_WIDE || format == CYC_TILES_COMPACT,
              "format must be CYC_TILES_AUTO, CYC_TILES_WIDE or CYC_TILES_COMPACT");
  std::lock_guard<std::mutex> g(t->mu);
  CYC_REQUIRE(t->n == 0 && t->fmt == CYC_TILES_AUTO,
              "the entry format is chosen before the first append");
  if (format != CYC_TILES_AUTO) return set_storage(t, format);
  return CYC_OK;
}

int32_t cyc_tiles_format(cyc_tiles t) { return t ? t->fmt : -1; }

int64_t cyc_tiles_entries(cyc_tiles t) { return t ? t->entries : -1; }

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
  cyc::DeviceBuffer keys, packed, keysOut, perm, tmp, counts, posb;
  // an append that fails leaves the layout as it was before it (the
  // segments it had written are rewritten by the next append of those rows)
  const int64_t nnz0 = t->nnz;
  int64_t entries0 = t->entries;
  int arc = [&]() -> int {
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
    const unsigned long long* pos = nullptr;    // compact: entry positions
    int64_t total = cnt;                        // entries of the sub-chunk
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
      rocprim::counting_iterator<uint32_t> cpos(0);
      CYC_HIP(rocprim::radix_sort_pairs(nullptr, tmpBytes, (const uint32_t*)keys.ptr,
                                        (uint32_t*)nullptr, cpos, (uint32_t*)nullptr, (size_t)cnt,
                                        0, endBit, st));
      if ((rc = tmp.reserve(tmpBytes))) return rc;
      CYC_HIP(rocprim::radix_sort_pairs(tmp.ptr, tmpBytes, (const uint32_t*)keys.ptr,
                                        (uint32_t*)keysOut.ptr, cpos, (uint32_t*)perm.ptr,
                                        (size_t)cnt, 0, endBit, st));
      if (t->fmt != CYC_TILES_WIDE) {
        // the compact entries this sub-chunk takes (fillers included)
        if ((rc = counts.reserve(sizeof(uint32_t) * (size_t)cnt)) ||
            (rc = posb.reserve(sizeof(unsigned long long) * (size_t)cnt)) ||
            (rc = t->scal.reserve(sizeof(int64_t))))
          return rc;
        hipLaunchKernelGGL(k_tile_fill_counts, dim3(8192), dim3(256), 0, st,
                           (const uint32_t*)keysOut.ptr, (const uint32_t*)perm.ptr,
                           (const uint32_t*)packed.ptr, cnt, (uint32_t*)counts.ptr);
        CYC_LAUNCH_CHECK("k_tile_fill_counts");
        size_t scanBytes = 0;
        CYC_HIP(rocprim::exclusive_scan(nullptr, scanBytes, (const uint32_t*)counts.ptr,
                                        (unsigned long long*)posb.ptr, 0ull, (size_t)cnt,
                                        rocprim::plus<unsigned long long>(), st));
        if ((rc = tmp.reserve(std::max(tmpBytes, scanBytes)))) return rc;
        CYC_HIP(rocprim::exclusive_scan(tmp.ptr, scanBytes, (const uint32_t*)counts.ptr,
                                        (unsigned long long*)posb.ptr, 0ull, (size_t)cnt,
                                        rocprim::plus<unsigned long long>(), st));
        hipLaunchKernelGGL(k_tile_total, dim3(1), dim3(1), 0, st, (const uint32_t*)counts.ptr,
                           (const unsigned long long*)posb.ptr, cnt, (int64_t*)t->scal.ptr);
        CYC_LAUNCH_CHECK("k_tile_total");
        CYC_HIP(hipMemcpyAsync(&total, t->scal.ptr, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        CYC_HIP(hipStreamSynchronize(st));
        if (t->fmt == CYC_TILES_AUTO) {
          // the first sub-chunk with nonzeros decides: compact when its
          // fillers are at most 1/32 of its nonzeros
          if ((rc = set_storage(t, (total - cnt) * 32 <= cnt ? CYC_TILES_COMPACT : CYC_TILES_WIDE)))
            return rc;
          t->autoFmt = true;
        }
        if (t->fmt == CYC_TILES_COMPACT && t->autoFmt && t->entries + total > t->capEntries) {
          // AUTO chose compact on denser rows than these: the whole layout
          // goes wide (this sub-chunk below in the wide form)
          if ((rc = demote_to_wide(t, (rb0 + a / kTileRows) * T, st))) return rc;
          entries0 = nnz0;
        }
      }
      if (t->fmt == CYC_TILES_COMPACT) {
        CYC_REQUIRE(t->entries + total <= t->capEntries,
                    "the compact layout's filler entries exceed its allowance (" +
                        std::to_string(t->capEntries - t->capNnz) + "): create it with "
                        "cyc_tiles_set_format(CYC_TILES_WIDE) for rows this sparse");
        pos = (const unsigned long long*)posb.ptr;
        hipLaunchKernelGGL(k_tile_compact, dim3(8192), dim3(256), 0, st,
                           (const uint32_t*)keysOut.ptr, (const uint32_t*)perm.ptr,
                           (const uint32_t*)packed.ptr, vals + (qa - q0), cnt, pos,
                           (uint16_t*)t->idx.ptr + t->entries, (double*)t->vals.ptr + t->entries);
        CYC_LAUNCH_CHECK("k_tile_compact");
      } else {
        total = cnt;
        hipLaunchKernelGGL(k_tile_gather, dim3(8192), dim3(256), 0, st, (const uint32_t*)perm.ptr,
                           cnt, (const uint32_t*)packed.ptr, vals + (qa - q0),
                           (uint32_t*)t->idx.ptr + t->entries, (double*)t->vals.ptr + t->entries);
        CYC_LAUNCH_CHECK("k_tile_gather");
      }
    }
    hipLaunchKernelGGL(k_tile_starts, dim3((unsigned)std::min<int64_t>((cnt + 256) / 256, 8192)),
                       dim3(256), 0, st, (const uint32_t*)keysOut.ptr, cnt, nkeys, seg0,
                       t->entries, pos, total, (int64_t*)t->segStart.ptr);
    CYC_LAUNCH_CHECK("k_tile_starts");
    t->nnz += cnt;
    t->entries += total;
    // scratch is reused by the next sub-chunk on this stream; freed on return
  }
  return CYC_OK;
  }();
  if (arc != CYC_OK) {
    t->nnz = nnz0;
    t->entries = entries0;
    return arc;
  }
  t->n += rows;
  if (t->n % kTileRows != 0) t->sealed = true;
  const int64_t segs = (t->n + kTileRows - 1) / kTileRows * T;
  hipLaunchKernelGGL(k_set_i64, dim3(1), dim3(1), 0, st, (int64_t*)t->segStart.ptr + segs,
                     t->entries);
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
