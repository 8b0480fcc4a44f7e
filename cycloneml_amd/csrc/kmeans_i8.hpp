// kmeans_i8.hpp -- tier 1 of the KMeans assignment (kmeans_i8.hip): an
// exact-integer screen of |x - c|^2 on the gfx950 i8 matrix cores, used when
// a per-fit row image exists (cyc_kmeans_rows) and d <= 512.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cyc {
namespace km8 {

constexpr int kMaxD = 512;    // |T| = |128 S_aa + S_ab| < 2^31 needs d <= 512
constexpr int kBM = 64;       // rows per workgroup
constexpr int kWaves = 4;     // waves per workgroup (centers split across them)

// Per-launch center constants, written on device by centers_prepare().
struct CenterParams {
  int ec;      // global center exponent: every |c_j| <= 2^ec * 127.5/128
  int ok;      // 0: some center is non-finite or beyond 2^50 (screen off)
  double mu;   // AM-GM balance of the separable error bound
  int k;       // centers (the padded tiles hold no center)
};

// 64-dim k-steps of the i8 MFMA, rounded up to even (the kernel's register
// rings alternate per step); the padding limbs are zero.
inline int ksteps(int d) { return ((d + 127) / 128) * 2; }

// d <= 256 screens with the 32x32x32 i8 form (row tiles of 32 in registers,
// 32-center tiles); larger d with the 16x16x64 form (64-row LDS tiles).
inline bool uses32(int d) { return d <= 256; }
// 32-center tiles of the 32x32 screen: even, and covered by the 16-center
// tile padding (a multiple of kWaves = 4 tiles, i.e. of 64 centers).
inline int tiles32(int k) { return 2 * ((k + 63) / 64); }

// Bytes per row of the image: three int8 limb planes of D = 64 ksteps(d).
inline int64_t image_row_bytes(int d) { return 3 * 64 * (int64_t)ksteps(d); }

// X (n x d, row-major fp64) -> img (n rows of image_row_bytes) and meta
// (per row: int exponent or INT32_MIN when the row cannot be screened, and
// the float bits of an upper bound of the 1-norm of the quantized row).
// scale (optional, n entries): image the rows x / scale[row] instead, and
// write their norms to unorm (the cosine plan's unit directions).
int rows_quantize(const double* X, int64_t n, int d, void* img, int2* meta, hipStream_t st,
                  const double* scale = nullptr, double* unorm = nullptr);

// Centers -> packed B fragments (Cb), per-center lower-bound constants cq
// (float, +inf for padding), error terms g (fp64) and the launch's params.
// scratch: >= 2k doubles + 1 int.  ktp: 16-center tiles, a multiple of kWaves.
// cq and g hold 3 ktp 16 entries: the 32x32 screen's two-limb pass keeps its
// constants in the second third, its one-limb pass in the last.
int centers_prepare(const double* C, const double* cnorm, int k, int d, int ktp, void* Cb,
                    float* cq, double* g, CenterParams* prm, double* scratch, hipStream_t st);

// Candidate pass of the d <= 256 screen: the two-limb pass hands each row
// it cannot certify, whose candidate set (the centers the certification
// test cannot exclude) has <= kCandMax members, to k_screen_cands: exact
// fp64 distances (any order, error-bounded) to those candidates, certified
// by a relative gap of `margin` (|x|^2 + |c|^2).  The rows and centers are
// the screened vectors: X / xnorm[row] when unit (the cosine plan), C as
// given (the screen's centers).
constexpr int kCandMax = 6;
// candidate centers per row the one-limb pass hands to the two-limb refinement
constexpr int kCand1 = 8;
struct CandArgs {
  const double* X;        // n x d fp64 rows
  const double* xnorm;    // unit: the row norms X is divided by
  const double* C;        // k x d screened centers
  const double* cnorm;    // their norms
  int k;
  bool unit;
  double margin;
  int32_t* candRows;      // n entries
  int32_t* cands;         // n * kCandMax entries
  unsigned int* candCount;
  // optional: the rows the three-limb candidate tier (k_screen_cands3)
  // leaves to the fp64 pass (n, n * kCandMax entries and their count)
  int32_t* candRows2 = nullptr;
  int32_t* cands2 = nullptr;
  unsigned int* candCount2 = nullptr;
};

// The one-limb pass + two-limb refinement of the d <= 256 screen (k > 96,
// k <= 4096; kmeans_i8.hip k_screen32r): the one-limb pass over every
// center lists each row it cannot certify with <= kCand1 candidates
// (cand1Rows / cand1, n and n kCand1 entries, cand1Count 1 counter); the
// refinement screens 32 listed rows at a time over the union of their
// candidates; rows neither pass can handle go to fullList (n entries,
// fullCount 2 counters: rows; union centers screened) for the full
// two-limb pass.  kstride = 32-center tiles x 32.
struct RefineArgs {
  int kstride;
  int32_t* cand1Rows;
  int32_t* cand1;
  unsigned int* cand1Count;
  int32_t* fullList;
  unsigned int* fullCount;
};

// Sharded appends.  A returning atomicAdd on ONE counter serialises at
// ~11 ns per wave-aggregated add across the chip (tools/atomic_probe.hip:
// 125k waves, one add each, 1.42 ms; 0.03 ms over 64 counters 256 B apart),
// which made every list-producing screen kernel counter-bound.  So the
// screen kernels append into kShards shards (one counter each; a wave's
// 32-row group picks shard group % kShards, so a shard holds at most `cap`
// entries), and compact() then moves the shards behind the list's current
// count in two small launches.  Lists keep no order either way (the atomic
// order was arbitrary too): nothing downstream depends on it.
constexpr int kShards = 64;
constexpr int kShardStride = 64;   // unsigned ints between two shard counters
enum { kSetRowsA = 0, kSetRowsB = 1, kSetCand = 2, kSetStat = 3, kSets = 4 };
struct AppendStage {
  int32_t* rowsA;       // kShards x cap row indices
  int32_t* rowsB;       // kShards x cap
  int32_t* candRows;    // kShards x cap
  int32_t* cands;       // kShards x cap x kCand1
  unsigned int* counts; // kSets x kShards x kShardStride, zero between uses
  unsigned int cap;     // entries per shard
  unsigned int* set(int s) const { return counts + (size_t)s * kShards * kShardStride; }
};
// entries per shard for kernels over at most n rows (32-row groups, or the
// candidate pass's grid-stride 4-row groups of <= 16384 waves)
inline unsigned int shard_cap(int64_t n) {
  return (unsigned int)((n + 32 * kShards - 1) / (32 * kShards) * 32 + 2048);
}
// Append the shards of count set `counts` (width-wide entries of src, and of
// src2 when given) behind *dstCount in dst (dst2); the shard counters are
// left zero.  dst == nullptr: only add the counters' total to *dstCount.
int compact(unsigned int* counts, unsigned int cap, const int32_t* src, int32_t* dst, int width,
            const int32_t* src2, int32_t* dst2, int width2, unsigned int* dstCount,
            hipStream_t st);

// Cross-iteration bounds of one fit (Hamerly's bounds, carried by the row
// image's owner, cyc_kmeans_rows): per row the pair (ub, lb) of f32
// DISTANCES (not squared), ub >= |x - c_a| for the row's assigned center a
// and lb <= |x - c| for every other center, both for the centers of the
// last call (kept in Cp); lb < 0 means "no bound".  The one-limb pass
// writes them for every row it screens (rows it certifies get the bounds its
// integer screen proves, the others lb = -1).  Before the next screen,
// bounds_filter moves the bounds by the centers' drift (triangle inequality:
// ub += |c_a' - c_a|, lb -= max over c != a of |c' - c|) and keeps a row's
// assignment only when lb^2 - ub^2 still exceeds the reference's rounding
// slack 2^-29 (|x|^2 + max |c|^2) -- the same standard as the candidate
// pass's 2^-30 certification: the true distance to c_a is then below every
// other center's by more than fp64 rounding, and the reference's pruned
// loop returns a (the argument of the screens).  The
// other rows are listed for the screen.
struct DriftParams {
  double d1, d2;     // the largest and second largest center drift (upper bounds)
  double cmax2;      // an upper bound of max |c|^2 over the current centers
  int i1;            // the center of d1
  int bad;           // a non-finite drift or center: no row keeps its bounds
};
// Carried candidate sets: a row the three-limb candidate tier certified
// keeps its set (<= kCandMax centers, sets) and the lower bound of every
// center outside it (lnc, a distance, moved by the drift like lb).  When its
// Hamerly bounds fail but lnc still stands, the row is re-checked against
// its set alone (k_screen_cands3<.., RC>) instead of a full screen.
struct Bounds {
  float2* ub_lb;               // n entries
  const int32_t* rowsIn;       // the rows to screen; nullptr: every row
  const unsigned int* rowsInCount;
  float* lnc = nullptr;        // n: the outside bound (< 0 or NaN: no set)
  int32_t* sets = nullptr;     // n x kCandMax
  unsigned char* state = nullptr;   // n: 0 kept, 1 full screen, 2 re-check, 3 re-check
                                    // against the center's neighbourhood (nbr)
  const int32_t* rcRows = nullptr;  // the re-check list (bounds_filter) and its count
  const unsigned int* rcCount = nullptr;
  const DriftParams* dp = nullptr;
  // the centers' neighbourhoods (k x kCandMax, k_center_nbrs) and their
  // outside bounds, for the state-3 re-checks (null: none)
  const int32_t* nbr = nullptr;
  const float* nbrR = nullptr;
  int dump = 0;                     // diagnostics: dump the state after the re-check
  // the filter already listed its state-1 rows in list / listCount (cum
  // counted): the re-check appends its failures there, no bounds_collect
  bool collected = false;
  // bounds_collect's scratch and output (rowsIn / rowsInCount), its count
  // of fully screened rows added to *cum
  int32_t* tmp = nullptr;
  unsigned int* bcount = nullptr;
  int32_t* list = nullptr;
  unsigned int* listCount = nullptr;
  unsigned long long* cum = nullptr;
  int64_t n = 0;
};
// Drift of the centers C against Cp (k x d, then Cp = C): delta (k doubles),
// ccs (k doubles of scratch) and *prm.
int centers_drift(const double* C, double* Cp, int k, int d, double* delta, double* ccs,
                  DriftParams* prm, hipStream_t st);
// The rows whose carried bounds still certify assign[row] keep it (their
// bounds moved by the drift, state 0); of the others, those with a carried
// set whose outside bound still stands go to the re-check list (rcList /
// *rcCount, in row order; state 2), the rest to a full screen (state 1;
// their sets dropped).  *rcCum (64-bit) accumulates the re-checked rows.
// stats (optional, the plan's computeStatistics of these centers): the
// centers' neighbourhoods first (nbr: k x kCandMax, a and its nearest
// others; nbrR: k, a lower bound of |c - c_a| for every c outside), and a
// row left for the screen whose nbrR[a] exceeds twice its moved upper bound
// (or that has none) goes to the re-check list as ~row (state 3): the
// re-check tests the neighbourhood, with |x - c| >= nbrR[a] - |x - c_a| for
// every center outside it, and certified rows keep it as their carried set.
// tmp: n entries; bcount: bounds_blocks(n) + 1 entries.  bounds_collect
// (in screen, after the re-check) lists the state-1 rows for the screen.
constexpr int kBndRows = 2048;   // rows per filter workgroup
inline int64_t bounds_blocks(int64_t n) { return (n + kBndRows - 1) / kBndRows; }
int bounds_filter(const int32_t* assign, float2* ub_lb, float* lnc, unsigned char* state,
                  const double* xnorm, int64_t n, int k, const double* delta,
                  const DriftParams* prm, int32_t* tmp, unsigned int* bcount, int32_t* rcList,
                  unsigned int* rcCount, unsigned long long* rcCum, const double* stats,
                  int32_t* nbr, float* nbrR, hipStream_t st, int32_t* tmp2 = nullptr,
                  unsigned int* bcount2 = nullptr, int32_t* list1 = nullptr,
                  unsigned int* list1Count = nullptr, unsigned long long* cum1 = nullptr);
// tmp2 .. cum1 (optional, with recheck_two_phase()): the filter also lists
// its state-1 rows (tmp2 / bcount2 scratch like tmp / bcount) into list1 /
// *list1Count, their count added to *cum1 -- the screen's list before the
// re-check appends the rows it fails (Bounds::collected).
bool recheck_two_phase();   // CYC_KMEANS_RECHECK != 1

// After the re-check (inside screen): the state-1 rows into bd.list /
// bd.listCount (the screen's rowsIn), their count added to *bd.cum.
int bounds_collect(const Bounds& bd, hipStream_t st);

// Screen every row: certified rows get assign[row]; the others are appended
// to list (listCount is NOT cleared here).  list2 / list2Count (n entries +
// one counter): scratch for the rows the 32x32 two-limb pass leaves.
// ca (d <= 256, optional): the candidate pass.  stg (optional, with ca; cap
// >= shard_cap(n)): the 32x32 kernels append through it.  bd (optional,
// with ra): the one-limb pass screens bd->rowsIn (every row when null) and
// writes the rows' bounds.
int screen(const void* img, const int2* meta, const double* xnorm, int64_t n, int d,
           const void* Cb, const float* cq, const double* g, const double* cnorm,
           const CenterParams* prm, int ktp, int32_t* assign, int32_t* list,
           unsigned int* listCount, int32_t* list2, unsigned int* list2Count, hipStream_t st,
           const CandArgs* ca = nullptr,
           const RefineArgs* ra = nullptr, const AppendStage* stg = nullptr,
           const Bounds* bd = nullptr);

}  // namespace km8
}  // namespace cyc
