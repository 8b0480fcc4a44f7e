// kmeans_i8.hip -- tier 1 of the KMeans assignment (EuclideanDistanceMeasure.
// findClosest, mllib/clustering/DistanceMeasure.scala:282-313) on gfx950: an
// exact-integer screen of the dot products x.c on the i8 matrix cores
// (v_mfma_i32_16x16x64_i8), with a rigorous error bound; fp64 only decides.
//
// Fixed-point split.  A row x (fp64) gets the exponent ex with every
// |x_j| 2^(7-ex) <= 127 and is written as three int8 limbs per element,
//   x_j 2^(7-ex) = a_j + b_j / 2^7 + c_j / 2^14 + r_j / 2^14,  |r_j| <= 1/2,
// a = rint(u), b = rint(128 (u - a)), c = rint(128 (128 (u - a) - b)): every
// step is exact in fp64, |a| <= 127, |b|, |c| <= 64, so |x_j - xh_j| <= 2^(ex-22).
// Centers use ONE exponent ec for the launch.  Then
//   xh.ch = 2^(ex+ec-14) (S1 + S2 / 2^7 + S3 / 2^14 + dropped),
//   S1 = a.a', S2 = a.b' + b.a', S3 = a.c' + b.b' + c.a'   (6 i8 MFMAs / 64 dims)
// accumulated EXACTLY in int32 (d <= 512: |128 S1 + S2| < 2^31), and
//   |x.c - 2^(ex+ec-14)(S1 + S2/2^7 + S3/2^14)|
//      <= Ax |c|_1 + Ac |xh|_1 + 1.004 d 2^22 Ax Ac,   Ax = 2^(ex-22), Ac = 2^(ec-22)
// (quantization of both operands, plus the dropped b.c', c.b', c.c' terms,
// |b|,|c| <= 64).  AM-GM with one balance mu > 0 per launch makes the bound
// separable: <= fx + gc with
//   fx = mu Ax^2 / 2 + |xh|_1^2 / (2 mu) + 0.502 d 2^22 Ax^2,   gc likewise.
// So every distance obeys
//   |x|^2 + |c|^2 - 2 s - 2 (fx + gc) <= |x - c|^2 <= |x|^2 + |c|^2 - 2 s + 2 (fx + gc),
//   2 s = 2^(ex+ec-20) (128 S1 + S2 + S3 / 2^7).
// The kernel keeps, per row, the two smallest of L'_c = cq_c - 2 s (f32,
// MODE rounding toward -inf; cq_c = |c|^2 (1 - epsF) - 2 gc rounded down) and
// the index of the smallest; f32 conversion / fma errors are below
// 2^-21 (|x|^2 + |c|^2) and absorbed by epsF = 2^-20.  A row is certified
// when  L'_2 - L'_1 > 4 (fx + g_1) + 2 epsF (|x|^2 + |c_1|^2) + slack: then
// its best center's upper bound lies below every other center's lower
// bound, the reference's pruned loop (whose prunes only skip centers that
// cannot win) returns the same index, and the row is assigned here.  Every
// other row (ties, near ties, NaN/Inf, |x_j| >= 2^50) is queued for the fp64
// MFMA screen and, behind it, the reference loop itself.
//
// The margin is ~1e-6 relative (vs ~2.5e-4 for a bf16 x3 split with f32
// accumulation), so practically only true near-ties reach the fp64 tiers.
//
// Data flow: the row image (3 D bytes per row, D = 64 ceil(d/64)) is built
// once per fit (rows_quantize; the reference likewise caches the rows with
// their norms once per fit, KMeans.scala:263-270); the center image (3 D
// bytes per center, ~0.75 MB at k=1024, d=256) is rebuilt per iteration and
// stays in each XCD's L2 while every workgroup streams it.
#include "kmeans_i8.hpp"

#include <climits>
#include <type_traits>
#include <cstdlib>

#include "common.hpp"

// tools/probe/screen1_probe.hip builds the one-limb pass with parts removed
// to time them (results then meaningless): bits 2 = no center DMA / waits,
// 4 = no reduction / certification tail, 8 = every wave's rows read from row
// 0 (no HBM stream).  0 in the library.
#ifndef CYC_PROBE_MODE
#define CYC_PROBE_MODE 0
#endif

namespace cyc {
namespace km8 {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

#ifndef CYC_QUANT_COAL
#define CYC_QUANT_COAL 1   // k_rows_quantize: 16 B coalesced row loads
#endif

// one f32 ulp toward -inf; f32 rounded down / up from fp64
__device__ __forceinline__ float ulp_dn(float f) {
  const int b = __float_as_int(f);
  if (f == 0.0f) return -__int_as_float(1);
  return __int_as_float(f > 0.0f ? b - 1 : b + 1);
}
__device__ __forceinline__ float fdown(double x) {
  const float f = (float)x;
  return ((double)f > x) ? ulp_dn(f) : f;
}
__device__ __forceinline__ float fup(double x) {
  const float f = (float)x;
  return ((double)f < x) ? -ulp_dn(-f) : f;
}

constexpr int kMinExp = -50, kMaxExp = 50;
constexpr double kEpsF = 0x1p-20;

__device__ __forceinline__ int choose_exp(double m) {
  if (!(m > 0.0)) return kMinExp;
  int E;
  const double f = __builtin_frexp(m, &E);   // m = f 2^E, f in [0.5, 1)
  const int e = (f * 128.0 >= 127.5) ? E + 1 : E;
  return e < kMinExp ? kMinExp : e;          // a coarser grid is always valid
}

// three limbs of v on the 2^(e-7) grid (exact fp64 steps)
__device__ __forceinline__ void quant3(double v, int e, int& a, int& b, int& c) {
  const double u = __builtin_ldexp(v, 7 - e);
  const double ar = __builtin_rint(u);
  const double t = (u - ar) * 128.0;
  const double br = __builtin_rint(t);
  const double cr = __builtin_rint((t - br) * 128.0);
  a = (int)ar;
  b = (int)br;
  c = (int)cr;
}

__device__ __forceinline__ unsigned pack4(const int* v) {
  return (unsigned)(v[0] & 0xff) | ((unsigned)(v[1] & 0xff) << 8) |
         ((unsigned)(v[2] & 0xff) << 16) | ((unsigned)(v[3] & 0xff) << 24);
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = __builtin_fmax(v, __shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// fx (or gc): separable half of the error bound (see the header comment)
__device__ __forceinline__ double err_term(int e, double n1, double mu, int d) {
  const double A = __builtin_ldexp(1.0, e - 22);
  const double kd = 0.502 * (double)d * 0x1p22;
  return (0.5 * mu * A * A + 0.5 * n1 * n1 / mu + kd * A * A) * (1.0 + 0x1p-40);
}

// The same for 16-byte aligned rows of even d <= 128 H, the next row's loads
// issued before this row's reductions and stores (software-pipelined: two
// rows in flight per wave; the row-at-a-time loop left the stream latency
// bound at ~3.4 TB/s of reads + writes).  Same limbs, exponents and meta.
template <int H>
__global__ __launch_bounds__(256) void k_rows_quantize_pf(const double* __restrict__ X, int64_t n,
                                                          int d, int D, unsigned* __restrict__ img,
                                                          int2* __restrict__ meta,
                                                          const double* __restrict__ scale,
                                                          double* __restrict__ unorm) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  v2d cur[H];
  auto load = [&](int64_t r, v2d (&w)[H]) {
    const double* x = X + (r < n ? r : 0) * d;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int j = h * 128 + 2 * lane;
      w[h] = j < d ? __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x + j)) : v2d{0.0, 0.0};
    }
  };
  if (row < n) load(row, cur);
  for (; row < n; row += nw) {
    v2d nxt[H];
    load(row + nw, nxt);   // in flight while this row is reduced and stored
    double v[2 * H];
    double m = 0.0, s1 = 0.0, s2 = 0.0;
    bool fin = true;
    const double sc = scale ? scale[row] : 1.0;
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        double t = q ? cur[h].y : cur[h].x;
        if (scale) t = t / sc;
        v[2 * h + q] = t;
        fin = fin && __builtin_isfinite(t);
        m = __builtin_fmax(m, __builtin_fabs(t));
        s1 += __builtin_fabs(t);
        s2 += t * t;
      }
    m = wave_max(m);
    s1 = wave_sum(s1);
    if (unorm) {
      s2 = wave_sum(s2);
      if (lane == 0) unorm[row] = __builtin_sqrt(s2);
    }
    const bool allFin = __all(fin);
    const int e = choose_exp(m);
    const bool bad = !allFin || e > kMaxExp;
    unsigned char* db = reinterpret_cast<unsigned char*>(img + row * (int64_t)(3 * D / 4));
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int j0 = h * 128 + 2 * lane;
      if (j0 < D) {
        int a[2], b[2], c[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (bad) a[q] = b[q] = c[q] = 0;
          else quant3(v[2 * h + q], e, a[q], b[q], c[q]);
        }
        *reinterpret_cast<unsigned short*>(db + j0) = (unsigned short)((a[0] & 0xff) | ((a[1] & 0xff) << 8));
        *reinterpret_cast<unsigned short*>(db + D + j0) = (unsigned short)((b[0] & 0xff) | ((b[1] & 0xff) << 8));
        *reinterpret_cast<unsigned short*>(db + 2 * D + j0) = (unsigned short)((c[0] & 0xff) | ((c[1] & 0xff) << 8));
      }
    }
    if (lane == 0) {
      const double n1 = bad ? 0.0 : s1 * (1.0 + 0x1p-40) + (double)d * __builtin_ldexp(1.0, e - 22);
      meta[row] = make_int2(bad ? INT_MIN : e, __float_as_int(fup(n1)));
    }
#pragma unroll
    for (int h = 0; h < H; ++h) cur[h] = nxt[h];
  }
}

// d % 4 == 0, d <= 256, rows 32-byte aligned: each lane quantises 4
// consecutive elements, so every limb plane leaves as one 4-byte store per
// lane (256 B per wave instruction; the 2-byte stores of k_rows_quantize_pf
// wrote half lines), the next row's loads in flight as there.
__global__ __launch_bounds__(256) void k_rows_quantize_q4(const double* __restrict__ X, int64_t n,
                                                          int d, int D, unsigned* __restrict__ img,
                                                          int2* __restrict__ meta,
                                                          const double* __restrict__ scale,
                                                          double* __restrict__ unorm) {
  const int lane = threadIdx.x & 63;
  const int j0 = 4 * lane;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  v2d cur[2];
  auto load = [&](int64_t r, v2d (&w)[2]) {
    const double* x = X + (r < n ? r : 0) * d + j0;
    w[0] = j0 < d ? __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x)) : v2d{0.0, 0.0};
    w[1] = j0 < d ? __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x + 2)) : v2d{0.0, 0.0};
  };
  if (row < n) load(row, cur);
  for (; row < n; row += nw) {
    v2d nxt[2];
    load(row + nw, nxt);   // in flight while this row is reduced and stored
    const double sc = scale ? scale[row] : 1.0;
    double v[4] = {cur[0].x, cur[0].y, cur[1].x, cur[1].y};
    double m = 0.0, s1 = 0.0, s2 = 0.0;
    bool fin = true;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (scale) v[q] = v[q] / sc;
      fin = fin && __builtin_isfinite(v[q]);
      m = __builtin_fmax(m, __builtin_fabs(v[q]));
      s1 += __builtin_fabs(v[q]);
      s2 += v[q] * v[q];
    }
    m = wave_max(m);
    s1 = wave_sum(s1);
    if (unorm) {
      s2 = wave_sum(s2);
      if (lane == 0) unorm[row] = __builtin_sqrt(s2);
    }
    const bool allFin = __all(fin);
    const int e = choose_exp(m);
    const bool bad = !allFin || e > kMaxExp;
    if (j0 < D) {
      int a[4], b[4], c[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (bad) a[q] = b[q] = c[q] = 0;
        else quant3(v[q], e, a[q], b[q], c[q]);
      }
      unsigned char* db = reinterpret_cast<unsigned char*>(img + row * (int64_t)(3 * D / 4));
      *reinterpret_cast<unsigned*>(db + j0) = pack4(a);
      *reinterpret_cast<unsigned*>(db + D + j0) = pack4(b);
      *reinterpret_cast<unsigned*>(db + 2 * D + j0) = pack4(c);
    }
    if (lane == 0) {
      const double n1 = bad ? 0.0 : s1 * (1.0 + 0x1p-40) + (double)d * __builtin_ldexp(1.0, e - 22);
      meta[row] = make_int2(bad ? INT_MIN : e, __float_as_int(fup(n1)));
    }
    cur[0] = nxt[0];
    cur[1] = nxt[1];
  }
}

// One wave per row: limbs into the image, exponent and |xh|_1 bound into meta.
// scale (optional): the row is x / scale[row] (the cosine plan's unit
// directions), whose norm goes to unorm[row] (any summation order: it only
// enters the certification margins, like the fp64 norms do).
__global__ __launch_bounds__(256) void k_rows_quantize(const double* __restrict__ X, int64_t n,
                                                       int d, int D, unsigned* __restrict__ img,
                                                       int2* __restrict__ meta,
                                                       const double* __restrict__ scale,
                                                       double* __restrict__ unorm, int vec) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; row < n; row += nw) {
    const double* x = X + row * d;
    double v[8];
    double m = 0.0, s1 = 0.0, s2 = 0.0;
    bool fin = true;
    const double sc = scale ? scale[row] : 1.0;
#if CYC_QUANT_COAL
    // lane holds elements 128 h + 2 lane + {0, 1}: one 16 B load per lane and
    // 1 KiB contiguous per wave instruction (vec: d even, X 16 B aligned)
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int j = h * 128 + 2 * lane;
      v2d w = {0.0, 0.0};
      if (vec) {
        if (j < d) w = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(x + j));
      } else {
        if (j < d) w.x = x[j];
        if (j + 1 < d) w.y = x[j + 1];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        double t = q ? w.y : w.x;
        if (scale) t = t / sc;
        v[2 * h + q] = t;
        fin = fin && __builtin_isfinite(t);
        m = __builtin_fmax(m, __builtin_fabs(t));
        s1 += __builtin_fabs(t);
        s2 += t * t;
      }
    }
#else
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = p * 256 + 4 * lane + q;
        double t = j < d ? x[j] : 0.0;
        if (scale) t = t / sc;
        v[4 * p + q] = t;
        fin = fin && __builtin_isfinite(t);
        m = __builtin_fmax(m, __builtin_fabs(t));
        s1 += __builtin_fabs(t);
        s2 += t * t;
      }
    }
#endif
    m = wave_max(m);
    s1 = wave_sum(s1);
    if (unorm) {
      s2 = wave_sum(s2);
      if (lane == 0) unorm[row] = __builtin_sqrt(s2);
    }
    const bool allFin = __all(fin);
    const int e = choose_exp(m);
    const bool bad = !allFin || e > kMaxExp;
#if CYC_QUANT_COAL
    unsigned char* db = reinterpret_cast<unsigned char*>(img + row * (int64_t)(3 * D / 4));
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int j0 = h * 128 + 2 * lane;
      if (j0 < D) {
        int a[2], b[2], c[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (bad) {
            a[q] = b[q] = c[q] = 0;
          } else {
            quant3(v[2 * h + q], e, a[q], b[q], c[q]);
          }
        }
        *reinterpret_cast<unsigned short*>(db + j0) = (unsigned short)((a[0] & 0xff) | ((a[1] & 0xff) << 8));
        *reinterpret_cast<unsigned short*>(db + D + j0) = (unsigned short)((b[0] & 0xff) | ((b[1] & 0xff) << 8));
        *reinterpret_cast<unsigned short*>(db + 2 * D + j0) = (unsigned short)((c[0] & 0xff) | ((c[1] & 0xff) << 8));
      }
    }
#else
    unsigned* dst = img + row * (int64_t)(3 * D / 4);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int j0 = p * 256 + 4 * lane;
      if (j0 < D) {
        int a[4], b[4], c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (bad) {
            a[q] = b[q] = c[q] = 0;
          } else {
            quant3(v[4 * p + q], e, a[q], b[q], c[q]);
          }
        }
        dst[j0 / 4] = pack4(a);
        dst[(D + j0) / 4] = pack4(b);
        dst[(2 * D + j0) / 4] = pack4(c);
      }
    }
#endif
    if (lane == 0) {
      // |xh|_1 <= |x|_1 + d 2^(e-22); the fp64 sum is rounded up generously
      const double n1 = bad ? 0.0 : s1 * (1.0 + 0x1p-40) + (double)d * __builtin_ldexp(1.0, e - 22);
      meta[row] = make_int2(bad ? INT_MIN : e, __float_as_int(fup(n1)));
    }
  }
}

// One wave per center: max |c_j|, |c|_1, finiteness.
__global__ __launch_bounds__(256) void k_centers_scan(const double* __restrict__ C, int k, int d,
                                                      double* __restrict__ cmax,
                                                      double* __restrict__ cn1) {
  const int lane = threadIdx.x & 63;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (c >= k) return;
  double m = 0.0, s1 = 0.0;
  bool fin = true;
  for (int j = lane; j < d; j += 64) {
    const double t = C[(int64_t)c * d + j];
    fin = fin && __builtin_isfinite(t);
    m = __builtin_fmax(m, __builtin_fabs(t));
    s1 += __builtin_fabs(t);
  }
  m = wave_max(m);
  s1 = wave_sum(s1);
  const bool allFin = __all(fin);
  if (lane == 0) {
    cmax[c] = allFin ? m : __builtin_inf();
    cn1[c] = s1 * (1.0 + 0x1p-40);
  }
}

// Single block: the launch's exponent, balance and on/off flag.
__global__ __launch_bounds__(256) void k_centers_params(int k, const double* __restrict__ cmax,
                                                        const double* __restrict__ cn1,
                                                        CenterParams* __restrict__ prm) {
  __shared__ double sm[256], sn[256];
  double m = 0.0, nmax = 0.0;
  for (int c = threadIdx.x; c < k; c += 256) {
    m = __builtin_fmax(m, cmax[c]);
    nmax = __builtin_fmax(nmax, cn1[c]);
    if (!(cmax[c] <= 0x1p60)) m = __builtin_inf();   // non-finite center
  }
  sm[threadIdx.x] = m;
  sn[threadIdx.x] = nmax;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      sm[threadIdx.x] = __builtin_fmax(sm[threadIdx.x], sm[threadIdx.x + off]);
      sn[threadIdx.x] = __builtin_fmax(sn[threadIdx.x], sn[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double gm = sm[0];
    const int ec = choose_exp(__builtin_isfinite(gm) ? gm : 0.0);
    CenterParams p;
    p.ok = (__builtin_isfinite(gm) && ec <= kMaxExp) ? 1 : 0;
    p.ec = ec;
    const double Ac = __builtin_ldexp(1.0, ec - 22);
    const double mu = sn[0] / Ac;
    p.mu = (mu > 0.0 && __builtin_isfinite(mu)) ? mu : 1.0;
    p.k = k;
    *prm = p;
  }
}

// Packed B fragments of v_mfma_i32_16x16x64_i8: lane l of 16-center tile ct,
// 64-dim step ks holds center ct*16 + (l & 15), dims ks*64 + 16 (l >> 4) + 0..15
// (the same element order as the rows' A fragments), limb planes a', b', c':
// Cb[((ct KS + ks) 3 + limb) 64 + l].  Plus cq (f32, rounded down) and g.
__global__ __launch_bounds__(256) void k_centers_pack(
    const double* __restrict__ C, const double* __restrict__ cnorm, int k, int d, int KS, int ktp,
    const double* __restrict__ cn1, const CenterParams* __restrict__ prm, uint4* __restrict__ Cb,
    float* __restrict__ cq, double* __restrict__ g) {
  const CenterParams p = *prm;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)ktp * KS * 64;
  if (idx < total) {
    const int lane = (int)(idx & 63);
    const int64_t t = idx >> 6;
    const int ks = (int)(t % KS), ct = (int)(t / KS);
    const int c = ct * 16 + (lane & 15), j0 = ks * 64 + 16 * (lane >> 4);
    int a[16], b[16], cc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int j = j0 + e;
      const double v = (p.ok && c < k && j < d) ? C[(int64_t)c * d + j] : 0.0;
      quant3(v, p.ec, a[e], b[e], cc[e]);
    }
    uint4 pa, pb, pc;
    pa.x = pack4(a); pa.y = pack4(a + 4); pa.z = pack4(a + 8); pa.w = pack4(a + 12);
    pb.x = pack4(b); pb.y = pack4(b + 4); pb.z = pack4(b + 8); pb.w = pack4(b + 12);
    pc.x = pack4(cc); pc.y = pack4(cc + 4); pc.z = pack4(cc + 8); pc.w = pack4(cc + 12);
    uint4* dst = Cb + (t * 3) * 64 + lane;
    dst[0] = pa;
    dst[64] = pb;
    dst[128] = pc;
  }
  if (idx < (int64_t)ktp * 16) {
    const int c = (int)idx;
    if (c < k && p.ok) {
      const double gc = err_term(p.ec, cn1[c], p.mu, d);
      const double cn = cnorm[c];
      g[c] = gc;
      cq[c] = fdown((cn * cn) * (1.0 - kEpsF) - 2.0 * gc);
    } else {
      g[c] = 0.0;
      cq[c] = __builtin_inff();
    }
  }
}

__device__ __forceinline__ v4i as_v4i(uint4 u) { return __builtin_bit_cast(v4i, u); }

// BM = 64 rows per workgroup (4 row tiles), 4 waves; wave w owns the 16-center
// tiles w, w+4, w+8, ...  The row image lives in LDS with a row stride of
// 12 KS + 2 16-byte chunks (== 2 mod 4: conflict-free ds_read_b128 fragment
// reads); B fragments come from L2 one 64-dim step ahead.
template <int KS>
__global__ __launch_bounds__(256, KS <= 4 ? 3 : 2) void k_screen(
    const uint4* __restrict__ Xq, const int2* __restrict__ meta, const double* __restrict__ xnorm,
    int64_t n, int d, const uint4* __restrict__ Cb, const float* __restrict__ cq,
    const double* __restrict__ g, const double* __restrict__ cnorm,
    const CenterParams* __restrict__ prm, int ktp, int32_t* __restrict__ assign,
    int32_t* __restrict__ list, unsigned int* __restrict__ listCount) {
  constexpr int BM = kBM, W = kWaves, CH = 12 * KS, STR = CH + 2;
  extern __shared__ __attribute__((aligned(16))) uint4 smem8[];
  uint4* As = smem8;                          // BM x STR chunks
  int* exS = (int*)(As + BM * STR);           // BM
  // after the main loop the row image is dead: the per-wave slot minima
  // reuse it (3 KB), so d <= 256 fits three workgroups per CU
  float* mL1 = (float*)As;                    // W x BM
  float* mL2 = mL1 + W * BM;                  // W x BM
  int* mI1 = (int*)(mL2 + W * BM);            // W x BM

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * BM;
  const int rows = (int)min<int64_t>(BM, n - row0);
  const CenterParams P = *prm;
  if (!P.ok) {
    if (tid < rows) list[atomicAdd(listCount, 1u)] = (int32_t)(row0 + tid);
    return;
  }
  {
    // every load in flight before the first LDS write (3 KS chunks per thread)
    constexpr int PER = BM * CH / 256;
    const uint4* src = Xq + row0 * CH;
    const int lim = rows * CH;
    v4u st[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i)
      st[i] = __builtin_nontemporal_load((const v4u*)(src + min(tid + 256 * i, lim - 1)));
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + 256 * i, r = e / CH, ch = e - r * CH;
      As[r * STR + ch] = e < lim ? make_uint4(st[i].x, st[i].y, st[i].z, st[i].w)
                                 : make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < BM) exS[tid] = tid < rows ? meta[row0 + tid].x : INT_MIN;
  }
  __syncthreads();

  // Per row slot q = 4 ta + r (row ta*16 + 4 (lane >> 4) + r): 2^(ex+ec-20).
  float F1[16];
#pragma unroll
  for (int ta = 0; ta < 4; ++ta) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ex = exS[ta * 16 + 4 * (lane >> 4) + r];
      F1[4 * ta + r] = ex == INT_MIN ? 0.0f : __builtin_ldexpf(1.0f, ex + P.ec - 20);
    }
  }
  float sL1[16], sL2[16];
  int sI1[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    sL1[q] = sL2[q] = __builtin_inff();
    sI1[q] = -1;
  }
  const uint4* ap = As + (lane & 15) * STR + (lane >> 4);
  const int nT = ktp / W;
  const uint4* cb = Cb + (size_t)wave * KS * 192 + lane;
  const size_t tstride = (size_t)W * KS * 192;
  // Register rings, all indices static after unrolling: B fragments one
  // 64-dim step ahead (KS is even, so a tile always starts on B0), A
  // fragments one (step, row tile) ahead (4 per step, so always on A0).
  v4i B0[3], B1[3], A0[3], A1[3];
#define CYC_LDB(DST, P)                                  \
  do {                                                   \
    DST[0] = as_v4i((P)[0]);                             \
    DST[1] = as_v4i((P)[64]);                            \
    DST[2] = as_v4i((P)[128]);                           \
  } while (0)
#define CYC_LDA(DST, KS_, TA_)                           \
  do {                                                   \
    const uint4* a_ = ap + (TA_) * 16 * STR + (KS_) * 4; \
    DST[0] = as_v4i(a_[0]);                              \
    DST[1] = as_v4i(a_[4 * KS]);                         \
    DST[2] = as_v4i(a_[8 * KS]);                         \
  } while (0)
#define CYC_MM(ACC, A, B)                                                    \
  do {                                                                       \
    ACC[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[0], ACC[0], 0, 0, 0); \
    ACC[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[1], ACC[1], 0, 0, 0); \
    ACC[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[0], ACC[1], 0, 0, 0); \
    ACC[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[2], ACC[2], 0, 0, 0); \
    ACC[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[1], ACC[2], 0, 0, 0); \
    ACC[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2], B[0], ACC[2], 0, 0, 0); \
  } while (0)
  // one (step, row tile): prefetch the next A, then 6 MFMAs
#define CYC_TA(KS_, TA_, AC, AN, BC)                                          \
  do {                                                                        \
    if ((TA_) < 3) CYC_LDA(AN, KS_, (TA_) + 1);                               \
    else CYC_LDA(AN, ((KS_) + 1 < KS ? (KS_) + 1 : 0), 0);                    \
    CYC_MM(acc[TA_], AC, BC);                                                 \
    __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);                        \
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);                        \
  } while (0)
#define CYC_KSTEP(KS_, BC, BN)                                                \
  do {                                                                        \
    CYC_LDB(BN, ((KS_) + 1 < KS ? cb + ((KS_) + 1) * 192 : cbn));             \
    __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);                        \
    CYC_TA(KS_, 0, A0, A1, BC);                                               \
    CYC_TA(KS_, 1, A1, A0, BC);                                               \
    CYC_TA(KS_, 2, A0, A1, BC);                                               \
    CYC_TA(KS_, 3, A1, A0, BC);                                               \
  } while (0)
  CYC_LDB(B0, cb);
  CYC_LDA(A0, 0, 0);

  // MODE.FP_ROUND single precision = toward -inf (the L' are lower bounds)
  __builtin_amdgcn_s_setreg(0x801, 2);
  for (int t = 0; t < nT; ++t) {
    const float cqv = cq[(t * W + wave) * 16 + (lane & 15)];
    // next tile's B (the last tile re-reads its own: harmless, branch free)
    const uint4* cbn = cb + (t + 1 < nT ? tstride : 0);
    v4i acc[4][3];
#pragma unroll
    for (int ta = 0; ta < 4; ++ta)
#pragma unroll
      for (int s = 0; s < 3; ++s) acc[ta][s] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int kp = 0; kp < KS; kp += 2) {
      CYC_KSTEP(kp, B0, B1);
      CYC_KSTEP(kp + 1, B1, B0);
    }
#undef CYC_KSTEP
#undef CYC_TA
#undef CYC_MM
#undef CYC_LDA
#undef CYC_LDB
    cb = cbn;
    const int c = (t * W + wave) * 16 + (lane & 15);
#pragma unroll
    for (int ta = 0; ta < 4; ++ta) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = 4 * ta + r;
        const int T = acc[ta][0][r] * 128 + acc[ta][1][r];
        const float V = __builtin_fmaf((float)acc[ta][2][r], 0x1p-7f, (float)T);
        const float L = __builtin_fmaf(-F1[q], V, cqv);
        // two smallest with sL1 <= sL2: the median of (sL1, sL2, L) is the
        // new second smallest
        const bool lt = L < sL1[q];
        sL2[q] = __builtin_amdgcn_fmed3f(sL1[q], sL2[q], L);
        sI1[q] = lt ? c : sI1[q];
        sL1[q] = __builtin_fminf(sL1[q], L);
      }
    }
  }
  __builtin_amdgcn_s_setreg(0x801, 0);

  // Reduce each slot over the 16 lanes (centers) that hold the same row.
#pragma unroll
  for (int q = 0; q < 16; ++q) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      const float oL1 = __shfl_xor(sL1[q], m), oL2 = __shfl_xor(sL2[q], m);
      const int oI1 = __shfl_xor(sI1[q], m);
      sL2[q] = __builtin_fminf(__builtin_fmaxf(sL1[q], oL1), __builtin_fminf(sL2[q], oL2));
      const bool take = oL1 < sL1[q] || (oL1 == sL1[q] && oI1 >= 0 && (sI1[q] < 0 || oI1 < sI1[q]));
      sI1[q] = take ? oI1 : sI1[q];
      sL1[q] = take ? oL1 : sL1[q];
    }
  }
  __syncthreads();   // every wave is done reading the row image (mL1.. alias it)
  if ((lane & 15) == 0) {
#pragma unroll
    for (int ta = 0; ta < 4; ++ta) {
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
  if (tid < rows) {
    const int row = tid;
    const int ex = exS[row];
    float L1 = __builtin_inff(), L2 = __builtin_inff();
    int I1 = -1;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const float oL1 = mL1[w * BM + row], oL2 = mL2[w * BM + row];
      const int oI1 = mI1[w * BM + row];
      L2 = __builtin_fminf(__builtin_fmaxf(L1, oL1), __builtin_fminf(L2, oL2));
      if (oL1 < L1 || (oL1 == L1 && oI1 >= 0 && (I1 < 0 || oI1 < I1))) {
        L1 = oL1;
        I1 = oI1;
      }
    }
    bool decided = false;
    if (ex != INT_MIN && I1 >= 0 && __builtin_isfinite(L1)) {
      const double xn = xnorm[row0 + row], cn = cnorm[I1];
      const double xx = xn * xn, cc = cn * cn;
      const double n1 = (double)__int_as_float(meta[row0 + row].y);
      const double fx = err_term(ex, n1, P.mu, d);
      const double l1 = (double)L1;
      const double M = (4.0 * (fx + g[I1]) + 2.0 * kEpsF * (xx + cc) +
                        0x1p-20 * (__builtin_fabs(l1) + cc + 2.0 * g[I1]) +
                        0x1p-24 * (2.0 * (xx + cc) + __builtin_fabs(l1) +
                                   __builtin_fmin(__builtin_fabs((double)L2), 0x1p120)) +
                        0x1p-90) *
                       (1.0 + 0x1p-30);
      // exact difference of two floats; L2 = +inf: no other real center
      decided = !__builtin_isfinite(L2) || ((double)L2 - l1) > M;
    }
    if (decided) {
      assign[row0 + row] = I1;
    } else {
      list[atomicAdd(listCount, 1u)] = (int32_t)(row0 + row);
    }
  }
}

// ---------------------------------------------------------------------------
// 32x32 form (d <= 256): v_mfma_i32_32x32x32_i8 holds the SIMD's issue for 8
// of its 32 cycles (the 16x16x64 form: 8 of 16), leaving room for the top-2
// epilogue (9 VALU per (row, center): ~3 per MFMA).
//
// One wave = 32 rows, held in REGISTERS in the MFMA A layout (lane l: row
// l & 31, dims 32 s + 16 (l >> 5) + 0..15 of substep s, three limbs: 96
// VGPRs at d = 256).  A workgroup of 4 waves (128 rows) sweeps every
// 32-center tile; each tile's B fragments (24 KiB at d = 256) are DMA'd
// into a ring of three LDS slots (global_load_lds, 1 KiB per wave-
// instruction, split over the waves, counted vmcnt + raw s_barrier so the
// next tile stays in flight) and read by conflict-free ds_read_b128.
// 252 VGPRs: two waves per SIMD (two workgroups per CU, 2 x 74.5 KB LDS).
// Measured at 10M x 256, k = 1024 (profiles/r02_kmeans_*): 14.4 ms per
// launch vs 14.0-15.4 for the 16x16x64 screen; PMC: 32 MFMA-busy cycles per
// MFMA, 53 % of the SIMD cycles at the 1.89 GHz the chip holds under this
// load.  Tried and slower: B fragments per wave straight from L2 (18.1 ms),
// one wave per SIMD with two accumulator sets so the epilogue of tile t
// interleaves tile t+1's MFMAs (18.1 ms), 8-wave workgroups (one tile load
// per 256 rows: 14.8-15.0 ms).
//
// B fragments: lane l of 32-center tile ct, 32-dim substep s holds center
// 32 ct + (l & 31), dims 32 s + 16 (l >> 5) + 0..15, limb planes a', b', c':
// Cb[((ct S + s) 3 + limb) 64 + l]; the tile count is even (padding centers
// are zero with cq = +inf).

__device__ __forceinline__ double err_term2(int e, double n1, double mu, int d);
__device__ __forceinline__ double err_term1(int e, double n1, double mu);
__global__ __launch_bounds__(256) void k_centers_pack32(
    const double* __restrict__ C, const double* __restrict__ cnorm, int k, int d, int S, int ktp,
    const double* __restrict__ cn1, const CenterParams* __restrict__ prm, uint4* __restrict__ Cb,
    float* __restrict__ cq, double* __restrict__ g, float* __restrict__ cq2,
    double* __restrict__ g2, float* __restrict__ cq1, double* __restrict__ g1) {
  const CenterParams p = *prm;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)ktp * S * 64;
  if (idx < total) {
    const int lane = (int)(idx & 63);
    const int64_t t = idx >> 6;
    const int s = (int)(t % S), ct = (int)(t / S);
    const int c = ct * 32 + (lane & 31), j0 = s * 32 + 16 * (lane >> 5);
    int a[16], b[16], cc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int j = j0 + e;
      const double v = (p.ok && c < k && j < d) ? C[(int64_t)c * d + j] : 0.0;
      quant3(v, p.ec, a[e], b[e], cc[e]);
    }
    uint4 pa, pb, pc;
    pa.x = pack4(a); pa.y = pack4(a + 4); pa.z = pack4(a + 8); pa.w = pack4(a + 12);
    pb.x = pack4(b); pb.y = pack4(b + 4); pb.z = pack4(b + 8); pb.w = pack4(b + 12);
    pc.x = pack4(cc); pc.y = pack4(cc + 4); pc.z = pack4(cc + 8); pc.w = pack4(cc + 12);
    uint4* dst = Cb + (t * 3) * 64 + lane;
    dst[0] = pa;
    dst[64] = pb;
    dst[128] = pc;
    // the center-major copy behind the fragments (k_screen32r's per-lane
    // gathers): center c's limb planes a', b', c' of D = 32 S bytes each,
    // dimensions in order, 6 S 16-byte pieces per center
    uint4* cr = Cb + (int64_t)ktp * S * 3 * 64 + (int64_t)c * (6 * S) + 2 * s + (lane >> 5);
    cr[0] = pa;
    cr[2 * S] = pb;
    cr[4 * S] = pc;
  }
  if (idx < (int64_t)ktp * 32) {
    const int c = (int)idx;
    if (c < k && p.ok) {
      const double gc = err_term(p.ec, cn1[c], p.mu, d);
      const double gc2 = err_term2(p.ec, cn1[c], p.mu * 0x1p-7, d);
      const double gc1 = err_term1(p.ec, cn1[c], p.mu * 0x1p-14);
      const double cn = cnorm[c];
      g[c] = gc;
      cq[c] = fdown((cn * cn) * (1.0 - kEpsF) - 2.0 * gc);
      g2[c] = gc2;
      cq2[c] = fdown((cn * cn) * (1.0 - kEpsF) - 2.0 * gc2);
      g1[c] = gc1;
      cq1[c] = fdown((cn * cn) * (1.0 - kEpsF) - 2.0 * gc1);
    } else {
      g[c] = g2[c] = g1[c] = 0.0;
      cq[c] = __builtin_inff();
      // finite: the integer passes keep index bits in L
      cq2[c] = cq1[c] = 0x1.fffffep127f;
    }
  }
}

typedef int v16i __attribute__((ext_vector_type(16)));

// fx / gc of the TWO-limb screen: |x_j - xh2_j| <= 2^(e-15) (u - a - b/128
// = (t - b)/128 with |t - b| <= 1/2), the dropped b.b' / 2^14 term <=
// d 2^(ex+ec-16) = d 2^14 A2x A2c <= 0.5 d 2^14 (A2x^2 + A2c^2) (AM-GM);
// A2 carries a 2^-7 slack.  n1 must bound |xh2|_1 (rows) or |c|_1 (centers).
// fx / gc of the ONE-limb screen: |x_j - xh1_j| <= 2^(e-8) (a = rint(u)),
// no dropped products (S1 = a.a' exactly): |x.c - xh1.ch1| <= A1x |c|_1 +
// A1c |xh1|_1, split by AM-GM as for the other limb counts; A1 carries a
// 2^-7 slack.  n1 must bound |xh1|_1 (rows) or |c|_1 (centers).
__device__ __forceinline__ double err_term1(int e, double n1, double mu) {
  const double A = __builtin_ldexp(1.0078125, e - 8);
  return (0.5 * mu * A * A + 0.5 * n1 * n1 / mu) * (1.0 + 0x1p-40);
}

__device__ __forceinline__ double err_term2(int e, double n1, double mu, int d) {
  const double A = __builtin_ldexp(1.0078125, e - 15);
  const double kd = 0.502 * (double)d * 0x1p14;
  return (0.5 * mu * A * A + 0.5 * n1 * n1 / mu + kd * A * A) * (1.0 + 0x1p-40);
}

// Carried bounds (kmeans_i8.hpp Bounds) from a screen's computed bounds.
// With Lt_c = |c|^2 - 2 x.c and L'_c = cq_c - 2 s_c its exact integer form
// (cq_c <= |c|^2 - 2 g_c, |x.c - s_c| <= fx + g_c): Lt_c >= L'_c - 2 fx, and
// a computed bound l is within enc of L' (the integer passes' index bits and
// floors; 0 for the three-limb f32 bounds, whose rounding the 2^-20 slack
// covers together with xx = xnorm^2, within 2^-44 xx of the true |x|^2).
// Every center whose computed bound is >= l therefore has
//   |x - c|^2 >= xx + l - enc - 2 fx                       (bnd_lb_sq)
// and the winner, bound l1, |x - c_w|^2 <= xx + l1 + enc + 2 fx + 4 g_w
// + eps |c_w|^2 (cq rounded down; the 2^-20 terms as in the margins M).
// `extra`: a further slack (the f32 three-limb bounds: 2^-20 max cq).
__device__ __forceinline__ double bnd_ub_sq(double xx, double cc, double l1, double fx, double gw,
                                            double enc) {
  return (xx + l1 + enc + 2.0 * fx + 4.0 * gw + 2.0 * kEpsF * (xx + cc) +
          0x1p-20 * (xx + __builtin_fabs(l1) + cc + 2.0 * gw) + 0x1p-90) *
         (1.0 + 0x1p-30);
}
__device__ __forceinline__ double bnd_lb_sq(double xx, double l, double fx, double enc,
                                            double extra) {
  return xx + l - enc - 2.0 * fx - 2.0 * kEpsF * xx -
         0x1p-20 * (xx + __builtin_fabs(l) + 2.0 * fx + enc) - extra;
}
// as f32 distances: up rounded up; a lower bound <= 0 (or NaN) is "none" (-1)
__device__ __forceinline__ float bnd_dist_up(double s2) {
  return fup(__builtin_sqrt(s2) * (1.0 + 0x1p-50));
}
__device__ __forceinline__ float bnd_dist_dn(double s2) {
  return s2 > 0.0 ? fdown(__builtin_sqrt(s2) * (1.0 - 0x1p-50)) : -1.0f;
}
// the largest of each row's per-lane values over its 32 lanes (the screens'
// register layout: lane (r, h) holds row (reg & 3) + 8 (reg >> 2) + 4 h of
// register reg): halving shuffles, then per row into out[32] (LDS)
__device__ __forceinline__ void rows_max32(int (&v)[16], int lane, int* out) {
#pragma unroll
  for (int lev = 0; lev < 4; ++lev) {
    const int half = 8 >> lev, m = 16 >> lev;
    const bool hi = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const int o = __shfl_xor(hi ? v[i] : v[i + half], m);
      v[i] = max(hi ? v[i + half] : v[i], o);
    }
  }
  v[0] = max(v[0], __shfl_xor(v[0], 1));
  if ((lane & 1) == 0) {
    const int q = (lane >> 1) & 15;
    out[(q & 3) + 8 * (q >> 2) + 4 * (lane >> 5)] = v[0];
  }
}

// One screen pass over 32-row groups.  LIMBS = 3: the exact-integer screen
// (S1, S2, S3: six MFMAs per 32-dim substep).  LIMBS = 2: the same over the
// a and b limbs only (S1, S2: three MFMAs), certified with err_term2 --
// config 2's rows certify 90 % of the time at this precision vs 99.9 % at
// three limbs, so the two-limb pass runs over every row and the three-limb
// pass only over its leftovers (LIST: rows taken from `rowsIn`, a device
// list of *rowsInCount row indices).  Both read the
// same center image (3 limb fragments per substep; LIMBS = 2 DMAs the first
// two) and write assign[] for certified rows, the rest to list.
// Two workgroups per CU; three for the two-limb pass (<= 168 VGPRs, LDS
// 3 x 49 KB at S = 8), measured 7 % faster than two.
// the one-limb pass screens a row whose exponent exceeds its wave's smallest
// by at most this much (larger shifts could overflow its 32-bit bounds)
constexpr int kShMax = 2;

template <int S, int W, int LIMBS, bool LIST>
__global__ __launch_bounds__(64 * W, W == 8 ? 2 : (LIMBS < 3 ? 12 : 8) / W) void k_screen32(
    const uint4* __restrict__ Xq, const int2* __restrict__ meta, const double* __restrict__ xnorm,
    int64_t n, int d, const uint4* __restrict__ Cb, const float* __restrict__ cq,
    const double* __restrict__ g, const double* __restrict__ cnorm,
    const CenterParams* __restrict__ prm, int ktp, const int32_t* __restrict__ rowsIn,
    const unsigned int* __restrict__ rowsInCount, int32_t* __restrict__ assign,
    int32_t* __restrict__ list, unsigned int* __restrict__ listCount,
    int32_t* __restrict__ candRows, int32_t* __restrict__ cands,
    unsigned int* __restrict__ candCount, unsigned int scap, float2* __restrict__ bnd) {
  constexpr int D = 32 * S, CH = 3 * D / 16;      // 16-byte chunks per image row
  // LIMBS = 1 takes two 32-center tiles per step (one barrier and one ring
  // slot per 64 centers: its tiles carry a third of the MFMAs)
  constexpr bool PAIR = LIMBS == 1;
  constexpr int FR = PAIR ? 2 * S : LIMBS * S;     // 1 KiB B fragments per ring step
  constexpr int TB = FR * 1024 + 256;              // tile slot: fragments, then 64 cq floats
  constexpr int G = FR / W;                        // fragment DMAs per wave per tile (+1: wave 0's cq)
  static_assert(FR % W == 0, "fragments split evenly over the waves");
  // ONE shared array (a second __shared__ object can make hipcc drain vmcnt
  // before every ds_read): three tile slots, reused for the final reduction.
  __shared__ __attribute__((aligned(16))) char lds[3 * TB];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const CenterParams P = *prm;
  // any mu > 0 is valid; scaled with each limb count's quantum
  const double mu = LIMBS == 3 ? P.mu : LIMBS == 2 ? P.mu * 0x1p-7 : P.mu * 0x1p-14;
  // integer bounds (LIMBS < 3) in units F1 = 2^(ex + ec - SH): 2 s = F1 T
  constexpr int SH = LIMBS == 1 ? 13 : 20;
  // candidate sets per row: the two-limb pass's for the fp64 candidate pass
  // (kCandMax), the one-limb pass's for the two-limb refinement (kCand1)
  constexpr int CMAX = LIMBS == 1 ? kCand1 : kCandMax;
  const int64_t total = LIST ? (int64_t)*rowsInCount : n;
  // one group of 32 W rows (positions)
  auto group = [&](int64_t grp) {
  const int64_t pos0 = (grp * W + wave) * 32;        // first position of this wave
  // waves past the end still take part in every barrier (zero rows)
  const int rows = (int)max<int64_t>(0, min<int64_t>(32, total - pos0));
  // scap > 0: list / cand appends go to this group's shard (kmeans_i8.hpp)
  const unsigned shard = (unsigned)((grp * W + wave) % kShards);
  int32_t* const listS = scap ? list + (size_t)shard * scap : list;
  unsigned int* const listCountS = scap ? listCount + shard * kShardStride : listCount;
  int32_t* const candRowsS = scap && candRows ? candRows + (size_t)shard * scap : candRows;
  int32_t* const candsS = scap && cands ? cands + (size_t)shard * scap * CMAX : cands;
  unsigned int* const candCountS =
      scap && candCount ? candCount + shard * kShardStride : candCount;
  auto rowAt = [&](int i) -> int64_t {   // global row of position pos0 + i (i < rows)
    if constexpr (LIST) return rowsIn[pos0 + i];
    else return pos0 + i;
  };
  if (!P.ok) {   // uniform over the grid
    if (lane < rows) {
      listS[atomicAdd(listCountS, 1u)] = (int32_t)rowAt(lane);
      if (LIMBS == 1 && bnd) bnd[rowAt(lane)] = make_float2(-1.0f, -1.0f);
    }
    return;
  }
  // tile t -> slot t % 3: each wave DMAs fragments wave, wave + W, ... and the
  // tile's cq (all waves write the same 256 bytes); past the last tile the
  // last one is re-read into the free slot, so every wave always has exactly
  // G DMAs per tile in flight and one counted wait fits all tiles.
  const int nsteps = PAIR ? ktp / 2 : ktp;          // ktp is even
  auto issue = [&](int t, int slot) {
    if constexpr (PAIR && (CYC_PROBE_MODE & 2)) return;
    const int tt = t < nsteps ? t : nsteps - 1;
    char* dst = lds + slot * TB;
#pragma unroll
    for (int j = 0; j < FR / W; ++j) {
      const int f = wave + W * j;
      // PAIR: fragment f = limb a of substep f % S of tile 2 tt + f / S;
      // else substep f / LIMBS, limb f % LIMBS of tile tt
      const int tile = PAIR ? 2 * tt + f / S : tt;
      const int piece = PAIR ? (f % S) * 3 : (f / LIMBS) * 3 + f % LIMBS;
      const char* src = (const char*)Cb + (size_t)tile * (3 * S) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)(src + piece * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + f * 1024),
                                       16, 0, 0);
    }
    if (wave == 0)   // the step's cq: 32 (lanes 32..63 repeat them) or PAIR's 64
      __builtin_amdgcn_global_load_lds(
          (const void*)(cq + (PAIR ? (size_t)tt * 64 + lane : (size_t)tt * 32 + r)),
          (__attribute__((address_space(3))) void*)(dst + FR * 1024), 4, 0, 0);
  };
  issue(0, 0);
  issue(1, 1);
  // A fragments of the wave's 32 rows, all substeps and limbs
  v4i A[S][LIMBS];
  const bool rowOk = r < rows;
  const int64_t myRow = rowOk ? rowAt(r) : 0;   // lane's row (row 0 exists: n > 0)
  {
    // loads from a valid row, zeroed after the load; the one-limb pass
    // with plain loads (3.40 -> 3.30 ms measured against nontemporal ones)
    const bool ok = rowOk;
    const uint4* src = Xq + ((PAIR && (CYC_PROBE_MODE & 8)) ? 0 : myRow) * CH + h;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int L = 0; L < LIMBS; ++L) {
        const v4u* a = (const v4u*)(src + L * (D / 16) + 2 * s);
        const v4u t = PAIR ? *a : __builtin_nontemporal_load(a);
        A[s][L] = ok ? __builtin_bit_cast(v4i, t) : v4i{0, 0, 0, 0};
      }
  }
  // row of accumulator register reg: (reg & 3) + 8 (reg >> 2) + 4 h
  const int exr = rowOk ? meta[myRow].x : INT_MIN;
  // LIMBS = 3: per-row unit F1 = 2^(ex + ec - 20) of T in f32 bounds.
  // LIMBS = 2: integer bounds in the same units: L / F1 = Q - T with
  // Q = cq / F1 rounded, from one per-lane base per tile at the wave's
  // smallest exponent exmin, shifted right by sh = ex - exmin per row.
  float F1[16];
  int sh[16];
  int exmin = 0;
  if constexpr (LIMBS == 3) {
    const float f = exr == INT_MIN ? 0.0f : __builtin_ldexpf(1.0f, exr + P.ec - 20);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) F1[reg] = __shfl(f, (reg & 3) + 8 * (reg >> 2) + 4 * h);
  } else {
    int e = exr == INT_MIN ? INT_MAX : exr;
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) e = min(e, __shfl_xor(e, m));
    exmin = __builtin_amdgcn_readfirstlane(e == INT_MAX ? 0 : e);
    const int s0 = exr == INT_MIN ? 31 : min(exr - exmin, 31);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) sh[reg] = __shfl(s0, (reg & 3) + 8 * (reg >> 2) + 4 * h);
  }
  // cq scaled to the units 2^(exmin + ec - SH)
  const float qscale = __builtin_ldexpf(1.0f, max(-160, min(160, SH - P.ec - exmin)));
  // |Q| clamp in those units: LIMBS = 1 keeps (Q << IB) in 31 bits
  constexpr float QCLAMP = LIMBS == 1 ? 0x1p25f : 0x1p30f;
  bool qbad = false;   // a cq below -QCLAMP units: the wave certifies nothing
  // LIMBS = 3: the two smallest f32 bounds; LIMBS = 2: the two largest
  // V = T - Q (the smallest L = -F1 V), tile index in the low IB bits
  float sL1[16], sL2[16];
  int sV1[16], sV2[16];
  int sI1[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    sL1[q] = sL2[q] = __builtin_inff();
    sV1[q] = sV2[q] = INT_MIN;
    sI1[q] = -1;
  }
  // tile ct from its slot: LIMBS = 3: six limb products per substep,
  // LIMBS = 2: three; B fragments by conflict-free ds_read_b128
  auto tile = [&](int slot, v16i (&acc)[LIMBS]) {   // acc: initialised by the caller
    const v4i* B = (const v4i*)(lds + slot * TB) + lane;
    // (reading the B fragments a substep ahead measured no faster)
#pragma unroll
    for (int s = 0; s < S; ++s) {
      v4i Bc[LIMBS];
#pragma unroll
      for (int L = 0; L < LIMBS; ++L) Bc[L] = B[(LIMBS * s + L) * 64];
      const v4i B0 = Bc[0], B1 = Bc[LIMBS >= 2 ? 1 : 0];
      // (separating the two acc[1] products by sched_barrier measured 3 % slower)
      acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], B0, acc[0], 0, 0, 0);
      if constexpr (LIMBS >= 2) {
        acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], B1, acc[1], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][1], B0, acc[1], 0, 0, 0);
      }
      if constexpr (LIMBS == 3) {
        const v4i B2 = Bc[2];
        acc[2] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], B2, acc[2], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][1], B1, acc[2], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][2], B0, acc[2], 0, 0, 0);
      }
    }
  };
  // LIMBS = 2 keeps the tile index in the low IB bits of V (moving it by
  // < 2^IB units either way, charged in the certification): a max and a med3
  // per (row, center) instead of a compare, a med3 and two selects.
  const int IB = 32 - __builtin_clz((unsigned)max(ktp - 1, 1));
  const unsigned IM = (1u << IB) - 1u;
  // LIMBS = 2, after the tile's MFMAs: acc[1] started at -Q
  int vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  auto epi2 = [&](int ct, const v16i (&acc)[LIMBS]) {
    // ct in a VGPR (one v_and_or_b32 may read only one SGPR, the mask), by
    // a VALU add to an opaque zero: no inline asm in the loop, which would
    // split its scheduling region
    const unsigned ctv = (unsigned)(vzero + ct);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      // T - Q (LIMBS = 1: acc[0] started at -Q)
      const int V = LIMBS == 1 ? acc[0][reg] : acc[0][reg] * 128 + acc[LIMBS - 1][reg];
      const int Ve = (int)(((unsigned)V & ~IM) | ctv);                  // ct < 2^IB
      sV2[reg] = max(min(sV1[reg], sV2[reg]), min(max(sV1[reg], sV2[reg]), Ve));   // v_med3_i32
      sV1[reg] = max(sV1[reg], Ve);
    }
  };
  auto epi = [&](int ct, float cqv, const v16i (&acc)[LIMBS]) {
    const int c = ct * 32 + r;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      if constexpr (LIMBS == 3) {
        const int T = acc[0][reg] * 128 + acc[1][reg];
        const float V = __builtin_fmaf((float)acc[2][reg], 0x1p-7f, (float)T);
        const float L = __builtin_fmaf(-F1[reg], V, cqv);
        const bool lt = L < sL1[reg];
        sL2[reg] = __builtin_amdgcn_fmed3f(sL1[reg], sL2[reg], L);
        sI1[reg] = lt ? c : sI1[reg];
        sL1[reg] = lt ? L : sL1[reg];   // L is never NaN: a select, no canonicalize
      }
    }
  };
  auto cq_of = [&](int slot, int half = 0) {
    return *(const float*)(lds + slot * TB + FR * 1024 + (half * 32 + r) * 4);
  };
  // tile t in `slot`: wait for this wave's DMAs of t (those of t + 1 may stay
  // in flight), barrier (every wave's part of t landed; every wave is past
  // t - 1, whose slot the DMAs of t + 2 now refill)
  auto arrive = [&](int t, int slot) {
    if constexpr (PAIR && (CYC_PROBE_MODE & 2)) {
      __builtin_amdgcn_s_barrier();
      return;
    }
    if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G + 1) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    __builtin_amdgcn_s_barrier();
    issue(t + 2, slot == 0 ? 2 : slot - 1);
  };
  auto next_slot = [](int slot) { return slot == 2 ? 0 : slot + 1; };

  // MODE.FP_ROUND single precision = toward -inf (the L' are lower bounds)
  __builtin_amdgcn_s_setreg(0x801, 2);
  // (software-pipelining the epilogue beside the next tile's MFMAs needs a
  // second accumulator set: 193 VGPRs, two waves per SIMD, 4 % slower than
  // this form at 168 VGPRs and three waves per SIMD)
  int sl = 0;
  if constexpr (PAIR) {
    // The one-limb bounds in the units 2^(exmin + ec - SH) of the wave's
    // smallest exponent, shifted left by IB with the tile index in the low
    // bits: Ve = (T << (sh + IB)) + ((-Q << IB) + ct), one v_lshl_add_u32 per
    // (row, center) on an accumulator started at 0 (the -Q start value of
    // the two-limb form is gone, and Q needs no per-row rounding).
    // |T| < 2^22 (d <= 256), sh <= kShMax (rows past it are not screened),
    // |Q| <= 2^25: |Ve| < 2^31.
    int shIB[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) shIB[reg] = min(sh[reg], kShMax) + IB;
    auto epi_reg = [&](int reg, int cpr, int T) {
      const int Ve = (int)(((unsigned)T << shIB[reg]) + (unsigned)cpr);
      sV2[reg] = max(min(sV1[reg], sV2[reg]), min(max(sV1[reg], sV2[reg]), Ve));   // v_med3_i32
      sV1[reg] = max(sV1[reg], Ve);
    };
    // Software-pipelined by hand: each gap between two MFMAs of one tile
    // carries the epilogue of 16 / S rows of the tile before (tile 2 st - 1's
    // beside 2 st's, across the barrier) and the B fragment of the next MFMA;
    // sched_barrier pins that order.  X1 starts as zero rows with cpr =
    // INT_MIN: an epilogue that changes no sV.
    constexpr int RPG = 16 / S;   // accumulator rows per MFMA gap
    static_assert(16 % S == 0, "the gaps split the 16 rows evenly");
    const v16i Z = {};
    v16i X0, X1 = Z;
    int cprPrev = INT_MIN;
    for (int st = 0; st < nsteps; ++st) {
      arrive(st, sl);
      // (-Q << IB) + ct of tiles 2 st and 2 st + 1
      int cpr[2];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float pf = cq_of(sl, hf) * qscale;
        qbad |= pf < -QCLAMP;
        const int nb = -(int)__builtin_floorf(__builtin_fminf(pf, QCLAMP));
        cpr[hf] = (int)(((unsigned)nb << IB) + (unsigned)(vzero + 2 * st + hf));
      }
      // opaque: one register each, not re-associated into every element's add
      asm volatile("" : "+v"(cpr[0]), "+v"(cpr[1]));
      const v4i* B = (const v4i*)(lds + sl * TB) + lane;
      v4i Bn = B[0];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const v4i Bc = Bn;
        Bn = B[(s + 1) * 64];   // s = S - 1: tile 2 st + 1's first fragment
        X0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], Bc, s == 0 ? Z : X0, 0, 0, 0);
#pragma unroll
        for (int q = RPG * s; q < RPG * (s + 1); ++q) epi_reg(q, cprPrev, X1[q]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const v4i Bc = Bn;
        if (s + 1 < S) Bn = B[(S + s + 1) * 64];
        X1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], Bc, s == 0 ? Z : X1, 0, 0, 0);
#pragma unroll
        for (int q = RPG * s; q < RPG * (s + 1); ++q) epi_reg(q, cpr[0], X0[q]);
        __builtin_amdgcn_sched_barrier(0);
      }
      cprPrev = cpr[1];
      sl = next_slot(sl);
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) epi_reg(reg, cprPrev, X1[reg]);
  }
  for (int ct = 0; ct < (PAIR ? 0 : ktp); ++ct) {
    v16i X[LIMBS];
    arrive(ct, sl);
    const float cqv = cq_of(sl);
    if constexpr (LIMBS < 3) {
      // -Q per row: ceil(floor(cq 2^k) / 2^sh) >= Q - 1 unit; cq above 2^30
      // units clamps (a smaller Q: still a lower bound)
      const float pf = cqv * qscale;   // exact (a power of two; round-down mode)
      qbad |= pf < -QCLAMP;
      const int nb = -(int)__builtin_floorf(__builtin_fminf(pf, QCLAMP));
      X[0] = v16i{};
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) X[LIMBS - 1][reg] = nb >> sh[reg];
      tile(sl, X);
      epi2(ct, X);
    } else {
#pragma unroll
      for (int L = 0; L < LIMBS; ++L) X[L] = v16i{};
      tile(sl, X);
      epi(ct, cqv, X);
    }
    sl = next_slot(sl);
  }
  __builtin_amdgcn_s_setreg(0x801, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing re-read DMAs
  if constexpr (PAIR && (CYC_PROBE_MODE & 4)) {   // probe: no reduction / certification
    if (lane < rows) assign[rowAt(lane)] = sV1[lane & 15] ^ sV2[(lane + 1) & 15];
    return;
  }

  // LIMBS = 2: each lane's own best and second best (one center column per
  // lane) before the reduction merges them: the candidate sets below
  int cV1[16], cV2[16];
  if constexpr (LIMBS < 3) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      sI1[q] = (int)((unsigned)sV1[q] & IM) * 32 + r;
      cV1[q] = sV1[q];
      cV2[q] = sV2[q];
    }
  }
  // each row's (L1, L2, I1) over the 32 lanes (centers) of its half: every
  // xor step halves the registers a lane keeps (lanes with the step's bit
  // keep the upper half and send the lower), so 16 rows cost 8 + 4 + 2 + 1 + 1
  // shuffles per quantity.  Equal L1 from two centers leave L2 = L1, which
  // never certifies, so the merge needs no index tie-break.
  auto mergeL = [](float& L1, float& L2, int& I1, float oL1, float oL2, int oI1) {
    L2 = __builtin_fminf(__builtin_fmaxf(L1, oL1), __builtin_fminf(L2, oL2));
    I1 = oL1 < L1 ? oI1 : I1;
    L1 = __builtin_fminf(L1, oL1);
  };
  auto mergeV = [](int& V1, int& V2, int& I1, int oV1, int oV2, int oI1) {
    V2 = max(min(V1, oV1), max(V2, oV2));
    I1 = oV1 > V1 ? oI1 : I1;
    V1 = max(V1, oV1);
  };
#define CYC_REDUCE(K1, K2, MERGE)                                                   \
  _Pragma("unroll") for (int lev = 0; lev < 4; ++lev) {                             \
    const int half = 8 >> lev, m = 16 >> lev;                                       \
    const bool hi = (lane & m) != 0;                                                \
    _Pragma("unroll") for (int i = 0; i < half; ++i) {                              \
      const auto o1 = __shfl_xor(hi ? K1[i] : K1[i + half], m);                     \
      const auto o2 = __shfl_xor(hi ? K2[i] : K2[i + half], m);                     \
      const int oI1 = __shfl_xor(hi ? sI1[i] : sI1[i + half], m);                   \
      auto k1 = hi ? K1[i + half] : K1[i];                                          \
      auto k2 = hi ? K2[i + half] : K2[i];                                          \
      int I1 = hi ? sI1[i + half] : sI1[i];                                         \
      MERGE(k1, k2, I1, o1, o2, oI1);                                               \
      K1[i] = k1;                                                                   \
      K2[i] = k2;                                                                   \
      sI1[i] = I1;                                                                  \
    }                                                                               \
  }                                                                                 \
  MERGE(K1[0], K2[0], sI1[0], __shfl_xor(K1[0], 1), __shfl_xor(K2[0], 1),           \
        __shfl_xor(sI1[0], 1));
  if constexpr (LIMBS < 3) {
    CYC_REDUCE(sV1, sV2, mergeV)
  } else {
    CYC_REDUCE(sL1, sL2, mergeL)
  }
#undef CYC_REDUCE
  // lane holds row register q = lane bits 1..4
  // per-wave reduction area in the (now idle) slots: L1, L2, I1 x 32 rows
  __syncthreads();
  float* redL1 = (float*)lds + wave * 96;   // LIMBS = 2: the V1, V2 bits
  float* redL2 = redL1 + 32;
  int* redI1 = (int*)(redL1 + 64);
  if ((lane & 1) == 0) {
    const int q = (lane >> 1) & 15;
    const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
    redL1[row] = LIMBS < 3 ? __int_as_float(sV1[0]) : sL1[0];
    redL2[row] = LIMBS < 3 ? __int_as_float(sV2[0]) : sL2[0];
    redI1[row] = sI1[0];
  }
  const bool waveBad = __builtin_amdgcn_ballot_w64(qbad) != 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  bool want = false;   // LIMBS < 3: an undecided row for the candidate pass
  int thrV = 0;
  int64_t grow = 0;
  // LIMBS = 1 with bnd: the row's terms for its candidate rows' bound
  double bxx = 0.0, bfx = 0.0, benc = 0.0, bf1 = 0.0;
  int bsb = 0;
  if (lane < rows) {
    grow = rowAt(lane);
    const int2 mt = meta[grow];
    const int I1 = redI1[lane];
    // L1, L2 as fp64 (LIMBS < 3: -F1 V; V2 = INT_MIN: no second)
    double l1, l2, f1 = 0.0;
    int v1 = 0;
    bool clamped = false, shOk = true;
    int sb = 0;   // LIMBS = 1: the row's Ve = V 2^sb (+ index bits)
    if constexpr (LIMBS < 3) {
      f1 = __builtin_ldexp(1.0, mt.x + P.ec - SH);
      v1 = __float_as_int(redL1[lane]);
      int v2 = __float_as_int(redL2[lane]);
      if constexpr (LIMBS == 1) {
        // back to the row's units, floored (< 1 unit, inside enc below)
        const int shr = mt.x - exmin;
        shOk = shr >= 0 && shr <= kShMax;
        sb = min(max(shr, 0), kShMax) + IB;
        if (v1 != INT_MIN) v1 >>= sb;
        if (v2 != INT_MIN) v2 >>= sb;
      }
      l1 = -f1 * (double)v1;
      l2 = v2 == INT_MIN ? __builtin_inf() : -f1 * (double)v2;
      // the winner's Q must not have clamped (its bound would be too low)
      if (I1 >= 0 && I1 < P.k)
        clamped = !((double)cq[I1] * (double)qscale <= (double)QCLAMP);
    } else {
      l1 = (double)redL1[lane];
      l2 = (double)redL2[lane];
    }
    bool decided = false, eligible = false;
    double M = 0.0;
    float2 bb = make_float2(-1.0f, -1.0f);   // LIMBS = 1 with bnd: the row's bounds (none)
    if (mt.x != INT_MIN && I1 >= 0 && I1 < P.k && !clamped && shOk && !waveBad &&
        __builtin_isfinite(l1)) {
      bsb = sb;
      bf1 = f1;
      const double xn = xnorm[grow], cn = cnorm[I1];
      const double xx = xn * xn, cc = cn * cn;
      const double n1 = (double)__int_as_float(mt.y);   // bounds |xh3|_1
      const double fx =
          LIMBS == 3 ? err_term(mt.x, n1, mu, d)
          : LIMBS == 2 ? err_term2(mt.x, n1 + (double)d * __builtin_ldexp(1.0078125, mt.x - 15), mu, d)
                       : err_term1(mt.x, n1 + (double)d * __builtin_ldexp(1.0078125, mt.x - 8), mu);
      // LIMBS = 2: the index bits move each V by < 2^IB units and the
      // rounded Q adds < 1 more: |L1 - L1'|, |L2 - L2'| < (2^IB + 1) F1
      // (LIMBS = 1: < 1 unit, the floor of V 2^sb)
      const double enc = LIMBS == 3 ? 0.0
                                    : __builtin_ldexp((double)(IM + 3u), mt.x + P.ec - SH);
      M = (4.0 * (fx + g[I1]) + 2.0 * kEpsF * (xx + cc) + 2.0 * enc +
           0x1p-20 * (__builtin_fabs(l1) + cc + 2.0 * g[I1]) +
           0x1p-24 * (2.0 * (xx + cc) + __builtin_fabs(l1) +
                      __builtin_fmin(__builtin_fabs(l2), 0x1p120)) +
           0x1p-90) *
          (1.0 + 0x1p-30);
      decided = !__builtin_isfinite(l2) || (l2 - l1) > M;
      eligible = __builtin_isfinite(M);
      if constexpr (LIMBS == 1) {
        bxx = xx;
        bfx = fx;
        benc = enc;
        // carried bounds of a certified row: every center but I1 has a
        // computed bound >= l2 (bnd_ub_sq / bnd_lb_sq)
        if (bnd && decided && __builtin_isfinite(l2)) {
          bb.x = bnd_dist_up(bnd_ub_sq(xx, cc, l1, fx, g[I1], enc));
          if (bb.x < 0x1p120f) bb.y = bnd_dist_dn(bnd_lb_sq(xx, l2, fx, enc, 0.0));
        }
      }
    }
    // (rows listed with candidates get their lower bound for the centers
    // outside the set below; every other undecided row none)
    if (LIMBS == 1 && bnd) bnd[grow] = bb;
    if (decided) {
      assign[grow] = I1;
    } else if (LIMBS < 3 && candRows != nullptr && eligible) {
      // candidates: the centers c with f1 (V1 - V_c) <= M, i.e. V_c >= v1 -
      // floor(M / f1) -- the certification test against I1, failed by
      // every candidate and passed by every other center
      const double tv = (double)v1 - __builtin_floor(M / f1);
      if (tv > (double)INT_MIN + 2.0) {
        want = true;
        thrV = (int)tv;
        // LIMBS = 1: in the lanes' Ve units (a lower threshold only adds
        // candidates)
        if constexpr (LIMBS == 1) thrV = (int)((unsigned)max(thrV, -(1 << 23)) << sb);
      } else {
        listS[atomicAdd(listCountS, 1u)] = (int32_t)grow;
      }
    } else {
      listS[atomicAdd(listCountS, 1u)] = (int32_t)grow;
    }
  }
  if constexpr (LIMBS < 3) {
    if (candRows != nullptr) {
      // Candidate sets of the undecided rows from the saved per-lane states:
      // lane (r, h) saw the centers 32 ct + r of row (reg & 3) + 8 (reg >> 2)
      // + 4 h; its best is a candidate when it reaches the row's threshold,
      // and a lane whose SECOND best reaches it too (an index not kept)
      // sends the row to the three-limb pass.  <= kCandMax candidates go to
      // the candidate list (exact fp64 distances, screen_cands).
      int* thrS = (int*)lds + W * 96 + wave * (64 + 32 * (CMAX + 1));
      int* wantS = thrS + 32;
      int* candS = thrS + 64;
      if (lane < 32) {
        thrS[lane] = thrV;
        wantS[lane] = want ? 1 : 0;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const bool w = wantS[row] != 0;
        const int t = thrS[row];
        const bool ok = w && cV1[reg] >= t;
        const bool ov = w && cV2[reg] >= t;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(ok);
        const unsigned long long mo = __builtin_amdgcn_ballot_w64(ov);
        const unsigned bits = (unsigned)(m >> (32 * h));
        if (ok) {
          const int slot = __builtin_popcount(bits & ((1u << r) - 1u));
          if (slot < CMAX)
            candS[row * (CMAX + 1) + 1 + slot] = (int)((unsigned)cV1[reg] & IM) * 32 + r;
        }
        if (r == 0 && w)
          candS[row * (CMAX + 1)] = (unsigned)(mo >> (32 * h)) ? -1 : __builtin_popcount(bits);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      // LIMBS = 1 with bnd: the best computed bound among the centers OUTSIDE
      // each candidate row's set -- per lane its best below the threshold
      // (a candidate row has at most one candidate per lane: cV2 is below),
      // the largest V over the row's lanes -- into thrS (read above)
      int* ncS = thrS;
      if constexpr (LIMBS == 1) {
        if (bnd) {
          int nc[16];
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int t = thrS[row];
            nc[reg] = cV1[reg] < t ? cV1[reg] : cV2[reg];
          }
          __builtin_amdgcn_wave_barrier();
          rows_max32(nc, lane, ncS);
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
      }
      if (want) {
        const int* cs = candS + lane * (CMAX + 1);
        const int cnt = cs[0];
        if (cnt >= 1 && cnt <= CMAX) {
          const unsigned idx = atomicAdd(candCountS, 1u);
          candRowsS[idx] = (int32_t)grow;
#pragma unroll
          for (int i = 0; i < CMAX; ++i) candsS[(size_t)idx * CMAX + i] = i < cnt ? cs[1 + i] : -1;
          if constexpr (LIMBS == 1) {
            if (bnd) {
              // (-2, lower bound of every center outside the set): the
              // refinement and the three-limb candidate tier finish it
              const int vnc = ncS[lane];
              const double lnc = vnc == INT_MIN ? __builtin_inf() : -bf1 * (double)(vnc >> bsb);
              bnd[grow] = make_float2(-2.0f, vnc == INT_MIN ? __builtin_inff()
                                                            : bnd_dist_dn(bnd_lb_sq(bxx, lnc, bfx, benc, 0.0)));
            }
          }
        } else {
          listS[atomicAdd(listCountS, 1u)] = (int32_t)grow;
        }
      }
    }
  }
  __syncthreads();   // the reduction area is the next group's tile ring
  };
  // LIST: the grid covers n rows; groups past the count leave at once (a
  // grid-stride loop here costs the three-limb S = 8 form ~30 spilled VGPRs)
  if ((int64_t)blockIdx.x * 32 * W < total) group(blockIdx.x);
}

template <int S, int W, int LIMBS, bool LIST>
int launch_screen32(const void* img, const int2* meta, const double* xnorm, int64_t n, int d,
                    const void* Cb, const float* cq, const double* g, const double* cnorm,
                    const CenterParams* prm, int ktp, const int32_t* rowsIn,
                    const unsigned int* rowsInCount, int32_t* assign, int32_t* list,
                    unsigned int* listCount, hipStream_t st, int32_t* candRows = nullptr,
                    int32_t* cands = nullptr, unsigned int* candCount = nullptr,
                    unsigned int scap = 0, float2* bnd = nullptr) {
  KernelTimer timer(LIMBS == 1 ? "k_kmeans_screen1" : LIMBS == 2 ? "k_kmeans_screen2"
                                                    : "k_kmeans_screen3", st);
  const int64_t wg = (n + 32 * W - 1) / (32 * W);   // W waves x 32 rows
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_screen32<S, W, LIMBS, LIST>), dim3((unsigned)wg),
                     dim3(64 * W), 0, st, (const uint4*)img, meta, xnorm, n, d, (const uint4*)Cb,
                     cq, g, cnorm, prm, ktp, rowsIn, rowsInCount, assign, list, listCount,
                     candRows, cands, candCount, scap, bnd);
  CYC_LAUNCH_CHECK("k_kmeans_screen32_i8");
  return CYC_OK;
}

// ---------------------------------------------------------------------------
// Two-limb refinement (d <= 256) of the one-limb pass.
//
// The one-limb pass (k_screen32<S, W, 1, false>: S1 = a.a' only, one MFMA
// per 32-dim substep, a third of the two-limb pass's) screens every row
// against every center.  It certifies the rows it can; for each other row
// it lists the centers its bounds cannot exclude (<= kCand1: rowsIn /
// candsIn) -- every other center c has a one-limb lower bound above the
// one-limb winner w1's upper bound, i.e. |x - c|^2 > |x - w1|^2 (by the
// certification margin).  Here each wave takes 32 listed rows, forms the
// UNION of their candidate sets (<= 32 kPruneTiles centers: virtual tiles
// of 32, B fragments gathered per lane from the center image) and runs the
// two-limb screen over that union only.  A row certified there (w2 beats
// every union center by the two-limb margin) beats w1 (in the union, or w2
// = w1), hence every center outside the union too, by more than the
// reference's fp64 rounding: the reference's pruned loop returns w2.  Its
// other rows get the two-limb pass's treatment: candidate sets (<=
// kCandMax, within the union) for the fp64 candidate pass, else the
// three-limb pass.  Waves whose union is too large go to fullList (the
// full two-limb pass over every center).
constexpr int kPruneTiles = 3;

template <int S>
__global__ __launch_bounds__(256, 2) void k_screen32r(
    const uint4* __restrict__ Xq, const int2* __restrict__ meta, const double* __restrict__ xnorm,
    int64_t n, int d, const uint4* __restrict__ Cb, const float* __restrict__ cq,
    const double* __restrict__ g, const double* __restrict__ cnorm,
    const CenterParams* __restrict__ prm, int kstride, const int32_t* __restrict__ rowsIn,
    const unsigned int* __restrict__ rowsInCount, const int32_t* __restrict__ candsIn,
    int32_t* __restrict__ assign, int32_t* __restrict__ list, unsigned int* __restrict__ listCount,
    int32_t* __restrict__ candRows, int32_t* __restrict__ cands,
    unsigned int* __restrict__ candCount, int32_t* __restrict__ fullList,
    unsigned int* __restrict__ fullCount, unsigned int* __restrict__ stat, unsigned int scap,
    float2* __restrict__ bnd) {
  constexpr int D = 32 * S, CH = 3 * D / 16;
  constexpr int W = 4;
  // per wave: the candidate list, then the candidate-set scratch (the union
  // bitmap, kstride bits, aliases the latter)
  constexpr int PER_WAVE = 32 * kPruneTiles + 64 + 32 * (kCandMax + 1);
  static_assert(64 + 32 * (kCandMax + 1) >= 4096 / 32, "bitmap fits the scratch");
  __shared__ int ldsw[W * PER_WAVE];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int* candL = ldsw + wave * PER_WAVE;
  const CenterParams P = *prm;
  const double mu = P.mu * 0x1p-7;
  const int64_t total = (int64_t)*rowsInCount;
  const int64_t pos0 = ((int64_t)blockIdx.x * W + wave) * 32;
  const int rows = (int)max<int64_t>(0, min<int64_t>(32, total - pos0));
  if (rows == 0) return;
  const bool rowOk = r < rows;
  const int64_t myRow = rowOk ? rowsIn[pos0 + r] : 0;
  // scap > 0: appends (and the stat adds) go to this wave's shard
  const unsigned shard = (unsigned)((blockIdx.x * W + wave) % kShards);
  if (scap) {
    list += (size_t)shard * scap;
    listCount += shard * kShardStride;
    fullList += (size_t)shard * scap;
    fullCount += shard * kShardStride;
    if (candRows) {
      candRows += (size_t)shard * scap;
      cands += (size_t)shard * scap * kCandMax;
      candCount += shard * kShardStride;
    }
    if (stat) stat += shard * kShardStride;
  }
  auto to_full = [&]() {
    if (lane < rows) {
      fullList[atomicAdd(fullCount, 1u)] = (int32_t)myRow;
      // the full two-limb pass keeps no bound for the centers it excludes
      if (bnd) bnd[myRow] = make_float2(-1.0f, -1.0f);
    }
  };
  if (!P.ok) {   // uniform over the grid: every row to the fp64 tier
    if (lane < rows) list[atomicAdd(listCount, 1u)] = (int32_t)myRow;
    return;
  }
  // the union of the rows' candidate sets: bitmap, then the compacted list
  unsigned* bm = (unsigned*)(candL + 32 * kPruneTiles);
  const int words = kstride >> 5;                      // <= 128
  for (int q = lane; q < words; q += 64) bm[q] = 0u;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  bool bad = false;
  if (lane < 32 && rowOk) {
    const int32_t* cs = candsIn + (pos0 + r) * kCand1;
#pragma unroll
    for (int i = 0; i < kCand1; ++i) {
      const int c = cs[i];
      if (c >= P.k) bad = true;
      if (c >= 0 && c < P.k) atomicOr(&bm[c >> 5], 1u << (c & 31));
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const unsigned wA = lane < words ? bm[lane] : 0u;
  const unsigned wB = lane + 64 < words ? bm[lane + 64] : 0u;
  const int cnt = __builtin_popcount(wA) + __builtin_popcount(wB);
  int pre = cnt;                                       // inclusive prefix over lanes
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const int t = __shfl_up(pre, m);
    if (lane >= m) pre += t;
  }
  const int ncand = __shfl(pre, 63);
  if (__builtin_amdgcn_ballot_w64(bad) != 0 || ncand > 32 * kPruneTiles || ncand == 0) {
    to_full();
    return;
  }
  {
    int o = pre - cnt;
    for (unsigned b = wA; b; b &= b - 1) candL[o++] = lane * 32 + __builtin_ffs((int)b) - 1;
    for (unsigned b = wB; b; b &= b - 1) candL[o++] = (lane + 64) * 32 + __builtin_ffs((int)b) - 1;
    const int nt = (ncand + 31) >> 5;
    for (int q = ncand + lane; q < nt * 32; q += 64) candL[q] = -1;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const int ntiles = (ncand + 31) >> 5;
  // A fragments of the wave's rows (two limbs)
  v4i A[S][2];
  {
    const uint4* src = Xq + myRow * CH + h;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int L = 0; L < 2; ++L) {
        const v4u t = __builtin_nontemporal_load((const v4u*)(src + L * (D / 16) + 2 * s));
        A[s][L] = rowOk ? __builtin_bit_cast(v4i, t) : v4i{0, 0, 0, 0};
      }
  }
  const int2 mt = rowOk ? meta[myRow] : make_int2(INT_MIN, 0);
  const int exr = mt.x;
  int e0 = exr == INT_MIN ? INT_MAX : exr;
#pragma unroll
  for (int m = 1; m < 32; m <<= 1) e0 = min(e0, __shfl_xor(e0, m));
  const int exmin = __builtin_amdgcn_readfirstlane(e0 == INT_MAX ? 0 : e0);
  int sh[16];
  {
    const int s0 = exr == INT_MIN ? 31 : min(exr - exmin, 31);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) sh[reg] = __shfl(s0, (reg & 3) + 8 * (reg >> 2) + 4 * h);
  }
  const float qscale = __builtin_ldexpf(1.0f, max(-160, min(160, 20 - P.ec - exmin)));
  bool qbad = false;
  double xxj = 0.0;
  if (lane < 32 && rowOk) {
    const double xn = xnorm[myRow];
    xxj = xn * xn;
  }
  // B fragments of center c (c < 0: a padding column, zero), from the
  // center-major copy behind the fragment image (k_centers_pack32): a lane's
  // 16 pieces of its center lie in 512 contiguous bytes (from the fragments
  // every piece was a separate cache line)
  const uint4* Cr = Cb + (size_t)(kstride >> 5) * S * 3 * 64;
  auto loadB = [&](int c, v4i (&B)[S][2]) {
    const bool on = c >= 0;
    const uint4* src = Cr + (size_t)(on ? c : 0) * (6 * S) + h;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int L = 0; L < 2; ++L) {
        const v4u t = *(const v4u*)(src + L * 2 * S + 2 * s);
        B[s][L] = on ? __builtin_bit_cast(v4i, t) : v4i{0, 0, 0, 0};
      }
  };
  // one virtual tile: column r holds center col (lane's), acc[1] from -Q
  auto tileMfma = [&](int col, const v4i (&B)[S][2], v16i (&X)[2]) {
    const float cqv = col >= 0 ? cq[col] : 0x1.fffffep127f;
    const float pf = cqv * qscale;
    qbad |= pf < -0x1p30f;
    const int nb = -(int)__builtin_floorf(__builtin_fminf(pf, 0x1p30f));
    X[0] = v16i{};
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) X[1][reg] = nb >> sh[reg];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      X[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], B[s][0], X[0], 0, 0, 0);
      X[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][0], B[s][1], X[1], 0, 0, 0);
      X[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s][1], B[s][0], X[1], 0, 0, 0);
    }
  };
  // the two-limb certification margin of row (mt, xx) against center c
  // (lower bounds l1, runner-up l2; IM: the index bits in V)
  auto margin = [&](int c, double xx, double l1, double l2, unsigned IM) {
    const double cn = cnorm[c];
    const double cc = cn * cn;
    const double n1 = (double)__int_as_float(mt.y);
    const double fx = err_term2(mt.x, n1 + (double)d * __builtin_ldexp(1.0078125, mt.x - 15), mu, d);
    const double enc = __builtin_ldexp((double)(IM + 3u), mt.x + P.ec - 20);
    return (4.0 * (fx + g[c]) + 2.0 * kEpsF * (xx + cc) + 2.0 * enc +
            0x1p-20 * (__builtin_fabs(l1) + cc + 2.0 * g[c]) +
            0x1p-24 * (2.0 * (xx + cc) + __builtin_fabs(l1) +
                       __builtin_fmin(__builtin_fabs(l2), 0x1p120)) +
            0x1p-90) *
           (1.0 + 0x1p-30);
  };
  __builtin_amdgcn_s_setreg(0x801, 2);     // f32 rounding toward -inf (lower bounds)
  const int total_ = ncand;
  // 4. the screen over the candidate tiles (top two V per row slot, the
  // virtual tile index in the low IB bits)
  const int IB = 32 - __builtin_clz((unsigned)max(ntiles - 1, 1));
  const unsigned IM = (1u << IB) - 1u;
  int sV1[16], sV2[16], sI1[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) sV1[q] = sV2[q] = INT_MIN;
  for (int t = 0; t < ntiles; ++t) {
    const int col = candL[t * 32 + r];
    v4i B[S][2];
    loadB(col, B);
    v16i X[2];
    tileMfma(col, B, X);
    unsigned ctv;
    asm("v_mov_b32 %0, %1" : "=v"(ctv) : "s"(t));
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int V = X[0][reg] * 128 + X[1][reg];
      const int Ve = (int)(((unsigned)V & ~IM) | ctv);
      sV2[reg] = max(min(sV1[reg], sV2[reg]), min(max(sV1[reg], sV2[reg]), Ve));
      sV1[reg] = max(sV1[reg], Ve);
    }
  }
  __builtin_amdgcn_s_setreg(0x801, 0);
  const bool waveBad = __builtin_amdgcn_ballot_w64(qbad) != 0;
  // each lane's own best / second best (its column) before the reduction:
  // the candidate sets; centers through the candidate list
  int cV1[16], cV2[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    sI1[q] = candL[(int)((unsigned)sV1[q] & IM) * 32 + r];
    cV1[q] = sV1[q];
    cV2[q] = sV2[q];
  }
  auto mergeV = [](int& V1, int& V2, int& I1, int oV1, int oV2, int oI1) {
    V2 = max(min(V1, oV1), max(V2, oV2));
    I1 = oV1 > V1 ? oI1 : I1;
    V1 = max(V1, oV1);
  };
#pragma unroll
  for (int lev = 0; lev < 4; ++lev) {
    const int half = 8 >> lev, m = 16 >> lev;
    const bool hi = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const int o1 = __shfl_xor(hi ? sV1[i] : sV1[i + half], m);
      const int o2 = __shfl_xor(hi ? sV2[i] : sV2[i + half], m);
      const int oI1 = __shfl_xor(hi ? sI1[i] : sI1[i + half], m);
      int k1 = hi ? sV1[i + half] : sV1[i];
      int k2 = hi ? sV2[i + half] : sV2[i];
      int I1 = hi ? sI1[i + half] : sI1[i];
      mergeV(k1, k2, I1, o1, o2, oI1);
      sV1[i] = k1;
      sV2[i] = k2;
      sI1[i] = I1;
    }
  }
  mergeV(sV1[0], sV2[0], sI1[0], __shfl_xor(sV1[0], 1), __shfl_xor(sV2[0], 1),
         __shfl_xor(sI1[0], 1));
  // lane holds row register q = lane bits 1..4: per-row results through LDS
  int* red = candL + 32 * kPruneTiles;                // 3 x 32 ints (reused below)
  int* redV1 = red;
  int* redV2 = red + 32;
  int* thrS = red;                                    // after the reads below
  int* wantS = red + 32;
  int* candS = red + 64;
  int* redI1 = candS;                                 // 32 ints, read before candS is written
  if ((lane & 1) == 0) {
    const int q = (lane >> 1) & 15;
    const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
    redV1[row] = sV1[0];
    redV2[row] = sV2[0];
    redI1[row] = sI1[0];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  bool want = false;
  int thrV = 0;
  // with bnd: the row's lower bound for the centers outside its one-limb
  // set (the one-limb pass left it in bnd[row].y), and its terms
  float lncPrev = -1.0f;
  double bfx = 0.0, benc = 0.0, bf1 = 0.0;
  if (lane < rows) {
    const int I1 = redI1[lane];
    const int v1 = redV1[lane];
    const int v2 = redV2[lane];
    const double f1 = __builtin_ldexp(1.0, exr + P.ec - 20);
    const double l1 = -f1 * (double)v1;
    const double l2 = v2 == INT_MIN ? __builtin_inf() : -f1 * (double)v2;
    bool decided = false, eligible = false;
    double M = 0.0;
    if (exr != INT_MIN && I1 >= 0 && I1 < P.k && !waveBad && __builtin_isfinite(l1) &&
        (double)cq[I1] * (double)qscale <= 0x1p30) {
      M = margin(I1, xxj, l1, l2, IM);
      decided = !__builtin_isfinite(l2) || (l2 - l1) > M;
      eligible = __builtin_isfinite(M);
      if (bnd) {
        const float2 pb = bnd[myRow];
        lncPrev = pb.x == -2.0f ? pb.y : -1.0f;
        const double n1 = (double)__int_as_float(mt.y);
        bfx = err_term2(mt.x, n1 + (double)d * __builtin_ldexp(1.0078125, mt.x - 15), mu, d);
        benc = __builtin_ldexp((double)(IM + 3u), mt.x + P.ec - 20);
        bf1 = f1;
        if (decided && __builtin_isfinite(l2) && lncPrev >= 0.0f) {
          // certified over the union: the union's other centers have
          // computed bounds >= l2, the rest the one-limb pass's bound
          const double cn = cnorm[I1];
          const float ub = bnd_dist_up(bnd_ub_sq(xxj, cn * cn, l1, bfx, g[I1], benc));
          const float lb = bnd_dist_dn(bnd_lb_sq(xxj, l2, bfx, benc, 0.0));
          bnd[myRow] = ub < 0x1p120f ? make_float2(ub, __builtin_fminf(lb, lncPrev))
                                     : make_float2(-1.0f, -1.0f);
        }
      }
    }
    if (decided) {
      assign[myRow] = I1;
    } else if (candRows != nullptr && eligible) {
      const double tv = (double)v1 - __builtin_floor(M / f1);
      if (tv > (double)INT_MIN + 2.0) {
        want = true;
        thrV = (int)tv;
      } else {
        list[atomicAdd(listCount, 1u)] = (int32_t)myRow;
      }
    } else {
      list[atomicAdd(listCount, 1u)] = (int32_t)myRow;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (candRows != nullptr) {
    // candidate sets of the undecided rows (as the full pass; the centers
    // pruned in step 3 are excluded by margin)
    if (lane < 32) {
      thrS[lane] = thrV;
      wantS[lane] = want ? 1 : 0;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
      const bool w = wantS[row] != 0;
      const int t = thrS[row];
      const bool ok = w && cV1[reg] >= t;
      const bool ov = w && cV2[reg] >= t;
      const unsigned long long m = __builtin_amdgcn_ballot_w64(ok);
      const unsigned long long mo = __builtin_amdgcn_ballot_w64(ov);
      const unsigned bts = (unsigned)(m >> (32 * h));
      if (ok) {
        const int slot = __builtin_popcount(bts & ((1u << r) - 1u));
        if (slot < kCandMax)
          candS[row * (kCandMax + 1) + 1 + slot] = candL[(int)((unsigned)cV1[reg] & IM) * 32 + r];
      }
      if (r == 0 && w)
        candS[row * (kCandMax + 1)] = (unsigned)(mo >> (32 * h)) ? -1 : __builtin_popcount(bts);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // with bnd: the best computed bound among the union's centers outside
    // each candidate row's set (the one-limb pass's ncS, over the union)
    int* ncS = thrS;
    if (bnd) {
      int nc[16];
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int t = thrS[row];
        nc[reg] = cV1[reg] < t ? cV1[reg] : cV2[reg];
      }
      __builtin_amdgcn_wave_barrier();
      rows_max32(nc, lane, ncS);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    if (want) {
      const int* cs = candS + lane * (kCandMax + 1);
      const int c0 = cs[0];
      if (c0 >= 1 && c0 <= kCandMax) {
        const unsigned idx = atomicAdd(candCount, 1u);
        candRows[idx] = (int32_t)myRow;
#pragma unroll
        for (int i = 0; i < kCandMax; ++i) cands[(size_t)idx * kCandMax + i] = i < c0 ? cs[1 + i] : -1;
        if (bnd) {
          // (-2, lower bound outside the set): the union's other centers and
          // (lncPrev) the centers outside the union; the three-limb
          // candidate tier finishes it
          const int vnc = ncS[lane];
          const float l2nc = vnc == INT_MIN ? __builtin_inff()
                                            : bnd_dist_dn(bnd_lb_sq(xxj, -bf1 * (double)vnc, bfx, benc, 0.0));
          bnd[myRow] = make_float2(-2.0f, lncPrev >= 0.0f ? __builtin_fminf(lncPrev, l2nc) : -1.0f);
        }
      } else {
        list[atomicAdd(listCount, 1u)] = (int32_t)myRow;
      }
    }
  }
  if (stat && lane == 0) atomicAdd(stat, (unsigned)total_);
}


// Candidate rows (one wave each): fp64 squared distances to the <= kCandMax
// candidates, summed over the lanes' dimensions (any order: the error is
// <= (d + 2) 2^-53 2 (|x|^2 + |c|^2) < 2^-40 (|x|^2 + |c|^2)); |c| from the
// screen's center norms (an fp64 norm: its rounding sits far inside margin).  The row is
// certified when the second smallest exceeds the smallest by margin (|x|^2
// + |c_best|^2) plus both errors: every other center was already excluded by
// the two-limb bounds (by the screen's own margin), so the best candidate
// is the reference loop's answer as for any certified row.  Ties and near
// ties go on to list (the fp64 screen, then the reference loop).
// 16-lane row sum by DPP row rotations (VALU, no LDS): every lane of the
// row ends with the total.
__device__ __forceinline__ double row16_sum(double v) {
#define CYC_ROR(CTRL)                                                                        \
  {                                                                                          \
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false); \
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false); \
    v += __hiloint2double(hi, lo);                                                           \
  }
  CYC_ROR(0x128) CYC_ROR(0x124) CYC_ROR(0x122) CYC_ROR(0x121)
#undef CYC_ROR
  return v;
}

__global__ __launch_bounds__(256) void k_screen_cands(
    const double* __restrict__ X, const double* __restrict__ xnorm, int d,
    const double* __restrict__ C, const double* __restrict__ cnorm, int k, bool unit,
    double margin, const int32_t* __restrict__ candRows, const int32_t* __restrict__ cands,
    const unsigned int* __restrict__ candCount, int32_t* __restrict__ assign,
    int32_t* __restrict__ list, unsigned int* __restrict__ listCount, unsigned int scap) {
  // 2 rows per wave, 32 lanes per row; lane s of a row holds the dimensions
  // s, s + 32, ... (each load instruction reads 256 contiguous bytes per
  // row), and every load of a row -- its x and all kCandMax candidate rows
  // -- is in flight at once: one memory latency per row after its indices
  // (4 rows x 16 lanes with the candidates in two batches took three)
  const unsigned cnt = *candCount;
  const int lane = threadIdx.x & 63, q = lane >> 5, sl = lane & 31;
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const unsigned w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (scap) {   // this wave's shard (<= 4 rows per grid stride: shard_cap)
    list += (size_t)(w0 % kShards) * scap;
    listCount += (w0 % kShards) * kShardStride;
  }
  for (unsigned base = w0 * 2; base < cnt; base += nw * 2) {
    const unsigned idx = base + q;
    const bool live = idx < cnt;
    const int64_t row = live ? candRows[idx] : 0;
    int ci[kCandMax];
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) ci[i] = live ? cands[(size_t)idx * kCandMax + i] : -1;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) bad = bad || ci[i] >= k;   // a padding center
    const double* x = X + row * d;
    double u[8], cv[kCandMax][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = e * 32 + sl;   // d <= 256
      u[e] = (live && j < d) ? x[j] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) {
      const int c = ci[i];
      const bool on = c >= 0 && c < k;
      const double* cr = C + (int64_t)(on ? c : 0) * d;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = e * 32 + sl;
        cv[i][e] = (on && j < d) ? cr[j] : 0.0;
      }
    }
    if (unit) {
      const double inv = live ? 1.0 / xnorm[row] : 0.0;
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = u[e] * inv;
    }
    double xx = 0.0;
#pragma unroll
    for (int e = 0; e < 8; ++e) xx += u[e] * u[e];
    double part[kCandMax];
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) {
      double s2 = 0.0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double t = cv[i][e] - u[e];
        s2 += t * t;
      }
      part[i] = s2;
    }
    // sums over the row's 32 lanes: within each 16-lane row by DPP, then
    // the two halves
    xx = row16_sum(xx);
    xx += __shfl_xor(xx, 16);
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) {
      part[i] = row16_sum(part[i]);
      part[i] += __shfl_xor(part[i], 16);
    }
    double best = __builtin_inf(), second = __builtin_inf();
    int bi = -1, si = -1;
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) {
      if (ci[i] < 0 || ci[i] >= k) continue;
      const double s2 = part[i];
      if (s2 < best) {
        second = best;
        si = bi;
        best = s2;
        bi = ci[i];
      } else if (s2 < second) {   // an equal distance lands here: no certification
        second = s2;
        si = ci[i];
      }
    }
    bool ok = !bad && bi >= 0 && __builtin_isfinite(best) && __builtin_isfinite(xx);
    if (ok && second != __builtin_inf()) {   // one candidate: certified as it is
      const double cb = cnorm[bi], cs = si >= 0 ? cnorm[si] : 0.0;
      const double ccb = cb * cb, ccs = cs * cs;
      const double M = margin * (xx + ccb) + 0x1p-40 * (2.0 * xx + ccb + ccs);
      ok = __builtin_isfinite(M) && (second - best) > M * (1.0 + 0x1p-30);
    }
    if (live && sl == 0) {
      if (ok) assign[row] = bi;
      else list[atomicAdd(listCount, 1u)] = (int32_t)row;
    }
  }
}

// Three-limb tier of the candidate rows, ahead of k_screen_cands: for each
// of a row's <= kCandMax candidates the exact integer limb products S1 =
// a.a', S2 = a.b' + b.a', S3 = a.c' + b.b' + c.a' of the row image and the
// center-major copy of the center image (v_dot4 over 2S lanes per row, 16
// dimensions a lane: 768 B per row and per candidate at d = 256, against
// 2 KB of fp64 each in k_screen_cands), bounded exactly as the three-limb
// pass bounds them (k_screen32<.., 3, ..>: the same f32 lower bounds L,
// rounded down, and the same certification margin M), over the candidates
// instead of every center.  A row is certified when its best candidate
// beats every other candidate by M: the candidates exclude every other
// center (by the two-limb margin against the two-limb winner, itself a
// candidate), so the best candidate is the reference loop's answer, as in
// k_screen_cands.  The other rows go on with their candidates to
// k_screen_cands (out*).
__device__ __forceinline__ int dot16(uint4 u, uint4 v, int acc) {
  acc = __builtin_amdgcn_sdot4((int)u.x, (int)v.x, acc, false);
  acc = __builtin_amdgcn_sdot4((int)u.y, (int)v.y, acc, false);
  acc = __builtin_amdgcn_sdot4((int)u.z, (int)v.z, acc, false);
  return __builtin_amdgcn_sdot4((int)u.w, (int)v.w, acc, false);
}
__device__ __forceinline__ int dot16(uint2 u, uint2 v, int acc) {
  acc = __builtin_amdgcn_sdot4((int)u.x, (int)v.x, acc, false);
  return __builtin_amdgcn_sdot4((int)u.y, (int)v.y, acc, false);
}

// 16-lane integer row sum by DPP row rotations: every lane of the row ends
// with the total
__device__ __forceinline__ int row16_isum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);   // row_ror:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);   // row_ror:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x122, 0xF, 0xF, false);   // row_ror:2
  return v + __builtin_amdgcn_update_dpp(0, v, 0x121, 0xF, 0xF, false);   // row_ror:1
}

// PB: bytes of a limb plane per lane (16: 2S lanes per row; 8: 4S lanes,
// measured 0.94 vs 0.59 ms at 5 waves per SIMD against 4)
// RC (the carried candidate sets, kmeans_i8.hpp Bounds): the rows of
// candRows re-checked against the candidate set their last screen left
// (cands = Bounds::sets, indexed by ROW), certified when the best candidate
// beats the others by M and its upper bound stays below the set's carried
// lower bound for every other center (Bounds::lnc, moved by the drift) by
// the reference's slack; state[row] = 0 (certified) or 1 (a full screen).
template <int S, int PB, bool RC = false>
__global__ __launch_bounds__(256) void k_screen_cands3(
    const uint4* __restrict__ Xq, const int2* __restrict__ meta, const double* __restrict__ xnorm,
    int d, const uint4* __restrict__ Cr, const float* __restrict__ cq,
    const double* __restrict__ g, const double* __restrict__ cnorm,
    const CenterParams* __restrict__ prm, const int32_t* __restrict__ candRows,
    const int32_t* __restrict__ cands, const unsigned int* __restrict__ candCount,
    int32_t* __restrict__ assign, int32_t* __restrict__ outRows, int32_t* __restrict__ outCands,
    unsigned int* __restrict__ outCount, unsigned int scap, float2* __restrict__ bnd,
    float* __restrict__ lncA, int32_t* __restrict__ sets, unsigned char* __restrict__ state,
    const DriftParams* __restrict__ dp, const int32_t* __restrict__ nbr,
    const float* __restrict__ nbrR) {
  using Pc = std::conditional_t<PB == 16, uint4, uint2>;
  constexpr int P16 = 32 * S / PB;    // pieces per limb plane = lanes per row
  constexpr int RPW = 64 / P16;       // rows per wave
  const unsigned cnt = *candCount;
  const int lane = threadIdx.x & 63, q = lane / P16, li = lane % P16;
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const unsigned w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (scap) {   // this wave's shard (<= RPW rows per grid stride: shard_cap)
    const unsigned sh = w0 % kShards;
    outRows += (size_t)sh * scap;
    outCands += (size_t)sh * scap * kCandMax;
    outCount += sh * kShardStride;
  }
  const CenterParams P = *prm;
  const auto cR = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Cr, (short)0, (int)std::min<int64_t>((int64_t)P.k * 3 * P16 * PB, 0x7fffffff),
      0x00020000);
  for (unsigned base = w0 * RPW; base < cnt; base += nw * RPW) {
    const unsigned idx = base + q;
    const bool live = idx < cnt;
    const int32_t rw = live ? candRows[idx] : 0;
    // RC: a row listed as ~row re-checks the neighbourhood of its center
    // (set slot 0 = that center; the filter's state 3)
    const bool nbrMode = RC && rw < 0;
    const int64_t row = nbrMode ? ~rw : rw;
    const int32_t* setp = nbrMode ? nbr + (size_t)assign[row] * kCandMax
                                  : cands + (size_t)(RC ? row : (int64_t)idx) * kCandMax;
    int ci[kCandMax];
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) ci[i] = live ? setp[i] : -1;
    const Pc* xr = (const Pc*)Xq + row * (3 * P16) + li;
    const Pc xa = xr[0], xb = xr[P16], xc = xr[2 * P16];
    // the row's and the candidates' scalars issued with the gathers (each
    // one waited for on its own after them cost a round trip apiece)
    const int2 mt = live ? meta[row] : make_int2(INT_MIN, 0);
    const double xnr = xnorm[row];
    float cqv[kCandMax];
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) cqv[i] = cq[(ci[i] >= 0 && ci[i] < P.k) ? ci[i] : 0];
    float lncR = 0.0f;
    float2 bndR = make_float2(0.0f, 0.0f);
    double cnA = 0.0, gA = 0.0;
    float RA = 0.0f;
    if (bnd) {
      if (RC) lncR = lncA[row];
      else bndR = bnd[row];
    }
    if (nbrMode) {   // the anchor's terms for its fresh upper bound
      const int a0 = (ci[0] >= 0 && ci[0] < P.k) ? ci[0] : 0;
      cnA = cnorm[a0];
      gA = g[a0];
      RA = nbrR[a0];
    }
    int s1[kCandMax], s2[kCandMax], s3[kCandMax];
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) {
      const int c = ci[i];
      Pc ca, cb, cc;
      if constexpr (PB == 16) {
        // empty slots fetch nothing: an out-of-range buffer offset reads
        // zeros without a memory access (the kernel is bound by these L2
        // gathers, 768 B per candidate), and every slot's loads stay in
        // flight together
        const unsigned off = (c >= 0 && c < P.k) ? (unsigned)(c * 3 * P16 + li) * 16u
                                                 : 0x80000000u;
        ca = __builtin_bit_cast(Pc, __builtin_amdgcn_raw_buffer_load_b128(cR, (int)off, 0, 0));
        cb = __builtin_bit_cast(Pc, __builtin_amdgcn_raw_buffer_load_b128(
                                        cR, (int)(off + 16u * P16), 0, 0));
        cc = __builtin_bit_cast(Pc, __builtin_amdgcn_raw_buffer_load_b128(
                                        cR, (int)(off + 32u * P16), 0, 0));
      } else {
        const Pc* cr = (const Pc*)Cr + (size_t)((c >= 0 && c < P.k) ? c : 0) * (3 * P16) + li;
        ca = cr[0];
        cb = cr[P16];
        cc = cr[2 * P16];
      }
      s1[i] = dot16(xa, ca, 0);
      s2[i] = dot16(xb, ca, dot16(xa, cb, 0));
      s3[i] = dot16(xc, ca, dot16(xb, cb, dot16(xa, cc, 0)));
    }
    // sums over the row's P16 lanes (integers: any order); 16 lanes: DPP
    // row rotations (VALU), else cross-lane permutes
    if constexpr (P16 == 16) {
#pragma unroll
      for (int i = 0; i < kCandMax; ++i) {
        s1[i] = row16_isum(s1[i]);
        s2[i] = row16_isum(s2[i]);
        s3[i] = row16_isum(s3[i]);
      }
    } else {
#pragma unroll
      for (int m = 1; m < P16; m <<= 1)
#pragma unroll
        for (int i = 0; i < kCandMax; ++i) {
          s1[i] += __shfl_xor(s1[i], m);
          s2[i] += __shfl_xor(s2[i], m);
          s3[i] += __shfl_xor(s3[i], m);
        }
    }
    // the three-limb pass's bounds: T = S1 2^7 + S2, V = T + S3 2^-7 and L =
    // cq - F1 V in f32 rounded toward -inf (lower bounds), F1 = 2^(ex + ec - 20)
    __builtin_amdgcn_s_setreg(0x801, 2);
    const float F1 = mt.x == INT_MIN ? 0.0f : __builtin_ldexpf(1.0f, mt.x + P.ec - 20);
    float L1 = __builtin_inff(), L2 = __builtin_inff();
    int I1 = -1;
    bool bad = false;
    float cqMax = 0.0f;   // the f32 bounds' rounding slack (carried bounds)
    float LA = __builtin_inff();   // the anchor's bound (slot 0, state-3 re-checks)
#pragma unroll
    for (int i = 0; i < kCandMax; ++i) {
      const int c = ci[i];
      bad = bad || c >= P.k;   // a padding center
      if (c < 0 || c >= P.k) continue;
      const int T = s1[i] * 128 + s2[i];
      const float V = __builtin_fmaf((float)s3[i], 0x1p-7f, (float)T);
      const float L = __builtin_fmaf(-F1, V, cqv[i]);
      if (i == 0) LA = L;
      cqMax = __builtin_fmaxf(cqMax, __builtin_fabsf(cqv[i]));
      const bool lt = L < L1;
      L2 = __builtin_amdgcn_fmed3f(L1, L2, L);
      I1 = lt ? c : I1;
      L1 = lt ? L : L1;
    }
    __builtin_amdgcn_s_setreg(0x801, 0);
    bool decided = false;
    const double l1 = (double)L1, l2 = (double)L2;
    if (live && P.ok && !bad && mt.x != INT_MIN && I1 >= 0 && __builtin_isfinite(l1)) {
      const double xn = xnr, cn = cnorm[I1];
      const double gw = g[I1];
      const double xx = xn * xn, cc = cn * cn;
      const double n1 = (double)__int_as_float(mt.y);   // bounds |xh3|_1
      const double fx = err_term(mt.x, n1, P.mu, d);
      const double M = (4.0 * (fx + gw) + 2.0 * kEpsF * (xx + cc) +
                        0x1p-20 * (__builtin_fabs(l1) + cc + 2.0 * gw) +
                        0x1p-24 * (2.0 * (xx + cc) + __builtin_fabs(l1) +
                                   __builtin_fmin(__builtin_fabs(l2), 0x1p120)) +
                        0x1p-90) *
                       (1.0 + 0x1p-30);
      decided = !__builtin_isfinite(l2) || (l2 - l1) > M;
      if (bnd && (decided || RC)) {
        // carried bounds: the other candidates' bounds are >= l2 (f32,
        // rounded down after a rounded-down V: slack 2^-20 max |cq|), the
        // centers outside the set below the earlier tiers' bound (RC: the
        // set's carried bound)
        float lnc0 = RC ? lncR : bndR.y;
        const bool mark = RC || bndR.x == -2.0f;
        const double ub2 = bnd_ub_sq(xx, cc, l1, fx, gw, 0.0) + 0x1p-20 * (double)cqMax;
        if (nbrMode) {
          // every center outside the neighbourhood: |x - c| >= |c - c_a| -
          // |x - c_a| >= nbrR[a] - (the anchor's fresh upper bound)
          const double ua2 = __builtin_isfinite(LA)
                                 ? bnd_ub_sq(xx, cnA * cnA, (double)LA, fx, gA, 0.0) +
                                       0x1p-20 * (double)cqMax
                                 : __builtin_inf();
          const double Ln = ((double)RA - __builtin_sqrt(ua2) * (1.0 + 0x1p-50)) * (1.0 - 0x1p-50);
          lnc0 = Ln > 0.0 ? fdown(Ln) : -1.0f;
        }
        if (RC && decided) {
          // every center outside the set: |x - c| >= lnc0, above the winner
          // by the reference's slack (the filter's test)
          const double L = (double)lnc0, tau = 0x1p-29 * (xx + dp->cmax2) + 0x1p-48 * (L * L + ub2);
          decided = lnc0 >= 0.0f && !dp->bad && L * L - ub2 > tau;
        }
        if (decided && mark && lnc0 >= 0.0f && li == 0) {
          const float ub = bnd_dist_up(ub2);
          // (l2 = +inf: a set of one, nothing but the outside bound)
          const float lb = __builtin_isfinite(l2)
                               ? bnd_dist_dn(bnd_lb_sq(xx, l2, fx, 0.0, 0x1p-20 * (double)cqMax))
                               : __builtin_inff();
          bnd[row] = ub < 0x1p120f ? make_float2(ub, __builtin_fminf(lb, lnc0))
                                   : make_float2(-1.0f, -1.0f);
          if ((!RC || nbrMode) && sets && ub < 0x1p120f) {
            // the set and its outside bound, for the next iterations' re-checks
            lncA[row] = lnc0;
#pragma unroll
            for (int i = 0; i < kCandMax; ++i) sets[(size_t)row * kCandMax + i] = ci[i];
          }
        }
      }
    }
    if (RC) decided = decided && bnd != nullptr;
    if (live && li == 0) {
      if (RC) {
        if (decided) assign[row] = I1;
        state[row] = decided ? 0 : 1;
      } else if (decided) {
        assign[row] = I1;
      } else {
        const unsigned o = atomicAdd(outCount, 1u);
        outRows[o] = (int32_t)row;
#pragma unroll
        for (int i = 0; i < kCandMax; ++i) outCands[(size_t)o * kCandMax + i] = ci[i];
      }
    }
  }
}

// The re-check of the carried candidate sets and neighbourhoods (the rows of
// bounds_filter's list; k_screen_cands3<.., RC>'s arithmetic, bit for bit)
// in two phases per batch of kRcBatch listed rows.  Phase A, 2S lanes a row
// as in k_screen_cands3: the limb products of the row's <= kCandMax
// candidates, their f32 lower bounds L, and the row's best two, its
// anchor's bound and its flags into LDS.  Phase B, one row a lane: the fp64
// certification, the outside-bound test, the bounds and the state.  In
// k_screen_cands3 every lane of a row ran that fp64 tail (~170 f64 of ~700
// VALU instructions a 4-row step): the kernel was VALU-issue bound (neither
// five waves per SIMD nor rows grouped by center changed its time).
constexpr int kRcBatch = 256;
template <int S>
__global__ __launch_bounds__(kRcBatch) void k_recheck(
    const uint4* __restrict__ Xq, const int2* __restrict__ meta, const double* __restrict__ xnorm,
    int d, const uint4* __restrict__ Cr, const float* __restrict__ cq,
    const double* __restrict__ g, const double* __restrict__ cnorm,
    const CenterParams* __restrict__ prm, const int32_t* __restrict__ candRows,
    const unsigned int* __restrict__ candCount, int32_t* __restrict__ assign,
    float2* __restrict__ bnd, float* __restrict__ lncA, int32_t* __restrict__ sets,
    unsigned char* __restrict__ state, const DriftParams* __restrict__ dp,
    const int32_t* __restrict__ nbr, const float* __restrict__ nbrR,
    int32_t* __restrict__ failList, unsigned int* __restrict__ failCount,
    unsigned long long* __restrict__ failCum) {
  constexpr int P16 = 2 * S;        // 16-byte pieces of a limb plane
  constexpr int LPR = 8;            // lanes per row, PPL pieces each
  __shared__ unsigned sFail, sFailBase;
  constexpr int PPL = P16 / LPR;
  constexpr int RPW = 64 / LPR;     // rows per wave and step; LPR steps fill a wave's 64 slots
  static_assert(P16 % LPR == 0, "whole pieces per lane");
  __shared__ int sRow[kRcBatch], sI1[kRcBatch], sA0[kRcBatch], sMx[kRcBatch], sMy[kRcBatch],
      sFl[kRcBatch];
  __shared__ float sL1[kRcBatch], sL2[kRcBatch], sLA[kRcBatch], sCq[kRcBatch];
  const unsigned cnt = *candCount;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, q = lane / LPR, li = lane % LPR;
  const CenterParams P = *prm;
  const auto cR = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Cr, (short)0, (int)std::min<int64_t>((int64_t)P.k * 3 * P16 * 16, 0x7fffffff),
      0x00020000);
  for (unsigned bb = blockIdx.x * kRcBatch; bb < cnt; bb += gridDim.x * kRcBatch) {
    if (t == 0) sFail = 0u;   // (ordered by the barrier after phase A)
    // ---- phase A
    for (int gi = 0; gi < LPR; ++gi) {
      const int slot = wave * 64 + gi * RPW + q;
      const unsigned idx = bb + slot;
      const bool live = idx < cnt;
      // (a slot past the list reads the batch's first entry, then drops it:
      // every load below is unconditional)
      const int32_t rw = candRows[live ? idx : bb];
      const bool nbrMode = rw < 0;   // ~row: the neighbourhood of its center
      const int64_t row = nbrMode ? ~(int64_t)rw : (int64_t)rw;
      const int32_t* setp = nbrMode ? nbr + (size_t)assign[row] * kCandMax
                                    : sets + (size_t)row * kCandMax;
      int ci[kCandMax];
      static_assert(kCandMax % 2 == 0, "sets read as int2");
#pragma unroll
      for (int i = 0; i < kCandMax; i += 2) {
        const int2 v = *reinterpret_cast<const int2*>(setp + i);   // 8-byte aligned rows
        ci[i] = live ? v.x : -1;
        ci[i + 1] = live ? v.y : -1;
      }
      const uint4* xr = Xq + row * (3 * P16) + li;
      uint4 xa[PPL], xb[PPL], xc[PPL];
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        xa[j] = xr[j * LPR];
        xb[j] = xr[P16 + j * LPR];
        xc[j] = xr[2 * P16 + j * LPR];
      }
      const int2 mt0 = meta[row];
      const int2 mt = live ? mt0 : make_int2(INT_MIN, 0);
      float cqv[kCandMax];
#pragma unroll
      for (int i = 0; i < kCandMax; ++i) cqv[i] = cq[(unsigned)ci[i] < (unsigned)P.k ? ci[i] : 0];
      // T = 2^7 S1 + S2 summed per lane (integers: exact in any order; the
      // row's total is k_screen_cands3's T), and S3
      int tt[kCandMax], s3[kCandMax];
#pragma unroll
      for (int i = 0; i < kCandMax; ++i) {
        const int c = ci[i];
        // an empty slot reads zeros without a memory access (out of range)
        const unsigned off =
            (unsigned)c < (unsigned)P.k ? (unsigned)(c * 3 * P16 + li) * 16u : 0x80000000u;
        int ti = 0, si = 0;
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
          const unsigned o = off + 16u * LPR * j;
          const uint4 ca = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(cR, (int)o, 0, 0));
          const uint4 cb = __builtin_bit_cast(
              uint4, __builtin_amdgcn_raw_buffer_load_b128(cR, (int)(o + 16u * P16), 0, 0));
          const uint4 cc = __builtin_bit_cast(
              uint4, __builtin_amdgcn_raw_buffer_load_b128(cR, (int)(o + 32u * P16), 0, 0));
          ti = dot16(xb[j], ca, dot16(xa[j], cb, ti + dot16(xa[j], ca, 0) * 128));
          si = dot16(xc[j], ca, dot16(xb[j], cb, dot16(xa[j], cc, si)));
        }
        tt[i] = ti;
        s3[i] = si;
      }
      // sums over the row's 8 lanes by DPP: quad_perm [1,0,3,2], [2,3,0,1],
      // then row_half_mirror (lane i of a half with lane 7 - i: the other quad)
#pragma unroll
      for (int i = 0; i < kCandMax; ++i) {
        tt[i] += __builtin_amdgcn_update_dpp(0, tt[i], 0xB1, 0xF, 0xF, false);
        s3[i] += __builtin_amdgcn_update_dpp(0, s3[i], 0xB1, 0xF, 0xF, false);
        tt[i] += __builtin_amdgcn_update_dpp(0, tt[i], 0x4E, 0xF, 0xF, false);
        s3[i] += __builtin_amdgcn_update_dpp(0, s3[i], 0x4E, 0xF, 0xF, false);
        tt[i] += __builtin_amdgcn_update_dpp(0, tt[i], 0x141, 0xF, 0xF, false);
        s3[i] += __builtin_amdgcn_update_dpp(0, s3[i], 0x141, 0xF, 0xF, false);
      }
      // the three-limb bounds L = cq - F1 (T + S3 2^-7), rounded toward -inf.
      // The empty asm statements pin every rounding operation between the
      // two mode switches (the compiler does not order FP arithmetic against
      // s_setreg: without them it scheduled five candidates' conversions and
      // FMAs after the switch back)
      __builtin_amdgcn_s_setreg(0x801, 2);
#pragma unroll
      for (int i = 0; i < kCandMax; ++i) asm volatile("" : "+v"(tt[i]), "+v"(s3[i]));
      const float F1 = mt.x == INT_MIN ? 0.0f : __builtin_ldexpf(1.0f, mt.x + P.ec - 20);
      float L1 = __builtin_inff(), L2 = __builtin_inff(), LA = __builtin_inff(), cqMax = 0.0f;
      int I1 = -1;
      bool bad = false;
      // (branch-free: an empty slot's L = +inf changes none of L1, L2, I1)
#pragma unroll
      for (int i = 0; i < kCandMax; ++i) {
        const int c = ci[i];
        const bool ok = c >= 0 && c < P.k;
        bad = bad || c >= P.k;   // a padding center
        const float V = __builtin_fmaf((float)s3[i], 0x1p-7f, (float)tt[i]);
        const float L = ok ? __builtin_fmaf(-F1, V, cqv[i]) : __builtin_inff();
        if (i == 0) LA = L;
        cqMax = ok ? __builtin_fmaxf(cqMax, __builtin_fabsf(cqv[i])) : cqMax;
        const bool lt = L < L1;
        L2 = __builtin_amdgcn_fmed3f(L1, L2, L);
        I1 = lt ? c : I1;
        L1 = lt ? L : L1;
      }
      asm volatile("" : "+v"(L1), "+v"(L2), "+v"(LA), "+v"(cqMax), "+v"(I1));
      __builtin_amdgcn_s_setreg(0x801, 0);
      if (li == 0) {
        sRow[slot] = live ? (int)row : -1;
        sI1[slot] = I1;
        sA0[slot] = ci[0];
        sMx[slot] = mt.x;
        sMy[slot] = mt.y;
        sFl[slot] = (bad ? 1 : 0) | (nbrMode ? 2 : 0);
        sL1[slot] = L1;
        sL2[slot] = L2;
        sLA[slot] = LA;
        sCq[slot] = cqMax;
      }
    }
    __syncthreads();
    // ---- phase B: row sRow[t]
    const int row = sRow[t];
    unsigned rank = ~0u;   // this row's place among the batch's failures
    if (row >= 0) {
      const int I1 = sI1[t], mx = sMx[t], fl = sFl[t];
      const bool bad = fl & 1, nbrMode = fl & 2;
      const double l1 = (double)sL1[t], l2 = (double)sL2[t];
      const float cqMax = sCq[t];
      bool decided = false;
      if (P.ok && !bad && mx != INT_MIN && I1 >= 0 && __builtin_isfinite(l1)) {
        const double xn = xnorm[row], cn = cnorm[I1];
        const double gw = g[I1];
        const double xx = xn * xn, cc = cn * cn;
        const double n1 = (double)__int_as_float(sMy[t]);   // bounds |xh3|_1
        const double fx = err_term(mx, n1, P.mu, d);
        const double M = (4.0 * (fx + gw) + 2.0 * kEpsF * (xx + cc) +
                          0x1p-20 * (__builtin_fabs(l1) + cc + 2.0 * gw) +
                          0x1p-24 * (2.0 * (xx + cc) + __builtin_fabs(l1) +
                                     __builtin_fmin(__builtin_fabs(l2), 0x1p120)) +
                          0x1p-90) *
                         (1.0 + 0x1p-30);
        decided = !__builtin_isfinite(l2) || (l2 - l1) > M;
        // every center outside the set at least lnc0 away (the carried bound,
        // or the neighbourhood's), the other members at least l2
        float lnc0 = lncA[row];
        const double ub2 = bnd_ub_sq(xx, cc, l1, fx, gw, 0.0) + 0x1p-20 * (double)cqMax;
        const int a0 = (sA0[t] >= 0 && sA0[t] < P.k) ? sA0[t] : 0;
        if (nbrMode) {
          // |x - c| >= |c - c_a| - |x - c_a| >= nbrR[a] - (the anchor's fresh upper bound)
          const float LA = sLA[t];
          const double cnA = cnorm[a0];
          const double ua2 = __builtin_isfinite(LA)
                                 ? bnd_ub_sq(xx, cnA * cnA, (double)LA, fx, g[a0], 0.0) +
                                       0x1p-20 * (double)cqMax
                                 : __builtin_inf();
          const double Ln =
              ((double)nbrR[a0] - __builtin_sqrt(ua2) * (1.0 + 0x1p-50)) * (1.0 - 0x1p-50);
          lnc0 = Ln > 0.0 ? fdown(Ln) : -1.0f;
        }
        if (decided) {
          // above the winner by the reference's slack (the filter's test)
          const double L = (double)lnc0, tau = 0x1p-29 * (xx + dp->cmax2) + 0x1p-48 * (L * L + ub2);
          decided = lnc0 >= 0.0f && !dp->bad && L * L - ub2 > tau;
        }
        if (decided) {
          const float ub = bnd_dist_up(ub2);
          // (l2 = +inf: a set of one, nothing but the outside bound)
          const float lb = __builtin_isfinite(l2)
                               ? bnd_dist_dn(bnd_lb_sq(xx, l2, fx, 0.0, 0x1p-20 * (double)cqMax))
                               : __builtin_inff();
          bnd[row] = ub < 0x1p120f ? make_float2(ub, __builtin_fminf(lb, lnc0))
                                   : make_float2(-1.0f, -1.0f);
          if (nbrMode && ub < 0x1p120f) {
            // the neighbourhood (slot 0: a itself) becomes the row's carried set
            lncA[row] = lnc0;
#pragma unroll
            for (int i = 0; i < kCandMax; ++i)
              sets[(size_t)row * kCandMax + i] = nbr[(size_t)a0 * kCandMax + i];
          }
        }
      }
      if (decided) assign[row] = I1;
      state[row] = decided ? 0 : 1;
      if (failList && !decided) rank = atomicAdd(&sFail, 1u);
    }
    if (failList) {
      // the failures behind the filter's state-1 rows in the screen's list:
      // one reservation per workgroup and batch
      __syncthreads();
      if (t == 0 && sFail) {
        sFailBase = atomicAdd(failCount, sFail);
        atomicAdd(failCum, (unsigned long long)sFail);
      }
      __syncthreads();
      if (rank != ~0u) failList[sFailBase + rank] = row;
    }
    __syncthreads();   // the records are rewritten by the next batch
  }
}

template <int S>
int launch_cands3(const CandArgs& ca, const void* img, const int2* meta, const double* xnorm,
                  int64_t n, int d, const void* Cb, const float* cq, const double* g,
                  const double* cnorm, const CenterParams* prm, int ktp, int32_t* assign,
                  int32_t* outRows, int32_t* outCands, unsigned int* outCount, hipStream_t st,
                  unsigned int scap, const Bounds* bd = nullptr) {
  KernelTimer timer("k_kmeans_cands3", st);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 127) / 128, 4096));
  // the center-major copy behind the fragment image (k_centers_pack32)
  const uint4* Cr = (const uint4*)Cb + (size_t)ktp * S * 3 * 64;
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_screen_cands3<S, 16>), dim3(grid), dim3(256), 0, st,
                     (const uint4*)img, meta, xnorm, d, Cr, cq, g, cnorm, prm,
                     (const int32_t*)ca.candRows, (const int32_t*)ca.cands,
                     (const unsigned int*)ca.candCount, assign, outRows, outCands, outCount, scap,
                     bd ? bd->ub_lb : nullptr, bd ? bd->lnc : nullptr, bd ? bd->sets : nullptr,
                     nullptr, nullptr, nullptr, nullptr);
  CYC_LAUNCH_CHECK("k_screen_cands3");
  return CYC_OK;
}

int launch_cands(const CandArgs& ca, int64_t n, int d, int32_t* assign, int32_t* list,
                 unsigned int* listCount, hipStream_t st, unsigned int scap = 0) {
  KernelTimer timer("k_kmeans_cands", st);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 127) / 128, 4096));
  hipLaunchKernelGGL(k_screen_cands, dim3(grid), dim3(256), 0, st, ca.X, ca.xnorm, d, ca.C,
                     ca.cnorm, ca.k, ca.unit, ca.margin, (const int32_t*)ca.candRows, (const int32_t*)ca.cands,
                     (const unsigned int*)ca.candCount, assign, list, listCount, scap);
  CYC_LAUNCH_CHECK("k_screen_cands");
  return CYC_OK;
}

// Sharded appends, compacted (kmeans_i8.hpp) in ONE launch: every block's
// first wave scans the kShards counters (64 values) for its shard's base
// behind *dstCount, the block copies that shard's entries there, and the last
// block to finish (a completion counter in shard 0's spare slot) clears the
// counters and advances *dstCount.  (A scan launch + a copy launch took ~5
// us each, nine pairs per screen call.)
struct CompactJob {
  unsigned int* counts;
  const int32_t* src;
  int32_t* dst;
  int width;
  const int32_t* src2;
  int32_t* dst2;
  int width2;
  unsigned int* dstCount;
};
constexpr int kMaxCompactJobs = 4;
struct CompactJobs {
  CompactJob j[kMaxCompactJobs];
};
__device__ __forceinline__ void shard_compact(const CompactJob& J, unsigned int cap) {
  __shared__ unsigned sb[2];
  const int j = blockIdx.y;
  unsigned int* counts = J.counts;
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    const unsigned c = counts[l * kShardStride];
    unsigned incl = c;
#pragma unroll
    for (int m = 1; m < kShards; m <<= 1) {
      const unsigned o = __shfl_up(incl, m);
      if (l >= m) incl += o;
    }
    if (l == j) {
      sb[0] = incl - c;
      sb[1] = c;
    }
  }
  const unsigned old = *J.dstCount;   // advanced only by the last block
  __syncthreads();
  if (J.dst) {
    const size_t base = (size_t)old + sb[0], c = sb[1];
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const int32_t* s1 = J.src + (size_t)j * cap * J.width;
    int32_t* d1 = J.dst + base * J.width;
    for (size_t i = t0; i < c * J.width; i += stride) d1[i] = s1[i];
    if (J.src2) {
      const int32_t* s2 = J.src2 + (size_t)j * cap * J.width2;
      int32_t* d2 = J.dst2 + base * J.width2;
      for (size_t i = t0; i < c * J.width2; i += stride) d2[i] = s2[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // no fence: this block's counter and count reads have returned (their
    // values were used above), and the copies reach the next launch at the
    // kernel boundary
    const unsigned blocks = gridDim.x * gridDim.y;
    if (atomicAdd(&counts[3], 1u) == blocks - 1) {
      // every block of this job has read the counters and *dstCount
      unsigned tot = 0;
      for (int l = 0; l < kShards; ++l) {
        tot += counts[l * kShardStride];
        counts[l * kShardStride] = 0u;
      }
      *J.dstCount = old + tot;
      counts[3] = 0u;
    }
  }
}
// Sharded appends, compacted (kmeans_i8.hpp) in ONE launch: every block's
// first wave scans the kShards counters (64 values) for its shard's base
// behind *dstCount, the block copies that shard's entries there, and the last
// block to finish (a completion counter in shard 0's spare slot) clears the
// counters and advances *dstCount.  (A scan launch + a copy launch took ~5
// us each, nine pairs per screen call.)  Up to kMaxCompactJobs independent
// compactions (distinct count sets and destination counters) share one
// launch, one per blockIdx.z.
__global__ __launch_bounds__(256) void k_shard_compact(CompactJobs jobs, unsigned int cap) {
  shard_compact(jobs.j[blockIdx.z], cap);
}

int compact_jobs(const CompactJob* jobs, int nj, unsigned int cap, hipStream_t st) {
  if (nj <= 0) return CYC_OK;
  KernelTimer timer("k_kmeans_compact", st);
  CompactJobs J{};
  bool anyDst = false;
  for (int i = 0; i < nj; ++i) {
    J.j[i] = jobs[i];
    anyDst = anyDst || jobs[i].dst;
  }
  // two blocks per shard: the completion counter's returning atomics
  // serialise (~11 ns each), 16 per shard measured 3x the two launches
  hipLaunchKernelGGL(k_shard_compact, anyDst ? dim3(2, kShards, nj) : dim3(1, 1, nj), dim3(256), 0,
                     st, J, cap);
  CYC_LAUNCH_CHECK("k_shard_compact");
  return CYC_OK;
}

int compact(unsigned int* counts, unsigned int cap, const int32_t* src, int32_t* dst, int width,
            const int32_t* src2, int32_t* dst2, int width2, unsigned int* dstCount,
            hipStream_t st) {
  const CompactJob j{counts, src, dst, width, src2, dst2, width2, dstCount};
  return compact_jobs(&j, 1, cap, st);
}

// Two-limb pass over every row; its undecided rows with a small candidate
// set get exact fp64 distances to those candidates (k_screen_cands), the
// others the three-limb pass.  With `stg` (and ca) every 32x32 kernel
// appends through its shards, compacted after each launch.
// Up to 8 counter ranges zeroed in one launch (a block per range).
struct ZeroArgs {
  unsigned int* p[8];
  int w[8];
  int n;
};
__global__ __launch_bounds__(256) void k_zero_counters(ZeroArgs z) {
  unsigned int* q = z.p[blockIdx.x];
  for (int i = threadIdx.x; i < z.w[blockIdx.x]; i += 256) q[i] = 0u;
}

template <int S, int W>
int screen32(const void* img, const int2* meta, const double* xnorm, int64_t n, int d,
             const void* Cb, const float* cq, const double* g, const double* cnorm,
             const CenterParams* prm, int ktp, int32_t* assign, int32_t* list,
             unsigned int* listCount, int32_t* list2, unsigned int* list2Count,
             const CandArgs* ca, hipStream_t st, const RefineArgs* ra = nullptr,
             const AppendStage* stg = nullptr, const Bounds* bd = nullptr) {
  const AppendStage* sg = ca ? stg : nullptr;
  const unsigned scap = sg ? sg->cap : 0u;
  {
    // every counter of the pass zeroed by one launch (six fills before)
    ZeroArgs z{};
    auto add = [&](unsigned int* q, int words) {
      if (q) {
        z.p[z.n] = q;
        z.w[z.n++] = words;
      }
    };
    add(list2Count, 1);
    if (ca) {
      add(ca->candCount, 1);
      add(ca->candCount2, 1);
    }
    if (ra && ca) {
      add(ra->cand1Count, 1);
      add(ra->fullCount, 2);
    }
    add(sg ? sg->counts : nullptr, kSets * kShards * kShardStride);
    if (z.n) {
      hipLaunchKernelGGL(k_zero_counters, dim3(z.n), dim3(256), 0, st, z);
      CYC_LAUNCH_CHECK("k_zero_counters");
    }
  }
  // append targets: the stage's shards, or the lists themselves
  auto A = [&](int32_t* staged, int32_t* direct) { return sg ? staged : direct; };
  auto N = [&](int set, unsigned int* direct) { return sg ? sg->set(set) : direct; };
  int rc;
  // the two-limb kernels' outputs: list2 (rows) and the candidate lists
  auto compact2 = [&]() -> int {
    if (!sg) return CYC_OK;
    const CompactJob jb[2] = {
        {sg->set(kSetRowsA), sg->rowsA, list2, 1, nullptr, nullptr, 0, list2Count},
        {sg->set(kSetCand), sg->candRows, ca->candRows, 1, sg->cands, ca->cands, kCandMax,
         ca->candCount}};
    return compact_jobs(jb, 2, scap, st);
  };
  if (ra && ca) {
    // one-limb pass over every center; the two-limb refinement over the
    // union of the listed rows' candidates; the full two-limb pass over the
    // rows neither can handle (fullList).  With carried bounds (bd) the
    // rows bounds_filter sent to a re-check against their carried candidate
    // sets go first (k_screen_cands3<.., true>), then the one-limb pass
    // screens only the rows that need a full screen.
    if (bd && bd->rcRows) {
      {
        KernelTimer timer("k_kmeans_recheck", st);
        // CYC_KMEANS_RECHECK=1: the one-phase form (k_screen_cands3<.., true>)
        static const bool onePhase = [] {
          const char* e = std::getenv("CYC_KMEANS_RECHECK");
          return e && e[0] == '1';
        }();
        if (onePhase) {
          const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 127) / 128, 4096));
          hipLaunchKernelGGL(HIP_KERNEL_NAME(k_screen_cands3<S, 16, true>), dim3(grid), dim3(256), 0,
                             st, (const uint4*)img, meta, xnorm, d,
                             (const uint4*)Cb + (size_t)ktp * S * 3 * 64, cq, g, cnorm, prm,
                             bd->rcRows, (const int32_t*)bd->sets, bd->rcCount, assign, nullptr,
                             nullptr, nullptr, 0u, bd->ub_lb, bd->lnc, bd->sets, bd->state, bd->dp,
                             bd->nbr, bd->nbrR);
          CYC_LAUNCH_CHECK("k_screen_cands3 (re-check)");
        } else {
          const unsigned grid = (unsigned)std::max<int64_t>(
              1, std::min<int64_t>((n + kRcBatch - 1) / kRcBatch, 2048));
          hipLaunchKernelGGL(HIP_KERNEL_NAME(k_recheck<S>), dim3(grid), dim3(kRcBatch), 0, st,
                             (const uint4*)img, meta, xnorm, d,
                             (const uint4*)Cb + (size_t)ktp * S * 3 * 64, cq, g, cnorm, prm,
                             bd->rcRows, bd->rcCount, assign, bd->ub_lb, bd->lnc, bd->sets,
                             bd->state, bd->dp, bd->nbr, bd->nbrR,
                             bd->collected ? bd->list : nullptr,
                             bd->collected ? bd->listCount : nullptr,
                             bd->collected ? bd->cum : nullptr);
          CYC_LAUNCH_CHECK("k_recheck");
        }
      }
      if (bd->dump) dump_dev("state_rc", bd->state, (size_t)bd->n, st);
      if (!(bd->collected && recheck_two_phase()) && (rc = bounds_collect(*bd, st))) return rc;
    }
    if (bd && bd->rowsIn)
      rc = launch_screen32<S, W, 1, true>(
          img, meta, xnorm, n, d, Cb, cq + (size_t)ktp * 64, g + (size_t)ktp * 64, cnorm, prm,
          ktp, bd->rowsIn, bd->rowsInCount, assign, A(sg ? sg->rowsA : nullptr, ra->fullList),
          N(kSetRowsA, ra->fullCount), st, A(sg ? sg->candRows : nullptr, ra->cand1Rows),
          A(sg ? sg->cands : nullptr, ra->cand1), N(kSetCand, ra->cand1Count), scap, bd->ub_lb);
    else
      rc = launch_screen32<S, W, 1, false>(
          img, meta, xnorm, n, d, Cb, cq + (size_t)ktp * 64, g + (size_t)ktp * 64, cnorm, prm,
          ktp, nullptr, nullptr, assign, A(sg ? sg->rowsA : nullptr, ra->fullList),
          N(kSetRowsA, ra->fullCount), st, A(sg ? sg->candRows : nullptr, ra->cand1Rows),
          A(sg ? sg->cands : nullptr, ra->cand1), N(kSetCand, ra->cand1Count), scap,
          bd ? bd->ub_lb : nullptr);
    if (rc) return rc;
    if (sg) {
      // (independent: distinct count sets and destinations, one launch)
      const CompactJob jb[2] = {
          {sg->set(kSetRowsA), sg->rowsA, ra->fullList, 1, nullptr, nullptr, 0, ra->fullCount},
          {sg->set(kSetCand), sg->candRows, ra->cand1Rows, 1, sg->cands, ra->cand1, kCand1,
           ra->cand1Count}};
      if ((rc = compact_jobs(jb, 2, scap, st))) return rc;
    }
    {
      KernelTimer timer("k_kmeans_refine2", st);
      hipLaunchKernelGGL(HIP_KERNEL_NAME(k_screen32r<S>), dim3((unsigned)((n + 127) / 128)),
                         dim3(256), 0, st, (const uint4*)img, meta, xnorm, n, d, (const uint4*)Cb,
                         cq + (size_t)ktp * 32, g + (size_t)ktp * 32, cnorm, prm, ra->kstride,
                         (const int32_t*)ra->cand1Rows, (const unsigned int*)ra->cand1Count,
                         (const int32_t*)ra->cand1, assign, A(sg ? sg->rowsA : nullptr, list2),
                         N(kSetRowsA, list2Count), A(sg ? sg->candRows : nullptr, ca->candRows),
                         A(sg ? sg->cands : nullptr, ca->cands), N(kSetCand, ca->candCount),
                         A(sg ? sg->rowsB : nullptr, ra->fullList), N(kSetRowsB, ra->fullCount),
                         N(kSetStat, ra->fullCount + 1), scap, bd ? bd->ub_lb : nullptr);
      CYC_LAUNCH_CHECK("k_screen32r");
    }
    if (sg) {
      // the refinement's four outputs: distinct count sets and counters
      const CompactJob jb[4] = {
          {sg->set(kSetRowsA), sg->rowsA, list2, 1, nullptr, nullptr, 0, list2Count},
          {sg->set(kSetCand), sg->candRows, ca->candRows, 1, sg->cands, ca->cands, kCandMax,
           ca->candCount},
          {sg->set(kSetRowsB), sg->rowsB, ra->fullList, 1, nullptr, nullptr, 0, ra->fullCount},
          {sg->set(kSetStat), nullptr, nullptr, 0, nullptr, nullptr, 0, ra->fullCount + 1}};
      if ((rc = compact_jobs(jb, 4, scap, st))) return rc;
    }
    rc = launch_screen32<S, W, 2, true>(
        img, meta, xnorm, n, d, Cb, cq + (size_t)ktp * 32, g + (size_t)ktp * 32, cnorm, prm, ktp,
        ra->fullList, ra->fullCount, assign, A(sg ? sg->rowsA : nullptr, list2),
        N(kSetRowsA, list2Count), st, A(sg ? sg->candRows : nullptr, ca->candRows),
        A(sg ? sg->cands : nullptr, ca->cands), N(kSetCand, ca->candCount), scap);
  } else {
    rc = launch_screen32<S, W, 2, false>(
        img, meta, xnorm, n, d, Cb, cq + (size_t)ktp * 32, g + (size_t)ktp * 32, cnorm, prm, ktp,
        nullptr, nullptr, assign, A(sg ? sg->rowsA : nullptr, list2), N(kSetRowsA, list2Count),
        st, ca ? A(sg ? sg->candRows : nullptr, ca->candRows) : nullptr,
        ca ? A(sg ? sg->cands : nullptr, ca->cands) : nullptr,
        ca ? N(kSetCand, ca->candCount) : nullptr, scap);
  }
  if (rc || (rc = compact2())) return rc;
  if (!ca)
    return launch_screen32<S, W, 3, true>(img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, ktp,
                                          list2, list2Count, assign, list, listCount, st);
  // the three-limb pass (rows with more than kCandMax candidates) and the
  // candidate pass touch disjoint rows and only append to `list` (through
  // two separate shard sets with a stage), so either order, or side by
  // side, gives the same result.  Side by side: a side stream of this host
  // thread (one per device: a host thread may drive plans on several GPUs;
  // the caller's DeviceGuard made `st`'s device current).
  // The three-limb pass (0.19 ms of work: ~115K rows on config 2) runs on
  // the main stream before the candidate pass: beside it on a side stream
  // (CYC_KMEANS_SIDE=1, the round-4 form) the two shared the CUs and the
  // iteration measured 9.77 vs 9.71 ms (same box, interleaved).
  // the three-limb tier of the candidate rows (CandArgs::candRows2 set):
  // the rows it cannot certify go on, with their candidates, to the fp64
  // candidate pass
  CandArgs caF = *ca;
  if (ca->candRows2) {
    if ((rc = launch_cands3<S>(*ca, img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, ktp, assign,
                               A(sg ? sg->candRows : nullptr, ca->candRows2),
                               A(sg ? sg->cands : nullptr, ca->cands2),
                               N(kSetCand, ca->candCount2), st, scap, bd)))
      return rc;
    if (sg && (rc = compact(sg->set(kSetCand), scap, sg->candRows, ca->candRows2, 1, sg->cands,
                            ca->cands2, kCandMax, ca->candCount2, st)))
      return rc;
    caF.candRows = ca->candRows2;
    caF.cands = ca->cands2;
    caF.candCount = ca->candCount2;
  }
  static const bool sideStream = [] {
    const char* e = std::getenv("CYC_KMEANS_SIDE");
    return e && e[0] == '1';
  }();
  if (!sideStream) {
    if ((rc = launch_screen32<S, W, 3, true>(img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, ktp,
                                             list2, list2Count, assign,
                                             A(sg ? sg->rowsA : nullptr, list),
                                             N(kSetRowsA, listCount), st, nullptr, nullptr,
                                             nullptr, scap)) ||
        (rc = launch_cands(caF, n, d, assign, A(sg ? sg->rowsB : nullptr, list),
                           N(kSetRowsB, listCount), st, scap)))
      return rc;
  } else {
  constexpr int kMaxDev = 64;
  thread_local hipStream_t sides[kMaxDev] = {};
  thread_local hipEvent_t forks[kMaxDev] = {}, joins[kMaxDev] = {};
  int dev = 0;
  CYC_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDev) {
    cyc::set_error("device index out of range");
    return CYC_ERR_INVALID_ARG;
  }
  if (!sides[dev]) {
    CYC_HIP(hipStreamCreateWithFlags(&sides[dev], hipStreamNonBlocking));
    CYC_HIP(hipEventCreateWithFlags(&forks[dev], hipEventDisableTiming));
    CYC_HIP(hipEventCreateWithFlags(&joins[dev], hipEventDisableTiming));
  }
  hipStream_t side = sides[dev];
  hipEvent_t fork = forks[dev], join = joins[dev];
  CYC_HIP(hipEventRecord(fork, st));
  CYC_HIP(hipStreamWaitEvent(side, fork, 0));
  if ((rc = launch_screen32<S, W, 3, true>(img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, ktp,
                                           list2, list2Count, assign,
                                           A(sg ? sg->rowsA : nullptr, list),
                                           N(kSetRowsA, listCount), side, nullptr, nullptr,
                                           nullptr, scap)))
    return rc;
  rc = launch_cands(caF, n, d, assign, A(sg ? sg->rowsB : nullptr, list), N(kSetRowsB, listCount),
                    st, scap);
  CYC_HIP(hipEventRecord(join, side));
  CYC_HIP(hipStreamWaitEvent(st, join, 0));
  if (rc) return rc;
  }
  if (sg && ((rc = compact(sg->set(kSetRowsA), scap, sg->rowsA, list, 1, nullptr, nullptr, 0,
                           listCount, st)) ||
             (rc = compact(sg->set(kSetRowsB), scap, sg->rowsB, list, 1, nullptr, nullptr, 0,
                           listCount, st))))
    return rc;
  return CYC_OK;
}

// ---------------------------------------------------------------------------
// Cross-iteration bounds (kmeans_i8.hpp Bounds).

// One wave per center: the drift |C_c - Cp_c| and |C_c|^2, both rounded up
// (fp64 sums of d <= 256 squares: relative error < (d + 2) 2^-53 < 2^-44),
// then Cp_c = C_c.
__global__ __launch_bounds__(256) void k_center_drift(const double* __restrict__ C,
                                                      double* __restrict__ Cp, int k, int d,
                                                      double* __restrict__ delta,
                                                      double* __restrict__ ccs) {
  const int lane = threadIdx.x & 63;
  const int c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (c >= k) return;
  double s = 0.0, q = 0.0;
  for (int j = lane; j < d; j += 64) {
    const double v = C[(int64_t)c * d + j], o = Cp[(int64_t)c * d + j];
    const double t = v - o;
    s += t * t;
    q += v * v;
    Cp[(int64_t)c * d + j] = v;
  }
  s = wave_sum(s);
  q = wave_sum(q);
  if (lane == 0) {
    delta[c] = __builtin_sqrt(s) * (1.0 + 0x1p-40) + 0x1p-500;
    ccs[c] = q * (1.0 + 0x1p-40);
  }
}

// Single block: the two largest drifts (and the largest one's center) and
// max |c|^2; any non-finite drift or norm sets `bad`.
__global__ __launch_bounds__(1024) void k_drift_top(const double* __restrict__ delta,
                                                    const double* __restrict__ ccs, int k,
                                                    DriftParams* __restrict__ prm) {
  __shared__ double s1[1024], s2[1024], sc[1024];
  __shared__ int si[1024];
  const int t = threadIdx.x;
  double d1 = 0.0, d2 = 0.0, cm = 0.0;
  int i1 = -1;
  bool bad = false;
  for (int c = t; c < k; c += 1024) {
    const double v = delta[c], q = ccs[c];
    bad = bad || !(v <= 0x1p1000) || !(q <= 0x1p1000);   // NaN, inf
    if (v > d1 || i1 < 0) {
      d2 = i1 < 0 ? 0.0 : d1;
      d1 = v;
      i1 = c;
    } else if (v > d2) {
      d2 = v;
    }
    cm = __builtin_fmax(cm, q);
  }
  s1[t] = d1;
  s2[t] = d2;
  si[t] = i1;
  sc[t] = cm;
  bad = __syncthreads_or(bad);
  for (int off = 512; off > 0; off >>= 1) {
    if (t < off && si[t + off] >= 0) {
      const double a1 = s1[t], a2 = s2[t], b1 = s1[t + off], b2 = s2[t + off];
      const bool aEmpty = si[t] < 0;
      if (aEmpty || b1 > a1) {
        s1[t] = b1;
        si[t] = si[t + off];
        s2[t] = aEmpty ? b2 : __builtin_fmax(a1, b2);
      } else {
        s2[t] = __builtin_fmax(a2, b1);
      }
      sc[t] = __builtin_fmax(sc[t], sc[t + off]);
    }
    __syncthreads();
  }
  if (t == 0) {
    DriftParams p;
    p.d1 = s1[0];
    p.d2 = s2[0];
    p.i1 = si[0];
    p.cmax2 = sc[0];
    p.bad = bad ? 1 : 0;
    *prm = p;
  }
}

// The listed rows of a kBndRows-row block in row order: tmp[block *
// kBndRows ...], their count in bcount[block] (masks: the wave's ballot of
// `listed` per 256-row step it, wc: IT x 4 counts in LDS)
constexpr int kBndIT = kBndRows / 256;
__device__ __forceinline__ void bnd_block_list(const unsigned long long (&masks)[kBndIT],
                                               unsigned* wc, int64_t base, int32_t* tmp,
                                               unsigned int* bcount,
                                               const unsigned long long* flips = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int it = 0; it < kBndIT; ++it) {
    unsigned before = 0;
    for (int j = 0; j < it * 4 + wave; ++j) before += wc[j];
    if ((masks[it] >> lane) & 1ull)
      tmp[base + before + (unsigned)__builtin_popcountll(masks[it] & below)] =
          (flips && ((flips[it] >> lane) & 1ull)) ? ~(int32_t)(base + it * 256 + tid)
                                                  : (int32_t)(base + it * 256 + tid);
  }
  if (tid == 0) {
    unsigned total = 0;
    for (int j = 0; j < kBndIT * 4; ++j) total += wc[j];
    bcount[blockIdx.x] = total;
  }
}

// Each center's neighbourhood (one wave per center) from the packed
// statistics 0.25 dist^2 (computeStatistics, exact to ~2^-45): nbr[a] =
// a and its kCandMax - 1 nearest other centers (-1 padding when k is
// smaller), nbrR[a] = a lower bound of the distance from c_a to every
// other center (the next nearest; +inf when none is left).
__global__ __launch_bounds__(64) void k_center_nbrs(const double* __restrict__ stats, int k,
                                                    int32_t* __restrict__ nbr,
                                                    float* __restrict__ nbrR) {
  const int a = blockIdx.x, lane = threadIdx.x;
  constexpr int T = kCandMax;   // kCandMax - 1 members + the next one
  double v[T];
  int ix[T];
#pragma unroll
  for (int i = 0; i < T; ++i) {
    v[i] = INFINITY;
    ix[i] = -1;
  }
  for (int j = lane; j < k; j += 64) {
    if (j == a) continue;
    const int64_t pi = a <= j ? (int64_t)j * (j + 1) / 2 + a : (int64_t)a * (a + 1) / 2 + j;
    double x = stats[pi];
    if (!(x >= 0.0)) x = INFINITY;   // NaN centers: the drift voids the bounds anyway
    // insert into the lane's sorted T smallest
    if (x < v[T - 1]) {
      double cv = x;
      int ci = j;
#pragma unroll
      for (int i = 0; i < T; ++i) {
        const bool sw = cv < v[i];
        const double tv = v[i];
        const int ti = ix[i];
        v[i] = sw ? cv : v[i];
        ix[i] = sw ? ci : ix[i];
        cv = sw ? tv : cv;
        ci = sw ? ti : ci;
      }
    }
  }
  // T rounds: the wave's smallest head, popped from its lane
  if (lane == 0) nbr[(int64_t)a * kCandMax] = a;
  for (int t = 0; t < T; ++t) {
    double bv = v[0];
    int bl = lane;
    for (int m = 32; m > 0; m >>= 1) {
      const double ov = __shfl_xor(bv, m);
      const int ol = __shfl_xor(bl, m);
      if (ov < bv || (ov == bv && ol < bl)) {
        bv = ov;
        bl = ol;
      }
    }
    const int bi = __shfl(ix[0], bl);
    if (lane == bl) {
#pragma unroll
      for (int i = 0; i < T - 1; ++i) {
        v[i] = v[i + 1];
        ix[i] = ix[i + 1];
      }
      v[T - 1] = INFINITY;
      ix[T - 1] = -1;
    }
    if (lane == 0) {
      if (t < T - 1) {
        nbr[(int64_t)a * kCandMax + 1 + t] = bv < INFINITY ? bi : -1;
      } else {
        // the next nearest: its distance, rounded down, bounds every center
        // outside the neighbourhood
        nbrR[a] = bv < INFINITY ? fdown(__builtin_sqrt(4.0 * bv) * (1.0 - 0x1p-40))
                                : __builtin_inff();
      }
    }
  }
}

// kBndRows rows per workgroup (8 per thread, coalesced): a row keeps its
// assignment when its moved bounds still certify it (kmeans_i8.hpp Bounds,
// state 0); else it is re-checked against its carried set when the set's
// moved outside bound still stands (state 2, listed here), else screened
// (state 1).  Every carried bound is moved by the drift.  Round 6: a row
// left for the screen whose center a has a usable neighbourhood (nbrR[a],
// a lower bound of the distance from c_a to every center outside a and its
// kCandMax - 1 nearest, over twice the row's moved upper bound, or no
// bound at all) is re-checked against that neighbourhood instead (state 3,
// listed as ~row).
__global__ __launch_bounds__(256) void k_bounds_filter(const int32_t* __restrict__ assign,
                                                       float2* __restrict__ bnd,
                                                       float* __restrict__ lnc,
                                                       unsigned char* __restrict__ state,
                                                       const double* __restrict__ xnorm,
                                                       int64_t n, int k,
                                                       const double* __restrict__ delta,
                                                       const DriftParams* __restrict__ prm,
                                                       int32_t* __restrict__ tmp,
                                                       unsigned int* __restrict__ bcount,
                                                       const float* __restrict__ nbrR,
                                                       int32_t* __restrict__ tmp2,
                                                       unsigned int* __restrict__ bcount2) {
  __shared__ unsigned wc[kBndIT * 4], wc2[kBndIT * 4];
  unsigned long long masks2[kBndIT];
  const DriftParams P = *prm;
  unsigned long long flips[kBndIT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kBndRows;
  unsigned long long masks[kBndIT];
#pragma unroll
  for (int it = 0; it < kBndIT; ++it) {
    const int64_t r = base + it * 256 + tid;
    int st = 1;
    if (r < n) {
      const int a = assign[r];
      const float2 b = bnd[r];
      const float ln = lnc[r];
      const bool okA = !P.bad && a >= 0 && a < k;
      if (okA && b.x >= 0.0f && b.y > 0.0f) {
        const double U = (double)b.x + delta[a];
        const double L = (double)b.y - (a == P.i1 ? P.d2 : P.d1);
        // |x| <= |x - c_a| + |c_a| <= U + max |c| (no norm read: 80 MB a
        // call at 10M rows)
        const double xr = U + __builtin_sqrt(P.cmax2);
        const double xx = xr * xr * (1.0 + 0x1p-50);
        const double U2 = U * U, L2 = L * L;
        // the reference's rounding slack, plus this test's own rounding
        const double tau = 0x1p-29 * (xx + P.cmax2) + 0x1p-48 * (L2 + U2) + 0x1p-1000;
        if (L > 0.0 && (L2 - U2) > tau) {
          st = 0;
          bnd[r] = make_float2(fup(U * (1.0 + 0x1p-50)), fdown(L * (1.0 - 0x1p-50)));
        }
      }
      // which re-check: a carried set whose moved outside bound still
      // clears the row's moved upper bound (it will most likely certify);
      // else the neighbourhood when nbrR[a] exceeds twice that bound (or
      // the row has none); else a carried set with any margin left.  Both
      // tests only pick the work: the re-check itself decides.
      const double Ln = ln >= 0.0f && okA ? ((double)ln - P.d1) * (1.0 - 0x1p-50) : -1.0;
      const double Um = okA && b.x >= 0.0f ? (double)b.x + delta[a] : 0.0;
      if (st == 1 && Ln > 0.0 && Ln > Um) st = 2;
      if (st == 1 && nbrR && okA) {
        // (a row without a bound: only when its center moved little
        // against its neighbourhood -- early in a fit such rows mostly fail)
        const double R = (double)nbrR[a];
        if (R > 0.0 && R > 2.0 * Um && (b.x >= 0.0f || delta[a] < 0.125 * R)) st = 3;
      }
      if (st == 1 && Ln > 0.0) st = 2;
      if (ln >= 0.0f)   // a carried set (NaN / negative: none) kept while it has a margin
        lnc[r] = (st == 0 || st == 2) && Ln > 0.0 ? fdown(Ln) : -1.0f;
      state[r] = (unsigned char)st;
    }
    masks[it] = __builtin_amdgcn_ballot_w64(st >= 2);
    flips[it] = __builtin_amdgcn_ballot_w64(st == 3);
    masks2[it] = __builtin_amdgcn_ballot_w64(r < n && st == 1);
    if (lane == 0) {
      wc[it * 4 + wave] = (unsigned)__builtin_popcountll(masks[it]);
      wc2[it * 4 + wave] = (unsigned)__builtin_popcountll(masks2[it]);
    }
  }
  bnd_block_list(masks, wc, base, tmp, bcount, flips);
  if (tmp2) bnd_block_list(masks2, wc2, base, tmp2, bcount2);
}

// The rows a full screen takes (state 1), listed as the filter lists its
// re-checks.
__global__ __launch_bounds__(256) void k_bounds_collect(const unsigned char* __restrict__ state,
                                                        int64_t n, int32_t* __restrict__ tmp,
                                                        unsigned int* __restrict__ bcount) {
  __shared__ unsigned wc[kBndIT * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t base = (int64_t)blockIdx.x * kBndRows;
  unsigned long long masks[kBndIT];
#pragma unroll
  for (int it = 0; it < kBndIT; ++it) {
    const int64_t r = base + it * 256 + tid;
    masks[it] = __builtin_amdgcn_ballot_w64(r < n && state[r] == 1);
    if (lane == 0) wc[it * 4 + wave] = (unsigned)__builtin_popcountll(masks[it]);
  }
  bnd_block_list(masks, wc, base, tmp, bcount);
}

// Single block: bcount[0..nb) -> exclusive offsets, bcount[nb] = *listCount
// = the total, added to *cum.
__global__ __launch_bounds__(1024) void k_bounds_scan(unsigned int* __restrict__ bcount, int64_t nb,
                                                      unsigned int* __restrict__ listCount,
                                                      unsigned long long* __restrict__ cum,
                                                      unsigned int* __restrict__ bcount2 = nullptr,
                                                      unsigned int* __restrict__ listCount2 = nullptr,
                                                      unsigned long long* __restrict__ cum2 = nullptr) {
  __shared__ unsigned part[1024];
  if (blockIdx.x == 1) {   // the second list of the same blocks
    bcount = bcount2;
    listCount = listCount2;
    cum = cum2;
  }
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
    bcount[nb] = part[1023];
    *listCount = part[1023];
    if (cum) *cum += (unsigned long long)part[1023];
  }
}

__global__ __launch_bounds__(256) void k_bounds_scatter(const int32_t* __restrict__ tmp,
                                                        const unsigned int* __restrict__ off,
                                                        int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ tmp2 = nullptr,
                                                        const unsigned int* __restrict__ off2 = nullptr,
                                                        int32_t* __restrict__ list2 = nullptr) {
  if (blockIdx.y == 1) {
    tmp = tmp2;
    off = off2;
    list = list2;
  }
  const int64_t b = blockIdx.x;
  const unsigned o = off[b], c = off[b + 1] - o;
  for (unsigned i = threadIdx.x; i < c; i += 256) list[o + i] = tmp[b * kBndRows + i];
}

template <int KS>
int launch_screen(const void* img, const int2* meta, const double* xnorm, int64_t n, int d,
                  const void* Cb, const float* cq, const double* g, const double* cnorm,
                  const CenterParams* prm, int ktp, int32_t* assign, int32_t* list,
                  unsigned int* listCount, hipStream_t st) {
  constexpr int STR = 12 * KS + 2;
  const size_t lds = (size_t)kBM * STR * 16 + (size_t)kBM * 4;   // slot minima alias the image
  static bool attr = false;
  if (!attr) {
    CYC_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_screen<KS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  KernelTimer timer("k_kmeans_screen3", st);
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_screen<KS>), dim3((unsigned)((n + kBM - 1) / kBM)),
                     dim3(256), lds, st, (const uint4*)img, meta, xnorm, n, d, (const uint4*)Cb,
                     cq, g, cnorm, prm, ktp, assign, list, listCount);
  CYC_LAUNCH_CHECK("k_kmeans_screen_i8");
  return CYC_OK;
}

}  // namespace

int rows_quantize(const double* X, int64_t n, int d, void* img, int2* meta, hipStream_t st,
                  const double* scale, double* unorm) {
  if (n <= 0) return CYC_OK;
  const int D = 64 * ksteps(d);
  const int64_t blocks = std::min<int64_t>((n + 3) / 4, 65536);
  const int vec = (d % 2 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0);
  static const bool pf = [] {   // CYC_QUANT_PF=0: the row-at-a-time kernel
    const char* e = std::getenv("CYC_QUANT_PF");
    return !(e && e[0] == '0');
  }();
  const bool q4 = d % 4 == 0 && reinterpret_cast<uintptr_t>(X) % 32 == 0;
  if (q4 && pf && d <= 256)
    hipLaunchKernelGGL(k_rows_quantize_q4, dim3((unsigned)blocks), dim3(256), 0, st, X, n, d, D,
                       (unsigned*)img, meta, scale, unorm);
  else if (vec && pf && d <= 256)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rows_quantize_pf<2>), dim3((unsigned)blocks), dim3(256), 0,
                       st, X, n, d, D, (unsigned*)img, meta, scale, unorm);
  else if (vec && pf)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rows_quantize_pf<4>), dim3((unsigned)blocks), dim3(256), 0,
                       st, X, n, d, D, (unsigned*)img, meta, scale, unorm);
  else
    hipLaunchKernelGGL(k_rows_quantize, dim3((unsigned)blocks), dim3(256), 0, st, X, n, d, D,
                       (unsigned*)img, meta, scale, unorm, vec);
  CYC_LAUNCH_CHECK("k_rows_quantize");
  return CYC_OK;
}

int centers_prepare(const double* C, const double* cnorm, int k, int d, int ktp, void* Cb,
                    float* cq, double* g, CenterParams* prm, double* scratch, hipStream_t st) {
  const int KS = ksteps(d);
  double* cmax = scratch;
  double* cn1 = scratch + k;
  hipLaunchKernelGGL(k_centers_scan, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, st, C, k, d,
                     cmax, cn1);
  CYC_LAUNCH_CHECK("k_centers_scan");
  hipLaunchKernelGGL(k_centers_params, dim3(1), dim3(256), 0, st, k, (const double*)cmax,
                     (const double*)cn1, prm);
  CYC_LAUNCH_CHECK("k_centers_params");
  if (uses32(d)) {
    // 32-center tiles, an even number of them (ktp 16-center tiles, a
    // multiple of kWaves = 4, cover them), 32-dim substeps
    const int ktp32 = tiles32(k), S = 2 * KS;
    const int64_t total = std::max<int64_t>((int64_t)ktp32 * S * 64, (int64_t)ktp32 * 32);
    hipLaunchKernelGGL(k_centers_pack32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       C, cnorm, k, d, S, ktp32, (const double*)cn1, (const CenterParams*)prm,
                       (uint4*)Cb, cq, g, cq + (size_t)ktp * 16, g + (size_t)ktp * 16,
                       cq + (size_t)ktp * 32, g + (size_t)ktp * 32);
    CYC_LAUNCH_CHECK("k_centers_pack32");
    return CYC_OK;
  }
  const int64_t total = std::max<int64_t>((int64_t)ktp * KS * 64, (int64_t)ktp * 16);
  hipLaunchKernelGGL(k_centers_pack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, C,
                     cnorm, k, d, KS, ktp, (const double*)cn1, (const CenterParams*)prm,
                     (uint4*)Cb, cq, g);
  CYC_LAUNCH_CHECK("k_centers_pack");
  return CYC_OK;
}

int centers_drift(const double* C, double* Cp, int k, int d, double* delta, double* ccs,
                  DriftParams* prm, hipStream_t st) {
  hipLaunchKernelGGL(k_center_drift, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, st, C, Cp, k, d,
                     delta, ccs);
  CYC_LAUNCH_CHECK("k_center_drift");
  hipLaunchKernelGGL(k_drift_top, dim3(1), dim3(1024), 0, st, (const double*)delta,
                     (const double*)ccs, k, prm);
  CYC_LAUNCH_CHECK("k_drift_top");
  return CYC_OK;
}

int bounds_filter(const int32_t* assign, float2* ub_lb, float* lnc, unsigned char* state,
                  const double* xnorm, int64_t n, int k, const double* delta,
                  const DriftParams* prm, int32_t* tmp, unsigned int* bcount, int32_t* rcList,
                  unsigned int* rcCount, unsigned long long* rcCum, const double* stats,
                  int32_t* nbr, float* nbrR, hipStream_t st, int32_t* tmp2,
                  unsigned int* bcount2, int32_t* list1, unsigned int* list1Count,
                  unsigned long long* cum1) {
  const int64_t nb = bounds_blocks(n);
  const bool two = tmp2 && bcount2 && list1 && list1Count;
  if (nb <= 0) return CYC_OK;
  KernelTimer timer("k_kmeans_bounds", st);
  if (stats) {
    hipLaunchKernelGGL(k_center_nbrs, dim3((unsigned)k), dim3(64), 0, st, stats, k, nbr, nbrR);
    CYC_LAUNCH_CHECK("k_center_nbrs");
  }
  hipLaunchKernelGGL(k_bounds_filter, dim3((unsigned)nb), dim3(256), 0, st, assign, ub_lb, lnc,
                     state, xnorm, n, k, delta, prm, tmp, bcount,
                     stats ? (const float*)nbrR : nullptr, two ? tmp2 : nullptr,
                     two ? bcount2 : nullptr);
  CYC_LAUNCH_CHECK("k_bounds_filter");
  // both lists' scans and scatters as one launch each (block / y index 1:
  // the state-1 list)
  hipLaunchKernelGGL(k_bounds_scan, dim3(two ? 2 : 1), dim3(1024), 0, st, bcount, nb, rcCount,
                     rcCum, two ? bcount2 : nullptr, two ? list1Count : nullptr,
                     two ? cum1 : nullptr);
  CYC_LAUNCH_CHECK("k_bounds_scan");
  hipLaunchKernelGGL(k_bounds_scatter, dim3((unsigned)nb, two ? 2 : 1), dim3(256), 0, st,
                     (const int32_t*)tmp, (const unsigned int*)bcount, rcList,
                     two ? (const int32_t*)tmp2 : nullptr,
                     two ? (const unsigned int*)bcount2 : nullptr, two ? list1 : nullptr);
  CYC_LAUNCH_CHECK("k_bounds_scatter");
  return CYC_OK;
}

bool recheck_two_phase() {
  static const bool two = [] {
    const char* e = std::getenv("CYC_KMEANS_RECHECK");
    return !(e && e[0] == '1');
  }();
  return two;
}

// After the re-check: the state-1 rows into the screen's list (bd.list).
int bounds_collect(const Bounds& bd, hipStream_t st) {
  const int64_t nb = bounds_blocks(bd.n);
  if (nb <= 0) return CYC_OK;
  hipLaunchKernelGGL(k_bounds_collect, dim3((unsigned)nb), dim3(256), 0, st,
                     (const unsigned char*)bd.state, bd.n, bd.tmp, bd.bcount);
  CYC_LAUNCH_CHECK("k_bounds_collect");
  hipLaunchKernelGGL(k_bounds_scan, dim3(1), dim3(1024), 0, st, bd.bcount, nb, bd.listCount,
                     bd.cum);
  CYC_LAUNCH_CHECK("k_bounds_scan");
  hipLaunchKernelGGL(k_bounds_scatter, dim3((unsigned)nb), dim3(256), 0, st,
                     (const int32_t*)bd.tmp, (const unsigned int*)bd.bcount, bd.list);
  CYC_LAUNCH_CHECK("k_bounds_scatter");
  return CYC_OK;
}

int screen(const void* img, const int2* meta, const double* xnorm, int64_t n, int d,
           const void* Cb, const float* cq, const double* g, const double* cnorm,
           const CenterParams* prm, int ktp, int32_t* assign, int32_t* list,
           unsigned int* listCount, int32_t* list2, unsigned int* list2Count, hipStream_t st,
           const CandArgs* ca, const RefineArgs* ra, const AppendStage* stg,
           const Bounds* bd) {
  if (n <= 0) return CYC_OK;
  if (stg && stg->cap < shard_cap(n)) {
    set_error("append stage smaller than shard_cap(n)");
    return CYC_ERR_INVALID_ARG;
  }
  if (bd && !(ra && ca && uses32(d))) {
    set_error("carried bounds need the one-limb pass (d <= 256, refinement, candidate pass)");
    return CYC_ERR_INVALID_ARG;
  }
  if (uses32(d)) {
    const int k32 = ktp * 16 / 32;   // launch over the padded center range (cq = +inf)
    switch (ksteps(d)) {
      case 2: return screen32<4, 4>(img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, k32, assign, list, listCount, list2, list2Count, ca, st, ra, stg, bd);
      default: return screen32<8, 4>(img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, k32, assign, list, listCount, list2, list2Count, ca, st, ra, stg, bd);
    }
  }
  switch (ksteps(d)) {
#define CYC_S8(K) \
  case K: return launch_screen<K>(img, meta, xnorm, n, d, Cb, cq, g, cnorm, prm, ktp, assign, list, listCount, st);
    CYC_S8(2) CYC_S8(4) CYC_S8(6) CYC_S8(8)
#undef CYC_S8
    default:
      set_error("the i8 screen supports d <= 512");
      return CYC_ERR_UNSUPPORTED;
  }
}

}  // namespace km8
}  // namespace cyc
