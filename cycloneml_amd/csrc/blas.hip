// blas.hip -- netlib-compatible per-call BLAS on gfx950 (layer 1 of the
// boundary): the Fortran-ABI symbols dev.ludovic.netlib's
// JNIBLAS binds when -Ddev.ludovic.netlib.blas.nativeLib[Path] points at
// libcyclone_blas.so (docs/ml-linalg-guide.md:59-75), plus cblas_* entry
// points.  Called from ml/linalg/BLAS.scala:85,145,284,336,422,630 and
// mllib/linalg/BLAS.scala:268,404,572.
//
// Host pointers in, host pointers out, synchronous, column-major, LP64 int32
// dimensions -- the netlib contract.  Every call stages its operands through
// a per-thread device scratch on a per-thread stream (reentrant across the
// executor threads that share the process-wide BLAS singleton,
// BLAS.scala:29-30).  The copies make this layer slow for 1 MiB blocks; it
// exists so that any netlib call site works unchanged.  The hot paths use
// the device-resident entry points of cyclone.h instead.
//
// Argument errors follow netlib's XERBLA numbering and are reported through
// cyc_last_error() (the call then returns without touching outputs).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cctype>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"

namespace {

constexpr int GT = 64;        // dgemm tile (GT x GT per workgroup, 4 waves x 32 x 32)
constexpr int GK = 16;        // k chunk
constexpr int AS = GK + 2;    // As row stride (== 2 mod 32 doubles)
constexpr int BS = GT + 16;   // Bs row stride (== 16 mod 32 doubles)

// C(m x n) = alpha op(A) op(B) + beta C, column-major, fp64 MFMA.
__global__ __launch_bounds__(256) void k_dgemm(int ta, int tb, int m, int n, int k, double alpha,
                                               const double* __restrict__ A, int lda,
                                               const double* __restrict__ B, int ldb,
                                               double beta, double* __restrict__ C, int ldc) {
  __shared__ double As[GT * AS];   // op(A)[i][p]
  __shared__ double Bs[GK * BS];   // op(B)[p][j]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.x * GT, j0 = blockIdx.y * GT;
  const int wi = (wave >> 1) * 32, wj = (wave & 1) * 32;
  cyc_double4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = cyc_double4{0.0, 0.0, 0.0, 0.0};
  for (int p0 = 0; p0 < k; p0 += GK) {
    __syncthreads();
    for (int e = tid; e < GT * GK; e += 256) {
      // op(A)[i][p]: A is m x k ('N') or k x m ('T')
      const int i = e / GK, p = e % GK;
      const int gi = i0 + i, gp = p0 + p;
      double v = 0.0;
      if (gi < m && gp < k) v = ta ? A[gi * (size_t)lda + gp] : A[gp * (size_t)lda + gi];
      As[i * AS + p] = v;
    }
    for (int e = tid; e < GT * GK; e += 256) {
      const int p = e / GT, j = e % GT;
      const int gj = j0 + j, gp = p0 + p;
      double v = 0.0;
      if (gj < n && gp < k) v = tb ? B[gp * (size_t)ldb + gj] : B[gj * (size_t)ldb + gp];
      Bs[p * BS + j] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        a[q] = As[(wi + q * 16 + (lane & 15)) * AS + kk + (lane >> 4)];
        b[q] = Bs[(kk + (lane >> 4)) * BS + wj + q * 16 + (lane & 15)];
      }
#pragma unroll
      for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          acc[qa][qb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[qa], b[qb], acc[qa][qb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = i0 + wi + qa * 16 + (lane >> 4) + 4 * r;
        const int gj = j0 + wj + qb * 16 + (lane & 15);
        if (gi < m && gj < n) {
          double* c = C + gj * (size_t)ldc + gi;
          // netlib: beta == 0 overwrites C (no 0*NaN), else alpha*temp + beta*c
          *c = (beta == 0.0) ? alpha * acc[qa][qb][r] : alpha * acc[qa][qb][r] + beta * *c;
        }
      }
}

__global__ void k_scale_matrix(int m, int n, double beta, double* C, int ldc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
  if (i < m) C[j * (size_t)ldc + i] = beta == 0.0 ? 0.0 : beta * C[j * (size_t)ldc + i];
}

// y(i) = beta y(i) + alpha sum_j A(i,j) x(j), one thread per row ('N').
__global__ void k_dgemv_n(int m, int n, double alpha, const double* __restrict__ A, int lda,
                          const double* __restrict__ x, double beta, double* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double t = 0.0;
  for (int j = 0; j < n; ++j) t += A[j * (size_t)lda + i] * x[j];
  const double yb = beta == 0.0 ? 0.0 : (beta == 1.0 ? y[i] : beta * y[i]);
  y[i] = yb + alpha * t;
}

// y(j) = beta y(j) + alpha sum_i A(i,j) x(i), one wave per column ('T').
__global__ void k_dgemv_t(int m, int n, double alpha, const double* __restrict__ A, int lda,
                          const double* __restrict__ x, double beta, double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (j >= n) return;
  double t = 0.0;
  for (int i = lane; i < m; i += 64) t += A[j * (size_t)lda + i] * x[i];
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) t += __shfl_xor(t, s);
  t = __shfl(t, 0);
  if (lane == 0) {
    const double yb = beta == 0.0 ? 0.0 : (beta == 1.0 ? y[j] : beta * y[j]);
    y[j] = yb + alpha * t;
  }
}

// netlib dspr / dsyr (upper or lower): a(i,j) += x(i) * (alpha x(j))
__global__ void k_dspr(int upper, int n, double alpha, const double* __restrict__ x,
                       double* __restrict__ ap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
  if (i >= n || x[j] == 0.0) return;
  const double t = alpha * x[j];
  if (upper) {
    if (i <= j) ap[(size_t)j * (j + 1) / 2 + i] += x[i] * t;
  } else {
    if (i >= j) ap[(size_t)j * (2 * (size_t)n - j + 1) / 2 + (i - j)] += x[i] * t;
  }
}

__global__ void k_dsyr(int upper, int n, double alpha, const double* __restrict__ x,
                       double* __restrict__ a, int lda) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
  if (i >= n || x[j] == 0.0) return;
  if (upper ? i <= j : i >= j) a[j * (size_t)lda + i] += x[i] * (alpha * x[j]);
}

__global__ void k_dger(int m, int n, double alpha, const double* __restrict__ x,
                       const double* __restrict__ y, double* __restrict__ a, int lda) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
  if (i >= m || y[j] == 0.0) return;
  a[j * (size_t)lda + i] += x[i] * (alpha * y[j]);
}

// y = alpha AP x + beta y, AP symmetric packed (netlib dspmv), thread per row.
__global__ void k_dspmv(int upper, int n, double alpha, const double* __restrict__ ap,
                        const double* __restrict__ x, double beta, double* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double t = 0.0;
  for (int j = 0; j < n; ++j) {
    const int r = upper ? min(i, j) : max(i, j), c = upper ? max(i, j) : min(i, j);
    const size_t idx = upper ? (size_t)c * (c + 1) / 2 + r
                             : (size_t)c * (2 * (size_t)n - c + 1) / 2 + (r - c);
    t += ap[idx] * x[j];
  }
  const double yb = beta == 0.0 ? 0.0 : (beta == 1.0 ? y[i] : beta * y[i]);
  y[i] = yb + alpha * t;
}

// Dot and sum of squares in a fixed order (bitwise reproducible): block b
// sums the grid-strided elements its threads own into out[1 + b] by a
// fixed tree; k_dot_final adds the blocks' partials in block order.
constexpr int kDotBlocks = 1024;
__global__ __launch_bounds__(256) void k_dot(int n, const double* __restrict__ x,
                                             const double* __restrict__ y,
                                             double* __restrict__ out, int square) {
  __shared__ double sh[256];
  double a = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    a += square ? x[i] * x[i] : x[i] * y[i];
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[1 + blockIdx.x] = sh[0];
}

__global__ void k_dot_final(int nb, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += out[1 + b];
  out[0] = s;
}

__global__ void k_axpy(int n, double a, const double* __restrict__ x, double* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = y[i] + a * x[i];
}

__global__ void k_scal(int n, double a, double* __restrict__ x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = a * x[i];
}

// ------------------------------------------------------------ host side
struct Ctx {
  hipStream_t st = nullptr;
  cyc::DeviceBuffer buf[4];
  double* reserve(int slot, size_t doubles) {
    if (buf[slot].reserve(sizeof(double) * std::max<size_t>(doubles, 1))) return nullptr;
    return (double*)buf[slot].ptr;
  }
};

// One context per calling thread.  Deliberately never destroyed: thread-exit
// destructors of the main thread run after the HIP runtime has torn down.
Ctx* ctx() {
  static thread_local Ctx* c = nullptr;
  if (!c) {
    Ctx* n = new Ctx();
    if (hipStreamCreateWithFlags(&n->st, hipStreamNonBlocking) != hipSuccess) {
      delete n;
      return nullptr;
    }
    c = n;
  }
  return c;
}

bool xerbla(const char* name, int info) {
  cyc::set_error(std::string(" ** On entry to ") + name + " parameter number " +
                 std::to_string(info) + " had an illegal value");
  return false;
}

inline char up(const char* c) { return (char)std::toupper((unsigned char)c[0]); }

// a contiguous view of a host vector: the caller's own memory when inc == 1
// (no host copy), else gathered into tmp by the BLAS negative-stride rule
const double* view(int n, const double* x, int inc, std::vector<double>& tmp);

// gather a strided host vector into a contiguous one (BLAS negative-stride rule)
std::vector<double> gather(int n, const double* x, int inc) {
  std::vector<double> v((size_t)std::max(n, 0));
  const long start = inc < 0 ? (long)(1 - n) * inc : 0;
  for (int i = 0; i < n; ++i) v[i] = x[start + (long)i * inc];
  return v;
}
void scatter(int n, const std::vector<double>& v, double* x, int inc) {
  const long start = inc < 0 ? (long)(1 - n) * inc : 0;
  for (int i = 0; i < n; ++i) x[start + (long)i * inc] = v[i];
}
const double* view(int n, const double* x, int inc, std::vector<double>& tmp) {
  if (inc == 1) return x;
  tmp = gather(n, x, inc);
  return tmp.data();
}
// the host destination of a device result: x itself when inc == 1, else tmp
// (scattered by scatter_back afterwards)
double* out_view(int n, double* x, int inc, std::vector<double>& tmp) {
  if (inc == 1) return x;
  tmp.assign((size_t)std::max(n, 0), 0.0);
  return tmp.data();
}
void scatter_back(int n, const std::vector<double>& tmp, double* x, int inc) {
  if (inc != 1) scatter(n, tmp, x, inc);
}

// copy a column-major host matrix (rows x cols, leading dim ld) to/from device
bool h2d(double* d, const double* h, int rows, int cols, int ld, hipStream_t st) {
  return hipMemcpy2DAsync(d, sizeof(double) * rows, h, sizeof(double) * ld, sizeof(double) * rows,
                          cols, hipMemcpyHostToDevice, st) == hipSuccess;
}
bool d2h(double* h, const double* d, int rows, int cols, int ld, hipStream_t st) {
  return hipMemcpy2DAsync(h, sizeof(double) * ld, d, sizeof(double) * rows, sizeof(double) * rows,
                          cols, hipMemcpyDeviceToHost, st) == hipSuccess;
}
bool fail(const char* what) {
  cyc::set_error(std::string("cyclone BLAS: ") + what + " failed: " +
                 hipGetErrorString(hipGetLastError()));
  return false;
}

bool gemm(char ta, char tb, int m, int n, int k, double alpha, const double* A, int lda,
          const double* B, int ldb, double beta, double* C, int ldc) {
  cyc::set_error("");
  const bool nota = ta == 'N', notb = tb == 'N';
  const int nrowa = nota ? m : k, nrowb = notb ? k : n;
  int info = 0;
  if (!nota && ta != 'C' && ta != 'T') info = 1;
  else if (!notb && tb != 'C' && tb != 'T') info = 2;
  else if (m < 0) info = 3;
  else if (n < 0) info = 4;
  else if (k < 0) info = 5;
  else if (lda < std::max(1, nrowa)) info = 8;
  else if (ldb < std::max(1, nrowb)) info = 10;
  else if (ldc < std::max(1, m)) info = 13;
  if (info) return xerbla("DGEMM ", info);
  if (m == 0 || n == 0 || ((alpha == 0.0 || k == 0) && beta == 1.0)) return true;
  Ctx* c = ctx();
  if (!c) return fail("stream");
  double* dC = c->reserve(2, (size_t)m * n);
  if (!dC || !h2d(dC, C, m, n, ldc, c->st)) return fail("copy C");
  if (alpha == 0.0 || k == 0) {
    hipLaunchKernelGGL(k_scale_matrix, dim3((m + 255) / 256, n), dim3(256), 0, c->st, m, n, beta,
                       dC, m);
  } else {
    const int ar = nota ? m : k, ac = nota ? k : m, br = notb ? k : n, bc = notb ? n : k;
    double* dA = c->reserve(0, (size_t)ar * ac);
    double* dB = c->reserve(1, (size_t)br * bc);
    if (!dA || !dB || !h2d(dA, A, ar, ac, lda, c->st) || !h2d(dB, B, br, bc, ldb, c->st))
      return fail("copy A/B");
    hipLaunchKernelGGL(k_dgemm, dim3((m + GT - 1) / GT, (n + GT - 1) / GT), dim3(256), 0, c->st,
                       nota ? 0 : 1, notb ? 0 : 1, m, n, k, alpha, dA, ar, dB, br, beta, dC, m);
  }
  if (!d2h(C, dC, m, n, ldc, c->st) || hipStreamSynchronize(c->st) != hipSuccess)
    return fail("dgemm");
  return true;
}

bool gemv(char t, int m, int n, double alpha, const double* A, int lda, const double* x, int incx,
          double beta, double* y, int incy) {
  cyc::set_error("");
  int info = 0;
  if (t != 'N' && t != 'T' && t != 'C') info = 1;
  else if (m < 0) info = 2;
  else if (n < 0) info = 3;
  else if (lda < std::max(1, m)) info = 6;
  else if (incx == 0) info = 8;
  else if (incy == 0) info = 11;
  if (info) return xerbla("DGEMV ", info);
  if (m == 0 || n == 0 || (alpha == 0.0 && beta == 1.0)) return true;
  const int lenx = t == 'N' ? n : m, leny = t == 'N' ? m : n;
  Ctx* c = ctx();
  if (!c) return fail("stream");
  std::vector<double> hx = gather(lenx, x, incx), hy = gather(leny, y, incy);
  double* dA = c->reserve(0, (size_t)m * n);
  double* dx = c->reserve(1, lenx);
  double* dy = c->reserve(2, leny);
  if (!dA || !dx || !dy || !h2d(dA, A, m, n, lda, c->st) ||
      hipMemcpyAsync(dx, hx.data(), sizeof(double) * lenx, hipMemcpyHostToDevice, c->st) ||
      hipMemcpyAsync(dy, hy.data(), sizeof(double) * leny, hipMemcpyHostToDevice, c->st))
    return fail("copy");
  const double a = alpha;
  if (t == 'N')
    hipLaunchKernelGGL(k_dgemv_n, dim3((m + 255) / 256), dim3(256), 0, c->st, m, n, a, dA, m, dx,
                       beta, dy);
  else
    hipLaunchKernelGGL(k_dgemv_t, dim3((n + 3) / 4), dim3(256), 0, c->st, m, n, a, dA, m, dx, beta,
                       dy);
  if (hipMemcpyAsync(hy.data(), dy, sizeof(double) * leny, hipMemcpyDeviceToHost, c->st) ||
      hipStreamSynchronize(c->st))
    return fail("dgemv");
  scatter(leny, hy, y, incy);
  return true;
}

// Packed / rank-1 updates share one shape: stage the matrix, x (and y), run.
bool rank1(const char* name, int kind, char uplo, int m, int n, double alpha, const double* x,
           int incx, const double* y, int incy, double* a, int lda) {
  cyc::set_error("");
  const bool upper = uplo == 'U';
  int info = 0;
  if (kind != 2 && uplo != 'U' && uplo != 'L') info = 1;
  else if (kind == 2 && m < 0) info = 1;
  else if (n < 0) info = 2;
  else if (incx == 0) info = 5;
  else if (kind == 2 && incy == 0) info = 7;
  else if (kind == 1 && lda < std::max(1, n)) info = 7;
  else if (kind == 2 && lda < std::max(1, m)) info = 9;
  if (info) return xerbla(name, info);
  const int rows = kind == 2 ? m : n;
  if (rows == 0 || n == 0 || alpha == 0.0) return true;
  Ctx* c = ctx();
  if (!c) return fail("stream");
  std::vector<double> hx = gather(rows, x, incx);
  std::vector<double> hy = kind == 2 ? gather(n, y, incy) : std::vector<double>();
  const size_t asz = kind == 0 ? (size_t)n * (n + 1) / 2 : (size_t)rows * n;
  double* dA = c->reserve(0, asz);
  double* dx = c->reserve(1, rows);
  double* dy = c->reserve(2, n);
  if (!dA || !dx || !dy) return fail("alloc");
  bool ok = (kind == 0 ? hipMemcpyAsync(dA, a, sizeof(double) * asz, hipMemcpyHostToDevice, c->st) ==
                             hipSuccess
                       : h2d(dA, a, rows, n, lda, c->st)) &&
            hipMemcpyAsync(dx, hx.data(), sizeof(double) * rows, hipMemcpyHostToDevice, c->st) ==
                hipSuccess;
  if (kind == 2)
    ok = ok && hipMemcpyAsync(dy, hy.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->st) ==
                   hipSuccess;
  if (!ok) return fail("copy");
  dim3 g((rows + 255) / 256, n);
  if (kind == 0) hipLaunchKernelGGL(k_dspr, g, dim3(256), 0, c->st, upper, n, alpha, dx, dA);
  else if (kind == 1) hipLaunchKernelGGL(k_dsyr, g, dim3(256), 0, c->st, upper, n, alpha, dx, dA, n);
  else hipLaunchKernelGGL(k_dger, g, dim3(256), 0, c->st, m, n, alpha, dx, dy, dA, m);
  ok = (kind == 0 ? hipMemcpyAsync(a, dA, sizeof(double) * asz, hipMemcpyDeviceToHost, c->st) ==
                        hipSuccess
                  : d2h(a, dA, rows, n, lda, c->st)) &&
       hipStreamSynchronize(c->st) == hipSuccess;
  return ok ? true : fail(name);
}

bool level1(int op, int n, double a, const double* x, int incx, double* y, int incy,
            double* result) {
  cyc::set_error("");
  // op: 0 dot, 1 axpy, 2 scal, 3 copy, 4 nrm2
  if (n <= 0) {
    if (result) *result = 0.0;
    return true;
  }
  if (op == 1 && a == 0.0) return true;
  if (op == 3) {
    std::vector<double> hx = gather(n, x, incx);
    scatter(n, hx, y, incy);
    return true;
  }
  Ctx* c = ctx();
  if (!c) return fail("stream");
  std::vector<double> tx, ty;
  const double* hx = view(n, x, incx, tx);
  const double* hy = (op == 0 || op == 1) ? view(n, y, incy, ty) : nullptr;
  double* dx = c->reserve(0, n);
  double* dy = c->reserve(1, n);
  double* dr = c->reserve(2, 1 + kDotBlocks);
  if (!dx || !dy || !dr ||
      hipMemcpyAsync(dx, hx, sizeof(double) * n, hipMemcpyHostToDevice, c->st))
    return fail("copy");
  if (hy && hipMemcpyAsync(dy, hy, sizeof(double) * n, hipMemcpyHostToDevice, c->st))
    return fail("copy");
  const dim3 g((n + 255) / 256);
  if (op == 0 || op == 4) {
    const int nb = (int)std::min<int64_t>(kDotBlocks, ((int64_t)n + 2047) / 2048);
    hipLaunchKernelGGL(k_dot, dim3(nb), dim3(256), 0, c->st, n, dx, dy, dr, op == 4);
    hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(64), 0, c->st, nb, dr);
    double r = 0.0;
    if (hipMemcpyAsync(&r, dr, sizeof(double), hipMemcpyDeviceToHost, c->st) ||
        hipStreamSynchronize(c->st))
      return fail("dot");
    *result = op == 4 ? std::sqrt(r) : r;
    return true;
  }
  if (op == 1) hipLaunchKernelGGL(k_axpy, g, dim3(256), 0, c->st, n, a, dx, dy);
  else hipLaunchKernelGGL(k_scal, g, dim3(256), 0, c->st, n, a, dx);
  double* src = op == 1 ? dy : dx;
  std::vector<double> to;
  double* dst = op == 1 ? out_view(n, y, incy, to) : out_view(n, const_cast<double*>(x), incx, to);
  if (hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToHost, c->st) ||
      hipStreamSynchronize(c->st))
    return fail("level1");
  if (op == 1) scatter_back(n, to, y, incy);
  else scatter_back(n, to, const_cast<double*>(x), incx);
  return true;
}

bool spmv(char uplo, int n, double alpha, const double* ap, const double* x, int incx,
          double beta, double* y, int incy) {
  cyc::set_error("");
  int info = 0;
  if (uplo != 'U' && uplo != 'L') info = 1;
  else if (n < 0) info = 2;
  else if (incx == 0) info = 6;
  else if (incy == 0) info = 9;
  if (info) return xerbla("DSPMV ", info);
  if (n == 0 || (alpha == 0.0 && beta == 1.0)) return true;
  Ctx* c = ctx();
  if (!c) return fail("stream");
  std::vector<double> hx = gather(n, x, incx), hy = gather(n, y, incy);
  const size_t asz = (size_t)n * (n + 1) / 2;
  double* dA = c->reserve(0, asz);
  double* dx = c->reserve(1, n);
  double* dy = c->reserve(2, n);
  if (!dA || !dx || !dy ||
      hipMemcpyAsync(dA, ap, sizeof(double) * asz, hipMemcpyHostToDevice, c->st) ||
      hipMemcpyAsync(dx, hx.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->st) ||
      hipMemcpyAsync(dy, hy.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->st))
    return fail("copy");
  hipLaunchKernelGGL(k_dspmv, dim3((n + 255) / 256), dim3(256), 0, c->st, uplo == 'U', n, alpha, dA,
                     dx, beta, dy);
  if (hipMemcpyAsync(hy.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost, c->st) ||
      hipStreamSynchronize(c->st))
    return fail("dspmv");
  scatter(n, hy, y, incy);
  return true;
}

enum { RowMajor = 101, ColMajor = 102 };
enum { NoTrans = 111, Trans = 112, ConjTrans = 113 };
enum { Upper = 121, Lower = 122 };
inline char tch(int t) { return t == NoTrans ? 'N' : 'T'; }

}  // namespace

extern "C" {

// ---- Fortran ABI (all arguments by reference; hidden string lengths ignored)
void dgemm_(const char* ta, const char* tb, const int* m, const int* n, const int* k,
            const double* alpha, const double* A, const int* lda, const double* B, const int* ldb,
            const double* beta, double* C, const int* ldc) {
  gemm(up(ta), up(tb), *m, *n, *k, *alpha, A, *lda, B, *ldb, *beta, C, *ldc);
}
void dgemv_(const char* t, const int* m, const int* n, const double* alpha, const double* A,
            const int* lda, const double* x, const int* incx, const double* beta, double* y,
            const int* incy) {
  gemv(up(t), *m, *n, *alpha, A, *lda, x, *incx, *beta, y, *incy);
}
void dspr_(const char* uplo, const int* n, const double* alpha, const double* x, const int* incx,
           double* ap) {
  rank1("DSPR  ", 0, up(uplo), *n, *n, *alpha, x, *incx, nullptr, 1, ap, *n);
}
void dsyr_(const char* uplo, const int* n, const double* alpha, const double* x, const int* incx,
           double* a, const int* lda) {
  rank1("DSYR  ", 1, up(uplo), *n, *n, *alpha, x, *incx, nullptr, 1, a, *lda);
}
void dger_(const int* m, const int* n, const double* alpha, const double* x, const int* incx,
           const double* y, const int* incy, double* a, const int* lda) {
  rank1("DGER  ", 2, 'U', *m, *n, *alpha, x, *incx, y, *incy, a, *lda);
}
void dspmv_(const char* uplo, const int* n, const double* alpha, const double* ap, const double* x,
            const int* incx, const double* beta, double* y, const int* incy) {
  spmv(up(uplo), *n, *alpha, ap, x, *incx, *beta, y, *incy);
}
double ddot_(const int* n, const double* x, const int* incx, const double* y, const int* incy) {
  double r = 0.0;
  level1(0, *n, 0.0, x, *incx, const_cast<double*>(y), *incy, &r);
  return r;
}
void daxpy_(const int* n, const double* a, const double* x, const int* incx, double* y,
            const int* incy) {
  level1(1, *n, *a, x, *incx, y, *incy, nullptr);
}
void dscal_(const int* n, const double* a, double* x, const int* incx) {
  if (*incx <= 0) return;   // netlib: no-op for incx <= 0
  level1(2, *n, *a, x, *incx, nullptr, 1, nullptr);
}
void dcopy_(const int* n, const double* x, const int* incx, double* y, const int* incy) {
  level1(3, *n, 0.0, x, *incx, y, *incy, nullptr);
}
double dnrm2_(const int* n, const double* x, const int* incx) {
  if (*incx <= 0) return 0.0;
  double r = 0.0;
  level1(4, *n, 0.0, x, *incx, nullptr, 1, &r);
  return r;
}

// ---- CBLAS
void cblas_dgemm(int layout, int ta, int tb, int m, int n, int k, double alpha, const double* A,
                 int lda, const double* B, int ldb, double beta, double* C, int ldc) {
  if (layout == ColMajor) gemm(tch(ta), tch(tb), m, n, k, alpha, A, lda, B, ldb, beta, C, ldc);
  else gemm(tch(tb), tch(ta), n, m, k, alpha, B, ldb, A, lda, beta, C, ldc);  // C^T = B^T A^T
}
void cblas_dgemv(int layout, int t, int m, int n, double alpha, const double* A, int lda,
                 const double* x, int incx, double beta, double* y, int incy) {
  if (layout == ColMajor) gemv(tch(t), m, n, alpha, A, lda, x, incx, beta, y, incy);
  else gemv(t == NoTrans ? 'T' : 'N', n, m, alpha, A, lda, x, incx, beta, y, incy);
}
void cblas_dspr(int layout, int uplo, int n, double alpha, const double* x, int incx,
                double* ap) {
  char u = uplo == Upper ? 'U' : 'L';
  if (layout == RowMajor) u = u == 'U' ? 'L' : 'U';  // row-major packed upper == col-major lower
  rank1("DSPR  ", 0, u, n, n, alpha, x, incx, nullptr, 1, ap, n);
}
void cblas_dsyr(int layout, int uplo, int n, double alpha, const double* x, int incx, double* a,
                int lda) {
  char u = uplo == Upper ? 'U' : 'L';
  if (layout == RowMajor) u = u == 'U' ? 'L' : 'U';
  rank1("DSYR  ", 1, u, n, n, alpha, x, incx, nullptr, 1, a, lda);
}
void cblas_dger(int layout, int m, int n, double alpha, const double* x, int incx,
                const double* y, int incy, double* a, int lda) {
  if (layout == ColMajor) rank1("DGER  ", 2, 'U', m, n, alpha, x, incx, y, incy, a, lda);
  else rank1("DGER  ", 2, 'U', n, m, alpha, y, incy, x, incx, a, lda);
}
double cblas_ddot(int n, const double* x, int incx, const double* y, int incy) {
  return ddot_(&n, x, &incx, y, &incy);
}
void cblas_daxpy(int n, double a, const double* x, int incx, double* y, int incy) {
  daxpy_(&n, &a, x, &incx, y, &incy);
}
void cblas_dscal(int n, double a, double* x, int incx) { dscal_(&n, &a, x, &incx); }
void cblas_dcopy(int n, const double* x, int incx, double* y, int incy) {
  dcopy_(&n, x, &incx, y, &incy);
}
double cblas_dnrm2(int n, const double* x, int incx) { return dnrm2_(&n, x, &incx); }

}  // extern "C"
