// abi_threads.cpp -- the C ABI driven the way a Spark local[N] executor drives
// it: many task threads of ONE process calling the libraries at once, no
// Python anywhere (tests/test_abi_threads.py runs it on the GPU box).
//
// The reference calls one process-wide netlib singleton from every task
// thread (mllib-local/src/main/scala/org/apache/spark/ml/linalg/BLAS.scala:
// 29-30, 42-56; docs/ml-linalg-guide.md:79-91), and each task aggregates its
// own partition.  Here:
//   part 1  16 pthreads call dgemm_ / dgemv_ / dspr_ / ddot_ (libcyclone_blas.so,
//           include/cyclone_blas.h: per-thread streams and scratch) on distinct
//           operands, three times each, while the others run;
//   part 2  16 pthreads each own a resident dataset (include/cyclone.h
//           cyc_dataset_*) and run four KMeans Lloyd iterations through
//           cyc_kmeans_iter (k = 128: the i8 screen with carried bounds) and
//           two cyc_logreg_binary_eval calls on a CSR dataset, concurrently.
// Every threaded result must equal the same call made alone on the main
// thread BIT FOR BIT, and the single-thread results must match the oracle
// (oracle/liboracle.so: netlib's ddot / dspr loops, findClosest + the Lloyd
// body, BinaryLogisticBlockAggregator.add): KMeans assignments exactly, the
// rest within 1e-10 relative (1e-12 for the BLAS loops).
// Exit status 0 and a last line "abi_threads OK" on success.
#include <pthread.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/cyclone.h"
#include "../include/cyclone_blas.h"

extern "C" {
double orc_ddot(const double* x, const double* y, int64_t n);
void orc_dspr_upper(int64_t n, double alpha, const double* x, double* ap);
double orc_norm2(const double* x, int64_t n);
void orc_kmeans_stats(const double* C, int64_t k, int64_t d, double* packed);
void orc_kmeans_partition(const double* X, const double* xnorm, const double* w, int64_t n,
                          int64_t d, const double* C, const double* cnorm, const double* stats,
                          int64_t k, int32_t* assign, double* dist, double* sums, double* wsum,
                          double* cost);
void orc_binary_logistic_add_csr(int64_t S, int64_t F, const int64_t* rowptr,
                                 const int32_t* colidx, const double* vals, const double* labels,
                                 const double* weights, const double* coef, int fitIntercept,
                                 int fitWithMean, const double* scaledMean, double* grad,
                                 double* lossSum, double* weightSum);
}

namespace {

constexpr int kThreads = 16;
int g_fail = 0;
pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

void fail(const char* what, int t) {
  pthread_mutex_lock(&g_mu);
  ++g_fail;
  std::fprintf(stderr, "FAIL thread %d: %s (%s)\n", t, what, cyc_last_error());
  pthread_mutex_unlock(&g_mu);
}

struct Rng {   // xorshift64*, one per thread
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
  uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 2685821657736338717ull;
  }
  double uni() { return (double)(next() >> 11) * 0x1p-53; }   // [0, 1)
  double sym() { return 2.0 * uni() - 1.0; }
};

bool same_bits(const double* a, const double* b, size_t n) {
  return std::memcmp(a, b, n * sizeof(double)) == 0;
}

bool close_rel(const double* got, const double* ref, size_t n, double tol) {
  double scale = 0.0;
  for (size_t i = 0; i < n; ++i) scale = std::fmax(scale, std::fabs(ref[i]));
  for (size_t i = 0; i < n; ++i)
    if (!(std::fabs(got[i] - ref[i]) <= tol * std::fmax(std::fabs(ref[i]), scale))) return false;
  return true;
}

// ------------------------------------------------------------- part 1: BLAS
struct BlasCase {
  int t;
  int m, n, k;
  char ta, tb, tv;
  std::vector<double> A, B, C0, Av, x, y0, xs, ap0, d1, d2;
  // single-thread results
  std::vector<double> Cref, yref, apref;
  double dref = 0.0;
};

void blas_make(BlasCase& c, int t) {
  Rng r(1000 + t);
  c.t = t;
  c.m = 96 + 8 * t;
  c.n = 80 + 4 * t;
  c.k = 64 + 16 * t;
  c.ta = (t & 1) ? 'T' : 'N';
  c.tb = (t & 2) ? 'T' : 'N';
  c.tv = (t & 1) ? 'T' : 'N';
  c.A.resize((size_t)c.m * c.k);
  c.B.resize((size_t)c.k * c.n);
  c.C0.resize((size_t)c.m * c.n);
  for (auto& v : c.A) v = r.sym();
  for (auto& v : c.B) v = r.sym();
  for (auto& v : c.C0) v = r.sym();
  c.Av.resize((size_t)(300 + t) * (200 + 2 * t));
  for (auto& v : c.Av) v = r.sym();
  c.x.resize(400);
  c.y0.resize(400);
  for (auto& v : c.x) v = r.sym();
  for (auto& v : c.y0) v = r.sym();
  c.xs.resize(200 + t);
  for (auto& v : c.xs) v = r.sym();
  c.ap0.resize(c.xs.size() * (c.xs.size() + 1) / 2);
  for (auto& v : c.ap0) v = r.sym();
  c.d1.resize(100000 + 37 * t);
  c.d2.resize(c.d1.size());
  for (auto& v : c.d1) v = r.sym();
  for (auto& v : c.d2) v = r.sym();
}

// one round of the four calls; outputs into C, y, ap, *dot
void blas_round(const BlasCase& c, std::vector<double>& C, std::vector<double>& y,
                std::vector<double>& ap, double* dot) {
  const double al = 0.7, be = 0.3;
  const int lda = c.ta == 'N' ? c.m : c.k, ldb = c.tb == 'N' ? c.k : c.n, ldc = c.m;
  C = c.C0;
  dgemm_(&c.ta, &c.tb, &c.m, &c.n, &c.k, &al, c.A.data(), &lda, c.B.data(), &ldb, &be, C.data(),
         &ldc);
  const int vm = 300 + c.t, vn = 200 + 2 * c.t, inc = 1;
  y = c.y0;
  dgemv_(&c.tv, &vm, &vn, &al, c.Av.data(), &vm, c.x.data(), &inc, &be, y.data(), &inc);
  const int sn = (int)c.xs.size();
  const double half = 0.5;
  ap = c.ap0;
  dspr_("U", &sn, &half, c.xs.data(), &inc, ap.data());
  const int dn = (int)c.d1.size();
  *dot = ddot_(&dn, c.d1.data(), &inc, c.d2.data(), &inc);
}

// netlib reference loops for dgemm / dgemv (column-major), the oracle's for
// dspr / ddot
bool blas_check_reference(const BlasCase& c) {
  const double al = 0.7, be = 0.3;
  std::vector<double> C = c.C0;
  for (int j = 0; j < c.n; ++j)
    for (int i = 0; i < c.m; ++i) {
      double s = 0.0;
      for (int l = 0; l < c.k; ++l) {
        const double a = c.ta == 'N' ? c.A[(size_t)l * c.m + i] : c.A[(size_t)i * c.k + l];
        const double b = c.tb == 'N' ? c.B[(size_t)j * c.k + l] : c.B[(size_t)l * c.n + j];
        s += a * b;
      }
      C[(size_t)j * c.m + i] = al * s + be * C[(size_t)j * c.m + i];
    }
  const int vm = 300 + c.t, vn = 200 + 2 * c.t;
  const int ylen = c.tv == 'N' ? vm : vn, xlen = c.tv == 'N' ? vn : vm;
  std::vector<double> y(c.y0.begin(), c.y0.begin() + ylen);
  for (int i = 0; i < ylen; ++i) {
    double s = 0.0;
    for (int l = 0; l < xlen; ++l)
      s += (c.tv == 'N' ? c.Av[(size_t)l * vm + i] : c.Av[(size_t)i * vm + l]) * c.x[l];
    y[i] = al * s + be * y[i];
  }
  std::vector<double> ap = c.ap0;
  orc_dspr_upper((int64_t)c.xs.size(), 0.5, c.xs.data(), ap.data());
  const double dot = orc_ddot(c.d1.data(), c.d2.data(), (int64_t)c.d1.size());
  double sabs = 0.0;   // the device sums in another order: bound by sum |x_i y_i|
  for (size_t i = 0; i < c.d1.size(); ++i) sabs += std::fabs(c.d1[i] * c.d2[i]);
  bool ok = close_rel(c.Cref.data(), C.data(), C.size(), 1e-12) &&
            close_rel(c.yref.data(), y.data(), (size_t)ylen, 1e-12) &&
            close_rel(c.apref.data(), ap.data(), ap.size(), 1e-12) &&
            std::fabs(c.dref - dot) <= 1e-12 * sabs;
  return ok;
}

void* blas_thread(void* arg) {
  BlasCase& c = *static_cast<BlasCase*>(arg);
  std::vector<double> C, y, ap;
  for (int rep = 0; rep < 3; ++rep) {
    double dot = 0.0;
    blas_round(c, C, y, ap, &dot);
    if (!same_bits(C.data(), c.Cref.data(), C.size())) fail("dgemm_ differs from its lone call", c.t);
    if (!same_bits(y.data(), c.yref.data(), y.size())) fail("dgemv_ differs from its lone call", c.t);
    if (!same_bits(ap.data(), c.apref.data(), ap.size())) fail("dspr_ differs from its lone call", c.t);
    if (std::memcmp(&dot, &c.dref, sizeof(double)) != 0) fail("ddot_ differs from its lone call", c.t);
  }
  return nullptr;
}

// ---------------------------------------------------------- part 2: datasets
struct DataCase {
  int t;
  // KMeans: n x d dense rows, k centers
  int64_t n = 20000;
  int d = 32, k = 128;
  std::vector<double> X;
  std::vector<double> C0;
  // per iteration (single-thread run): centers used, assign, sums, wsum, cost
  std::vector<std::vector<double>> Cs, sums, wsums;
  std::vector<std::vector<int32_t>> assigns;
  std::vector<double> costs;
  // binary LR on CSR rows
  int64_t m = 20000;
  int F = 3000;
  std::vector<int64_t> rowptr;
  std::vector<int32_t> colidx;
  std::vector<double> vals, labels, weights, coef, scaledMean;
  std::vector<std::vector<double>> grads;
  std::vector<double> losses, wts;
};

void data_make(DataCase& c, int t) {
  Rng r(5000 + t);
  c.t = t;
  // 64 well-separated blobs: near-ties where two centers share a blob
  std::vector<double> blob(64 * (size_t)c.d);
  for (auto& v : blob) v = 6.0 * r.sym();
  c.X.resize((size_t)c.n * c.d);
  for (int64_t i = 0; i < c.n; ++i) {
    const size_t b = (size_t)(r.next() % 64);
    for (int j = 0; j < c.d; ++j) c.X[(size_t)i * c.d + j] = blob[b * c.d + j] + r.sym();
  }
  c.C0.assign(c.X.begin(), c.X.begin() + (size_t)c.k * c.d);
  c.rowptr.assign(1, 0);
  for (int64_t i = 0; i < c.m; ++i) {
    int col = (int)(r.next() % 40);
    while (col < c.F) {
      c.colidx.push_back(col);
      c.vals.push_back(r.sym());
      col += 1 + (int)(r.next() % 360);
    }
    c.rowptr.push_back((int64_t)c.colidx.size());
  }
  c.labels.resize(c.m);
  c.weights.resize(c.m);
  for (int64_t i = 0; i < c.m; ++i) {
    c.labels[i] = r.uni() < 0.4 ? 1.0 : 0.0;
    c.weights[i] = 0.25 + r.uni();
  }
  c.coef.resize(c.F + 1);
  for (auto& v : c.coef) v = 0.2 * r.sym();
  c.scaledMean.resize(c.F);
  for (auto& v : c.scaledMean) v = 0.01 * r.uni();
}

// the Lloyd loop over a dataset: 4 iterations, host centroid update; returns
// false on a library error.  record: keep the per-iteration outputs in c
// (single-thread reference) or compare with them (threaded).
bool data_run(DataCase& c, bool record) {
  cyc_dataset km = nullptr, lr = nullptr;
  if (cyc_dataset_dense_create(c.d, c.n, 0, 0, &km) ||
      cyc_dataset_append_dense(km, c.X.data(), nullptr, nullptr, c.n)) {
    fail("dense dataset", c.t);
    return false;
  }
  std::vector<double> C = c.C0, sums((size_t)c.k * c.d), wsum(c.k);
  std::vector<int32_t> a(c.n);
  bool ok = true;
  for (int it = 0; it < 4 && ok; ++it) {
    std::fill(sums.begin(), sums.end(), 0.0);
    std::fill(wsum.begin(), wsum.end(), 0.0);
    double cost = 0.0;
    if (cyc_kmeans_iter(km, C.data(), c.k, sums.data(), wsum.data(), &cost, a.data())) {
      fail("cyc_kmeans_iter", c.t);
      ok = false;
      break;
    }
    if (record) {
      c.Cs.push_back(C);
      c.assigns.push_back(a);
      c.sums.push_back(sums);
      c.wsums.push_back(wsum);
      c.costs.push_back(cost);
    } else if (a != c.assigns[it] || !same_bits(sums.data(), c.sums[it].data(), sums.size()) ||
               !same_bits(wsum.data(), c.wsums[it].data(), wsum.size()) ||
               std::memcmp(&cost, &c.costs[it], sizeof(double)) != 0) {
      fail("cyc_kmeans_iter differs from its lone run", c.t);
      ok = false;
    }
    for (int q = 0; q < c.k; ++q)   // centroid (DistanceMeasure.scala:200-203)
      if (wsum[q] > 0)
        for (int j = 0; j < c.d; ++j) C[(size_t)q * c.d + j] = (1.0 / wsum[q]) * sums[(size_t)q * c.d + j];
  }
  cyc_dataset_destroy(km);
  if (!ok) return false;
  if (cyc_dataset_csr_create(c.F, c.m, (int64_t)c.colidx.size(), 1, 1, &lr) ||
      cyc_dataset_append_csr(lr, c.rowptr.data(), c.colidx.data(), c.vals.data(),
                             c.labels.data(), c.weights.data(), c.m)) {
    fail("csr dataset", c.t);
    return false;
  }
  for (int ev = 0; ev < 2 && ok; ++ev) {
    std::vector<double> grad(c.F + 1, 0.0), coef = c.coef;
    for (auto& v : coef) v *= 1.0 + ev;
    double loss = 0.0, wt = 0.0;
    if (cyc_logreg_binary_eval(lr, coef.data(), 1, 1, c.scaledMean.data(), grad.data(), &loss,
                               &wt)) {
      fail("cyc_logreg_binary_eval", c.t);
      ok = false;
      break;
    }
    if (record) {
      c.grads.push_back(grad);
      c.losses.push_back(loss);
      c.wts.push_back(wt);
    } else if (!same_bits(grad.data(), c.grads[ev].data(), grad.size()) ||
               std::memcmp(&loss, &c.losses[ev], sizeof(double)) != 0 ||
               std::memcmp(&wt, &c.wts[ev], sizeof(double)) != 0) {
      fail("cyc_logreg_binary_eval differs from its lone run", c.t);
      ok = false;
    }
  }
  cyc_dataset_destroy(lr);
  return ok;
}

bool data_check_reference(const DataCase& c) {
  std::vector<double> xn(c.n);
  for (int64_t i = 0; i < c.n; ++i) xn[i] = orc_norm2(c.X.data() + (size_t)i * c.d, c.d);
  for (size_t it = 0; it < c.Cs.size(); ++it) {
    const std::vector<double>& C = c.Cs[it];
    std::vector<double> cn(c.k), st((size_t)c.k * (c.k + 1) / 2), sums((size_t)c.k * c.d, 0.0),
        wsum(c.k, 0.0), dist(c.n);
    for (int q = 0; q < c.k; ++q) cn[q] = orc_norm2(C.data() + (size_t)q * c.d, c.d);
    orc_kmeans_stats(C.data(), c.k, c.d, st.data());
    std::vector<int32_t> a(c.n);
    double cost = 0.0;
    orc_kmeans_partition(c.X.data(), xn.data(), nullptr, c.n, c.d, C.data(), cn.data(),
                         st.data(), c.k, a.data(), dist.data(), sums.data(), wsum.data(), &cost);
    if (a != c.assigns[it]) {
      std::fprintf(stderr, "thread %d iteration %zu: assignments differ from the oracle\n", c.t, it);
      return false;
    }
    if (!close_rel(c.sums[it].data(), sums.data(), sums.size(), 1e-10) ||
        !same_bits(c.wsums[it].data(), wsum.data(), wsum.size()) ||
        std::fabs(c.costs[it] - cost) > 1e-10 * cost) {
      std::fprintf(stderr, "thread %d iteration %zu: sums / weights / cost off\n", c.t, it);
      return false;
    }
  }
  for (size_t ev = 0; ev < c.grads.size(); ++ev) {
    std::vector<double> grad(c.F + 1, 0.0), coef = c.coef;
    for (auto& v : coef) v *= 1.0 + ev;
    double loss = 0.0, wt = 0.0;
    orc_binary_logistic_add_csr(c.m, c.F, c.rowptr.data(), c.colidx.data(), c.vals.data(),
                                c.labels.data(), c.weights.data(), coef.data(), 1, 1,
                                c.scaledMean.data(), grad.data(), &loss, &wt);
    if (!close_rel(c.grads[ev].data(), grad.data(), grad.size(), 1e-10) ||
        std::fabs(c.losses[ev] - loss) > 1e-10 * std::fabs(loss) ||
        std::fabs(c.wts[ev] - wt) > 1e-12 * wt) {
      std::fprintf(stderr, "thread %d evaluation %zu: logistic state off the oracle\n", c.t, ev);
      return false;
    }
  }
  return true;
}

void* data_thread(void* arg) {
  data_run(*static_cast<DataCase*>(arg), false);
  return nullptr;
}

int run_threads(void* (*fn)(void*), void* base, size_t stride) {
  pthread_t th[kThreads];
  for (int t = 0; t < kThreads; ++t)
    if (pthread_create(&th[t], nullptr, fn, static_cast<char*>(base) + t * stride)) return 1;
  for (int t = 0; t < kThreads; ++t) pthread_join(th[t], nullptr);
  return 0;
}

}  // namespace

int main() {
  // part 1: per-call BLAS
  std::vector<BlasCase> bc(kThreads);
  for (int t = 0; t < kThreads; ++t) {
    blas_make(bc[t], t);
    blas_round(bc[t], bc[t].Cref, bc[t].yref, bc[t].apref, &bc[t].dref);   // alone
    if (!blas_check_reference(bc[t])) fail("BLAS result off the reference loops", t);
  }
  if (run_threads(blas_thread, bc.data(), sizeof(BlasCase))) return 2;
  std::printf("part 1: %d threads x 3 rounds of dgemm_/dgemv_/dspr_/ddot_: %s\n", kThreads,
              g_fail ? "FAILED" : "bitwise equal to lone calls");
  // part 2: one resident dataset per thread
  std::vector<DataCase> dc(kThreads);
  for (int t = 0; t < kThreads; ++t) {
    data_make(dc[t], t);
    if (!data_run(dc[t], true)) return 1;   // alone
    if (!data_check_reference(dc[t])) fail("dataset results off the oracle", t);
  }
  if (run_threads(data_thread, dc.data(), sizeof(DataCase))) return 2;
  std::printf("part 2: %d threads x (4 cyc_kmeans_iter + 2 cyc_logreg_binary_eval): %s\n",
              kThreads, g_fail ? "FAILED" : "bitwise equal to lone runs");
  if (g_fail) return 1;
  std::printf("abi_threads OK\n");
  return 0;
}
