// libsvm.cpp -- LIBSVM text -> CSR rows for the device.
//
// Restates MLUtils.parseLibSVMFile / parseLibSVMRecord /
// computeNumFeatures (mllib/util/MLUtils.scala:91-151): lines are trimmed
// (java.lang.String.trim: every char <= ' ' at both ends), empty lines and
// lines starting with '#' are dropped, a line splits on single spaces, the
// first item is the label (Double.parseDouble), every further non-empty item
// is "index:value" with a one-based int index; indices must be strictly
// ascending (the reference's require message, verbatim).  numFeatures =
// max(last index of each row, or 0) + 1 unless given.
//
// The text is cut into per-thread ranges at line boundaries and parsed in
// parallel; the rows concatenate in file order, so the CSR equals a
// sequential parse.  Values parse with strtod (correctly rounded, like
// Double.parseDouble), so they are bit-identical to the JVM's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "common.hpp"

struct cyc_libsvm_s {
  int64_t n = 0, nnz = 0;
  int32_t numFeatures = 0;
  std::vector<double> labels, values;
  std::vector<int64_t> rowptr;
  std::vector<int32_t> colidx;
};

namespace {

struct Part {
  std::vector<double> labels, values;
  std::vector<int64_t> rowEnd;   // nnz count after each row (part-local)
  std::vector<int32_t> colidx;
  int32_t maxIndex = -1;         // max over rows of the last index (-1: none)
  std::string error;
};

inline bool is_ws(char c) { return (unsigned char)c <= ' '; }

// Double.parseDouble: surrounding whitespace allowed, optional trailing
// d/D/f/F type suffix; "NaN", "Infinity" with sign.  Everything must be used.
bool parse_double(const char* b, const char* e, double* out) {
  while (b < e && is_ws(*b)) ++b;
  while (e > b && is_ws(e[-1])) --e;
  if (b == e) return false;
  if (e - b > 1 && (e[-1] == 'd' || e[-1] == 'D' || e[-1] == 'f' || e[-1] == 'F') &&
      !(e - b >= 8 && std::memcmp(e - 8, "Infinity", 8) == 0))
    --e;
  const char* p = b;
  bool neg = false;
  if (*p == '+' || *p == '-') neg = *p++ == '-';
  const size_t rest = (size_t)(e - p);
  if (rest == 3 && std::memcmp(p, "NaN", 3) == 0) { *out = NAN; return true; }
  if (rest == 8 && std::memcmp(p, "Infinity", 8) == 0) {
    *out = neg ? -INFINITY : INFINITY;
    return true;
  }
  // strtod would take "inf"/"nan" spellings the JVM rejects
  for (const char* q = p; q < e; ++q)
    if (*q == 'n' || *q == 'N' || *q == 'i' || *q == 'I') {
      if (!(q > p && (q[-1] == 'x' || q[-1] == 'X'))) return false;
    }
  std::string tmp(b, e);
  char* end = nullptr;
  errno = 0;
  const double v = std::strtod(tmp.c_str(), &end);
  if (end != tmp.c_str() + tmp.size()) return false;
  *out = v;
  return true;
}

// Integer.parseInt: optional sign, decimal digits, int32 range, nothing else.
bool parse_int(const char* b, const char* e, int32_t* out) {
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = *b == '-';
    ++b;
    if (b == e) return false;
  }
  int64_t v = 0;
  for (; b < e; ++b) {
    if (*b < '0' || *b > '9') return false;
    v = v * 10 + (*b - '0');
    if (v > (int64_t)INT32_MAX + 1) return false;
  }
  if (neg) v = -v;
  if (v < INT32_MIN || v > INT32_MAX) return false;
  *out = (int32_t)v;
  return true;
}

void parse_range(const char* text, int64_t b, int64_t e, Part& out) {
  int64_t pos = b;
  while (pos < e && out.error.empty()) {
    const char* nl = (const char*)std::memchr(text + pos, '\n', (size_t)(e - pos));
    const int64_t le = nl ? nl - text : e;
    const char* s = text + pos;
    const char* t = text + le;
    pos = le + 1;
    while (s < t && is_ws(*s)) ++s;        // String.trim
    while (t > s && is_ws(t[-1])) --t;
    if (s == t || *s == '#') continue;     // MLUtils.scala:102
    // items = line.split(' '): label first, then the non-empty "i:v" items
    const char* sp = (const char*)std::memchr(s, ' ', (size_t)(t - s));
    const char* le0 = sp ? sp : t;
    double label;
    if (!parse_double(s, le0, &label)) {
      out.error = "For input string: \"" + std::string(s, le0) + "\" (label); line=\"" +
                  std::string(s, t) + "\"";
      return;
    }
    out.labels.push_back(label);
    int32_t previous = -1;
    const char* q = le0;
    while (q < t) {
      while (q < t && *q == ' ') ++q;
      if (q >= t) break;
      const char* ie = (const char*)std::memchr(q, ' ', (size_t)(t - q));
      if (!ie) ie = t;
      const char* colon = (const char*)std::memchr(q, ':', (size_t)(ie - q));
      int32_t idx1;
      double v;
      if (!colon || !parse_int(q, colon, &idx1)) {
        out.error = "For input string: \"" + std::string(q, colon ? colon : ie) +
                    "\" (index); line=\"" + std::string(s, t) + "\"";
        return;
      }
      // indexAndValue(1): the text up to a second ':' if any (split(':'))
      const char* c2 = (const char*)std::memchr(colon + 1, ':', (size_t)(ie - colon - 1));
      if (!parse_double(colon + 1, c2 ? c2 : ie, &v)) {
        out.error = "For input string: \"" + std::string(colon + 1, c2 ? c2 : ie) +
                    "\" (value); line=\"" + std::string(s, t) + "\"";
        return;
      }
      const int32_t current = idx1 - 1;   // one-based -> zero-based
      if (!(current > previous)) {        // MLUtils.scala:142-143
        out.error = "indices should be one-based and in ascending order; found current=" +
                    std::to_string(current) + ", previous=" + std::to_string(previous) +
                    "; line=\"" + std::string(s, t) + "\"";
        return;
      }
      previous = current;
      out.colidx.push_back(current);
      out.values.push_back(v);
      q = ie;
    }
    // computeNumFeatures: indices.lastOption.getOrElse(0)
    out.maxIndex = std::max(out.maxIndex, previous >= 0 ? previous : 0);
    out.rowEnd.push_back((int64_t)out.colidx.size());
  }
}

int parse_text(const char* text, int64_t len, int32_t numFeatures, int nthreads,
               cyc_libsvm_s* r) {
  nthreads = std::max(1, std::min(nthreads, 64));
  if (len < (int64_t)1 << 20) nthreads = 1;
  std::vector<int64_t> cut(nthreads + 1, len);
  cut[0] = 0;
  for (int t = 1; t < nthreads; ++t) {
    int64_t c = std::max(cut[t - 1], len * t / nthreads);
    while (c < len && c > 0 && text[c - 1] != '\n') ++c;
    cut[t] = c;
  }
  std::vector<Part> parts(nthreads);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] { parse_range(text, cut[t], cut[t + 1], parts[t]); });
  for (auto& x : th) x.join();
  int64_t n = 0, nnz = 0;
  int32_t maxIndex = -1;
  for (auto& p : parts) {
    if (!p.error.empty()) {
      cyc::set_error("requirement failed: " + p.error);
      return CYC_ERR_INVALID_ARG;
    }
    n += (int64_t)p.labels.size();
    nnz += (int64_t)p.colidx.size();
    maxIndex = std::max(maxIndex, p.maxIndex);
  }
  r->n = n;
  r->nnz = nnz;
  r->numFeatures = numFeatures > 0 ? numFeatures : (n ? maxIndex + 1 : 1);
  if (numFeatures > 0 && maxIndex >= numFeatures) {
    cyc::set_error("requirement failed: You may not write an element to index " +
                   std::to_string(maxIndex) + " because the declared size of your vector is " +
                   std::to_string(numFeatures));
    return CYC_ERR_INVALID_ARG;
  }
  r->labels.reserve(n);
  r->values.reserve(nnz);
  r->colidx.reserve(nnz);
  r->rowptr.reserve(n + 1);
  r->rowptr.push_back(0);
  for (auto& p : parts) {
    const int64_t base = (int64_t)r->colidx.size();
    r->labels.insert(r->labels.end(), p.labels.begin(), p.labels.end());
    r->values.insert(r->values.end(), p.values.begin(), p.values.end());
    r->colidx.insert(r->colidx.end(), p.colidx.begin(), p.colidx.end());
    for (int64_t e : p.rowEnd) r->rowptr.push_back(base + e);
  }
  return CYC_OK;
}

}  // namespace

extern "C" {

int cyc_libsvm_parse(const char* text, int64_t len, int32_t numFeatures, int nthreads,
                     cyc_libsvm* out) {
  CYC_REQUIRE(out != nullptr && (text != nullptr || len == 0), "text and out must not be null");
  CYC_REQUIRE(len >= 0, "len >= 0");
  auto* r = new cyc_libsvm_s();
  int rc = parse_text(text, len, numFeatures, nthreads, r);
  if (rc) {
    delete r;
    return rc;
  }
  *out = r;
  return CYC_OK;
}

int cyc_libsvm_load_file(const char* path, int32_t numFeatures, int nthreads, cyc_libsvm* out) {
  CYC_REQUIRE(path != nullptr && out != nullptr, "path and out must not be null");
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) {
    cyc::set_error(std::string("cannot open ") + path + ": " + std::strerror(errno));
    return CYC_ERR_INVALID_ARG;
  }
  struct stat st;
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    cyc::set_error(std::string("cannot stat ") + path);
    return CYC_ERR_INVALID_ARG;
  }
  const int64_t len = (int64_t)st.st_size;
  const char* text = nullptr;
  void* m = MAP_FAILED;
  if (len > 0) {
    m = ::mmap(nullptr, (size_t)len, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      ::close(fd);
      cyc::set_error(std::string("cannot map ") + path);
      return CYC_ERR_INVALID_ARG;
    }
    text = (const char*)m;
  }
  const int rc = cyc_libsvm_parse(text ? text : "", len, numFeatures, nthreads, out);
  if (m != MAP_FAILED) ::munmap(m, (size_t)len);
  ::close(fd);
  return rc;
}

int cyc_libsvm_sizes(cyc_libsvm h, int64_t* n, int64_t* nnz, int32_t* numFeatures) {
  CYC_REQUIRE(h != nullptr, "handle must not be null");
  if (n) *n = h->n;
  if (nnz) *nnz = h->nnz;
  if (numFeatures) *numFeatures = h->numFeatures;
  return CYC_OK;
}

int cyc_libsvm_copy(cyc_libsvm h, double* labels, int64_t* rowptr, int32_t* colidx,
                    double* values) {
  CYC_REQUIRE(h != nullptr, "handle must not be null");
  // (an empty parse has empty vectors, whose data() may be null: no memcpy)
  if (labels && h->n) std::memcpy(labels, h->labels.data(), sizeof(double) * (size_t)h->n);
  if (rowptr) std::memcpy(rowptr, h->rowptr.data(), sizeof(int64_t) * (size_t)(h->n + 1));
  if (colidx && h->nnz) std::memcpy(colidx, h->colidx.data(), sizeof(int32_t) * (size_t)h->nnz);
  if (values && h->nnz) std::memcpy(values, h->values.data(), sizeof(double) * (size_t)h->nnz);
  return CYC_OK;
}

int cyc_libsvm_upload(cyc_libsvm h, double* labels, int64_t* rowptr, int32_t* colidx,
                      double* values, void* stream) {
  CYC_REQUIRE(h != nullptr, "handle must not be null");
  hipStream_t st = cyc::as_stream(stream);
  if (labels && h->n)
    CYC_HIP(hipMemcpyAsync(labels, h->labels.data(), sizeof(double) * (size_t)h->n,
                           hipMemcpyHostToDevice, st));
  if (rowptr)
    CYC_HIP(hipMemcpyAsync(rowptr, h->rowptr.data(), sizeof(int64_t) * (size_t)(h->n + 1),
                           hipMemcpyHostToDevice, st));
  if (colidx && h->nnz)
    CYC_HIP(hipMemcpyAsync(colidx, h->colidx.data(), sizeof(int32_t) * (size_t)h->nnz,
                           hipMemcpyHostToDevice, st));
  if (values && h->nnz)
    CYC_HIP(hipMemcpyAsync(values, h->values.data(), sizeof(double) * (size_t)h->nnz,
                           hipMemcpyHostToDevice, st));
  CYC_HIP(hipStreamSynchronize(st));   // the host arrays may be freed right after
  return CYC_OK;
}

int cyc_libsvm_destroy(cyc_libsvm h) {
  delete h;
  return CYC_OK;
}

}  // extern "C"
