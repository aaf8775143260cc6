// Matrix Market (coordinate) reader / writer.
//
// The north-star configs ask for Matrix-Market I/O next to the reference's own
// folder format (BASELINE.json).  Reader: header and size line parsed
// serially, entries by the parallel tokenizer (textio.hpp) straight into
// caller buffers (0-based int64 coordinates, float64 values).  Symmetric
// expansion and COO -> CSR happen on the device / in torch afterwards.
// Writer: parallel formatting with shortest round-trip float text.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "textio.hpp"

#define SPMM_HOST_EXPORT extern "C" __attribute__((visibility("default")))

using namespace spmm_host;

namespace {

struct MtxHandle {
  MappedFile f;
  int64_t rows = 0, cols = 0, nnz = 0;
  int field = 0;      // 0 real, 1 integer, 2 pattern, 3 complex
  int symmetry = 0;   // 0 general, 1 symmetric, 2 skew-symmetric, 3 hermitian
  size_t body = 0;
};

void set_err(char* err, int errlen, const std::string& msg) {
  if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", msg.c_str());
}

std::string lower(std::string s) {
  for (char& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

}  // namespace

SPMM_HOST_EXPORT void* spmm_mtx_open(const char* path, int64_t* rows, int64_t* cols, int64_t* nnz,
                                     int* field, int* symmetry, char* err, int errlen) {
  auto h = std::make_unique<MtxHandle>();
  if (!h->f.open(path)) { set_err(err, errlen, h->f.error); return nullptr; }
  const char* p = h->f.data;
  const char* end = p + h->f.size;
  // Banner: %%MatrixMarket matrix coordinate <field> <symmetry>
  const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
  std::string banner(p, nl ? nl : end);
  std::string b = lower(banner);
  if (b.rfind("%%matrixmarket", 0) != 0) { set_err(err, errlen, "missing %%MatrixMarket banner"); return nullptr; }
  if (b.find("coordinate") == std::string::npos) { set_err(err, errlen, "only coordinate format is supported"); return nullptr; }
  if (b.find("complex") != std::string::npos) h->field = 3;
  else if (b.find("pattern") != std::string::npos) h->field = 2;
  else if (b.find("integer") != std::string::npos) h->field = 1;
  else h->field = 0;
  if (b.find("skew-symmetric") != std::string::npos) h->symmetry = 2;
  else if (b.find("hermitian") != std::string::npos) h->symmetry = 3;
  else if (b.find("symmetric") != std::string::npos) h->symmetry = 1;
  else h->symmetry = 0;
  if (h->field == 3) { set_err(err, errlen, "complex matrices are not supported"); return nullptr; }
  // Skip comment lines.
  p = nl ? nl + 1 : end;
  while (p < end && (*p == '%' || *p == '\n' || *p == '\r')) {
    const char* q = (const char*)memchr(p, '\n', (size_t)(end - p));
    p = q ? q + 1 : end;
  }
  int64_t sz[3];
  for (int i = 0; i < 3; ++i) {
    while (p < end && is_space(*p)) ++p;
    if (p >= end) { set_err(err, errlen, "truncated size line"); return nullptr; }
    p = parse_i64(p, end, &sz[i]);
  }
  h->rows = sz[0]; h->cols = sz[1]; h->nnz = sz[2];
  h->body = (size_t)(p - h->f.data);
  *rows = h->rows; *cols = h->cols; *nnz = h->nnz;
  *field = h->field; *symmetry = h->symmetry;
  return h.release();
}

// Fills 0-based coordinates and values (1.0 for pattern files).
SPMM_HOST_EXPORT int spmm_mtx_fill(void* handle, int64_t* ri, int64_t* ci, double* v, int nthreads,
                                   char* err, int errlen) {
  MtxHandle* h = (MtxHandle*)handle;
  const int per = (h->field == 2) ? 2 : 3;
  const int64_t need = h->nnz * per;
  if (h->field == 2) {
    for (int64_t e = 0; e < h->nnz; ++e) v[e] = 1.0;
  }
  const int64_t ntok = parallel_tokens(h->f.data, h->body, h->f.size, nthreads,
                                       [&](int64_t g, const char* p, const char* end) {
                                         if (g >= need) return;
                                         const int64_t e = g / per, o = g % per;
                                         if (o < 2) {
                                           int64_t x;
                                           parse_i64(p, end, &x);
                                           (o == 0 ? ri : ci)[e] = x - 1;
                                         } else {
                                           const char* q = skip_token(p, end);
                                           double d = 0.0;
                                           std::from_chars(*p == '+' ? p + 1 : p, q, d);
                                           v[e] = d;
                                         }
                                       });
  if (ntok < need) {
    set_err(err, errlen, "file has " + std::to_string(ntok) + " entry tokens, expected " + std::to_string(need));
    return -1;
  }
  return 0;
}

SPMM_HOST_EXPORT void spmm_mtx_close(void* handle) { delete (MtxHandle*)handle; }

// Part `part` of `nparts` of the entry section, for a distributed read: the
// byte range [*b0, *b1) cut at line starts (every rank parses 1/nparts of
// the text, not the whole file) and its entry count (tokens / entry width).
// Returns -1 if the part does not hold whole entries.
SPMM_HOST_EXPORT int spmm_mtx_part(void* handle, int part, int nparts, int64_t* b0, int64_t* b1, int64_t* entries,
                                   int nthreads) {
  MtxHandle* h = (MtxHandle*)handle;
  const char* d = h->f.data;
  const size_t size = h->f.size, body = h->body;
  auto cut = [&](int r) -> size_t {   // first line start at or after the even split point
    if (r <= 0) return body;
    if (r >= nparts) return size;
    size_t x = body + (size - body) * (size_t)r / (size_t)nparts;
    if (x > body && d[x - 1] != '\n') {
      const char* q = (const char*)memchr(d + x, '\n', size - x);
      x = q ? (size_t)(q - d) + 1 : size;
    }
    return x;
  };
  const size_t lo = cut(part), hi = cut(part + 1);
  const int per = (h->field == 2) ? 2 : 3;
  const int64_t ntok = parallel_tokens(d, lo, hi, nthreads, [](int64_t, const char*, const char*) {});
  *b0 = (int64_t)lo;
  *b1 = (int64_t)hi;
  *entries = ntok / per;
  return ntok % per ? -1 : 0;
}

// Entries of the byte range [b0, b1) (from spmm_mtx_part), as spmm_mtx_fill,
// at most `entries` of them (the caller's buffers).  Returns the number of
// entry tokens found in the range, so the caller can check it against the
// count spmm_mtx_part reported (a file changed in between, or a short part).
SPMM_HOST_EXPORT int64_t spmm_mtx_fill_part(void* handle, int64_t b0, int64_t b1, int64_t entries, int64_t* ri,
                                            int64_t* ci, double* v, int nthreads) {
  MtxHandle* h = (MtxHandle*)handle;
  const int per = (h->field == 2) ? 2 : 3;
  const int64_t need = entries * per;
  return parallel_tokens(h->f.data, (size_t)b0, (size_t)b1, nthreads, [&](int64_t g, const char* p, const char* end) {
    if (g >= need) return;
    const int64_t e = g / per, o = g % per;
    if (o < 2) {
      int64_t x;
      parse_i64(p, end, &x);
      (o == 0 ? ri : ci)[e] = x - 1;
    } else {
      const char* q = skip_token(p, end);
      double dv = 0.0;
      std::from_chars(*p == '+' ? p + 1 : p, q, dv);
      v[e] = dv;
    }
  });   // (pattern files: the caller fills unit values)
}

// Writer: header, then row panels appended in order (a distributed run
// streams the panels of C to rank 0 one at a time), then close.  Formatting
// is parallel over each panel's entries; the bytes do not depend on how C was
// split into panels.
namespace {
struct MtxWriter {
  int fd = -1;
  int64_t off = 0;
  int rc = 0;
  bool values = true;
};
}  // namespace

SPMM_HOST_EXPORT void* spmm_mtx_write_begin(const char* path, int64_t m, int64_t n, int64_t nnz, int pattern) {
  auto w = std::make_unique<MtxWriter>();
  w->values = !pattern;
  w->fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (w->fd < 0) return nullptr;
  const std::string head = std::string("%%MatrixMarket matrix coordinate ") + (pattern ? "pattern" : "real") +
                           " general\n% written by spmm_amd\n" + std::to_string(m) + " " + std::to_string(n) +
                           " " + std::to_string(nnz) + "\n";
  if (::pwrite(w->fd, head.data(), head.size(), 0) != (ssize_t)head.size()) w->rc = -EIO;
  w->off = (int64_t)head.size();
  return w.release();
}

// Rows row0 .. row0 + mp of C: rp[0 .. mp] (any base), ci / v indexed by rp.
SPMM_HOST_EXPORT int spmm_mtx_write_panel(void* handle, int64_t row0, int64_t mp, const int64_t* rp,
                                          const int32_t* ci, const float* v, int nthreads) {
  MtxWriter* w = (MtxWriter*)handle;
  const float* vv = w->values ? v : nullptr;
  const int64_t base = rp[0], nnz = rp[mp] - base;
  if (nnz <= 0) return w->rc;
  int T = nthreads > 0 ? nthreads : omp_get_max_threads();
  if (nnz < 4096) T = 1;
  std::vector<std::string> bufs((size_t)T);
  std::vector<int64_t> sizes((size_t)T + 1, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int64_t e0 = base + nnz * t / T, e1 = base + nnz * (t + 1) / T;   // balanced entry ranges
    std::string& s = bufs[(size_t)t];
    s.resize((size_t)((e1 - e0) * 48 + 16));
    char* o = s.data();
    int64_t row = std::upper_bound(rp, rp + mp + 1, e0) - rp - 1;
    for (int64_t e = e0; e < e1; ++e) {
      while (rp[row + 1] <= e) ++row;
      o = std::to_chars(o, o + 20, row0 + row + 1).ptr; *o++ = ' ';
      o = std::to_chars(o, o + 20, (int64_t)ci[e - base] + 1).ptr;
      if (vv) { *o++ = ' '; o = std::to_chars(o, o + 24, vv[e - base]).ptr; }
      *o++ = '\n';
    }
    s.resize((size_t)(o - s.data()));
    sizes[(size_t)t + 1] = (int64_t)s.size();
  }
  sizes[0] = w->off;
  for (int t = 0; t < T; ++t) sizes[(size_t)t + 1] += sizes[(size_t)t];
  int rc = 0;
#pragma omp parallel for num_threads(T)
  for (int t = 0; t < T; ++t) {
    const std::string& s = bufs[(size_t)t];
    size_t done = 0;
    while (done < s.size()) {
      ssize_t k = ::pwrite(w->fd, s.data() + done, s.size() - done, (off_t)(sizes[(size_t)t] + (int64_t)done));
      if (k <= 0) { rc = -EIO; break; }
      done += (size_t)k;
    }
  }
  w->off = sizes[(size_t)T];
  if (rc) w->rc = rc;
  return w->rc;
}

SPMM_HOST_EXPORT int spmm_mtx_write_end(void* handle) {
  MtxWriter* w = (MtxWriter*)handle;
  int rc = w->rc;
  if (::close(w->fd) != 0 && rc == 0) rc = -EIO;
  delete w;
  return rc;
}

// Writes a general real coordinate file from CSR (int64 rowptr, int32 cols,
// float32 values; values == nullptr writes a pattern file).
SPMM_HOST_EXPORT int spmm_mtx_write(const char* path, int64_t m, int64_t n, const int64_t* rp,
                                    const int32_t* ci, const float* v, int nthreads) {
  void* w = spmm_mtx_write_begin(path, m, n, rp[m] - rp[0], v ? 0 : 1);
  if (!w) return -errno;
  spmm_mtx_write_panel(w, 0, m, rp, ci, v, nthreads);
  return spmm_mtx_write_end(w);
}
