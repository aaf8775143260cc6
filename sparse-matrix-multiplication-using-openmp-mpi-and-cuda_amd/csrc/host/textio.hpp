// Parallel whitespace-token scanner over a memory-mapped text file.
//
// The reference parses each matrix file with `ifstream >>`, one OpenMP task per
// file (sparse_matrix_mult.cu:334-397), so a single large file is parsed by
// one thread.  Here every file is split into byte ranges parsed by all
// threads: pass 1 counts the tokens that START in each range, an exclusive
// scan gives every range its first global token index, and pass 2 parses each
// token and hands it to a visitor together with its global index, which is
// enough to know where it belongs (header, key, or value slot).
#pragma once
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace spmm_host {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  std::string error;

  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) { error = std::string("cannot open ") + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0) { error = std::string("cannot stat ") + path; return false; }
    size = (size_t)st.st_size;
    if (size == 0) { data = ""; return true; }
    // no MAP_POPULATE: the scanning threads fault their own ranges in, in parallel
    void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (p == MAP_FAILED) { error = std::string("cannot mmap ") + path; return false; }
    madvise(p, size, MADV_WILLNEED);
    data = (const char*)p;
    return true;
  }
  ~MappedFile() {
    if (data && size) munmap((void*)data, size);
    if (fd >= 0) ::close(fd);
  }
};

inline bool is_space(char c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t' || c == '\f' || c == '\v'; }

// Parse an unsigned 64-bit decimal token the way `istream >> uint64_t` does for
// well-formed input: wraps on a leading '-', like strtoull.
inline const char* parse_u64(const char* p, const char* end, uint64_t* out) {
  bool neg = false;
  if (p < end && (*p == '-' || *p == '+')) { neg = (*p == '-'); ++p; }
  uint64_t v = 0;
  while (p < end && (unsigned)(*p - '0') < 10u) { v = v * 10u + (uint64_t)(*p - '0'); ++p; }
  *out = neg ? (uint64_t)(0 - v) : v;
  return p;
}

// SWAR: 8 ASCII digits in one 64-bit word (first digit in the low byte).
inline bool eight_digits(uint64_t w) {
  return ((w & 0xF0F0F0F0F0F0F0F0ull) == 0x3030303030303030ull) &&
         (((w + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) == 0x3030303030303030ull);
}
inline uint32_t eight_digits_value(uint64_t w) {
  w -= 0x3030303030303030ull;
  w = (w * 10) + (w >> 8);   // pairs of digits
  w = (((w & 0x000000FF000000FFull) * (100 + (1000000ull << 32))) +
       (((w >> 16) & 0x000000FF000000FFull) * (1 + (10000ull << 32)))) >> 32;
  return (uint32_t)w;
}

// parse_u64 with 8 digits per step where 8 bytes remain; v*10^8 + d8 mod 2^64
// equals eight v*10 + d steps mod 2^64, so the wrap semantics are unchanged.
inline const char* parse_u64_fast(const char* p, const char* end, uint64_t* out) {
  if (p < end && (*p == '-' || *p == '+')) return parse_u64(p, end, out);
  uint64_t v = 0;
  while (end - p >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    if (!eight_digits(w)) break;
    v = v * 100000000ull + eight_digits_value(w);
    p += 8;
  }
  while (p < end && (unsigned)(*p - '0') < 10u) { v = v * 10u + (uint64_t)(*p - '0'); ++p; }
  *out = v;
  return p;
}

inline const char* parse_i64(const char* p, const char* end, int64_t* out) {
  bool neg = false;
  if (p < end && (*p == '-' || *p == '+')) { neg = (*p == '-'); ++p; }
  int64_t v = 0;
  while (p < end && (unsigned)(*p - '0') < 10u) { v = v * 10 + (*p - '0'); ++p; }
  *out = neg ? -v : v;
  return p;
}

inline const char* skip_token(const char* p, const char* end) {
  while (p < end && !is_space(*p)) ++p;
  return p;
}

// Visits tokens [first_token, ...) of data[begin, end) in parallel.  Visitor is
// called as v(global_token_index, token_ptr, text_end) from many threads.
// Returns the total number of tokens in the range.
template <class Visitor>
int64_t parallel_tokens(const char* data, size_t begin, size_t end, int nthreads, Visitor&& v) {
  if (end <= begin) return 0;
  const size_t n = end - begin;
  int T = nthreads > 0 ? nthreads : omp_get_max_threads();
  if (n < (size_t)(1 << 20)) T = 1;                  // small files: not worth forking
  std::vector<int64_t> counts(T + 1, 0);
  auto range_lo = [&](int t) { return begin + n * (size_t)t / (size_t)T; };
  const char* text_end = data + end;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const size_t lo = range_lo(t), hi = range_lo(t + 1);
    int64_t c = 0;
    bool prev_space = (lo == begin) ? true : is_space(data[lo - 1]);
    for (size_t i = lo; i < hi; ++i) {
      const bool sp = is_space(data[i]);
      c += (prev_space && !sp);
      prev_space = sp;
    }
    counts[t + 1] = c;
#pragma omp barrier
#pragma omp single
    {
      for (int q = 0; q < T; ++q) counts[q + 1] += counts[q];
    }
    int64_t g = counts[t];
    const char* p = data + lo;
    const char* h = data + hi;
    if (lo != begin && !is_space(data[lo - 1])) {     // token owned by the previous range
      p = skip_token(p, text_end);
    }
    while (p < h) {
      while (p < h && is_space(*p)) ++p;
      if (p >= h) break;
      v(g++, p, text_end);
      p = skip_token(p, text_end);
    }
  }
  return counts[T];
}

// Token separator of the fast scanner: any byte <= ' ' (space, \t \n \v \f \r
// and the other control bytes, which never occur in a well-formed file).
inline bool is_sep(unsigned char c) { return c <= ' '; }

// Cursor-based variant of parallel_tokens for the hot reference-format loader.
// Each thread gets its own copy of `proto`, positioned once with
// cur.seek(first_global_token) and then fed its tokens in order through
// cur.token(p, text_end), which parses the token and returns where it ended
// (no per-token division to locate the slot, no second scan to skip it).
// Pass 1 is a branch-free separator->token transition count the compiler
// vectorises.
template <class Cursor>
int64_t parallel_scan(const char* data, size_t begin, size_t end, int nthreads, const Cursor& proto) {
  if (end <= begin) return 0;
  const size_t n = end - begin;
  int T = nthreads > 0 ? nthreads : omp_get_max_threads();
  if (n < (size_t)(1 << 20)) T = 1;
  std::vector<int64_t> counts(T + 1, 0);
  auto range_lo = [&](int t) { return begin + n * (size_t)t / (size_t)T; };
  const unsigned char* d = reinterpret_cast<const unsigned char*>(data);
  const char* text_end = data + end;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const size_t lo = range_lo(t), hi = range_lo(t + 1);
    int64_t c = 0;
    if (lo < hi) {
      c = ((lo == begin) || is_sep(d[lo - 1])) && !is_sep(d[lo]);
      for (size_t base = lo + 1; base < hi;) {   // 32-bit partial sums over 1 MiB blocks
        const size_t e = (hi - base) > (size_t(1) << 20) ? base + (size_t(1) << 20) : hi;
        uint32_t cc = 0;
        for (size_t i = base; i < e; ++i) cc += (uint32_t)((d[i - 1] <= ' ') & (d[i] > ' '));
        c += cc;
        base = e;
      }
    }
    counts[t + 1] = c;
#pragma omp barrier
#pragma omp single
    {
      for (int q = 0; q < T; ++q) counts[q + 1] += counts[q];
    }
    Cursor cur = proto;
    cur.seek(counts[t]);
    const char* p = data + lo;
    const char* h = data + hi;
    if (lo != begin && !is_sep(d[lo - 1]))   // token owned by the previous range
      while (p < text_end && !is_sep((unsigned char)*p)) ++p;
    while (p < h) {
      while (p < h && is_sep((unsigned char)*p)) ++p;
      if (p >= h) break;
      const char* q = cur.token(p, text_end);
      while (q < text_end && !is_sep((unsigned char)*q)) ++q;   // malformed tail of a token
      p = q;
    }
  }
  return counts[T];
}

}  // namespace spmm_host
