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
    void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (p == MAP_FAILED) { error = std::string("cannot mmap ") + path; return false; }
    madvise(p, size, MADV_SEQUENTIAL);
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

}  // namespace spmm_host
