// Reference-format block-sparse matrix reader / writer.
//
// Format (reader sparse_matrix_mult.cu:342-391, writer
// :595-608):
//   rows cols
//   blocks
//   repeat blocks times:  r c  then k*k unsigned 64-bit values, row-major
// The writer emits exactly the reference's bytes: "R C\n", "n\n", then per
// tile "r c\n" and k lines of single-space separated values with no trailing
// space.
//
// Reader: mmap + parallel two-pass tokenizer (textio.hpp), values parsed
// straight into caller-provided (typically pinned) buffers so the device
// upload can start without another host copy; 8 digits per step (SWAR).
// Writer: a sizing pass gives every thread its exact byte range, then all
// threads format straight into a shared mapping of the output file.
#include <fcntl.h>
#include <unistd.h>

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

struct RefHandle {
  MappedFile f;
  int64_t rows = 0, cols = 0, blocks = 0;
  size_t body = 0;   // byte offset of the first block token
  int k = 0;
  std::string error;
};

void set_err(char* err, int errlen, const std::string& msg) {
  if (err && errlen > 0) {
    std::snprintf(err, (size_t)errlen, "%s", msg.c_str());
  }
}

}  // namespace

// Opens a reference matrix file and parses its 3-token header.
// Returns an opaque handle or nullptr (message in err).
SPMM_HOST_EXPORT void* spmm_ref_open(const char* path, int k, int64_t* rows, int64_t* cols,
                                     int64_t* blocks, char* err, int errlen) {
  auto h = std::make_unique<RefHandle>();
  h->k = k;
  if (!h->f.open(path)) { set_err(err, errlen, h->f.error); return nullptr; }
  const char* p = h->f.data;
  const char* end = p + h->f.size;
  int64_t hdr[3];
  for (int i = 0; i < 3; ++i) {
    while (p < end && is_space(*p)) ++p;
    if (p >= end) { set_err(err, errlen, std::string("truncated header in ") + path); return nullptr; }
    p = parse_i64(p, end, &hdr[i]);
  }
  if (hdr[2] < 0) { set_err(err, errlen, std::string("negative block count in ") + path); return nullptr; }
  h->rows = hdr[0]; h->cols = hdr[1]; h->blocks = hdr[2];
  h->body = (size_t)(p - h->f.data);
  *rows = h->rows; *cols = h->cols; *blocks = h->blocks;
  return h.release();
}

// Fills keys [blocks][2] (int32, file order) and vals [blocks][k][k] (uint64).
// Returns 0 on success, -1 on a short file (message in err).
SPMM_HOST_EXPORT int spmm_ref_fill(void* handle, int32_t* keys, uint64_t* vals, int nthreads,
                                   char* err, int errlen) {
  RefHandle* h = (RefHandle*)handle;
  const int64_t kk = (int64_t)h->k * h->k;
  const int64_t per = 2 + kk;
  const int64_t need = h->blocks * per;
  // Per-thread position in the block stream: block b, token o of the block
  // (0, 1 = tile key, 2.. = values).
  struct Cursor {
    int32_t* keys;
    uint64_t* vals;
    int64_t kk, per, blocks, b = 0, o = 0;
    void seek(int64_t g) { b = g / per; o = g % per; }
    const char* token(const char* p, const char* end) {
      if (b >= blocks) return p;   // trailing tokens are ignored, as `>>` would never read them
      if (o < 2) {
        int64_t x;
        p = parse_i64(p, end, &x);
        keys[2 * b + o] = (int32_t)x;
      } else {
        p = parse_u64_fast(p, end, &vals[b * kk + (o - 2)]);
      }
      if (++o == per) { o = 0; ++b; }
      return p;
    }
  };
  const int64_t ntok = parallel_scan(h->f.data, h->body, h->f.size, nthreads,
                                     Cursor{keys, vals, kk, per, h->blocks});
  if (ntok < need) {
    set_err(err, errlen, "file has " + std::to_string(ntok) + " block tokens, expected " +
                             std::to_string(need));
    return -1;
  }
  return 0;
}

SPMM_HOST_EXPORT void spmm_ref_close(void* handle) { delete (RefHandle*)handle; }

namespace {

// Decimal digits of v (1..20): bit length -> estimate, one table compare.
inline int u64_digits(uint64_t v) {
  static const uint64_t p10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                   100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                   1000000000000ull, 10000000000000ull, 100000000000000ull,
                                   1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                   1000000000000000000ull, 10000000000000000000ull};
  const int bits = 64 - __builtin_clzll(v | 1);   // 1..64
  const int t = (bits * 1233) >> 12;              // 0..19, digits are t or t + 1
  return t + (v >= p10[t] ? 1 : 0) + (v == 0 ? 1 : 0);
}

inline int i32_len(int32_t x) {
  char b[16];
  return (int)(std::to_chars(b, b + 16, x).ptr - b);
}

// Bytes of tile b in the output layout: "r c\n" + k lines of k values.
inline int64_t tile_bytes(const int32_t* keys, const uint64_t* v, int64_t kk, int64_t b) {
  int64_t n = i32_len(keys[2 * b]) + 1 + i32_len(keys[2 * b + 1]) + 1;
  for (int64_t e = 0; e < kk; ++e) n += u64_digits(v[b * kk + e]) + 1;   // value + ' ' or '\n'
  return n;
}

}  // namespace

SPMM_HOST_EXPORT int spmm_ref_write_buffered(const char* path, int64_t R, int64_t C, int64_t nb,
                                             const int32_t* keys, const uint64_t* vals, int k, int nthreads);

// Writes the reference output layout with every thread formatting straight
// into a shared mapping of the output file: a sizing pass gives each thread's
// exact byte range, so there is no intermediate buffer and no serialised
// write(2).  Returns 0 or -errno.
SPMM_HOST_EXPORT int spmm_ref_write(const char* path, int64_t R, int64_t C, int64_t nb,
                                    const int32_t* keys, const uint64_t* vals, int k,
                                    int nthreads) {
  const int64_t kk = (int64_t)k * k;
  int T = nthreads > 0 ? nthreads : omp_get_max_threads();
  if (nb < 64) T = 1;
  char head[64];
  const int hl = std::snprintf(head, sizeof head, "%lld %lld\n%lld\n", (long long)R, (long long)C, (long long)nb);
  std::vector<int64_t> off((size_t)T + 1, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int64_t b0 = nb * t / T, b1 = nb * (t + 1) / T;
    int64_t n = 0;
    for (int64_t b = b0; b < b1; ++b) n += tile_bytes(keys, vals, kk, b);
    off[(size_t)t + 1] = n;
  }
  off[0] = hl;
  for (int t = 0; t < T; ++t) off[(size_t)t + 1] += off[(size_t)t];
  const int64_t total = off[(size_t)T];

  int fd = ::open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -errno;
  if (::ftruncate(fd, (off_t)total) != 0) { const int e = errno; ::close(fd); return -e; }
  void* map = mmap(nullptr, (size_t)total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (map == MAP_FAILED) { ::close(fd); return spmm_ref_write_buffered(path, R, C, nb, keys, vals, k, nthreads); }
  char* out = static_cast<char*>(map);
  std::memcpy(out, head, (size_t)hl);
  int bad = 0;
#pragma omp parallel num_threads(T) reduction(| : bad)
  {
    const int t = omp_get_thread_num();
    const int64_t b0 = nb * t / T, b1 = nb * (t + 1) / T;
    char* o = out + off[(size_t)t];
    char* lim = out + off[(size_t)t + 1];
    for (int64_t b = b0; b < b1; ++b) {
      o = std::to_chars(o, lim, keys[2 * b]).ptr; *o++ = ' ';
      o = std::to_chars(o, lim, keys[2 * b + 1]).ptr; *o++ = '\n';
      const uint64_t* v = vals + b * kk;
      for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) {
          o = std::to_chars(o, lim, v[r * k + c]).ptr;
          *o++ = (c + 1 < k) ? ' ' : '\n';
        }
    }
    bad |= (o != lim);
  }
  int rc = bad ? -EIO : 0;
  if (munmap(map, (size_t)total) != 0 && rc == 0) rc = -errno;
  if (::close(fd) != 0 && rc == 0) rc = -EIO;
  return rc;
}

// Buffered fallback (filesystems that cannot map the output).
SPMM_HOST_EXPORT int spmm_ref_write_buffered(const char* path, int64_t R, int64_t C, int64_t nb,
                                             const int32_t* keys, const uint64_t* vals, int k, int nthreads) {
  const int64_t kk = (int64_t)k * k;
  int T = nthreads > 0 ? nthreads : omp_get_max_threads();
  if (nb < 64) T = 1;
  std::vector<std::string> bufs((size_t)T);
  std::vector<int64_t> sizes((size_t)T + 1, 0);

  char head[64];
  int hl = std::snprintf(head, sizeof head, "%lld %lld\n%lld\n", (long long)R, (long long)C, (long long)nb);

#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const int64_t b0 = nb * t / T, b1 = nb * (t + 1) / T;
    std::string& s = bufs[(size_t)t];
    s.resize((size_t)((b1 - b0) * (24 + kk * 21)));
    char* o = s.data();
    for (int64_t b = b0; b < b1; ++b) {
      o = std::to_chars(o, o + 12, keys[2 * b]).ptr; *o++ = ' ';
      o = std::to_chars(o, o + 12, keys[2 * b + 1]).ptr; *o++ = '\n';
      const uint64_t* v = vals + b * kk;
      for (int r = 0; r < k; ++r) {
        for (int c = 0; c < k; ++c) {
          o = std::to_chars(o, o + 21, v[r * k + c]).ptr;
          *o++ = (c + 1 < k) ? ' ' : '\n';
        }
      }
    }
    s.resize((size_t)(o - s.data()));
    sizes[(size_t)t + 1] = (int64_t)s.size();
  }
  sizes[0] = hl;
  for (int t = 0; t < T; ++t) sizes[(size_t)t + 1] += sizes[(size_t)t];

  int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -errno;
  int rc = 0;
  if (::pwrite(fd, head, (size_t)hl, 0) != hl) rc = -EIO;
#pragma omp parallel for num_threads(T) schedule(static)
  for (int t = 0; t < T; ++t) {
    const std::string& s = bufs[(size_t)t];
    size_t done = 0;
    while (done < s.size()) {
      ssize_t w = ::pwrite(fd, s.data() + done, s.size() - done, (off_t)(sizes[(size_t)t] + (int64_t)done));
      if (w <= 0) { rc = -EIO; break; }
      done += (size_t)w;
    }
  }
  if (::close(fd) != 0 && rc == 0) rc = -EIO;
  return rc;
}
