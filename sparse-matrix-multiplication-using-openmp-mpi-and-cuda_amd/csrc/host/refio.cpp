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
// Writer: a sizing pass gives every thread its exact byte range; threads
// format into small private buffers and pwrite them at their offsets.
#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <algorithm>
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

// "00".."99"
struct Digits2 {
  char d[200];
  constexpr Digits2() : d() {
    for (int i = 0; i < 100; ++i) {
      d[2 * i] = (char)('0' + i / 10);
      d[2 * i + 1] = (char)('0' + i % 10);
    }
  }
};
constexpr Digits2 kDig2{};

inline void put2(char* o, uint32_t x) { std::memcpy(o, kDig2.d + 2 * x, 2); }
inline void put8(char* o, uint32_t x) {   // exactly 8 digits, leading zeros kept
  const uint32_t hi = x / 10000, lo = x - hi * 10000;
  put2(o, hi / 100);
  put2(o + 2, hi % 100);
  put2(o + 4, lo / 100);
  put2(o + 6, lo % 100);
}

// Decimal text of v at o (no terminator); returns the end.  Two-digit table
// and 8-digit blocks: several times faster than std::to_chars for 20-digit
// values (the formatter is the writer's bottleneck).
inline char* fmt_u64(char* o, uint64_t v) {
  char* const end = o + u64_digits(v);
  char* p = end;
  while (v >= 100000000ull) {
    const uint64_t q = v / 100000000ull;
    p -= 8;
    put8(p, (uint32_t)(v - q * 100000000ull));
    v = q;
  }
  uint32_t x = (uint32_t)v;
  while (x >= 100) {
    const uint32_t q = x / 100;
    p -= 2;
    put2(p, x - q * 100);
    x = q;
  }
  if (x >= 10) {
    p -= 2;
    put2(p, x);
  } else {
    *--p = (char)('0' + x);
  }
  return end;
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

// Writes the reference output layout.  keys/vals must already be sorted and
// pruned by the caller.  A sizing pass gives every thread the exact byte
// offset of its tile range; each thread then formats into a small private
// buffer (cache resident, never zero-filled) and pwrite()s it at its running
// offset whenever the next tile might not fit, so formatting and the
// page-cache copies of all threads overlap.  Returns 0 or -errno.
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

  int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -errno;
  int rc = (::pwrite(fd, head, (size_t)hl, 0) == hl) ? 0 : -EIO;
  const size_t tile_max = 24 + (size_t)kk * 21;
  const size_t cap = std::max<size_t>(size_t(4) << 20, 2 * tile_max);
  int bad = 0;
#pragma omp parallel num_threads(T) reduction(| : bad)
  {
    const int t = omp_get_thread_num();
    const int64_t b0 = nb * t / T, b1 = nb * (t + 1) / T;
    std::unique_ptr<char[]> buf(new char[cap]);
    char* const base = buf.get();
    char* o = base;
    int64_t at = off[(size_t)t];
    auto flush = [&]() {
      size_t n = (size_t)(o - base), done = 0;
      while (done < n) {
        const ssize_t w = ::pwrite(fd, base + done, n - done, (off_t)(at + (int64_t)done));
        if (w <= 0) { bad = 1; break; }
        done += (size_t)w;
      }
      at += (int64_t)n;
      o = base;
    };
    for (int64_t b = b0; b < b1; ++b) {
      if ((size_t)(o - base) + tile_max > cap) flush();
      o = std::to_chars(o, o + 12, keys[2 * b]).ptr; *o++ = ' ';
      o = std::to_chars(o, o + 12, keys[2 * b + 1]).ptr; *o++ = '\n';
      const uint64_t* v = vals + b * kk;
      for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) {
          o = fmt_u64(o, v[r * k + c]);
          *o++ = (c + 1 < k) ? ' ' : '\n';
        }
    }
    flush();
    bad |= (at != off[(size_t)t + 1]);
  }
  if (bad && rc == 0) rc = -EIO;
  if (::close(fd) != 0 && rc == 0) rc = -EIO;
  return rc;
}
