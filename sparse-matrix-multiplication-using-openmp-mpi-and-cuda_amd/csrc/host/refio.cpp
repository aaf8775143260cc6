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
// upload can start without another host copy.  Writer: tiles are formatted by
// all threads into private buffers, then written with pwrite at prefix-summed
// offsets.
#include <fcntl.h>
#include <unistd.h>

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
  const int64_t ntok = parallel_tokens(
      h->f.data, h->body, h->f.size, nthreads,
      [&](int64_t g, const char* p, const char* end) {
        if (g >= need) return;   // trailing tokens are ignored, as `>>` would never read them
        const int64_t b = g / per, o = g % per;
        if (o < 2) {
          int64_t x;
          parse_i64(p, end, &x);
          keys[2 * b + o] = (int32_t)x;
        } else {
          parse_u64(p, end, &vals[b * kk + (o - 2)]);
        }
      });
  if (ntok < need) {
    set_err(err, errlen, "file has " + std::to_string(ntok) + " block tokens, expected " +
                             std::to_string(need));
    return -1;
  }
  return 0;
}

SPMM_HOST_EXPORT void spmm_ref_close(void* handle) { delete (RefHandle*)handle; }

// Writes the reference output layout.  keys/vals must already be sorted and
// pruned by the caller.  Returns 0 or -errno.
SPMM_HOST_EXPORT int spmm_ref_write(const char* path, int64_t R, int64_t C, int64_t nb,
                                    const int32_t* keys, const uint64_t* vals, int k,
                                    int nthreads) {
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
