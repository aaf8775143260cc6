// CPU block-sparse engine of the native `a4` (OpenMP): the same join, order
// and pruning as bsr_engine.hip, for `--device cpu` and GPU-less tests.
// The numeric phase is libspmm_host.so's spmm_cpu_bsr_u64_numeric.
#include <algorithm>
#include <numeric>

#include "rt.hpp"

namespace a4 {

void canonicalize(Mat& M) {
  const int64_t n = M.nb();
  if (n <= 1) return;
  bool sorted = true;
  for (int64_t i = 1; i < n && sorted; ++i)
    sorted = encode_key(M.keys[2 * i - 2], M.keys[2 * i - 1]) < encode_key(M.keys[2 * i], M.keys[2 * i + 1]);
  if (sorted) return;
  // std::map semantics of the reference loader (:383): later duplicates win
  std::vector<int64_t> idx((size_t)n);
  std::iota(idx.begin(), idx.end(), 0);
  auto code = [&](int64_t i) { return encode_key(M.keys[2 * i], M.keys[2 * i + 1]); };
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return code(a) < code(b); });
  const int64_t kk = (int64_t)M.k * M.k;
  Mat out;
  out.rows = M.rows; out.cols = M.cols; out.k = M.k;
  for (int64_t i = 0; i < n; ++i) {
    if (i + 1 < n && code(idx[i]) == code(idx[i + 1])) continue;   // keep the last of a run
    const int64_t s = idx[i];
    out.keys.push_back(M.keys[2 * s]);
    out.keys.push_back(M.keys[2 * s + 1]);
    out.vals.insert(out.vals.end(), M.vals.begin() + s * kk, M.vals.begin() + (s + 1) * kk);
  }
  M = std::move(out);
}

Mat cpu_prune(Mat M) {
  const int64_t n = M.nb(), kk = (int64_t)M.k * M.k;
  int64_t d = 0;
  for (int64_t t = 0; t < n; ++t) {
    bool any = false;
    for (int64_t e = 0; e < kk && !any; ++e) any = M.vals[t * kk + e] != 0;
    if (!any) continue;
    if (d != t) {
      M.keys[2 * d] = M.keys[2 * t];
      M.keys[2 * d + 1] = M.keys[2 * t + 1];
      std::copy(M.vals.begin() + t * kk, M.vals.begin() + (t + 1) * kk, M.vals.begin() + d * kk);
    }
    ++d;
  }
  M.keys.resize((size_t)d * 2);
  M.vals.resize((size_t)(d * kk));
  return M;
}

Mat cpu_multiply(const Mat& A, const Mat& B, int nthreads, int64_t* tile_pairs) {
  A4_CHECK(A.k == B.k, "tile size mismatch");
  Mat C;
  C.rows = A.rows; C.cols = B.cols; C.k = A.k;
  const int64_t na = A.nb(), nb = B.nb(), kk = (int64_t)C.k * C.k;
  // B tile-row ranges (B sorted by (r, c))
  std::vector<int64_t> lo((size_t)na), cnt((size_t)na);
  int64_t np = 0;
  for (int64_t a = 0; a < na; ++a) {
    const int32_t j = A.keys[2 * a + 1];
    int64_t l = 0, h = nb;
    while (l < h) { const int64_t m = (l + h) / 2; if (B.keys[2 * m] < j) l = m + 1; else h = m; }
    const int64_t f = l;
    h = nb;
    while (l < h) { const int64_t m = (l + h) / 2; if (B.keys[2 * m] <= j) l = m + 1; else h = m; }
    lo[a] = f;
    cnt[a] = l - f;
    np += cnt[a];
  }
  if (tile_pairs) *tile_pairs = np;
  if (np == 0) return C;
  std::vector<uint64_t> code((size_t)np);
  std::vector<int64_t> pidx((size_t)np);
  std::vector<int32_t> pa0((size_t)np), pb0((size_t)np);
  {
    int64_t p = 0;
    for (int64_t a = 0; a < na; ++a)
      for (int64_t t = 0; t < cnt[a]; ++t, ++p) {
        const int64_t b = lo[a] + t;
        code[p] = encode_key(A.keys[2 * a], B.keys[2 * b + 1]);
        pa0[p] = (int32_t)a;
        pb0[p] = (int32_t)b;
        pidx[p] = p;
      }
  }
  // stable: ascending middle index inside each output tile (reference order)
  std::stable_sort(pidx.begin(), pidx.end(), [&](int64_t x, int64_t y) { return code[x] < code[y]; });
  std::vector<int32_t> pa((size_t)np), pb((size_t)np);
  std::vector<int64_t> tile_ptr(1, 0);
  for (int64_t i = 0; i < np; ++i) {
    const int64_t p = pidx[i];
    pa[i] = pa0[p];
    pb[i] = pb0[p];
    if (i == 0 || code[p] != code[pidx[i - 1]]) {
      if (i) tile_ptr.push_back(i);
      C.keys.push_back(key_r(code[p]));
      C.keys.push_back(key_c(code[p]));
    }
  }
  tile_ptr.push_back(np);
  const int64_t nt = C.nb();
  C.vals.resize((size_t)(nt * kk));
  std::vector<int32_t> nz((size_t)nt);
  if (spmm_cpu_bsr_u64_numeric(A.vals.data(), B.vals.data(), pa.data(), pb.data(), tile_ptr.data(), C.vals.data(),
                               nz.data(), C.k, nt, nthreads) != 0)
    throw Error("spmm_cpu_bsr_u64_numeric failed");
  return cpu_prune(std::move(C));
}

}  // namespace a4
