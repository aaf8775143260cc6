// OpenMP CPU backend.
//
// 1. BSR uint64 tile-pair multiply with the reference's exact arithmetic and
//    per-element order (sparse_matrix_mult.cu:54-62).  This is the CPU-only
//    backend the report's Table 1 "CPU-Only" column describes but the
//    reference never shipped (report.pdf p.3), and the host fallback that lets
//    every non-GPU test run the same engine code.
// 2. CSR SpGEMM fp32 (Gustavson, sparse accumulator per thread, sorted output
//    columns): the north-star plumbing config "1024x1024 CSR x CSR at 1 % on
//    CPU/OpenMP" (BASELINE.json) and the measured CPU baseline.
// 3. CSR SpMM fp32 accumulate (sparse x dense) reference for tests.
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#define SPMM_HOST_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t ref_mac(uint64_t acc, uint64_t a, uint64_t b) {
  uint64_t t = a * b;
  t = (t == ~0ull) ? 0ull : t;
  uint64_t s = acc + t;
  return (s == ~0ull) ? 0ull : s;
}

inline int threads_or_default(int n) { return n > 0 ? n : omp_get_max_threads(); }

}  // namespace

SPMM_HOST_EXPORT int spmm_cpu_bsr_u64_numeric(const uint64_t* A, const uint64_t* B, const int32_t* pa,
                                              const int32_t* pb, const int64_t* tile_ptr, uint64_t* C,
                                              int32_t* nz_flag, int k, int64_t ntiles, int nthreads) {
  const int64_t kk = (int64_t)k * k;
#pragma omp parallel num_threads(threads_or_default(nthreads))
  {
    std::vector<uint64_t> acc((size_t)kk);
#pragma omp for schedule(dynamic, 4)
    for (int64_t t = 0; t < ntiles; ++t) {
      std::fill(acc.begin(), acc.end(), 0ull);
      for (int64_t p = tile_ptr[t]; p < tile_ptr[t + 1]; ++p) {
        const uint64_t* a = A + (int64_t)pa[p] * kk;
        const uint64_t* b = B + (int64_t)pb[p] * kk;
        for (int r = 0; r < k; ++r) {
          uint64_t* cr = acc.data() + (int64_t)r * k;
          for (int j = 0; j < k; ++j) {
            const uint64_t av = a[(int64_t)r * k + j];
            const uint64_t* br = b + (int64_t)j * k;
            for (int c = 0; c < k; ++c) cr[c] = ref_mac(cr[c], av, br[c]);
          }
        }
      }
      uint64_t any = 0;
      for (int64_t e = 0; e < kk; ++e) any |= acc[(size_t)e];
      std::memcpy(C + t * kk, acc.data(), (size_t)kk * sizeof(uint64_t));
      nz_flag[t] = any != 0;
    }
  }
  return 0;
}

SPMM_HOST_EXPORT int spmm_cpu_bsr_u64_nonzero(const uint64_t* vals, int k, int64_t ntiles,
                                              int32_t* nz_flag, int nthreads) {
  const int64_t kk = (int64_t)k * k;
#pragma omp parallel for num_threads(threads_or_default(nthreads)) schedule(static)
  for (int64_t t = 0; t < ntiles; ++t) {
    uint64_t any = 0;
    for (int64_t e = 0; e < kk; ++e) any |= vals[t * kk + e];
    nz_flag[t] = any != 0;
  }
  return 0;
}

// Intermediate-product count per row: nprod[i] = sum_{j in A(i,:)} nnz(B(j,:)).
// 2 * sum(nprod) is the FLOP count used for every SpGEMM GFLOP/s figure.
SPMM_HOST_EXPORT int64_t spmm_cpu_csr_nprod(int64_t m, const int64_t* Arp, const int32_t* Aci,
                                            const int64_t* Brp, int64_t* nprod, int nthreads) {
  int64_t total = 0;
#pragma omp parallel for num_threads(threads_or_default(nthreads)) schedule(dynamic, 256) reduction(+ : total)
  for (int64_t i = 0; i < m; ++i) {
    int64_t s = 0;
    for (int64_t e = Arp[i]; e < Arp[i + 1]; ++e) s += Brp[Aci[e] + 1] - Brp[Aci[e]];
    nprod[i] = s;
    total += s;
  }
  return total;
}

// Symbolic phase: Crp[i+1] = |union of B rows|; Crp becomes the row pointer
// after the caller's scan (done here).  Returns nnz(C).
SPMM_HOST_EXPORT int64_t spmm_cpu_csr_spgemm_symbolic(int64_t m, int64_t n, const int64_t* Arp,
                                                      const int32_t* Aci, const int64_t* Brp,
                                                      const int32_t* Bci, int64_t* Crp, int nthreads) {
  Crp[0] = 0;
#pragma omp parallel num_threads(threads_or_default(nthreads))
  {
    std::vector<int64_t> mark((size_t)n, -1);
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < m; ++i) {
      int64_t cnt = 0;
      for (int64_t e = Arp[i]; e < Arp[i + 1]; ++e) {
        const int32_t j = Aci[e];
        for (int64_t f = Brp[j]; f < Brp[j + 1]; ++f) {
          const int32_t c = Bci[f];
          if (mark[(size_t)c] != i) { mark[(size_t)c] = i; ++cnt; }
        }
      }
      Crp[i + 1] = cnt;
    }
  }
  for (int64_t i = 0; i < m; ++i) Crp[i + 1] += Crp[i];
  return Crp[m];
}

// Numeric phase into the symbolic layout; columns sorted ascending per row.
// Products are accumulated in A's row order then B's row order (a fixed,
// deterministic order).
SPMM_HOST_EXPORT int spmm_cpu_csr_spgemm_numeric(int64_t m, int64_t n, const int64_t* Arp,
                                                 const int32_t* Aci, const float* Av, const int64_t* Brp,
                                                 const int32_t* Bci, const float* Bv, const int64_t* Crp,
                                                 int32_t* Cci, float* Cv, int nthreads) {
#pragma omp parallel num_threads(threads_or_default(nthreads))
  {
    std::vector<int64_t> mark((size_t)n, -1);
    std::vector<float> accum((size_t)n, 0.f);
    std::vector<int32_t> cols;
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < m; ++i) {
      cols.clear();
      for (int64_t e = Arp[i]; e < Arp[i + 1]; ++e) {
        const int32_t j = Aci[e];
        const float a = Av[e];
        for (int64_t f = Brp[j]; f < Brp[j + 1]; ++f) {
          const int32_t c = Bci[f];
          if (mark[(size_t)c] != i) { mark[(size_t)c] = i; accum[(size_t)c] = 0.f; cols.push_back(c); }
          accum[(size_t)c] += a * Bv[f];
        }
      }
      std::sort(cols.begin(), cols.end());
      int64_t o = Crp[i];
      for (int32_t c : cols) { Cci[o] = c; Cv[o] = accum[(size_t)c]; ++o; }
    }
  }
  return 0;
}

// Y[m][d] = A (CSR, fp32 values) x X[n][d] (fp32), accumulate in fp32.
SPMM_HOST_EXPORT int spmm_cpu_csr_spmm(int64_t m, int64_t d, const int64_t* Arp, const int32_t* Aci,
                                       const float* Av, const float* X, float* Y, int nthreads) {
#pragma omp parallel for num_threads(threads_or_default(nthreads)) schedule(dynamic, 64)
  for (int64_t i = 0; i < m; ++i) {
    float* y = Y + i * d;
    for (int64_t c = 0; c < d; ++c) y[c] = 0.f;
    for (int64_t e = Arp[i]; e < Arp[i + 1]; ++e) {
      const float a = Av[e];
      const float* x = X + (int64_t)Aci[e] * d;
      for (int64_t c = 0; c < d; ++c) y[c] += a * x[c];
    }
  }
  return 0;
}
