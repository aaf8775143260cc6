// Device-resident CSR SpGEMM engine of the native `a4 --format mtx` chain
// (csr_engine.cpp): the operands and every intermediate product stay in HBM;
// the host sees only plan statistics and a few per-row arrays.  The Python
// engine's paths (ops/spgemm.py) driven from C++ through the kernels' C ABI:
//   bitmap-rank  count -> scan -> numeric (csr_spgemm_bitmap.hip) for products
//                whose rows look uniform (the 1M / 65536^2 configs);
//   binned       symbolic + numeric LDS tables (csr_spgemm.hip spgemm_lds)
//                for short / medium rows, and the column-chunked long-row
//                pipeline (long_route / long_wg_scan / long_dense /
//                long_place) for hub rows (R-MAT) -- any row of any length.
// The reference has no CSR path; its per-product host round trips
// (sparse_matrix_mult.cu:181-270) are what this replaces.
#pragma once

#include <cstdint>
#include <vector>

#include "rt.hpp"

namespace a4 {

// Host CSR (fp32): row pointer, column indices, values.
struct Csr {
  int64_t m = 0, n = 0;
  std::vector<int64_t> rp{0};
  std::vector<int32_t> ci;
  std::vector<float> v;
  int64_t nnz() const { return (int64_t)ci.size(); }
};

// Device CSR: rows sorted by column unless `unsorted_rows` lists some.
struct DCsr {
  int64_t m = 0, n = 0, nnz = 0;
  DevBuf<int64_t> rp;
  DevBuf<int32_t> ci;
  DevBuf<float> v;
};

struct EngineStats {
  int64_t bitmap = 0, binned = 0, long_rows = 0, resorted_rows = 0;   // resorted_rows: on the host (none since round 5)
  int64_t device_sorted_rows = 0;   // flagged rows re-sorted by csr_rowsort.hip
};

DCsr dcsr_upload(const Csr& H, hipStream_t s);
Csr dcsr_download(const DCsr& D, hipStream_t s);
// C = A . B on the device, B's rows column-sorted; C's rows column-sorted.
DCsr dev_spgemm(const DCsr& A, const DCsr& B, hipStream_t s, EngineStats* st, int64_t* products);

}  // namespace a4
