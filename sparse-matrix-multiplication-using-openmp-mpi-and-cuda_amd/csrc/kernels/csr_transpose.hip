// CSR transpose on gfx950 (SURVEY.md §2.3 north-star additions: "csr_transpose:
// for A.A^T"; the R-MAT config multiplies A by its transpose).  The reference
// has no CSR at all; its only re-layout is the host-side tile flattening of
// sparse_matrix_mult.cu:102-138.
//
// Pipeline (the host wrapper is ops/csr.py:transpose_gpu):
//   1. csr_col_count   column histogram (one thread per stored entry)
//   2. device scan     -> row pointer of A^T (torch cumsum on the stream)
//   3. csr_t_scatter   one wave per row of A: every entry claims a slot in its
//                      column's segment with an atomic cursor and stores its
//                      SOURCE index e (int64).  Slot order inside a segment is
//                      arbitrary...
//   4. ...so each segment is sorted by e afterwards; A is row-sorted, so
//      ascending e == ascending row index, the canonical order of A^T:
//        csr_t_sort_wave  segments of <= 64: one wave, bitonic over lanes
//                         (DPP/ds_swizzle shuffles, no LDS);
//        csr_t_sort_lds   segments of 65..2048: one workgroup, bitonic in LDS;
//        longer segments (R-MAT hub columns) go to a device radix sort on the
//        host side (few rows, most of their bytes).
//   Columns / values of A^T are then gathers by e (row id of e, val[e]), so
//   the kernels are value-type agnostic (fp32 SpGEMM and bf16 SpMM operands).
#include "common.hpp"

namespace {

constexpr int kSortLds = 2048;   // largest segment sorted in LDS

__global__ __launch_bounds__(256) void csr_col_count(const int32_t* __restrict__ col, int64_t nnz,
                                                     int64_t* __restrict__ cnt) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += stride)
    atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[col[e]]), 1ull);
}

// cursor: a copy of A^T's row pointer (start of every segment), advanced
// atomically as entries land.
__global__ __launch_bounds__(256) void csr_t_scatter(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                     int64_t m, unsigned long long* __restrict__ cursor,
                                                     int64_t* __restrict__ src) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < m; r += nw) {
    const int64_t e1 = rp[r + 1];
    for (int64_t e = rp[r] + lane; e < e1; e += 64) {
      const unsigned long long pos = atomicAdd(&cursor[col[e]], 1ull);
      src[pos] = e;
    }
  }
}

__device__ __forceinline__ int64_t shfl_xor64(int64_t v, int mask) {
  const int lo = __shfl_xor((int)(uint32_t)v, mask), hi = __shfl_xor((int)(v >> 32), mask);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// One wave per segment of 2..64 entries: lane i holds entry i (padding lanes
// hold INT64_MAX), bitonic network across lanes.
__global__ __launch_bounds__(256) void csr_t_sort_wave(const int64_t* __restrict__ trp,
                                                       const int64_t* __restrict__ rows, int64_t nrows,
                                                       int64_t* __restrict__ src) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nrows) return;   // wave-uniform
  const int64_t r = rows[i], s = trp[r];
  const int len = (int)(trp[r + 1] - s);
  int64_t v = lane < len ? src[s + lane] : INT64_MAX;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int64_t o = shfl_xor64(v, j);
      const bool lower = (lane & j) == 0, up = (lane & k) == 0;
      // the lower lane of a pair keeps the min when sorting up
      v = (lower == up) ? (o < v ? o : v) : (o > v ? o : v);
    }
  }
  if (lane < len) src[s + lane] = v;
}

// One 256-thread workgroup per segment of 65..2048 entries, bitonic in LDS
// over the next power of two.
__global__ __launch_bounds__(256) void csr_t_sort_lds(const int64_t* __restrict__ trp,
                                                      const int64_t* __restrict__ rows, int64_t* __restrict__ src) {
  __shared__ int64_t sh[kSortLds];
  const int tid = threadIdx.x;
  const int64_t r = rows[blockIdx.x], s = trp[r];
  const int len = (int)(trp[r + 1] - s);
  int n = 128;
  while (n < len) n <<= 1;
  for (int i = tid; i < n; i += 256) sh[i] = i < len ? src[s + i] : INT64_MAX;
  __syncthreads();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n; i += 256) {
        const int p = i ^ j;
        if (p > i) {
          const int64_t a = sh[i], b = sh[p];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            sh[i] = b;
            sh[p] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < len; i += 256) src[s + i] = sh[i];
}

}  // namespace

SPMM_EXPORT int spmm_csr_col_count(const int32_t* col, int64_t nnz, int64_t* cnt, void* stream) {
  if (nnz <= 0) return 0;
  const int64_t blocks = (nnz + 255) / 256;
  hipLaunchKernelGGL(csr_col_count, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                     (hipStream_t)stream, col, nnz, cnt);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_csr_t_scatter(const int64_t* rp, const int32_t* col, int64_t m, int64_t* cursor, int64_t* src,
                                   void* stream) {
  if (m <= 0) return 0;
  const int64_t blocks = (m + 3) / 4;
  hipLaunchKernelGGL(csr_t_scatter, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                     (hipStream_t)stream, rp, col, m, reinterpret_cast<unsigned long long*>(cursor), src);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// rows: segments of 2..64 entries (wave = 0) or 65..2048 (wave = 1)
SPMM_EXPORT int spmm_csr_t_sort(int lds, const int64_t* trp, const int64_t* rows, int64_t nrows, int64_t* src,
                                void* stream) {
  if (nrows <= 0) return 0;
  if (lds) {
    if (nrows > 0x7fffffffll) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(csr_t_sort_lds, dim3((unsigned)nrows), dim3(256), 0, (hipStream_t)stream, trp, rows, src);
  } else {
    hipLaunchKernelGGL(csr_t_sort_wave, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, trp,
                       rows, nrows, src);
  }
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_csr_t_sort_max() { return kSortLds; }
