// Device row utilities of the binned SpGEMM path: row binning by the shared bin table, flagged-row
// selection, and the re-sort of listed CSR rows (the SpGEMM rows whose LDS table could not keep
// its output column-sorted, flag 1): one engine for the Python front end
// (ops/csr.py sort_rows) and the native chain (csrc/runtime/csr_engine.cpp), which
// re-sorted them on the host one row at a time (round 4).  The reference keeps its
// output ordered through std::map on the host (sparse_matrix_mult.cu:287-327).
//
// Entries are packed as int64 keys (column << 32 | value bits): a row's columns are
// distinct, so sorting the keys sorts by column and carries the value along.
//   rs_pack      one wave per listed row: keys into a compact buffer at toff[i]
//   rs_sort_wave rows of <= 64 entries: bitonic across the lanes of one wave
//   rs_sort_lds  rows of 65..kRsLds entries: one 1024-thread workgroup, bitonic in LDS
//   (longer)     every listed row at once through the in-tree radix sort (prim.hip)
//                on (row index << 31 | column) keys
//   rs_unpack    keys back into the row
#include "common.hpp"

#include <algorithm>

extern "C" {
int spmm_prim_scan(const void* in, int in_bytes, int64_t n, int64_t* out, int inclusive, void* ws, void* stream);
size_t spmm_prim_scan_ws(int64_t n);
size_t spmm_prim_sort_ws(int64_t n);
int spmm_prim_sort_pairs_u64(uint64_t* keys, uint64_t* vals, int64_t n, int bits, void* ws, void* stream);
int spmm_spgemm_bin_caps(int numeric, double load, double load_sliced, int64_t esc_min, int64_t* caps);
}

namespace {

constexpr int kRsLds = 16384;   // 128 KB of LDS
constexpr int kRsNt = 1024;

__global__ __launch_bounds__(256) void rs_lens(const int64_t* __restrict__ rp, const int64_t* __restrict__ rows,
                                               int64_t nrows, int64_t* __restrict__ len,
                                               unsigned long long* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nrows) len[i] = rp[rows[i] + 1] - rp[rows[i]];
  if (i == 0) cnt[i] = 0;
}

// radix: key = (i << 31) | column, value = value bits; otherwise key = column << 32 | bits
template <bool RADIX>
__global__ __launch_bounds__(256) void rs_pack(const int64_t* __restrict__ rp, const int64_t* __restrict__ rows,
                                               int64_t nrows, const int64_t* __restrict__ toff,
                                               const int32_t* __restrict__ ci, const uint32_t* __restrict__ v,
                                               uint64_t* __restrict__ key, uint64_t* __restrict__ val) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nrows) return;
  const int64_t s = rp[rows[i]], n = rp[rows[i] + 1] - s, d = toff[i];
  for (int64_t e = lane; e < n; e += 64) {
    const uint64_t c = (uint32_t)ci[s + e];
    if (RADIX) {
      key[d + e] = ((uint64_t)i << 31) | c;
      val[d + e] = v[s + e];
    } else {
      key[d + e] = (c << 32) | v[s + e];
    }
  }
}

template <bool RADIX>
__global__ __launch_bounds__(256) void rs_unpack(const int64_t* __restrict__ rp, const int64_t* __restrict__ rows,
                                                 int64_t nrows, const int64_t* __restrict__ toff,
                                                 const uint64_t* __restrict__ key, const uint64_t* __restrict__ val,
                                                 int32_t* __restrict__ ci, uint32_t* __restrict__ v) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nrows) return;
  const int64_t s = rp[rows[i]], n = rp[rows[i] + 1] - s, d = toff[i];
  for (int64_t e = lane; e < n; e += 64) {
    const uint64_t k = key[d + e];
    if (RADIX) {
      ci[s + e] = (int32_t)(k & 0x7fffffffu);
      v[s + e] = (uint32_t)val[d + e];
    } else {
      ci[s + e] = (int32_t)(k >> 32);
      v[s + e] = (uint32_t)k;
    }
  }
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int mask) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, mask), hi = (uint32_t)__shfl_xor((int)(x >> 32), mask);
  return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void rs_sort_wave(const int64_t* __restrict__ toff, int64_t nrows,
                                                    uint64_t* __restrict__ key) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nrows) return;   // wave-uniform
  const int64_t s = toff[i];
  const int64_t len = toff[i + 1] - s;
  if (len < 2 || len > 64) return;
  uint64_t x = lane < len ? key[s + lane] : ~0ull;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint64_t o = shfl_xor_u64(x, j);
      const bool lower = (lane & j) == 0, up = (lane & k) == 0;
      x = (lower == up) ? (o < x ? o : x) : (o > x ? o : x);
    }
  }
  if (lane < len) key[s + lane] = x;
}

// the listed rows of 65..kRsLds entries, appended to mid[0 .. *cnt) (any order; *cnt zeroed by rs_lens)
__global__ __launch_bounds__(256) void rs_select_mid(const int64_t* __restrict__ toff, int64_t nrows,
                                                     int32_t* __restrict__ mid, unsigned long long* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t len = 0;
  if (i < nrows) len = toff[i + 1] - toff[i];
  const bool hit = len > 64 && len <= kRsLds;
  const unsigned long long b = __ballot(hit);
  if (!b) return;
  const int lane = threadIdx.x & 63, first = __ffsll((long long)b) - 1;
  unsigned long long base = 0;
  if (lane == first) base = atomicAdd(cnt, (unsigned long long)__popcll(b));
  base = __shfl(base, first);
  if (hit) mid[base + __popcll(b & ((1ull << lane) - 1ull))] = (int32_t)i;
}

// One 1024-thread workgroup per row of mid (a grid of at most one workgroup per CU looping over
// the list: the 128 KB of LDS admits one per CU, so a workgroup per listed row -- most of them
// short -- spent a slot on every row just to exit)
__global__ __launch_bounds__(kRsNt) void rs_sort_lds(const int64_t* __restrict__ toff, const int32_t* __restrict__ mid,
                                                     const unsigned long long* __restrict__ cnt,
                                                     uint64_t* __restrict__ key) {
  __shared__ uint64_t sh[kRsLds];
  const int tid = threadIdx.x;
  const int64_t nmid = (int64_t)*cnt;
  for (int64_t r = blockIdx.x; r < nmid; r += gridDim.x) {
    const int64_t row = mid[r];
    const int64_t s = toff[row];
    const int len = (int)(toff[row + 1] - s);
    int n = 128;
    while (n < len) n <<= 1;
    for (int i = tid; i < n; i += kRsNt) sh[i] = i < len ? key[s + i] : ~0ull;
    __syncthreads();
    for (int k = 2; k <= n; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < n; i += kRsNt) {
          const int p = i ^ j;
          if (p > i) {
            const uint64_t a = sh[i], b = sh[p];
            if ((a > b) == ((i & k) == 0)) {
              sh[i] = b;
              sh[p] = a;
            }
          }
        }
        __syncthreads();
      }
    }
    for (int i = tid; i < len; i += kRsNt) key[s + i] = sh[i];
    __syncthreads();   // the row's LDS reads done before the next row's loads
  }
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// ---- row binning of the binned SpGEMM path (the native engine's device planner) ----------
struct Caps {
  int64_t c[11];
};

// key = bin + 1 (0: empty row, 1..11: LDS bins 0..10, 12: long-row path); hist[key] counts
__global__ __launch_bounds__(256) void rb_keys(const int64_t* __restrict__ nprod, int64_t m, Caps caps,
                                               uint64_t* __restrict__ key, uint64_t* __restrict__ val,
                                               unsigned long long* __restrict__ hist) {
  __shared__ unsigned int h[13];
  if (threadIdx.x < 13) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < m) {
    const int64_t p = nprod[r];
    int k = 12;
    if (p == 0) {
      k = 0;
    } else {
      for (int b = 10; b >= 0; --b)
        if (p <= caps.c[b]) k = b + 1;
    }
    key[r] = (uint64_t)k;
    val[r] = (uint64_t)r;
    atomicAdd(&h[k], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 13 && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void rb_order(const uint64_t* __restrict__ val, int64_t m, int32_t* __restrict__ order) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < m) order[i] = (int32_t)val[i];
}

// rows r with flags[r] & mask, appended at out[*count] (any order)
__global__ __launch_bounds__(256) void rb_select(const int32_t* __restrict__ flags, int64_t m, int mask,
                                                 int32_t* __restrict__ out, unsigned long long* __restrict__ count) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool hit = r < m && (flags[r] & mask) != 0;
  const unsigned long long b = __ballot(hit);
  if (!b) return;
  const int lane = threadIdx.x & 63;
  unsigned long long base = 0;
  if (lane == __ffsll((long long)b) - 1) base = atomicAdd(count, (unsigned long long)__popcll(b));
  base = __shfl(base, __ffsll((long long)b) - 1);
  if (hit) out[base + __popcll(b & ((1ull << lane) - 1ull))] = (int32_t)r;
}

}  // namespace

SPMM_EXPORT size_t spmm_spgemm_bin_rows_ws(int64_t m) {
  return align256((size_t)m * 8) * 2 + align256(spmm_prim_sort_ws(m));
}

// The rows of the binned path ordered by bin (stable: ascending row ids inside a bin), with the
// bin table of spmm_spgemm_bin_caps: order[m] (int32), hist[13] (int64, device) = empty rows,
// then bins 0..10, then the long-row path.  Launches only (ops/spgemm.py _bins + _group).
SPMM_EXPORT int spmm_spgemm_bin_rows(const int64_t* nprod, int64_t m, int numeric, double load, double load_sliced,
                                     int64_t esc_min, int32_t* order, int64_t* hist, void* ws, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(hist, 0, 13 * sizeof(int64_t), s) != hipSuccess) return (int)hipErrorUnknown;
  if (m <= 0) return 0;
  if (m >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  Caps caps;
  spmm_spgemm_bin_caps(numeric, load, load_sliced, esc_min, caps.c);
  char* p = (char*)ws;
  uint64_t* key = (uint64_t*)p;
  p += align256((size_t)m * 8);
  uint64_t* val = (uint64_t*)p;
  p += align256((size_t)m * 8);
  const dim3 g((unsigned)((m + 255) / 256));
  hipLaunchKernelGGL(rb_keys, g, dim3(256), 0, s, nprod, m, caps, key, val, (unsigned long long*)hist);
  SPMM_LAUNCH_CHECK();
  const int rc = spmm_prim_sort_pairs_u64(key, val, m, 4, p, s);
  if (rc) return rc;
  hipLaunchKernelGGL(rb_order, g, dim3(256), 0, s, val, m, order);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Rows whose flag word has a bit of mask: out[0 .. *count) (device count, zeroed here; any order).
SPMM_EXPORT int spmm_rows_with_flag(const int32_t* flags, int64_t m, int mask, int32_t* out, int64_t* count,
                                    void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(count, 0, sizeof(int64_t), s) != hipSuccess) return (int)hipErrorUnknown;
  if (m <= 0) return 0;
  hipLaunchKernelGGL(rb_select, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, flags, m, mask, out,
                     (unsigned long long*)count);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Workspace bytes of spmm_csr_sort_rows for nrows listed rows holding total entries.
SPMM_EXPORT size_t spmm_csr_sort_rows_ws(int64_t nrows, int64_t total, int64_t maxlen) {
  size_t b = align256((size_t)(nrows + 1) * 8) * 2 + align256(spmm_prim_scan_ws(nrows + 1)) +
             align256((size_t)total * 8) + align256((size_t)nrows * 4) + 256;
  if (maxlen > kRsLds) b += align256((size_t)total * 8) + align256(spmm_prim_sort_ws(total));
  return b;
}

// Sort the entries of rows[0..nrows) (int64 row ids, device) of the CSR (rp, ci, v) by column,
// in place.  total = sum of their lengths, maxlen = the longest (host values: the caller
// sizes the workspace with spmm_csr_sort_rows_ws from them).  Launches only.
SPMM_EXPORT int spmm_csr_sort_rows(const int64_t* rp, const int64_t* rows, int64_t nrows, int64_t total, int64_t maxlen,
                                   int32_t* ci, float* v, void* ws, void* stream) {
  if (nrows <= 0 || total <= 0 || maxlen < 2) return 0;
  if (nrows >= ((int64_t)1 << 32) || (nrows + 3) / 4 > (int64_t)UINT32_MAX) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  char* p = (char*)ws;
  int64_t* len = (int64_t*)p;
  p += align256((size_t)(nrows + 1) * 8);
  int64_t* toff = (int64_t*)p;
  p += align256((size_t)(nrows + 1) * 8);
  char* scan_ws = p;
  p += align256(spmm_prim_scan_ws(nrows + 1));
  uint64_t* key = (uint64_t*)p;
  p += align256((size_t)total * 8);
  int32_t* mid = (int32_t*)p;   // rows for the LDS sort, and their count
  p += align256((size_t)nrows * 4);
  unsigned long long* nmid = (unsigned long long*)p;
  p += 256;
  const bool radix = maxlen > kRsLds;
  hipLaunchKernelGGL(rs_lens, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, rp, rows, nrows, len, nmid);
  SPMM_LAUNCH_CHECK();
  (void)hipMemsetAsync(len + nrows, 0, 8, s);
  int rc = spmm_prim_scan(len, 8, nrows + 1, toff, 0, scan_ws, s);   // exclusive: toff[nrows] = total
  if (rc) return rc;
  const dim3 gw((unsigned)((nrows + 3) / 4));
  if (radix) {
    uint64_t* val = (uint64_t*)p;
    p += align256((size_t)total * 8);
    hipLaunchKernelGGL(rs_pack<true>, gw, dim3(256), 0, s, rp, rows, nrows, toff, ci, (const uint32_t*)v, key, val);
    SPMM_LAUNCH_CHECK();
    int bits = 31;
    while (bits < 63 && ((int64_t)1 << (bits - 31)) < nrows) ++bits;
    rc = spmm_prim_sort_pairs_u64(key, val, total, bits, p, s);
    if (rc) return rc;
    hipLaunchKernelGGL(rs_unpack<true>, gw, dim3(256), 0, s, rp, rows, nrows, toff, key, val, ci, (uint32_t*)v);
  } else {
    hipLaunchKernelGGL(rs_pack<false>, gw, dim3(256), 0, s, rp, rows, nrows, toff, ci, (const uint32_t*)v, key,
                       nullptr);
    SPMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(rs_sort_wave, gw, dim3(256), 0, s, toff, nrows, key);
    SPMM_LAUNCH_CHECK();
    if (maxlen > 64) {
      hipLaunchKernelGGL(rs_select_mid, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, toff, nrows, mid, nmid);
      SPMM_LAUNCH_CHECK();
      int dev = 0, ncu = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
      hipLaunchKernelGGL(rs_sort_lds, dim3((unsigned)std::min<int64_t>(nrows, ncu)), dim3(kRsNt), 0, s, toff, mid,
                         nmid, key);
      SPMM_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(rs_unpack<false>, gw, dim3(256), 0, s, rp, rows, nrows, toff, key, nullptr, ci, (uint32_t*)v);
  }
  SPMM_LAUNCH_CHECK();
  return 0;
}
