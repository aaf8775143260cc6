// GPU block-sparse engine of the native `a4`: C = A (x) B on one stream.
//
// Replaces the reference's `helper` (sparse_matrix_mult.cu:97-286), which
// joins tile keys on the host with hash maps (:140-156), copies every
// contributing (A, B) tile pair into an 8 GB staging buffer in rounds of 500
// output tiles (:181-253) and unpacks into a std::map (:259-269).  Here every
// phase runs in HBM:
//   symbolic  k_count (binary search of A's tile column in B's sorted tile
//             rows) -> scan -> k_fill (pair codes) -> stable radix sort by
//             output key (keeps ascending middle index per output tile, the
//             reference's summation order) -> run-length encode = tile_ptr
//   numeric   spmm_bsr_u64_numeric (csrc/kernels/bsr_u64.hip: LDS-tiled
//             gfx950 kernel, exact per-element order) + fused nonzero flags
//   prune     scan of the flags + tile gather (output-preserving)
// Host syncs: pair total, output tile count, kept tile count.
#include <hipcub/hipcub.hpp>

#include "rt.hpp"

namespace a4 {
namespace {

constexpr int TPB = 256;

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

__global__ void k_count(const int32_t* __restrict__ akeys, int64_t na, const int32_t* __restrict__ bkeys, int64_t nb,
                        int64_t* __restrict__ cnt, int64_t* __restrict__ lo) {
  const int64_t a = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (a >= na) return;
  const int32_t j = akeys[2 * a + 1];
  int64_t l = 0, h = nb;
  while (l < h) {   // first B tile with row >= j
    const int64_t m = (l + h) >> 1;
    if (bkeys[2 * m] < j) l = m + 1; else h = m;
  }
  const int64_t first = l;
  h = nb;
  while (l < h) {   // first B tile with row > j
    const int64_t m = (l + h) >> 1;
    if (bkeys[2 * m] <= j) l = m + 1; else h = m;
  }
  cnt[a] = l - first;
  lo[a] = first;
}

// Pair p of A tile a: output key (A.row, B.col), payload (a << 32 | b).
__global__ void k_fill(const int32_t* __restrict__ akeys, const int32_t* __restrict__ bkeys, int64_t na,
                       const int64_t* __restrict__ start, const int64_t* __restrict__ lo,
                       uint64_t* __restrict__ code, uint64_t* __restrict__ ab) {
  const int64_t a = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (a >= na) return;
  const int32_t r = akeys[2 * a];
  const int64_t p0 = start[a], n = start[a + 1] - p0, b0 = lo[a];
  for (int64_t t = 0; t < n; ++t) {
    const int64_t b = b0 + t;
    code[p0 + t] = encode_key(r, bkeys[2 * b + 1]);
    ab[p0 + t] = ((uint64_t)a << 32) | (uint64_t)b;
  }
}

__global__ void k_split(const uint64_t* __restrict__ ab, int64_t n, int32_t* __restrict__ pa, int32_t* __restrict__ pb) {
  const int64_t p = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (p >= n) return;
  pa[p] = (int32_t)(ab[p] >> 32);
  pb[p] = (int32_t)(ab[p] & 0xffffffffu);
}

__global__ void k_decode(const uint64_t* __restrict__ code, int64_t n, int32_t* __restrict__ keys) {
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= n) return;
  keys[2 * t] = key_r(code[t]);
  keys[2 * t + 1] = key_c(code[t]);
}

// Kept tiles: dst slot = exclusive scan of the flags.
__global__ void k_gather_tiles(const int32_t* __restrict__ keys, const uint64_t* __restrict__ vals,
                               const int32_t* __restrict__ flag, const int64_t* __restrict__ pos, int64_t n,
                               int64_t kk, int32_t* __restrict__ okeys, uint64_t* __restrict__ ovals) {
  const int64_t t = blockIdx.x;
  if (t >= n || !flag[t]) return;
  const int64_t d = pos[t];
  if (threadIdx.x == 0) {
    okeys[2 * d] = keys[2 * t];
    okeys[2 * d + 1] = keys[2 * t + 1];
  }
  for (int64_t e = threadIdx.x; e < kk; e += blockDim.x) ovals[d * kk + e] = vals[t * kk + e];
}

// Largest A / B tile index referenced by the sorted pairs, + 1 (0 = none):
// the host checks them against the operand sizes before the numeric kernel
// gathers tiles by these indices.
__global__ void k_pair_bounds(const uint64_t* __restrict__ ab, int64_t n, unsigned long long* __restrict__ bounds) {
  const int64_t p = (int64_t)blockIdx.x * TPB + threadIdx.x;
  unsigned long long a = 0, b = 0;
  if (p < n) {
    a = (ab[p] >> 32) + 1;
    b = (ab[p] & 0xffffffffu) + 1;
  }
  for (int d = 32; d > 0; d >>= 1) {
    a = max(a, (unsigned long long)__shfl_xor(a, d));
    b = max(b, (unsigned long long)__shfl_xor(b, d));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&bounds[0], a);
    atomicMax(&bounds[1], b);
  }
}

// A few pinned int64 slots per host thread for the size read-backs.
int64_t* pinned_scratch() {
  thread_local int64_t* p = nullptr;
  if (!p) A4_HIP(hipHostMalloc(reinterpret_cast<void**>(&p), 8 * sizeof(int64_t), hipHostMallocDefault));
  return p;
}

// Copies n (<= 8) int64 values from the device and waits for them.
const int64_t* read_back_n(const int64_t* dptr, int n, hipStream_t s) {
  int64_t* h = pinned_scratch();
  A4_HIP(hipMemcpyAsync(h, dptr, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  A4_HIP(hipStreamSynchronize(s));
  return h;
}

int64_t read_back(const int64_t* dptr, hipStream_t s) { return read_back_n(dptr, 1, s)[0]; }

template <typename F>
DevBuf<char> cub_temp(F&& query, hipStream_t s) {
  size_t bytes = 0;
  A4_HIP(query(nullptr, bytes));
  return DevBuf<char>(bytes ? bytes : 1, s);
}

}  // namespace

DevMat dev_upload(const Mat& M, hipStream_t s) {
  DevMat D;
  D.rows = M.rows; D.cols = M.cols; D.k = M.k; D.nb = M.nb();
  D.keys = DevBuf<int32_t>(M.keys.size(), s);
  D.vals = DevBuf<uint64_t>(M.vals.size(), s);
  if (D.nb) {
    A4_HIP(hipMemcpyAsync(D.keys.get(), M.keys.data(), M.keys.size() * 4, hipMemcpyHostToDevice, s));
    A4_HIP(hipMemcpyAsync(D.vals.get(), M.vals.data(), M.vals.size() * 8, hipMemcpyHostToDevice, s));
  }
  return D;
}

Mat dev_download(const DevMat& D, hipStream_t s) {
  Mat M;
  M.rows = D.rows; M.cols = D.cols; M.k = D.k;
  M.keys.resize((size_t)D.nb * 2);
  M.vals.resize((size_t)D.nb * D.k * D.k);
  if (D.nb) {
    A4_HIP(hipMemcpyAsync(M.keys.data(), D.keys.get(), M.keys.size() * 4, hipMemcpyDeviceToHost, s));
    A4_HIP(hipMemcpyAsync(M.vals.data(), D.vals.get(), M.vals.size() * 8, hipMemcpyDeviceToHost, s));
  }
  A4_HIP(hipStreamSynchronize(s));
  return M;
}

static DevMat prune_with_flags(DevMat C, const int32_t* flag, hipStream_t s) {
  const int64_t n = C.nb;
  if (n == 0) return C;
  DevBuf<int64_t> pos((size_t)n + 1, s);
  A4_HIP(hipMemsetAsync(pos.get(), 0, sizeof(int64_t), s));
  {
    // inclusive sum of flags into pos[1..n] -> pos[t] = exclusive prefix
    auto q = [&](void* t, size_t& b) {
      return hipcub::DeviceScan::InclusiveSum(t, b, flag, pos.get() + 1, (int)n, s);
    };
    DevBuf<char> tmp = cub_temp(q, s);
    size_t b = tmp.size();
    A4_HIP(hipcub::DeviceScan::InclusiveSum(tmp.get(), b, flag, pos.get() + 1, (int)n, s));
  }
  const int64_t kept = read_back(pos.get() + n, s);
  if (kept == n) return C;
  const int64_t kk = (int64_t)C.k * C.k;
  DevMat P;
  P.rows = C.rows; P.cols = C.cols; P.k = C.k; P.nb = kept;
  P.keys = DevBuf<int32_t>((size_t)kept * 2, s);
  P.vals = DevBuf<uint64_t>((size_t)kept * kk, s);
  if (kept)
    hipLaunchKernelGGL(k_gather_tiles, dim3((unsigned)n), dim3(TPB), 0, s, C.keys.get(), C.vals.get(), flag,
                       pos.get(), n, kk, P.keys.get(), P.vals.get());
  A4_HIP(hipGetLastError());
  return P;
}

DevMat dev_prune(DevMat M, hipStream_t s) {
  if (M.nb == 0) return M;
  DevBuf<int32_t> flag((size_t)M.nb, s);
  A4_HIP(hipMemsetAsync(flag.get(), 0, (size_t)M.nb * 4, s));
  if (spmm_bsr_u64_nonzero(M.vals.get(), M.k, M.nb, flag.get(), s) != 0) throw Error("spmm_bsr_u64_nonzero failed");
  return prune_with_flags(std::move(M), flag.get(), s);
}

DevMat dev_multiply(const DevMat& A, const DevMat& B, hipStream_t s, int64_t* tile_pairs) {
  A4_CHECK(A.k == B.k, "tile size mismatch");
  DevMat C;
  C.rows = A.rows; C.cols = B.cols; C.k = A.k; C.nb = 0;
  if (tile_pairs) *tile_pairs = 0;
  const int64_t na = A.nb, nbB = B.nb;
  if (na == 0 || nbB == 0) return C;

  // ---- symbolic: pair counts and their offsets
  DevBuf<int64_t> cnt((size_t)na, s), lo((size_t)na, s), start((size_t)na + 1, s);
  hipLaunchKernelGGL(k_count, dim3(blocks_for(na)), dim3(TPB), 0, s, A.keys.get(), na, B.keys.get(), nbB, cnt.get(),
                     lo.get());
  A4_HIP(hipGetLastError());
  A4_HIP(hipMemsetAsync(start.get(), 0, sizeof(int64_t), s));
  {
    auto q = [&](void* t, size_t& b) {
      return hipcub::DeviceScan::InclusiveSum(t, b, cnt.get(), start.get() + 1, (int)na, s);
    };
    DevBuf<char> tmp = cub_temp(q, s);
    size_t b = tmp.size();
    A4_HIP(hipcub::DeviceScan::InclusiveSum(tmp.get(), b, cnt.get(), start.get() + 1, (int)na, s));
  }
  const int64_t np = read_back(start.get() + na, s);
  if (tile_pairs) *tile_pairs = np;
  if (np == 0) return C;
  A4_CHECK(np < (int64_t)INT32_MAX, "tile pair count exceeds the sort's 2^31 limit");

  DevBuf<uint64_t> code((size_t)np, s), ab((size_t)np, s);
  hipLaunchKernelGGL(k_fill, dim3(blocks_for(na)), dim3(TPB), 0, s, A.keys.get(), B.keys.get(), na, start.get(),
                     lo.get(), code.get(), ab.get());
  A4_HIP(hipGetLastError());
  cnt.reset(); lo.reset(); start.reset();

  // stable radix sort by output key: ascending middle index survives inside a tile
  DevBuf<uint64_t> code2((size_t)np, s), ab2((size_t)np, s);
  {
    auto q = [&](void* t, size_t& b) {
      return hipcub::DeviceRadixSort::SortPairs(t, b, code.get(), code2.get(), ab.get(), ab2.get(), (int)np, 0, 64, s);
    };
    DevBuf<char> tmp = cub_temp(q, s);
    size_t b = tmp.size();
    A4_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.get(), b, code.get(), code2.get(), ab.get(), ab2.get(), (int)np, 0,
                                              64, s));
  }
  code.reset(); ab.reset();

  // output tiles = runs of equal keys
  DevBuf<uint64_t> uniq((size_t)np, s);
  DevBuf<int64_t> runs((size_t)np + 1, s);
  DevBuf<int64_t> nruns(1, s);
  {
    auto q = [&](void* t, size_t& b) {
      return hipcub::DeviceRunLengthEncode::Encode(t, b, code2.get(), uniq.get(), runs.get() + 1, nruns.get(), (int)np, s);
    };
    DevBuf<char> tmp = cub_temp(q, s);
    size_t b = tmp.size();
    A4_HIP(hipcub::DeviceRunLengthEncode::Encode(tmp.get(), b, code2.get(), uniq.get(), runs.get() + 1, nruns.get(),
                                                 (int)np, s));
  }
  const int64_t nt = read_back(nruns.get(), s);
  code2.reset();
  DevBuf<int64_t> tile_ptr((size_t)nt + 1, s);
  A4_HIP(hipMemsetAsync(tile_ptr.get(), 0, sizeof(int64_t), s));
  {
    auto q = [&](void* t, size_t& b) {
      return hipcub::DeviceScan::InclusiveSum(t, b, runs.get() + 1, tile_ptr.get() + 1, (int)nt, s);
    };
    DevBuf<char> tmp = cub_temp(q, s);
    size_t b = tmp.size();
    A4_HIP(hipcub::DeviceScan::InclusiveSum(tmp.get(), b, runs.get() + 1, tile_ptr.get() + 1, (int)nt, s));
  }
  runs.reset();
  // Host-side guard of the numeric kernel's assumptions: the groups cover
  // exactly the np pairs and every pair indexes existing A / B tiles.
  {
    DevBuf<int64_t> chk(3, s);
    A4_HIP(hipMemsetAsync(chk.get(), 0, 2 * sizeof(int64_t), s));
    hipLaunchKernelGGL(k_pair_bounds, dim3(blocks_for(np)), dim3(TPB), 0, s, ab2.get(), np,
                       reinterpret_cast<unsigned long long*>(chk.get()));
    A4_HIP(hipGetLastError());
    A4_HIP(hipMemcpyAsync(chk.get() + 2, tile_ptr.get() + nt, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    const int64_t* h = read_back_n(chk.get(), 3, s);
    A4_CHECK(h[2] == np && h[0] >= 1 && h[0] <= na && h[1] >= 1 && h[1] <= nbB,
             "bsr symbolic phase produced inconsistent pairs (groups " + std::to_string(h[2]) + "/" +
                 std::to_string(np) + ", max A tile " + std::to_string(h[0] - 1) + "/" + std::to_string(na) +
                 ", max B tile " + std::to_string(h[1] - 1) + "/" + std::to_string(nbB) + ")");
  }
  DevBuf<int32_t> pa((size_t)np, s), pb((size_t)np, s);
  hipLaunchKernelGGL(k_split, dim3(blocks_for(np)), dim3(TPB), 0, s, ab2.get(), np, pa.get(), pb.get());
  A4_HIP(hipGetLastError());
  ab2.reset();

  // ---- numeric
  C.nb = nt;
  C.keys = DevBuf<int32_t>((size_t)nt * 2, s);
  C.vals = DevBuf<uint64_t>((size_t)nt * C.k * C.k, s);
  hipLaunchKernelGGL(k_decode, dim3(blocks_for(nt)), dim3(TPB), 0, s, uniq.get(), nt, C.keys.get());
  A4_HIP(hipGetLastError());
  uniq.reset();
  DevBuf<int32_t> nz((size_t)nt, s);
  A4_HIP(hipMemsetAsync(nz.get(), 0, (size_t)nt * 4, s));
  if (spmm_bsr_u64_numeric(A.vals.get(), B.vals.get(), pa.get(), pb.get(), tile_ptr.get(), C.vals.get(), nz.get(),
                           C.k, nt, s) != 0)
    throw Error("spmm_bsr_u64_numeric failed");

  // ---- prune intermediate zero tiles (output-preserving)
  return prune_with_flags(std::move(C), nz.get(), s);
}

}  // namespace a4
