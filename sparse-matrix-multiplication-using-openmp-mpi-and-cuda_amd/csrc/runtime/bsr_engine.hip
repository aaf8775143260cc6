// GPU block-sparse engine of the native `a4`: C = A (x) B on one stream.
//
// Replaces the reference's `helper` (sparse_matrix_mult.cu:97-286), which
// joins tile keys on the host with hash maps (:140-156), copies every
// contributing (A, B) tile pair into an 8 GB staging buffer in rounds of 500
// output tiles (:181-253) and unpacks into a std::map (:259-269).  Here every
// phase runs in HBM:
//   symbolic  spmm_bsr_sym_plan / spmm_bsr_sym_build (csrc/kernels/prim.hip,
//             shared with the Python engine): pair counts by binary search of
//             A's tile column in B's sorted tile rows -> scan -> pair fill with
//             compact output keys -> in-tree stable LSD radix sort (keeps the
//             ascending middle index per output tile, the reference's
//             summation order) -> run-length encode = tile_ptr
//   numeric   spmm_bsr_u64_numeric (csrc/kernels/bsr_u64.hip: LDS-tiled
//             gfx950 kernel, exact per-element order) + fused nonzero flags
//   prune     in-tree scan of the flags + tile gather (output-preserving,
//             SURVEY §2.4)
// Host syncs: pair total, output tile count, kept tile count.
#include "rt.hpp"

namespace a4 {
namespace {

constexpr int TPB = 256;

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

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
    DevBuf<char> ws(spmm_prim_scan_ws(n), s);
    if (spmm_prim_scan(flag, 4, n, pos.get() + 1, 1, ws.get(), s) != 0) throw Error("spmm_prim_scan failed");
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

  // ---- symbolic (shared with ops/bsr.py): pairs grouped by output tile
  DevBuf<int64_t> start((size_t)na + 1, s), lo((size_t)na, s);
  int64_t plan[5] = {0, 0, 0, 0, 0};
  {
    DevBuf<char> ws(spmm_bsr_sym_plan_ws(na), s);
    const int rc = spmm_bsr_sym_plan(A.keys.get(), na, B.keys.get(), nbB, start.get(), lo.get(), ws.get(), plan, s);
    A4_CHECK(rc == 0, "spmm_bsr_sym_plan failed (" + std::to_string(rc) + ")");
  }
  const int64_t np = plan[0];
  if (tile_pairs) *tile_pairs = np;
  if (np == 0) return C;
  A4_CHECK(np < (int64_t)INT32_MAX, "tile pair count exceeds the int32 pair indices");
  DevBuf<int32_t> okeys((size_t)np * 2, s), pa((size_t)np, s), pb((size_t)np, s);
  DevBuf<int64_t> tile_ptr((size_t)np + 1, s);
  int64_t nt = 0;
  {
    DevBuf<char> ws(spmm_bsr_sym_build_ws(np), s);
    const int rc = spmm_bsr_sym_build(A.keys.get(), B.keys.get(), na, start.get(), lo.get(), plan, ws.get(),
                                      okeys.get(), tile_ptr.get(), pa.get(), pb.get(), &nt, s);
    A4_CHECK(rc == 0, "spmm_bsr_sym_build failed (" + std::to_string(rc) + ")");
  }
  start.reset(); lo.reset();
  A4_CHECK(nt >= 1 && nt <= np, "bsr symbolic phase produced " + std::to_string(nt) + " tiles for " +
                                    std::to_string(np) + " pairs");

  // ---- numeric
  C.nb = nt;
  C.keys = DevBuf<int32_t>((size_t)nt * 2, s);
  C.vals = DevBuf<uint64_t>((size_t)nt * C.k * C.k, s);
  A4_HIP(hipMemcpyAsync(C.keys.get(), okeys.get(), (size_t)nt * 2 * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  okeys.reset();
  DevBuf<int32_t> nz((size_t)nt, s);
  A4_HIP(hipMemsetAsync(nz.get(), 0, (size_t)nt * 4, s));
  if (spmm_bsr_u64_numeric(A.vals.get(), B.vals.get(), pa.get(), pb.get(), tile_ptr.get(), C.vals.get(), nz.get(),
                           C.k, nt, s) != 0)
    throw Error("spmm_bsr_u64_numeric failed");

  // ---- prune intermediate zero tiles (output-preserving)
  return prune_with_flags(std::move(C), nz.get(), s);
}

}  // namespace a4
