// Native runtime core for the `a4` executable (SURVEY.md §7.1 csrc/core +
// csrc/format): error checking, RAII device buffers, the block-sparse matrix
// types and the engine / communicator interfaces.
//
// Reference parity: the reference is one C++/CUDA/MPI translation unit
// (sparse_matrix_mult.cu) whose `one_matrix` is a std::map of k x k uint64
// tiles (:26-32).  Here a matrix is sorted block-COO with contiguous
// [nb][k][k] values, on the host (Mat, std::vector) or in HBM (DevMat).
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace a4 {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define A4_HIP(call)                                                                                 \
  do {                                                                                               \
    hipError_t e_ = (call);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      throw ::a4::Error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" + \
                        std::to_string(__LINE__) + ": " #call);                                      \
  } while (0)

#define A4_CHECK(cond, msg)                          \
  do {                                               \
    if (!(cond)) throw ::a4::Error(std::string(msg)); \
  } while (0)

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Scoped roctx range: the phases the reference times with chrono and never
// prints (sparse_matrix_mult.cu:160-274) show up as named ranges in
// `rocprofv3 --marker-trace` timelines (load / multiply / send / recv / write).
class Range {
 public:
  explicit Range(const std::string& name) { roctxRangePushA(name.c_str()); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// Device memory arena (alloc.cpp): a caching allocator with explicit event
// ordering, in place of HIP's stream-ordered pool (hipMallocAsync).  A
// released block carries an event recorded on the stream of its last use; the
// next allocation that takes it makes its own stream wait on that event, so
// reuse is ordered after every earlier use whatever streams are involved, and
// nothing is returned to the driver before trim() (HBM is 288 GB).
// Streams that recorded a release must stay alive until trim().
class Arena {
 public:
  static Arena& get();
  void* alloc(size_t bytes, hipStream_t s);
  void release(void* p, size_t bytes, hipStream_t s);
  void trim();   // device-synchronises, frees every cached block
  size_t cached_bytes() const { return cached_; }
  size_t peak_bytes() const { return peak_; }

 private:
  struct Block {
    void* p;
    size_t bytes;
    hipEvent_t ev;
  };
  std::vector<Block> free_;   // small: a linear best-fit scan is cheap
  size_t cached_ = 0, live_ = 0, peak_ = 0;
  std::mutex mu_;
};

// Device buffer from the arena, released on the stream that last used it.
// Move-only.
template <typename T>
class DevBuf {
 public:
  DevBuf() = default;
  DevBuf(size_t n, hipStream_t s) : n_(n), s_(s) {
    if (n_) p_ = static_cast<T*>(Arena::get().alloc(n_ * sizeof(T), s_));
  }
  DevBuf(DevBuf&& o) noexcept : p_(o.p_), n_(o.n_), s_(o.s_) { o.p_ = nullptr; o.n_ = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { reset(); p_ = o.p_; n_ = o.n_; s_ = o.s_; o.p_ = nullptr; o.n_ = 0; }
    return *this;
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { reset(); }
  void reset() {
    if (p_) Arena::get().release(p_, n_ * sizeof(T), s_);
    p_ = nullptr;
    n_ = 0;
  }
  // the release is ordered after the work of `s` (the last user)
  void retarget(hipStream_t s) { s_ = s; }
  T* get() const { return p_; }
  size_t size() const { return n_; }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
  hipStream_t s_ = nullptr;
};

// Host matrix in the reference's logical layout: tiles sorted by (r, c),
// keys [nb][2], values [nb][k][k].
struct Mat {
  int64_t rows = 0, cols = 0;
  int k = 0;
  std::vector<int32_t> keys;
  std::vector<uint64_t> vals;
  int64_t nb() const { return (int64_t)keys.size() / 2; }
  size_t bytes() const { return keys.size() * 4 + vals.size() * 8; }
};

// Device matrix (HBM resident).
struct DevMat {
  int64_t rows = 0, cols = 0;
  int k = 0;
  int64_t nb = 0;
  DevBuf<int32_t> keys;    // [nb][2]
  DevBuf<uint64_t> vals;   // [nb][k][k]
  size_t bytes() const { return (size_t)nb * (8 + (size_t)k * k * 8); }
};

// Order-preserving uint64 code of a signed (r, c) pair.
__host__ __device__ inline uint64_t encode_key(int32_t r, int32_t c) {
  return ((uint64_t)((uint32_t)r ^ 0x80000000u) << 32) | (uint64_t)((uint32_t)c ^ 0x80000000u);
}
__host__ __device__ inline int32_t key_r(uint64_t code) { return (int32_t)((uint32_t)(code >> 32) ^ 0x80000000u); }
__host__ __device__ inline int32_t key_c(uint64_t code) { return (int32_t)((uint32_t)code ^ 0x80000000u); }

// ---- engines ---------------------------------------------------------------
// GPU engine (bsr_engine.hip): C = A (x) B with the reference arithmetic,
// zero tiles pruned.  All work is ordered on `s`; returns after the output
// sizes are known (one host sync per phase).
DevMat dev_multiply(const DevMat& A, const DevMat& B, hipStream_t s, int64_t* tile_pairs);
DevMat dev_upload(const Mat& M, hipStream_t s);
Mat dev_download(const DevMat& M, hipStream_t s);
DevMat dev_prune(DevMat M, hipStream_t s);
// CPU engine (cpu_engine.cpp, OpenMP).
Mat cpu_multiply(const Mat& A, const Mat& B, int nthreads, int64_t* tile_pairs);
Mat cpu_prune(Mat M);
void canonicalize(Mat& M);   // sort by (r, c), last duplicate wins (std::map insert semantics)

}  // namespace a4

// Kernels exported by libspmm_hip.so / libspmm_host.so (csrc/kernels, csrc/host).
extern "C" {
int spmm_bsr_u64_numeric(const void* Avals, const void* Bvals, const int32_t* pa, const int32_t* pb,
                         const int64_t* tile_ptr, void* Cvals, int32_t* nz_flag, int k, int64_t ntiles,
                         void* stream);
int spmm_bsr_u64_nonzero(const void* vals, int k, int64_t ntiles, int32_t* nz_flag, void* stream);
// in-tree primitives and the shared symbolic phase (csrc/kernels/prim.hip)
size_t spmm_prim_scan_ws(int64_t n);
int spmm_prim_scan(const void* in, int in_bytes, int64_t n, int64_t* out, int inclusive, void* ws, void* stream);
size_t spmm_bsr_sym_plan_ws(int64_t na);
int spmm_bsr_sym_plan(const int32_t* akeys, int64_t na, const int32_t* bkeys, int64_t nb, int64_t* start, int64_t* lo,
                      void* ws, int64_t* plan, void* stream);
size_t spmm_bsr_sym_build_ws(int64_t np);
int spmm_bsr_sym_build(const int32_t* akeys, const int32_t* bkeys, int64_t na, const int64_t* start, const int64_t* lo,
                       const int64_t* plan, void* ws, int32_t* okeys, int64_t* tile_ptr, int32_t* pa, int32_t* pb,
                       int64_t* nt, void* stream);
int spmm_cpu_bsr_u64_numeric(const uint64_t* A, const uint64_t* B, const int32_t* pa, const int32_t* pb,
                             const int64_t* tile_ptr, uint64_t* C, int32_t* nz_flag, int k, int64_t ntiles,
                             int nthreads);
void* spmm_ref_open(const char* path, int k, int64_t* rows, int64_t* cols, int64_t* blocks, char* err, int errlen);
int spmm_ref_fill(void* handle, int32_t* keys, uint64_t* vals, int nthreads, char* err, int errlen);
void spmm_ref_close(void* handle);
int spmm_ref_write(const char* path, int64_t R, int64_t C, int64_t nb, const int32_t* keys, const uint64_t* vals,
                   int k, int nthreads);
}
