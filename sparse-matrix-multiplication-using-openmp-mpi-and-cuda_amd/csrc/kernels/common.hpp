// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of spmm_amd.
//
// Every launcher is exported with C linkage and takes raw device pointers plus
// the hipStream_t the caller (PyTorch's current stream, or the C++ runtime's
// stream pool) wants the work on.  Launchers return a hipError_t as int and
// never synchronise, so they can be captured into hipGraphs.
//
// Error handling replaces the reference's CUDA_CHECK (sparse_matrix_mult.cu:33-41),
// which only guarded allocations: here every launch is followed by a
// hipGetLastError() check.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SPMM_EXPORT extern "C" __attribute__((visibility("default")))

#define SPMM_LAUNCH_CHECK()                          \
  do {                                               \
    hipError_t _e = hipGetLastError();               \
    if (_e != hipSuccess) return (int)_e;            \
  } while (0)

namespace spmm {

constexpr int kWave = 64;      // CDNA wavefront width
constexpr int kNumXcd = 8;     // MI355X: 8 XCDs, 32 CUs each

// The reference's element step (sparse_matrix_mult.cu:57-61):
//   t = (a*b) % MAX; acc = (acc + t) % MAX;   MAX = 2^64-1
// where a*b and acc+t first wrap mod 2^64.  x % (2^64-1) for a 64-bit x is x
// unless x == 2^64-1, where it is 0, so the step is two compare/selects with
// no 64-bit division.
__device__ __forceinline__ uint64_t ref_mac(uint64_t acc, uint64_t a, uint64_t b) {
  uint64_t t = a * b;
  t = (t == ~0ull) ? 0ull : t;
  uint64_t s = acc + t;
  return (s == ~0ull) ? 0ull : s;
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): consecutive logical ids land on the same
// XCD so neighbouring work shares that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {
  if (nwg < kNumXcd) return orig;
  int64_t q = nwg / kNumXcd, r = nwg % kNumXcd;
  int64_t xcd = orig % kNumXcd, idx = orig / kNumXcd;
  int64_t base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace spmm
