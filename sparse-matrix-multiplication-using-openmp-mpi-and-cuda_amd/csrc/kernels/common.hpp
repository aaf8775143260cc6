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

#ifndef SPMM_CHAIN_CROSS_MUL   // speculative MAC: cross terms by v_mul_lo_u32 (1) or v_mad_u64_u32 (0)
#define SPMM_CHAIN_CROSS_MUL 1
#endif
#ifndef SPMM_CHAIN_SPEC   // chain tile kernel: speculative wrapping MAC + exact recompute (1) or exact only (0)
#define SPMM_CHAIN_SPEC 1
#endif

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

// Speculative form of ref_mac: the plain wrapping acc + a*b in three VALU ops
// (v_mad_u64_u32 folds the low product and the 64-bit add; the two cross
// terms land in the high word), plus a conservative flag for the two events
// where the reference's collapse could differ from wrapping arithmetic:
// t = a*b == 2^64-1 needs t_lo == 0xffffffff (t_lo = r_lo - acc_lo), and
// s = acc + t == 2^64-1 needs s_lo == 0xffffffff.  When no lane of a tile
// ever raises the flag the wrapped result IS the reference's (no collapse
// fired); otherwise the caller recomputes the tile with ref_mac.
// Returns s = acc + a*b (wrapping); ``m`` accumulates max(s_lo, t_lo) so the
// caller tests a whole group of MACs with one compare (max == 0xffffffff iff
// some s_lo or t_lo was all-ones).
__device__ __forceinline__ uint64_t spec_mac(uint64_t acc, uint64_t a, uint64_t b, uint32_t& m) {
  const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
  // four VALU ops: r = alo*blo + acc;  c = alo*bhi;  x = ahi*blo + c (its low
  // word = the cross terms mod 2^32);  s_hi = r_hi + x_lo (32-bit add into the
  // high half; opaque so the compiler does not rebuild it as a 64-bit add)
  // (64-bit v_mad_u64_u32 destinations are early-clobber: a destination pair
  // overlapping a source is unsafe, so the register allocator must not reuse one)
  uint64_t r, k0;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=&s"(k0) : "v"(alo), "v"(blo), "v"(acc));
  uint32_t hi;
#if SPMM_CHAIN_CROSS_MUL
  // cross terms as two v_mul_lo_u32 + one v_add3_u32
  uint32_t c1, c2;
  asm("v_mul_lo_u32 %0, %1, %2" : "=v"(c1) : "v"(alo), "v"(bhi));
  asm("v_mul_lo_u32 %0, %1, %2" : "=v"(c2) : "v"(ahi), "v"(blo));
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(r >> 32)), "v"(c1), "v"(c2));
#else
  uint64_t c, x, k1, k2;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=&v"(c), "=&s"(k1) : "v"(alo), "v"(bhi));
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(x), "=&s"(k2) : "v"(ahi), "v"(blo), "v"(c));
  asm("v_add_u32 %0, %1, %2" : "=v"(hi) : "v"((uint32_t)(r >> 32)), "v"((uint32_t)x));
#endif
  const uint32_t lo = (uint32_t)r;
  const uint64_t s = ((uint64_t)hi << 32) | lo;
  const uint32_t tlo = lo - (uint32_t)acc;
  const uint32_t q = lo > tlo ? lo : tlo;
  m = m > q ? m : q;   // (one v_max3_u32)
  return s;
}

// LDS float adds: one read + compare-swap try, ds_add_f32 only for the lanes that lost it.
// gfx950 executes ds_add_f32 at ~3 LDS cycles per active lane (~193 CU-cycles per full
// wave-instruction, any address pattern) while a ds_read_b32 + ds_cmpst_rtn_b32 pair takes ~23
// on distinct addresses (tools/probes/lds_atomic.hip, PERF_LOG round 5).  A compare-swap LOOP
// collapses on hot addresses (one winner per LDS round trip: R-MAT 15 -> 34 s per step), so
// losers take the hardware-serialised add instead: never much worse than ds_add_f32 alone
// (~210 cycles with 48 of 64 lanes losing), ~8x better when few lanes collide.  Used where
// every product is an add (long_dense); the bitmap kernels' duplicate adds and long_rank's
// keep ds_add_f32: their adding lanes mostly collide (1M step 61.4 vs 62.6 ms with the try).
// N independent adds base[idx[u]] += v[u] (idx < 0: none): all reads, then all compare-swap
// tries in flight together, then ds_add_f32 for the lanes that lost.
// (Two / three tries before the fallback measured within run-to-run spread: one try.)
// fresh[u]: the slot is known to hold +0.0 (its occupancy bit was clear): no read.
template <int N>
__device__ __forceinline__ void lds_fadd_n(float* base, const int (&idx)[N], const float (&v)[N],
                                           const bool (&fresh)[N]) {
  uint32_t* q = reinterpret_cast<uint32_t*>(base);
  uint32_t old[N];
#pragma unroll
  for (int u = 0; u < N; ++u) old[u] = (idx[u] >= 0 && !fresh[u]) ? q[idx[u]] : 0u;
  bool lost[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    lost[u] = false;
    if (idx[u] >= 0) {
      const uint32_t prev = atomicCAS(q + idx[u], old[u], __float_as_uint(__uint_as_float(old[u]) + v[u]));
      lost[u] = prev != old[u];
      old[u] = prev;
    }
  }
#pragma unroll
  for (int u = 0; u < N; ++u)
    if (lost[u]) atomicAdd(base + idx[u], v[u]);
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
