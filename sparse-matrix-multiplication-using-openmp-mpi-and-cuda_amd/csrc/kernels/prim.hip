// In-tree device primitives for gfx950 (no hipCUB / rocPRIM): scan, stable
// LSD radix sort of (key, payload) pairs, and the block-sparse symbolic phase
// built on them, shared by the native `a4` engine (csrc/runtime/bsr_engine.hip)
// and the Python engine (ops/bsr.py).
//
// The reference joins tiles on the host with hash maps and std::map ordering
// (sparse_matrix_mult.cu:140-156, :259-269); SURVEY §2.3 K-scan / K-sort.
//
//   scan   3-phase: per-tile sums (2048 items, 256 threads x 8), recursive
//          exclusive scan of the tile sums, tile-local scan + carry (int64
//          wave scans by shuffles, one LDS word per wave).
//   sort   LSD, 8-bit digits, stable.  Per pass: per-tile digit histograms
//          (digit-major, so ONE exclusive scan of 256 x tiles counters gives
//          every (digit, tile) its output base), then each tile re-reads its
//          keys in 8 striped rounds (round r covers items r*256 .. r*256+255,
//          so rounds and lanes are in input order = stability) and ranks each
//          key among the same-digit keys of its wave with 8 ballots (the
//          64-lane match), wave offsets per digit from LDS.  Only the bits that
//          differ are sorted: the symbolic phase compacts tile keys first.
//   bsr    symbolic phase of C = A (x) B on sorted tile keys: pair counts by
//          binary search, scan, pair fill with compact output codes, stable
//          sort (ascending middle index survives within an output tile: the
//          reference's summation order), run-length encode -> tile_ptr.
#include "common.hpp"

namespace {

constexpr int PT = 256;            // threads per block
constexpr int PI = 8;              // items per thread
constexpr int TILE = PT * PI;      // 2048 items per tile
constexpr int PW = PT / 64;

__device__ __forceinline__ int64_t prim_wave_incl(int64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

// exclusive block scan of one int64 per thread; *total = block sum
__device__ __forceinline__ int64_t prim_block_excl(int64_t v, int64_t* wsum, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t incl = prim_wave_incl(v);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int64_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int64_t s = wsum[i];
    pre += (i < w) ? s : 0;
    tot += s;
  }
  *total = tot;
  return pre + incl - v;
}

template <typename T>
__global__ __launch_bounds__(PT) void scan_reduce(const T* __restrict__ in, int64_t n, int64_t* __restrict__ part) {
  __shared__ int64_t wsum[PW];
  const int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * PI;
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < PI; ++i)
    if (base + i < n) s += (int64_t)in[base + i];
  int64_t tot;
  prim_block_excl(s, wsum, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// carry[b] = exclusive prefix of the tiles before b (nullptr: one tile)
template <typename T>
__global__ __launch_bounds__(PT) void scan_apply(const T* __restrict__ in, int64_t n, const int64_t* __restrict__ carry,
                                                 int64_t* __restrict__ out, int inclusive) {
  __shared__ int64_t wsum[PW];
  const int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * PI;
  int64_t v[PI];
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    v[i] = base + i < n ? (int64_t)in[base + i] : 0;
    s += v[i];
  }
  int64_t tot;
  int64_t run = prim_block_excl(s, wsum, &tot) + (carry ? carry[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    if (base + i < n) out[base + i] = inclusive ? run + v[i] : run;
    run += v[i];
  }
}

int64_t tiles_of(int64_t n) { return (n + TILE - 1) / TILE; }

// workspace (bytes) of scan(n): the tile sums of every level
size_t scan_ws(int64_t n) {
  size_t b = 0;
  for (int64_t t = tiles_of(n); t > 1; t = tiles_of(t)) b += (size_t)t * 2 * sizeof(int64_t);
  return b + 16;
}

template <typename T>
void scan(const T* in, int64_t n, int64_t* out, int inclusive, char* ws, hipStream_t s) {
  if (n <= 0) return;
  const int64_t t = tiles_of(n);
  if (t == 1) {
    hipLaunchKernelGGL(scan_apply<T>, dim3(1), dim3(PT), 0, s, in, n, (const int64_t*)nullptr, out, inclusive);
    return;
  }
  int64_t* part = reinterpret_cast<int64_t*>(ws);
  int64_t* carry = part + t;
  hipLaunchKernelGGL(scan_reduce<T>, dim3((unsigned)t), dim3(PT), 0, s, in, n, part);
  scan<int64_t>(part, t, carry, 0, ws + (size_t)t * 2 * sizeof(int64_t), s);
  hipLaunchKernelGGL(scan_apply<T>, dim3((unsigned)t), dim3(PT), 0, s, in, n, (const int64_t*)carry, out, inclusive);
}

// ---- radix sort -------------------------------------------------------------
__global__ __launch_bounds__(PT) void rs_hist(const uint64_t* __restrict__ keys, int64_t n, int shift, int64_t ntiles,
                                             int64_t* __restrict__ hist) {
  __shared__ int h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE;
#pragma unroll
  for (int r = 0; r < PI; ++r) {
    const int64_t i = base + r * PT + threadIdx.x;
    if (i < n) atomicAdd(&h[(int)((keys[i] >> shift) & 255u)], 1);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];   // digit-major
}

__global__ __launch_bounds__(PT) void rs_scatter(const uint64_t* __restrict__ kin, const uint64_t* __restrict__ vin,
                                                uint64_t* __restrict__ kout, uint64_t* __restrict__ vout, int64_t n,
                                                int shift, int64_t ntiles, const int64_t* __restrict__ offs) {
  __shared__ int64_t run[256];
  __shared__ int wcnt[PW][256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  run[tid] = offs[(int64_t)tid * ntiles + blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int r = 0; r < PI; ++r) {
    const int64_t i = base + r * PT + tid;
    const bool ok = i < n;
    uint64_t k = 0, v = 0;
    if (ok) { k = kin[i]; v = vin[i]; }
    const int d = (int)((k >> shift) & 255u);
#pragma unroll
    for (int q = 0; q < PW; ++q) wcnt[q][tid] = 0;
    __syncthreads();   // run[] written / wcnt cleared; previous round's reads done
    unsigned long long m = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const unsigned long long bb = __ballot((d >> b) & 1);
      m &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(m & below);
    if (ok && rank == 0) wcnt[w][d] = __popcll(m);   // the digit's first lane in this wave
    __syncthreads();
    if (ok) {
      int64_t pos = run[d] + rank;
#pragma unroll
      for (int q = 0; q < PW; ++q) pos += (q < w) ? wcnt[q][d] : 0;
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();   // every read of run[] for this round done
    int add = 0;
#pragma unroll
    for (int q = 0; q < PW; ++q) add += wcnt[q][tid];
    run[tid] += add;
  }
}

size_t sort_ws(int64_t n) {
  const int64_t t = tiles_of(n);
  return (size_t)n * 2 * sizeof(uint64_t) + (size_t)256 * t * 2 * sizeof(int64_t) + scan_ws(256 * t) + 64;
}

// Sorts bits [0, bits) of (k0, v0) stably; the result ends in (k0, v0) or
// (k1, v1) = the ws copies: returns 0 if in k0/v0, 1 if in the ws buffers.
int sort_pairs(uint64_t* k0, uint64_t* v0, int64_t n, int bits, char* ws, hipStream_t s, uint64_t** kr, uint64_t** vr) {
  const int64_t t = tiles_of(n);
  uint64_t* k1 = reinterpret_cast<uint64_t*>(ws);
  uint64_t* v1 = k1 + n;
  int64_t* hist = reinterpret_cast<int64_t*>(v1 + n);
  int64_t* offs = hist + 256 * t;
  char* sws = reinterpret_cast<char*>(offs + 256 * t);
  uint64_t *ka = k0, *va = v0, *kb = k1, *vb = v1;
  for (int shift = 0; shift < bits; shift += 8) {
    hipLaunchKernelGGL(rs_hist, dim3((unsigned)t), dim3(PT), 0, s, ka, n, shift, t, hist);
    scan<int64_t>(hist, 256 * t, offs, 0, sws, s);
    hipLaunchKernelGGL(rs_scatter, dim3((unsigned)t), dim3(PT), 0, s, ka, va, kb, vb, n, shift, t, offs);
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  *kr = ka;
  *vr = va;
  return ka == k0 ? 0 : 1;
}

// ---- block-sparse symbolic phase --------------------------------------------
__global__ __launch_bounds__(PT) void bsr_count(const int32_t* __restrict__ akeys, int64_t na,
                                               const int32_t* __restrict__ bkeys, int64_t nb,
                                               int64_t* __restrict__ cnt, int64_t* __restrict__ lo) {
  const int64_t a = (int64_t)blockIdx.x * PT + threadIdx.x;
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

// min / max of B's tile columns (out[0] = min, out[1] = max; int64, preset)
__global__ __launch_bounds__(PT) void bsr_col_range(const int32_t* __restrict__ bkeys, int64_t nb,
                                                   unsigned long long* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * PT + threadIdx.x;
  // order-preserving unsigned image of int32
  unsigned long long lo = ~0ull, hi = 0;
  if (i < nb) lo = hi = (unsigned long long)((uint32_t)bkeys[2 * i + 1] ^ 0x80000000u);
  for (int d = 32; d > 0; d >>= 1) {
    lo = min(lo, (unsigned long long)__shfl_xor(lo, d));
    hi = max(hi, (unsigned long long)__shfl_xor(hi, d));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&out[0], lo);
    atomicMax(&out[1], hi);
  }
}

// pairs of A tile a: compact output code (r - rmin) * crange + (c - cmin),
// payload a << 32 | b
__global__ __launch_bounds__(PT) void bsr_fill(const int32_t* __restrict__ akeys, const int32_t* __restrict__ bkeys,
                                              int64_t na, const int64_t* __restrict__ start,
                                              const int64_t* __restrict__ lo, int64_t rmin, int64_t cmin,
                                              int64_t crange, uint64_t* __restrict__ code, uint64_t* __restrict__ ab) {
  const int64_t a = (int64_t)blockIdx.x * PT + threadIdx.x;
  if (a >= na) return;
  const uint64_t rbase = (uint64_t)((int64_t)akeys[2 * a] - rmin) * (uint64_t)crange;
  const int64_t p0 = start[a], n = start[a + 1] - p0, b0 = lo[a];
  for (int64_t t = 0; t < n; ++t) {
    const int64_t b = b0 + t;
    code[p0 + t] = rbase + (uint64_t)((int64_t)bkeys[2 * b + 1] - cmin);
    ab[p0 + t] = ((uint64_t)a << 32) | (uint64_t)b;
  }
}

__global__ __launch_bounds__(PT) void rle_heads(const uint64_t* __restrict__ code, int64_t n, int32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * PT + threadIdx.x;
  if (i < n) head[i] = (i == 0 || code[i] != code[i - 1]) ? 1 : 0;
}

// run heads -> output tile t: keys and first pair; every pair -> pa / pb
__global__ __launch_bounds__(PT) void bsr_emit(const uint64_t* __restrict__ code, const uint64_t* __restrict__ ab,
                                              const int32_t* __restrict__ head, const int64_t* __restrict__ pos,
                                              int64_t n, int64_t rmin, int64_t cmin, int64_t crange,
                                              int32_t* __restrict__ okeys, int64_t* __restrict__ tile_ptr,
                                              int32_t* __restrict__ pa, int32_t* __restrict__ pb) {
  const int64_t i = (int64_t)blockIdx.x * PT + threadIdx.x;
  if (i >= n) return;
  pa[i] = (int32_t)(ab[i] >> 32);
  pb[i] = (int32_t)(ab[i] & 0xffffffffu);
  if (head[i]) {
    const int64_t t = pos[i] - 1;   // inclusive scan of the heads
    const uint64_t c = code[i];
    okeys[2 * t] = (int32_t)((int64_t)(c / (uint64_t)crange) + rmin);
    okeys[2 * t + 1] = (int32_t)((int64_t)(c % (uint64_t)crange) + cmin);
    tile_ptr[t] = i;
  }
  if (i == n - 1) tile_ptr[pos[i]] = n;
}

unsigned grid(int64_t n) { return (unsigned)((n + PT - 1) / PT); }

// One wave that returns after `ticks` of the 100 MHz real-time counter (a bounded wait: the
// loop ends whatever the clock does, after at most 2^31 polls): a stand-in for a link
// transfer's duration on a stream (tools/rank_emulate.py models the all-gather with it).
__global__ __launch_bounds__(64) void prim_spin(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < (1 << 31) - 1; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace

// Stream-ordered delay of `us` microseconds on one wave (diagnostics / emulation).
SPMM_EXPORT int spmm_prim_spin(double us, void* stream) {
  if (!(us > 0)) return 0;
  hipLaunchKernelGGL(prim_spin, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint64_t)(us * 100.0));
  SPMM_LAUNCH_CHECK();
  return 0;
}

// ---- exports ----------------------------------------------------------------
SPMM_EXPORT size_t spmm_prim_scan_ws(int64_t n) { return scan_ws(n); }

// out[i] = sum of in[0..i] (inclusive) or in[0..i-1]; int32 or int64 input
SPMM_EXPORT int spmm_prim_scan(const void* in, int in_bytes, int64_t n, int64_t* out, int inclusive, void* ws,
                               void* stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (in_bytes == 4) scan<int32_t>((const int32_t*)in, n, out, inclusive, (char*)ws, s);
  else if (in_bytes == 8) scan<int64_t>((const int64_t*)in, n, out, inclusive, (char*)ws, s);
  else return (int)hipErrorInvalidValue;
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT size_t spmm_prim_sort_ws(int64_t n) { return sort_ws(n); }

// Stable sort of (keys, vals) by bits [0, bits) of the keys, in place.
SPMM_EXPORT int spmm_prim_sort_pairs_u64(uint64_t* keys, uint64_t* vals, int64_t n, int bits, void* ws, void* stream) {
  if (n <= 1 || bits <= 0) return 0;
  if (bits > 64 || n >= ((int64_t)1 << 40)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  uint64_t *kr, *vr;
  if (sort_pairs(keys, vals, n, bits, (char*)ws, s, &kr, &vr)) {
    (void)hipMemcpyAsync(keys, kr, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(vals, vr, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
  }
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Symbolic phase, step 1 of C = A (x) B (tile keys int32 [n][2], sorted
// (row, col), unique).  start[na + 1] (exclusive pair offsets) and lo[na]
// (first B tile of each A tile's row) are caller buffers; ws: caller buffer
// of spmm_bsr_sym_plan_ws(na) bytes.  plan[0..4] (host) = pair count, row
// min, column min, column range, key bits.  One host synchronisation.
SPMM_EXPORT size_t spmm_bsr_sym_plan_ws(int64_t na) { return (size_t)na * 8 + scan_ws(na) + 64; }

SPMM_EXPORT int spmm_bsr_sym_plan(const int32_t* akeys, int64_t na, const int32_t* bkeys, int64_t nb, int64_t* start,
                                  int64_t* lo, void* ws, int64_t* plan, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < 5; ++i) plan[i] = 0;
  if (na <= 0 || nb <= 0) return 0;
  int64_t* cnt = reinterpret_cast<int64_t*>(ws);
  unsigned long long* rng = reinterpret_cast<unsigned long long*>(cnt + na);
  char* sws = reinterpret_cast<char*>(rng + 4);
  hipLaunchKernelGGL(bsr_count, dim3(grid(na)), dim3(PT), 0, s, akeys, na, bkeys, nb, cnt, lo);
  (void)hipMemsetAsync(start, 0, sizeof(int64_t), s);
  scan<int64_t>(cnt, na, start + 1, 1, sws, s);
  (void)hipMemsetAsync(rng, 0xff, sizeof(unsigned long long), s);   // min <- all ones
  (void)hipMemsetAsync(rng + 1, 0, sizeof(unsigned long long), s);  // max <- 0
  hipLaunchKernelGGL(bsr_col_range, dim3(grid(nb)), dim3(PT), 0, s, bkeys, nb, rng);
  SPMM_LAUNCH_CHECK();
  // one read-back: pair total, B column range, A's first / last tile row
  int64_t h[3] = {0, 0, 0};
  unsigned long long r2[2] = {0, 0};
  int32_t a_first = 0, a_last = 0;
  (void)hipMemcpyAsync(h, start + na, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  (void)hipMemcpyAsync(r2, rng, sizeof r2, hipMemcpyDeviceToHost, s);
  (void)hipMemcpyAsync(&a_first, akeys, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  (void)hipMemcpyAsync(&a_last, akeys + 2 * (na - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s);
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return (int)e;
  const int64_t cmin = (int64_t)(int32_t)((uint32_t)r2[0] ^ 0x80000000u);
  const int64_t cmax = (int64_t)(int32_t)((uint32_t)r2[1] ^ 0x80000000u);
  const int64_t crange = cmax - cmin + 1, rrange = (int64_t)a_last - a_first + 1;
  if (crange <= 0 || rrange <= 0 || rrange > ((int64_t)1 << 62) / crange) return (int)hipErrorInvalidValue;
  const unsigned long long top = (unsigned long long)rrange * (unsigned long long)crange - 1ull;
  plan[0] = h[0];
  plan[1] = a_first;
  plan[2] = cmin;
  plan[3] = crange;
  plan[4] = top ? 64 - __builtin_clzll(top) : 0;
  return 0;
}

SPMM_EXPORT size_t spmm_bsr_sym_build_ws(int64_t np) {
  return (size_t)np * (8 + 8 + 4 + 8) + sort_ws(np) + scan_ws(np) + 128;
}

// Step 2: the np pairs grouped by output tile.  Outputs (caller buffers sized
// for np): okeys [np][2], tile_ptr [np + 1], pa / pb [np]; *nt (host) = output
// tiles.  plan: from step 1.  One host synchronisation.
SPMM_EXPORT int spmm_bsr_sym_build(const int32_t* akeys, const int32_t* bkeys, int64_t na, const int64_t* start,
                                   const int64_t* lo, const int64_t* plan, void* ws, int32_t* okeys,
                                   int64_t* tile_ptr, int32_t* pa, int32_t* pb, int64_t* nt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t np = plan[0], rmin = plan[1], cmin = plan[2], crange = plan[3];
  const int bits = (int)plan[4];
  *nt = 0;
  if (np <= 0) return 0;
  if (np >= (int64_t)INT32_MAX) return (int)hipErrorInvalidValue;   // pa / pb are int32 tile indices
  uint64_t* code = reinterpret_cast<uint64_t*>(ws);
  uint64_t* ab = code + np;
  int64_t* pos = reinterpret_cast<int64_t*>(ab + np);
  int32_t* head = reinterpret_cast<int32_t*>(pos + np);
  char* sws = reinterpret_cast<char*>(head + np + (np & 1));
  hipLaunchKernelGGL(bsr_fill, dim3(grid(na)), dim3(PT), 0, s, akeys, bkeys, na, start, lo, rmin, cmin, crange, code,
                     ab);
  uint64_t *kr, *vr;
  sort_pairs(code, ab, np, bits, sws, s, &kr, &vr);
  hipLaunchKernelGGL(rle_heads, dim3(grid(np)), dim3(PT), 0, s, kr, np, head);
  scan<int32_t>(head, np, pos, 1, sws + sort_ws(np), s);
  hipLaunchKernelGGL(bsr_emit, dim3(grid(np)), dim3(PT), 0, s, kr, vr, head, pos, np, rmin, cmin, crange, okeys,
                     tile_ptr, pa, pb);
  SPMM_LAUNCH_CHECK();
  int64_t h = 0;
  (void)hipMemcpyAsync(&h, pos + np - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return (int)e;
  *nt = h;
  return 0;
}
