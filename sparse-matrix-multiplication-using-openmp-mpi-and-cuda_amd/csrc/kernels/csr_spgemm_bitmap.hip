// Bitmap-rank CSR SpGEMM (fp32) for gfx950: the fast path for rows whose
// column windows each hold a few thousand intermediate products (BASELINE
// configs 2 and 4: uniform random A, B; compression nnz(C) / products ~ 1).
//
// The reference has no CSR path; its tile-level analogue is the host join +
// per-tile kernel of sparse_matrix_mult.cu:140-253.
//
// Columns are cut into windows of W = 2^LGW; a UNIT is (row i of A, window q).
// Two persistent kernels, no cross-workgroup waits:
//   count   per unit: OR every product's column into an LDS bitmap of the
//           window (one fire-and-forget ds_or per product); popcount = the
//           exact nnz of C(i, window q).  B's values are not read.  A count
//           workgroup covers NSUB windows of one row at once (one staging of
//           the A row for up to 8 windows).
//   (host)  exclusive scan of the unit counts = the final offset of every
//           unit; the row pointer is every nwin-th entry.
//   numeric per unit: the products (column, a*b) are fetched ONCE into
//           registers; pass 1 ORs them into the bitmap, a popcount scan gives
//           a 16-bit rank prefix per 64-bit bitmap word, pass 2 turns every
//           product into its output slot (prefix + popcount of the bits below
//           it) and accumulates a*b there with an LDS float atomic; the unit's
//           slots are then copied to C at the offset fixed by the count
//           kernel: coalesced, no sort, no look-back, no compaction copy.
//           Units too big for the register / LDS budget are deferred to a
//           list and finished by the same code with a 1-workgroup-per-CU
//           budget that re-reads B in pass 2 (the "reload" mode).
// Output rows are column-sorted by construction (rank order = column order).
// Per product: count 4 B of B + 1 LDS op; numeric 8 B of B + 5 LDS ops + 8 B
// of C; per unit O(W / 64) LDS words of scan.  Window bounds inside every B
// row come from one binary-search kernel (bm_window_splits), uint32 indices;
// it and B's other layout kernels (packed bounds, padded arrays, the
// gathered-operand unpack) are in csr_bitmap_layout.hip.
#include "bitmap_common.hpp"
#include "common.hpp"

#include <cstdlib>
#include <type_traits>

using namespace spmm_bitmap;

// Wave priority while a kernel stages the next unit and issues its gathers: the other
// workgroups of the CU are in their VALU / LDS phases, so the raised waves get their
// requests out first.  1M step 60.8-60.9 -> 58.8-58.9 ms, rank 0 of 8 9.43-9.51 -> 9.10-9.24 ms;
// any level 1-3 measures the same (PERF_LOG round 5).
#define SPMM_BM_PRIO_HI() __builtin_amdgcn_s_setprio(3)
#define SPMM_BM_PRIO_LO() __builtin_amdgcn_s_setprio(0)

// Row schedule of the pipelined numeric row kernel: ticket rows (1, the default) or static
// rows me, me + NG, ... (0, diagnostic builds).  1M step: static 58.5 ms, tickets 54.7 ms
// (PERF_LOG round 6).
#ifndef SPMM_BM_TICKETS
#define SPMM_BM_TICKETS 1
#endif

// Build-time geometry (every value below was swept in PERF_LOG rounds 3-5; tools/bm_variants.py
// builds diagnostic variants of these, normal builds never override them):
#ifndef SPMM_BM_ROWS_R   // register rounds of the row-major numeric kernel (chunk capacity 16 * R per unit)
#define SPMM_BM_ROWS_R 10
#endif
// numeric rank prefix: bitmap words per lane and scan step (2 and 4 measured identical)
constexpr int kSweepG = 2;
// per-unit pass 2: rank lookups in flight per group of rounds (and the skip granularity;
// 65536^2: 2 = 1.547 / 1.556 ms vs 4 = 1.562 / 1.586, 7 spills)
constexpr int kP2G = 2;

#define BM_OUT(ptr, val) __builtin_nontemporal_store((val), (ptr))

namespace {

// Block-wide exclusive scan of a non-negative int (+ total); DPP inside the
// wave, one LDS word per wave.  Ends synchronised; the caller must put a
// barrier between two scans that share wsum.
template <int NT>
__device__ __forceinline__ int bm_scan(int v, int* wsum, int* total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = bm_wave_incl(v);
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int s = wsum[i];
    pre += (i < w) ? s : 0;
    tot += s;
  }
  *total = tot;
  return pre + x - v;
}

// Two block-wide exclusive scans with one barrier (wsum holds 2 * NW ints).
template <int NT>
__device__ __forceinline__ void bm_scan2(int a, int b, int* wsum, int& pa, int& pb, int& ta, int& tb) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int xa = bm_wave_incl(a), xb = bm_wave_incl(b);
  if (lane == 63) {
    wsum[w] = xa;
    wsum[NW + w] = xb;
  }
  __syncthreads();
  int qa = 0, qb = 0;
  ta = 0;
  tb = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int sa = wsum[i], sb = wsum[NW + i];
    qa += (i < w) ? sa : 0;
    qb += (i < w) ? sb : 0;
    ta += sa;
    tb += sb;
  }
  pa = qa + xa - a;
  pb = qb + xb - b;
}

__device__ __forceinline__ int bm_wave_sum(int x) {
  return __builtin_amdgcn_readlane(bm_wave_incl(x), 63);
}

__device__ __forceinline__ int64_t bm_rfl64(int64_t x) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// A unit's slots items[0, lim) to C[off, off + lim) (one store per entry and
// array; 16-byte stores of four entries measured neutral, PERF_LOG round 4).
template <int NT>
__device__ __forceinline__ void bm_write_unit(const unsigned long long* items, int lim, int32_t* __restrict__ cci,
                                              float* __restrict__ cv, int64_t off, uint32_t cmask) {
  for (int i = threadIdx.x; i < lim; i += NT) {
    const unsigned long long it = items[i];
    BM_OUT(cci + (off + i), (int32_t)((uint32_t)it & cmask));
    BM_OUT(cv + (off + i), __uint_as_float((uint32_t)(it >> 32)));
  }
}


// Diagnostic phase stamps, compiled in only with -DSPMM_BM_STAMPS (the
// accumulators cost registers): thread 0 of every workgroup adds the
// shader-clock cycles of each phase of a unit, measured between the barriers
// that delimit it, in registers, flushed once at the end; [7] counts units.
__device__ int g_bm_stamp_on = 0;
__device__ unsigned long long g_bm_stamps[8];
// per workgroup of the numeric kernel (pipelined row or per-unit; stamps build): start / end on
// the 100 MHz real-time counter (one clock for every XCD), XCD id << 32 | units formed
constexpr int kBmWgMax = 8192;
__device__ unsigned long long g_bm_wg[3 * kBmWgMax];
#ifdef SPMM_BM_STAMPS
#define BM_STAMP_DECL                                                              \
  const int stamp_on = g_bm_stamp_on;                                              \
  unsigned long long t_prev = stamp_on ? __builtin_amdgcn_s_memtime() : 0ull;      \
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define BM_STAMP(i)                                                                \
  do {                                                                             \
    if (stamp_on) {                                                                \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();                  \
      st_acc[i] += _t - t_prev;                                                    \
      t_prev = _t;                                                                 \
    }                                                                              \
  } while (0)
#define BM_STAMP_UNIT() st_acc[7] += 1
#define BM_STAMP_FLUSH()                                                           \
  if (stamp_on && threadIdx.x == 0)                                                \
    for (int i = 0; i < 8; ++i) atomicAdd(&g_bm_stamps[i], st_acc[i])
#define BM_WG_DECL const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
#define BM_WG_FLUSH()                                                              \
  if (stamp_on && threadIdx.x == 0 && blockIdx.x < kBmWgMax) {                      \
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();                 \
    const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u; \
    atomicExch(&g_bm_wg[3 * blockIdx.x], wg_t0);                                    \
    atomicExch(&g_bm_wg[3 * blockIdx.x + 1], t1);                                   \
    atomicExch(&g_bm_wg[3 * blockIdx.x + 2], ((unsigned long long)xcc << 32) | st_acc[7]); \
  }
#else
#define BM_STAMP_DECL
#define BM_STAMP(i) do {} while (0)
#define BM_STAMP_UNIT() do {} while (0)
#define BM_STAMP_FLUSH() do {} while (0)
#define BM_WG_DECL
#define BM_WG_FLUSH() do {} while (0)
#endif

// ---- deterministic mode (DET kernels) ---------------------------------------
// The fast path folds a column's products into its output slot with LDS float
// atomics, so with three or more products per slot the fp32 sum depends on
// the atomics' order.  One product needs no add, and two commute exactly
// (fl(a + b) = fl(b + a)), so only slots of >= 3 products are order-
// sensitive; they are rare (~0.03 per unit at the 1M config).  DET kernels
// mark them in the slot's column word (columns < 2^30: bits 30 / 31 free):
//   bit 31 (kDupBit): the slot has received a duplicate; a duplicate that
//          finds it already set means >= 3 products -> the unit is "fixed";
//   bit 30 (kOwnBit): reload kernel only (no owner store): a product has
//          claimed the slot.
// Fix: every product of a marked slot appends {slot << 17 | key, value} to a
// small LDS list (key = its position in the unit's Gustavson order: chunk
// index << lg | lane in chunk, < 2^17), and wave 0 re-sums each listed slot
// in key order.  The result is then the sequential Gustavson sum
// (A entries in order, B entries in order), bit for bit: the CPU engine's
// order.  A unit whose list would overflow is deferred (fast kernels) or
// flagged (reload: err bit 4 -> the host recomputes the product on the CPU
// engine, same order).
constexpr uint32_t kDupBit = 1u << 31, kOwnBit = 1u << 30, kColMask = (1u << 30) - 1u;
constexpr uint32_t kKeyBits = 17, kKeyMask = (1u << kKeyBits) - 1u;

// wave-level: re-sum the n listed products per slot in key order into items
__device__ __forceinline__ void bm_det_sum(const uint2* list, int n, unsigned long long* items, int lane) {
  for (int i = lane; i < n; i += 64) {
    const uint2 e = list[i];
    const uint32_t slot = e.x >> kKeyBits, key = e.x & kKeyMask;
    bool head = true;   // the slot's first product in key order sums the slot
    for (int j = 0; j < n; ++j) {
      const uint32_t f = list[j].x;
      head &= !((f >> kKeyBits) == slot && (f & kKeyMask) < key);
    }
    if (!head) continue;
    float s = __uint_as_float(e.y);
    uint32_t cur = key;
    for (;;) {
      uint32_t best = 0xFFFFFFFFu;
      float bv = 0.f;
      for (int j = 0; j < n; ++j) {
        const uint2 f = list[j];
        const uint32_t fk = f.x & kKeyMask;
        if ((f.x >> kKeyBits) == slot && fk > cur && fk < best) {
          best = fk;
          bv = __uint_as_float(f.y);
        }
      }
      if (best == 0xFFFFFFFFu) break;
      s += bv;
      cur = best;
    }
    reinterpret_cast<float*>(&items[slot])[1] = s;
  }
}

// One instantiation's geometry.  MODE 0: count (NSUB windows per unit);
// 1: numeric, products held in R register rounds; 2: numeric reload
// (deferred units, B re-read in pass 2).
template <int LGW, int NSUB, int NT, int PCAP, int R, int CCAP, int MODE>
struct BmGeom {
  static constexpr int NWORD = (NSUB << LGW) / 64;   // 64-bit bitmap words
  static constexpr int WPW = NWORD / (NT / 64);      // words per wave (scan: a wave owns a contiguous block)
  static constexpr int WPT = WPW >= 64 ? WPW / 64 : 1;
  static constexpr int NCLR = NWORD / 2;             // 16-byte clears
  static_assert(NWORD % 64 == 0 && (WPW % 64 == 0 || NWORD < NT), "bitmap words split over the waves");
  static_assert(MODE != 0 || (NWORD / NSUB) % 64 == 0, "count: 64-word rows stay inside one window");
  static_assert(MODE == 0 || NSUB == 1, "numeric units are single windows");
  static_assert(MODE == 0 || NWORD >= NT, "numeric: every wave owns bitmap words");
  static_assert(PCAP < 65536, "16-bit rank prefix");
  static_assert(NT <= 1024 && NT % 64 == 0, "workgroup size");
};

struct BmArgs {
  const int64_t* Arp;
  const int32_t* Aci;
  const float* Av;
  const uint32_t* ws;      // [mb][nwin + 1] window bounds inside every B row (absolute indices)
  const int32_t* Bci;
  const float* Bv;
  int64_t m;               // rows of A
  int nwin;                // windows per row
  int lg;                  // log2 lanes per product chunk
  int32_t* ucnt;           // count: [m * nwin] distinct columns per unit
  const int64_t* uoff;     // numeric: [m * nwin + 1] exclusive unit offsets into C
  int32_t* Cci;
  float* Cv;
  int32_t* ovf;            // numeric: deferred units
  uint32_t* novf;          //          and their count
  int64_t ovf_cap;
  int64_t cap;             // numeric: entries allocated for C (a unit outside it is an error, never a write)
  const uint2* Bcv;        // row-major numeric: B as interleaved (column, value bits), or null
                           // (per-unit WIDE numeric: the padded pair array)
  int32_t* err;            // bit 0: a deferred unit exceeds the reload budget (host falls back)
                           // bit 1: count / numeric disagree (kernel invariant)
                           // bit 2: deferred list full (host falls back)
  const uint4* ws8 = nullptr;   // per-unit WIDE numeric: packed window bounds + padded pair bases
  int32_t chunk = 0;            // numeric: 0 = persistent grid, else `chunk` consecutive units a workgroup
};

// CV: B read as interleaved (column, value bits) pairs (p.Bcv): one 8-byte load
// per product instead of two 4-byte ones (numeric modes only)
// WIDE (fast numeric, padded pairs): two pairs per lane and 16-byte loads, as
// in the row kernel; the window bounds come from ws8 (padded segment starts).
template <int LGW, int NSUB, int NT, int PCAP, int R, int CCAP, int MODE, bool DET = false, bool CV = false,
          bool WIDE = false>
__global__ __launch_bounds__(NT, 4) void spgemm_bm(BmArgs p) {
  using Gm = BmGeom<LGW, NSUB, NT, PCAP, R, CCAP, MODE>;
  constexpr int NW = NT / 64;
  constexpr bool VALUES = MODE != 0;
  constexpr int NWORD = Gm::NWORD, WPW = Gm::WPW, WPT = Gm::WPT;
  constexpr int RR = MODE == 1 ? R : (MODE == 0 ? 16 : 8);   // product slots per lane
  constexpr int PPL = WIDE ? 2 : 1;   // pairs per lane and load
  constexpr int RL = RR / PPL;        // load rounds
  static_assert(!WIDE || (MODE != 0 && CV && !DET && RR % 2 == 0), "wide loads: numeric / reload, padded pairs");
  // deterministic fix-up list: the fast kernel defers a unit that overflows
  // it to the reload kernel, whose list is larger (it has one CU's LDS)
  constexpr int LCAP = !DET ? 1 : (MODE == 2 ? 1024 : 64);
  static_assert(!DET || MODE != 0, "DET: numeric kernels only");
  static_assert(!DET || (CCAP << 6) <= (1 << kKeyBits), "DET keys fit 17 bits");

  // LDS.  bm: the window's column bitmap.  pre16: exclusive rank prefix of
  // every 64-bit word.  items: (column, value) of every output slot.
  // desc: chunk descriptors {first B index, valid lanes, a(i, j) bits}.
  __shared__ __attribute__((aligned(16))) unsigned long long bm[NWORD];
  __shared__ __attribute__((aligned(16))) uint16_t pre16[VALUES ? NWORD : 1];
  __shared__ __attribute__((aligned(16))) unsigned long long items[VALUES ? PCAP : 1];
  using Desc = typename std::conditional<VALUES, uint4, uint2>::type;
  __shared__ __attribute__((aligned(16))) Desc desc[CCAP];
  __shared__ __attribute__((aligned(8))) uint2 dlist[LCAP];
  __shared__ int wsum[2 * NW];
  __shared__ int scnt[NSUB];
  __shared__ int sdup, sfix, snl;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lgc = p.lg;                  // log2 pairs per chunk
  const int lg = lgc - (WIDE ? 1 : 0);   // log2 lanes per chunk
  const int Gc = 1 << lgc;
  const int Gl = 1 << lg;
  const int ngrp = NW << (6 - lg);
  const int gid = (w << (6 - lg)) + (lane >> lg);
  const int gl = lane & (Gl - 1);
  const int nwin = p.nwin;
  const int64_t nw1 = nwin + 1;
  uint32_t* const bm32 = reinterpret_cast<uint32_t*>(bm);
  // A zero the compiler cannot see through: indices built with it look
  // divergent, so the prefetch loads below are VECTOR loads (vmcnt).  As
  // scalar loads they would share lgkmcnt with every LDS wait and stall the
  // first LDS read after them for a full memory latency.
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  BM_STAMP_DECL
  BM_WG_DECL
  if constexpr (MODE != 0) {
    // numeric / reload after a row count that stood down (ws8 lengths
    // truncated, err bit 3; the host reruns the product on the per-unit count):
    // the unit offsets are not valid, so nothing is formed (uniform exit)
    if (*p.err & 8) return;
  }

  // bitmap clear: 16-byte stores, consecutive lanes on consecutive slots (conflict-free)
  auto clear_bm = [&]() {
    for (int i = tid; i < Gm::NCLR; i += NT) reinterpret_cast<uint4*>(bm)[i] = make_uint4(0, 0, 0, 0);
  };
  clear_bm();
  if (tid < NSUB) scnt[tid] = 0;
  if (tid == 0) {
    sdup = 0;
    sfix = 0;
    snl = 0;
  }

  // Unit schedule.  Count / numeric: static and persistent; iteration k of
  // workgroup g takes unit k * gridDim + perm(g), perm putting consecutive
  // units (the windows of one row: same A row, neighbouring B lines) on one
  // XCD (blocks b and b + 8 share one; speed only).  Reload: the deferred list.
  // Chunked numeric (p.chunk > 0): workgroup g takes units g * chunk .. + chunk
  // and exits, and the grid is ~16x the resident slots, so the dispatcher
  // hands the freed slots new workgroups: the workgroups of a CU are served
  // unequally, and a persistent grid's fixed share leaves a 16 % tail
  // (65536^2, PERF_LOG round 6).
  const int64_t nsw = MODE == 0 ? (nwin + NSUB - 1) / NSUB : nwin;   // units per row
  int64_t nunits = MODE == 2 ? (int64_t)__hip_atomic_load(p.novf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : p.m * nsw;
  if (MODE == 2 && nunits > p.ovf_cap) nunits = p.ovf_cap;
  const int64_t NG = gridDim.x;
  const int64_t me = (MODE != 2 && NG % 8 == 0) ? (int64_t)(blockIdx.x % 8) * (NG / 8) + blockIdx.x / 8
                                                : (int64_t)blockIdx.x;
  const int64_t CU = MODE == 1 ? p.chunk : 0;
  const int64_t SU = CU > 0 ? 1 : NG;   // unit stride of this workgroup's sequence
  const int64_t u_first = CU > 0 ? (int64_t)blockIdx.x * CU : me;
  const int64_t u_lim = CU > 0 ? min(nunits, u_first + CU) : nunits;

  // ---- software pipeline over this workgroup's units ----------------------
  // Three units ahead, every load issued unconditionally at the top of an
  // iteration (one control path, so no conservative waits): at the top of
  // unit k, the window bounds and output offsets of unit k+1 (needs k+1's A
  // columns, loaded one iteration earlier), the A entries of unit k+2 (needs
  // its row pointers, one iteration earlier) and the row pointers of unit
  // k+3.  Unit k's staging then finds its inputs in registers.
  struct Head {   // wave-uniform identity of a unit (m * nwin < 2^31, checked by the host)
    int slot, u, row, qi;   // qi: unit index inside its row
  };
  auto first_head = [&](int64_t slot) {
    Head h{(int)(slot < u_lim ? slot : u_lim), 0, 0, 0};
    if (slot < u_lim) {
      h.u = MODE == 2 ? p.ovf[slot] : (int)slot;
      h.row = (int)(h.u / nsw);
      h.qi = (int)(h.u - (int64_t)h.row * nsw);
    }
    return h;
  };
  const int step_q = (int)(SU % nsw), step_row = (int)(SU / nsw);
  auto next_head = [&](const Head& h) {
    if constexpr (MODE == 2) {
      return first_head((int64_t)h.slot + NG);
    } else {
      Head n{h.slot, h.u, h.row, h.qi};
      if ((int64_t)h.slot + SU >= u_lim) {
        n.slot = (int)u_lim;
        return n;
      }
      n.slot = (int)(h.slot + SU);
      n.u = (int)(h.u + SU);
      n.row = h.row + step_row;
      n.qi = h.qi + step_q;
      if (n.qi >= nsw) {
        n.qi -= (int)nsw;
        ++n.row;
      }
      return n;
    }
  };
  auto live = [&](const Head& h) { return (int64_t)h.slot < u_lim; };
  auto q0_of = [&](const Head& h) { return h.qi * (MODE == 0 ? NSUB : 1); };
  auto q1_of = [&](const Head& h) { return MODE == 0 ? min(h.qi * NSUB + NSUB, nwin) : h.qi + 1; };
  Head h0 = first_head(u_first);
  Head h1 = next_head(h0), h2 = next_head(h1), h3 = next_head(h2);
  // row start / length of A (vector registers; nnz(A) < 2^31, checked by the host)
  int ra0 = 0, rb0 = 0, ra1 = 0, rb1 = 0, ra2 = 0, rb2 = 0, ra3 = 0, rb3 = 0;
  int jj1 = 0, jj2 = 0;                   // A columns of units k+1 (landed) and k+2 (in flight)
  float av0 = 0.f, av1 = 0.f, av2 = 0.f;  // A values of units k, k+1, k+2
  uint32_t b00 = 0, b10 = 0, b01 = 0, b11 = 0;   // window bounds of units k and k+1
  int64_t oa0 = 0, oa1 = 0;   // uoff of units k and k+1, and the low words of the next entry
  int ob0 = 0, ob1 = 0;
  auto ld_arp = [&](const Head& h, int& ra, int& rb) {
    if (live(h)) {
      ra = (int)p.Arp[h.row + vz];
      rb = (int)p.Arp[h.row + 1 + vz];
    }
  };
  auto ld_entries = [&](const Head& h, int ra, int rb, int& j, float& av) {
    if (live(h)) {
      const int a0 = __builtin_amdgcn_readfirstlane(ra), na = __builtin_amdgcn_readfirstlane(rb) - a0;
      if (tid < na) {
        j = p.Aci[a0 + tid];
        if constexpr (VALUES) av = p.Av[a0 + tid];
      }
    }
  };
  auto ld_bounds = [&](const Head& h, int ra, int rb, int j, uint32_t& b0, uint32_t& b1, int64_t& oa, int& ob) {
    if (live(h)) {
      const int na = __builtin_amdgcn_readfirstlane(rb) - __builtin_amdgcn_readfirstlane(ra);
      if (tid < na) {
        if constexpr (WIDE) {   // the unit's segment in the padded pair array
          const uint4 wa = p.ws8[2 * (int64_t)j];
          const uint32_t wb = p.ws8[2 * (int64_t)j + 1].x;
          uint32_t st = p.ws8[2 * (int64_t)j + 1].y;
          const int q = q0_of(h);
          uint32_t ln = 0;
#pragma unroll
          for (int qq = 0; qq < 8; ++qq) {
            const uint32_t word = qq < 2 ? wa.y : qq < 4 ? wa.z : qq < 6 ? wa.w : wb;
            const uint32_t l = (word >> (16 * (qq & 1))) & 0xffffu;
            if (qq < q) st += ((l + (1u << kPadLg) - 1) >> kPadLg) << kPadLg;
            if (qq == q) ln = l;
          }
          b0 = st;
          b1 = st + ln;
        } else {
          const uint32_t* wr = p.ws + (int64_t)j * nw1;
          b0 = wr[q0_of(h)];
          b1 = wr[q1_of(h)];
        }
      }
      if constexpr (VALUES) {
        oa = p.uoff[h.u + vz];
        ob = (int)p.uoff[h.u + 1 + vz];   // low word: the unit's count is (ob - oa) mod 2^32
      }
    }
  };
  // prologue: units 0, 1, 2 staged to the depth the loop expects
  ld_arp(h0, ra0, rb0);
  ld_arp(h1, ra1, rb1);
  ld_arp(h2, ra2, rb2);
  ld_entries(h0, ra0, rb0, jj1, av0);
  ld_bounds(h0, ra0, rb0, jj1, b00, b10, oa0, ob0);
  ld_entries(h1, ra1, rb1, jj1, av1);
  ld_entries(h2, ra2, rb2, jj2, av2);
  ld_arp(h3, ra3, rb3);
  __syncthreads();

  // Products of chunk rounds [i0, i0 + RR) of this lane group: descriptor
  // reads for every round (LDS broadcasts, clamped index: all in flight
  // together), B loads only for rounds that exist (wave-uniform guards),
  // every load before any use.
  int c[RR];
  float v[RR];
  auto fetch = [&](int i0, int nr, int TC, int clo) {
    Desc ds[RL];
#pragma unroll
    for (int d = 0; d < RL; ++d) {
      const int t = gid + (i0 + d) * ngrp;
      ds[d] = desc[t < TC ? t : TC - 1];
    }
    uint32_t f[RL];
    uint32_t okm = 0;   // bit s: product slot s (round s / PPL, pair s % PPL) is in its segment
#pragma unroll
    for (int d = 0; d < RL; ++d) {
      const int t = gid + (i0 + d) * ngrp;
      const int nv = (int)ds[d].y - PPL * gl;
      const bool ok = (t < TC) & (nv > 0);
      okm |= (ok ? 1u : 0u) << (d * PPL);
      if constexpr (WIDE) okm |= ((ok & (nv > 1)) ? 1u : 0u) << (d * PPL + 1);
      f[d] = ds[d].x + (ok ? (uint32_t)(PPL * gl) : 0u);
    }
    int x[RR];
    float b[RR];
#pragma unroll
    for (int d = 0; d < RL; ++d) {
#pragma unroll
      for (int hh = 0; hh < PPL; ++hh) {
        x[d * PPL + hh] = 0;
        b[d * PPL + hh] = 0.f;
      }
      if (i0 + d < nr) {   // wave-uniform
        if constexpr (WIDE) {   // one 16-byte load: two pairs (segments start on 128-byte lines)
          const uint4 e = *reinterpret_cast<const uint4*>(p.Bcv + f[d]);
          x[2 * d] = (int)e.x;
          b[2 * d] = __uint_as_float(e.y);
          x[2 * d + 1] = (int)e.z;
          b[2 * d + 1] = __uint_as_float(e.w);
        } else if constexpr (CV && VALUES) {
          const uint2 e = p.Bcv[f[d]];
          x[d] = (int)e.x;
          b[d] = __uint_as_float(e.y);
        } else {
          x[d] = p.Bci[f[d]];
          if constexpr (VALUES) b[d] = p.Bv[f[d]];
        }
      }
    }
#pragma unroll
    for (int d = 0; d < RR; ++d) {
      c[d] = ((okm >> d) & 1u) ? x[d] - clo : -1;
      if constexpr (VALUES) v[d] = __uint_as_float(reinterpret_cast<const uint4&>(ds[d / PPL]).z) * b[d];
    }
  };
  // OR the columns into the bitmap.  Numeric mode keeps the old words: a
  // product whose bit was already set is a duplicate (returned as a mask);
  // the first product of every column is its slot's owner.
  auto or_all = [&]() {
    uint32_t dupm = 0;
    if constexpr (MODE == 0) {
#pragma unroll
      for (int d = 0; d < RR; ++d)
        if (c[d] >= 0) atomicOr(bm32 + (c[d] >> 5), 1u << (c[d] & 31));
    } else {
      uint32_t old[RR];
#pragma unroll
      for (int d = 0; d < RR; ++d) {
        old[d] = 0u;
        if (c[d] >= 0) old[d] = atomicOr(bm32 + (c[d] >> 5), 1u << (c[d] & 31));
      }
#pragma unroll
      for (int d = 0; d < RR; ++d) dupm |= (c[d] >= 0 ? (old[d] >> (c[d] & 31)) & 1u : 0u) << d;
    }
    return dupm;
  };

  while (live(h0)) {
    // ---- unit k = h0: inputs in registers; issue the loads of k+1..k+3 ----
    const Head h = h0;
    const int64_t a0 = __builtin_amdgcn_readfirstlane(ra0);
    const int64_t na = __builtin_amdgcn_readfirstlane(rb0) - (int)a0;
    const int64_t off = bm_rfl64(oa0);
    const int want = __builtin_amdgcn_readfirstlane(ob0) - (int)(uint32_t)off;
    const float avk = av0;
    const uint32_t bk0 = b00, bk1 = b10;
    {
      const Head h4 = next_head(h3);
      int ra4 = 0, rb4 = 0;
      int jj3 = 0;
      float av3 = 0.f;
      ld_bounds(h1, ra1, rb1, jj1, b01, b11, oa1, ob1);
      ld_entries(h3, ra3, rb3, jj3, av3);
      ld_arp(h4, ra4, rb4);
      // rotate the pipeline registers
      h0 = h1; h1 = h2; h2 = h3; h3 = h4;
      ra0 = ra1; rb0 = rb1; ra1 = ra2; rb1 = rb2; ra2 = ra3; rb2 = rb3; ra3 = ra4; rb3 = rb4;
      av0 = av1; av1 = av2; av2 = av3;
      jj1 = jj2; jj2 = jj3;
      b00 = b01; b10 = b11;
      oa0 = oa1; ob0 = ob1;
    }
    const int64_t row = h.row;
    const int q0 = q0_of(h), q1 = q1_of(h);
    const int clo = q0 << LGW;

    if constexpr (MODE == 0) {
      // ---- count: batches of NT entries, descriptors in windows of CCAP ----
      int64_t P = 0;
      for (int64_t bat = 0; bat < na; bat += NT) {
        const int nb = (int)((na - bat) < NT ? (na - bat) : NT);
        int len = 0, nch = 0;
        uint32_t b0 = 0;
        if (tid < nb) {
          if (bat == 0) {   // from the pipeline registers
            b0 = bk0;
            len = (int)(bk1 - bk0);
          } else {
            const uint32_t* wr = p.ws + (int64_t)p.Aci[a0 + bat + tid] * nw1;
            b0 = wr[q0];
            len = (int)(wr[q1] - b0);
          }
          nch = (len + Gl - 1) >> lg;
        }
        int pre, plen, TCall, Pb;
        bm_scan2<NT>(nch, len, wsum, pre, plen, TCall, Pb);
        P += Pb;
        for (int cb = 0; cb < TCall; cb += CCAP) {
          const int TC = TCall - cb < CCAP ? TCall - cb : CCAP;
          const int k0 = max(cb - pre, 0), k1 = min(cb + CCAP - pre, nch);
          for (int kk = k0; kk < k1; ++kk) {
            const int rem = len - (kk << lg);
            Desc dd{};
            dd.x = b0 + ((uint32_t)kk << lg);
            dd.y = (uint32_t)(rem < Gl ? rem : Gl);
            desc[pre + kk - cb] = dd;
          }
          __syncthreads();
          const int nr = (TC + ngrp - 1) / ngrp;
          for (int i0 = 0; i0 < nr; i0 += RR) {
            fetch(i0, nr, TC, clo);
            or_all();
          }
          __syncthreads();   // descriptors consumed before they are rewritten
        }
      }
      BM_STAMP(5);
      if (P == 0) {   // uniform
        if (tid < q1 - q0) p.ucnt[row * nwin + q0 + tid] = 0;
        continue;
      }
      // popcount per window: rows of 64 words, consecutive lanes on
      // consecutive words (conflict-free), each row inside one window
      constexpr int WORDS_PER_WIN = NWORD / NSUB;
      for (int r0 = w * 64; r0 < NWORD; r0 += NT) {
        const int cnt = bm_wave_sum(__popcll(bm[r0 + lane]));
        if (lane == 0) atomicAdd(&scnt[r0 / WORDS_PER_WIN], cnt);
      }
      __syncthreads();
      if (tid < NSUB) {
        if (q0 + tid < q1) p.ucnt[row * nwin + q0 + tid] = scnt[tid];
        scnt[tid] = 0;
      }
      clear_bm();
      __syncthreads();   // cleared before the next unit's ORs
      BM_STAMP(6);
    } else {
      // ---- numeric staging: the whole row in one batch, from registers -----
      int len = 0, nch = 0;
      if (tid < na && tid < NT) {
        len = (int)(bk1 - bk0);
        nch = (len + Gc - 1) >> lgc;
      }
      int pre, plen, TC, P;
      bm_scan2<NT>(nch, len, wsum, pre, plen, TC, P);
      if (P == 0) {   // uniform; the count kernel wrote 0 for this unit
        continue;
      }
      const bool too_big = na > NT || P > PCAP || TC > CCAP || (MODE == 1 && TC > RL * ngrp);
      if (too_big) {   // uniform
        if (tid == 0) {
          if (MODE == 1) {
            const uint32_t at = atomicAdd(p.novf, 1u);
            if ((int64_t)at < p.ovf_cap) p.ovf[at] = h.u;
            else atomicOr(p.err, 4);
          } else {
            atomicOr(p.err, 1);
          }
        }
        __syncthreads();   // wsum reads done before the next unit's scan
        continue;
      }
      for (int kk = 0; kk < nch; ++kk) {
        const int rem = len - (kk << lgc);
        Desc dd{};
        dd.x = bk0 + ((uint32_t)kk << lgc);
        dd.y = (uint32_t)(rem < Gc ? rem : Gc);
        reinterpret_cast<uint4&>(dd).z = __float_as_uint(avk);
        desc[pre + kk] = dd;
      }
      __syncthreads();
      BM_STAMP(0);
      // ---- pass 1: products into registers, columns into the bitmap -------
      const int nr = (TC + ngrp - 1) / ngrp;
      uint32_t dupm = 0;
      if constexpr (MODE == 1) {
        SPMM_BM_PRIO_HI();
        fetch(0, nr, TC, clo);
        SPMM_BM_PRIO_LO();
        dupm = or_all();
      } else {
        for (int i0 = 0; i0 < nr; i0 += RL) {
          fetch(i0, nr, TC, clo);
          or_all();
        }
      }
      if (dupm) sdup = 1;
      __syncthreads();
      BM_STAMP(1);
      // ---- rank prefix per 64-bit word: wave w owns words [w*WPW, (w+1)*WPW)
      // (groups: a lane takes SG adjacent words per step -- 16-byte reads, ONE
      // wave scan of their sum, 16-bit prefixes stored SG at a time)
      constexpr int SG = (kSweepG > 1 && WPW % (64 * kSweepG) == 0) ? kSweepG : 1;
      constexpr bool PAIRS = SG > 1;
      int run[WPT];   // groups: [SG * kk] = group prefix inside the wave, [SG * kk + i] = local prefix of word i
      int wtot = 0;
      if constexpr (PAIRS) {
#pragma unroll
        for (int kk = 0; kk < WPT / SG; ++kk) {
          const ulonglong2* src = reinterpret_cast<const ulonglong2*>(&bm[w * WPW + kk * 64 * SG + SG * lane]);
          int c[SG];
#pragma unroll
          for (int h = 0; h < SG / 2; ++h) {
            const ulonglong2 x = src[h];
            c[2 * h] = __popcll(x.x);
            c[2 * h + 1] = __popcll(x.y);
          }
          int sum = 0;
#pragma unroll
          for (int i = 0; i < SG; ++i) {
            if (i > 0) run[SG * kk + i] = sum;
            sum += c[i];
          }
          const int incl = bm_wave_incl(sum);
          run[SG * kk] = wtot + incl - sum;
          wtot += __builtin_amdgcn_readlane(incl, 63);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < WPT; ++kk) {
          const int cnt = __popcll(bm[w * WPW + kk * 64 + lane]);
          const int incl = bm_wave_incl(cnt);
          run[kk] = wtot + incl - cnt;
          wtot += __builtin_amdgcn_readlane(incl, 63);
        }
      }
      const int any_dup = sdup;
      if (lane == 0) wsum[w] = wtot;
      __syncthreads();
      int base = 0, total = 0;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const int sw = wsum[i];
        base += (i < w) ? sw : 0;
        total += sw;
      }
      if constexpr (PAIRS) {
#pragma unroll
        for (int kk = 0; kk < WPT / SG; ++kk) {
          const uint32_t g0 = (uint32_t)(base + run[SG * kk]);
          uint32_t pk[SG / 2];
#pragma unroll
          for (int h = 0; h < SG / 2; ++h) {
            const uint32_t lo = g0 + (h > 0 ? (uint32_t)run[SG * kk + 2 * h] : 0u);
            const uint32_t hi = g0 + (uint32_t)run[SG * kk + 2 * h + 1];
            pk[h] = (lo & 0xffffu) | (hi << 16);
          }
          uint16_t* dst = &pre16[w * WPW + kk * 64 * SG + SG * lane];
          if constexpr (SG == 2) {
            *reinterpret_cast<uint32_t*>(dst) = pk[0];
          } else if constexpr (SG == 4) {
            *reinterpret_cast<uint2*>(dst) = make_uint2(pk[0], pk[1]);
          } else {
            static_assert(SG == 8, "sweep group of 2, 4 or 8 words");
            *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          }
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < WPT; ++kk) pre16[w * WPW + kk * 64 + lane] = (uint16_t)(base + run[kk]);
      }
      if (tid == 0) sdup = 0;
      __syncthreads();
      BM_STAMP(2);
      // ---- pass 2: rank -> slot; owners store (column, value), duplicates
      // add their value after a barrier (bit set by an earlier product)
      auto rank = [&](int cc) {
        const int wd = cc >> 6;
        return (int)pre16[wd] + __popcll(bm[wd] & ((1ull << (cc & 63)) - 1ull));
      };
      if constexpr (MODE == 1) {
        // ranks of P2G rounds at a time (their LDS reads in flight together)
        constexpr int P2G = kP2G;
#pragma unroll
        for (int d0 = 0; d0 < RR; d0 += P2G) {
          if (d0 >= nr * PPL) break;   // uniform: slots past the unit's chunks hold no product
          int r[P2G];
#pragma unroll
          for (int dd = 0; dd < P2G && d0 + dd < RR; ++dd) r[dd] = rank(c[d0 + dd] >= 0 ? c[d0 + dd] : 0);
#pragma unroll
          for (int dd = 0; dd < P2G && d0 + dd < RR; ++dd) {
            const int d = d0 + dd;
            if (c[d] >= 0 && !((dupm >> d) & 1u))
              items[r[dd]] = ((unsigned long long)__float_as_uint(v[d]) << 32) | (uint32_t)(c[d] + clo);
          }
        }
        if (any_dup) {   // uniform
          __syncthreads();
          if constexpr (DET) {   // duplicates mark their slot; a second duplicate flags the unit
            bool tri = false;
#pragma unroll
            for (int d = 0; d < RR; ++d)
              if ((dupm >> d) & 1u) {
                unsigned long long* it = &items[rank(c[d])];
                tri |= (atomicOr(reinterpret_cast<uint32_t*>(it), kDupBit) & kDupBit) != 0u;
                atomicAdd(reinterpret_cast<float*>(it) + 1, v[d]);
              }
            if (tri) sfix = 1;
          } else {
#pragma unroll
            for (int d = 0; d < RR; ++d)
              if ((dupm >> d) & 1u) atomicAdd(reinterpret_cast<float*>(&items[rank(c[d])]) + 1, v[d]);
          }
        }
      } else {
        // reload: B re-read; every product adds into a zeroed slot
        for (int i = tid; i < total; i += NT) items[i] = 0ull;
        __syncthreads();
        bool tri = false;
        for (int i0 = 0; i0 < nr; i0 += RL) {
          fetch(i0, nr, TC, clo);
          // the value adds: one compare-swap try each, ds_add_f32 for the lanes that lost (the
          // reload's adds land on distinct slots almost always: ~3x fewer LDS cycles than
          // ds_add_f32 alone, common.hpp lds_fadd_n)
          int ri[RR];
          float rv[RR];
          bool rf[RR];
#pragma unroll
          for (int d = 0; d < RR; ++d) {
            ri[d] = -1;
            rv[d] = v[d];
            rf[d] = false;
            if (c[d] >= 0) {
              const int rr = rank(c[d]);
              uint32_t* cw = reinterpret_cast<uint32_t*>(&items[rr]);
              if constexpr (DET) {   // first product claims the slot, a third one flags the unit
                if (atomicOr(cw, (uint32_t)(c[d] + clo) | kOwnBit) & kOwnBit)
                  tri |= (atomicOr(cw, kDupBit) & kDupBit) != 0u;
              } else {
                cw[0] = (uint32_t)(c[d] + clo);
              }
              ri[d] = 2 * rr + 1;
            }
          }
          spmm::lds_fadd_n(reinterpret_cast<float*>(items), ri, rv, rf);
        }
        if (DET && tri) sfix = 1;
      }
      __syncthreads();
      bool skip = false;
      if constexpr (DET) {
        if (sfix) {   // uniform, rare: re-sum the slots of >= 3 products in Gustavson order
          auto append = [&](int i0) {
#pragma unroll
            for (int d = 0; d < RR; ++d) {
              if (c[d] >= 0) {
                const int rr = rank(c[d]);
                if (reinterpret_cast<const uint32_t*>(&items[rr])[0] & kDupBit) {
                  const int at = atomicAdd(&snl, 1);
                  const uint32_t key = ((uint32_t)(gid + (i0 + d) * ngrp) << lg) | (uint32_t)gl;
                  if (at < LCAP) dlist[at] = make_uint2(((uint32_t)rr << kKeyBits) | key, __float_as_uint(v[d]));
                }
              }
            }
          };
          if constexpr (MODE == 1) {
            append(0);
          } else {
            for (int i0 = 0; i0 < nr; i0 += RL) {   // the products again (B re-read)
              fetch(i0, nr, TC, clo);
              append(i0);
            }
          }
          __syncthreads();
          const int nl = snl;
          if (nl <= LCAP && w == 0) bm_det_sum(dlist, nl, items, lane);
          skip = nl > LCAP;
          if (skip && tid == 0) {
            if (MODE == 1) {   // the reload kernel redoes the unit with a larger list
              const uint32_t at = atomicAdd(p.novf, 1u);
              if ((int64_t)at < p.ovf_cap) p.ovf[at] = h.u;
              else atomicOr(p.err, 4);
            } else {
              atomicOr(p.err, 16);   // the host recomputes the product on the CPU engine
            }
          }
          __syncthreads();
          if (tid == 0) {
            sfix = 0;
            snl = 0;
          }
        }
      }
      BM_STAMP(3);
      // ---- the unit's slots to C at its final offset; clear the bitmap -----
      int lim = skip ? 0 : total;
      if (!skip && (want != total || off < 0 || off + total > p.cap)) {   // never write outside the unit or C
        if (tid == 0) atomicOr(p.err, 2);
        lim = (off < 0 || off + total > p.cap) ? 0 : (total < want ? total : (int)want);
      }
      bm_write_unit<NT>(items, lim, p.Cci, p.Cv, off, DET ? kColMask : 0xFFFFFFFFu);
      clear_bm();
      __syncthreads();   // cleared (and items read) before the next unit's pass 1
      BM_STAMP(4);
      BM_STAMP_UNIT();
    }
  }
  BM_STAMP_FLUSH();
  if constexpr (MODE == 1) BM_WG_FLUSH();
}

// ---- row-major kernels (nwin <= 8) -----------------------------------------
// A workgroup takes whole rows and runs their windows back to back, so the A
// row and all its window bounds are loaded ONCE per row, rows ahead (see the
// row pipeline in spgemm_bm_rows_pipe).
// ws8[j] = {first index of B row j, 16-bit lengths of windows 0..7} (uint4 x 2);
// ws8[2j + 1].y = first index of row j in the padded pair array (below).
//
// Padded B (``Bcv`` with ``pad`` = 1): the numeric kernel's (column, value)
// pairs with every (row, window) segment starting on a 128-byte line (16
// pairs), so a segment of L pairs touches ceil(L / 16) lines instead of ~1 +
// 8L / 128: random segment gathers run at a fixed rate of LINES, and the
// 1M config's ~13-pair segments gather 1.39x faster aligned (4.64 vs 3.35
// TB/s useful, tools/probes/seg_gather.hip, profiles/r4/seg_gather.md).
// (The unpipelined row kernels -- flat numeric, flat count, their
// deterministic forms -- were removed in round 6: the planner sends every
// product the pipelined ones cannot take to the per-unit kernels.)
struct BmRowArgs {
  BmArgs a;
  const uint4* ws8;
  int pad;   // numeric: Bcv is the padded pair array
};

// First B index of window q0 inside this entry's B row: the row start plus
// the packed 16-bit lengths of windows 0 .. q0-1.
__device__ __forceinline__ uint32_t bm_window_start(const uint4& wa, uint32_t wb, int q0) {
  uint32_t b = wa.x;
  for (int q = 0; q < q0; ++q) {
    const uint32_t wl = q < 2 ? wa.y : q < 4 ? wa.z : q < 6 ? wa.w : wb;
    b += (wl >> (16 * (q & 1))) & 0xffffu;
  }
  return b;
}

// ---- pipelined row-major numeric kernel (padded pairs, unordered sum) -------
// The per-unit kernel's work on whole rows (two padded pairs per 16-byte
// lane load) in a software pipeline that hides the B gathers: unit k+1 is staged (scan, descriptors) and its B loads
// are issued right after unit k's pass 2, BEFORE unit k's write-out, so the
// gathers travel while unit k's slots are copied to C.  Unit k+1's pass 1
// then finds its products landed (the flat kernel waited a full memory
// latency at every pass 1: ~35 % of a unit's cycles, shader-clock stamps,
// PERF_LOG round 5).  Memory is addressed through buffer descriptors with
// 32-bit offsets: B gathers as buffer_load_dwordx4 (no 64-bit address
// arithmetic per load), and the write-out as a FIXED count of 16-byte
// buffer_store_dwordx4 per lane whose range check (num_records = the unit's
// entries) drops the lanes past the unit -- a fixed store count lets the
// compiler wait for the next unit's loads with vmcnt(#stores) and leave the
// write-out stores in flight.  Four barriers per unit instead of six.
typedef uint32_t bm_v4u __attribute__((ext_vector_type(4)));

struct BmPipeArgs {
  BmRowArgs r;
  uint32_t bcv_bytes;   // bytes of the padded pair array (< 2^32: checked by the host)
  int64_t annz;         // nnz(A) > 0
  int32_t* ticket;      // row ticket counter, zero at launch
};


template <int LGW, int NT, int PCAP, int R, int CCAP, int WPE = 4>
__global__ __launch_bounds__(NT, WPE) void spgemm_bm_rows_pipe(BmPipeArgs pa) {
  const BmRowArgs& ra = pa.r;
  const BmArgs& p = ra.a;
  constexpr int NW = NT / 64;
  constexpr int NWORD = (1 << LGW) / 64, WPW = NWORD / NW, WPT = WPW / 64;
  constexpr int RR = R;          // product slots per lane
  constexpr int RL = RR / 2;     // load rounds (two pairs per lane and load)
  constexpr int NWR = (PCAP + 4 * NT - 1) / (4 * NT);   // write-out rounds: four entries per lane and round
  static_assert(RR % 2 == 0 && WPW % 64 == 0 && PCAP < 65536, "geometry");
  constexpr int SG = (kSweepG > 1 && WPW % (64 * kSweepG) == 0) ? kSweepG : 1;
  constexpr bool PAIRS = SG > 1;

  __shared__ __attribute__((aligned(16))) unsigned long long bm[NWORD];
  __shared__ __attribute__((aligned(16))) uint16_t pre16[NWORD];
  __shared__ __attribute__((aligned(16))) unsigned long long items[NWR * 4 * NT];
  __shared__ __attribute__((aligned(16))) uint2 desc[CCAP];   // chunk: {first B pair, valid pairs}
  __shared__ float dval[CCAP];                                 //        a(i, j)
  __shared__ int wsum[NW];        // rank sweep: word totals per wave
  __shared__ int wscan[2 * NW];   // staging scan
  __shared__ __attribute__((aligned(8))) int64_t suo[9];   // unit offsets of the staged row (uoff[row * nwin + q])
  __shared__ int sdup;
  __shared__ int s_tk[2];   // row tickets: row ids, double-buffered (see next_row)

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lgc = p.lg;          // log2 pairs per chunk
  const int lg = lgc - 1;        // log2 lanes per chunk
  const int Gc = 1 << lgc;
  const int Gl = 1 << lg;
  const int ngrp = NW << (6 - lg);
  const int gid = (w << (6 - lg)) + (lane >> lg);
  const int gl = lane & (Gl - 1);
  const int nwin = p.nwin;
  uint32_t* const bm32 = reinterpret_cast<uint32_t*>(bm);
  BM_STAMP_DECL
  BM_WG_DECL
  if (*p.err & 8) return;   // ws8 lengths truncated: the host takes the per-unit kernels (uniform exit)
  const auto rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2*>(p.Bcv), 0, (int)pa.bcv_bytes, 0x00020000);

  for (int i = tid; i < NWORD / 2; i += NT) reinterpret_cast<uint4*>(bm)[i] = make_uint4(0, 0, 0, 0);
  if (tid == 0) sdup = 0;

  // 32-bit row indices: the host takes this path only for m * nwin < 2^31
  const int NG = (int)gridDim.x;
  const int me = (NG % 8 == 0) ? (int)(blockIdx.x % 8) * (NG / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
  const int m = (int)p.m;
  const int annz = (int)pa.annz;   // > 0 (checked by the host)
  // Row schedule.  The first six rows of a workgroup are static (me, me + NG, ..), every
  // later one is a ticket: 6 NG + a global counter.  Equal rows per workgroup are not equal
  // time: the four workgroups of a CU arbitrate unequally and the statically scheduled grid's
  // ends spread over +-13 % of the kernel (tools/bm_wg_times.py, PERF_LOG round 6), so the
  // faster workgroups take more rows and every slot stays busy to the end.  Thread 0 fetches
  // a ticket at the top of a row's last unit (a global atomic into a unit-local register)
  // and writes it to LDS at the end of that unit -- straight-line code, so hipcc's wait for
  // the atomic there covers only what was issued after it; the slot is read two rows later
  // (the row pointers of row k + 4 are loaded in row k's last unit).  A buffer atomic whose
  // result crosses the loop back-edge got no wait from hipcc: garbage row ids.
  int kl = 0;   // last units (rows) done by this workgroup
  // a zero hipcc cannot see through: the ticket atomic's offset looks divergent, so the atomic
  // optimizer leaves it alone (it would combine the lanes and wait for the result on the spot);
  // a buffer atomic keeps the address in scalar registers
  int tkz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(tkz));
  const auto rtk = __builtin_amdgcn_make_buffer_rsrc(pa.ticket, 0, 4, 0x00020000);
  int id1 = me, id2 = me + NG, id3 = me + 2 * NG;   // rows in the "1" / "2" / "3" pipeline registers
  auto next_row = [&]() {   // row k + 4 in row k's last unit
    if constexpr (!SPMM_BM_TICKETS) return id3 + NG;
    return kl < 2 ? me + (kl + 4) * NG : __builtin_amdgcn_readfirstlane(s_tk[kl & 1]);
  };

  // ---- row pipeline --------------------------------------------------------
  // The per-row inputs (A entries, packed window bounds, unit offsets) are
  // loaded ONCE per row, unconditionally at the top of the row loop, each
  // from values that landed during the previous row: the next row's bounds
  // (from its A columns), the row after's A entries (from its row pointers),
  // the third row's row pointers (rows in the order of the row schedule).  No load sits under a branch inside the
  // loops and none is consumed in the row that issues it, so hipcc never
  // merges or copies a register whose load is still in flight (a merge it
  // materialises as copies that wait for the load: a full memory latency
  // per row).  Indices are clamped into range (values past the matrix or the
  // row are never used).
  auto arp2 = [&](int r, int& a, int& b) {   // row pointers of row r (clamped; low words: nnz(A) < 2^31)
    const int rr = r < m ? r : m - 1;
    const int* lo = reinterpret_cast<const int*>(p.Arp);
    a = lo[2 * rr];
    b = lo[2 * rr + 2];
  };
  auto entry = [&](int a, int b) {   // this thread's A entry of the row [a, b) (clamped)
    const int a0 = __builtin_amdgcn_readfirstlane(a), na = __builtin_amdgcn_readfirstlane(b) - a0;
    const int e = a0 + (tid < na ? tid : 0);
    return e < annz ? e : annz - 1;
  };
  auto uoff_of = [&](int r) {   // lane q <= nwin: uoff[r * nwin + q] (clamped)
    const int rr = r < m ? r : m - 1;
    return p.uoff[(int64_t)rr * nwin + (lane <= nwin ? lane : nwin)];
  };
  int a1 = 0, b1 = 0, a2 = 0, b2 = 0, a3 = 0, b3 = 0;
  arp2(id1, a1, b1);
  int e2 = entry(a1, b1);
  uint32_t jj1 = (uint32_t)p.Aci[e2];   // row me: A column / value of this thread's entry
  float av1 = p.Av[e2];
  uint4 wa1 = ra.ws8[2 * (int64_t)jj1];   // ... its packed bounds and the row's unit offsets
  uint2 wb1 = *reinterpret_cast<const uint2*>(ra.ws8 + 2 * (int64_t)jj1 + 1);
  int64_t uo1 = uoff_of(id1);
  int na1 = __builtin_amdgcn_readfirstlane(b1 - a1);
  arp2(id2, a2, b2);
  e2 = entry(a2, b2);
  uint32_t jj2 = (uint32_t)p.Aci[e2];   // row me + NG: its A entries
  float av2 = p.Av[e2];
  int na2 = b2 - a2;
  arp2(id3, a3, b3);                    // row me + 2 NG: its row pointers
  // Once per row, in the LAST unit of the current row (after its pass 1, with
  // loads that land while the unit finishes): the next row's inputs are taken
  // into the staging registers, then the row after's bounds and offsets are
  // loaded from its A columns (landed one row ago), the third row's A entries
  // from its row pointers (idem) and the fourth row's row pointers.  No load
  // sits under a branch and none is consumed in the unit that issues it.
  auto row_block = [&](int next_id) {
    id1 = id2;
    id2 = id3;
    id3 = next_id;
    jj1 = jj2;
    wa1 = ra.ws8[2 * (int64_t)jj1];
    wb1 = *reinterpret_cast<const uint2*>(ra.ws8 + 2 * (int64_t)jj1 + 1);
    uo1 = uoff_of(id1);
    av1 = av2;
    na1 = __builtin_amdgcn_readfirstlane(na2);
    e2 = entry(a3, b3);
    jj2 = (uint32_t)p.Aci[e2];
    av2 = p.Av[e2];
    na2 = b3 - a3;
    arp2(id3, a3, b3);
  };

  // staging registers of the row being staged
  int cna = 0, cid = me;   // (cid: its row id)
  float cav = 0.f;
  uint32_t cl0 = 0, cl1 = 0, cl2 = 0, cl3 = 0;   // 16-bit window lengths, two per word; cl0 = the word
                                                  // of the window being staged (shifted down every two
                                                  // windows: no run-time indexing, which hipcc would
                                                  // put in scratch)
  uint32_t bq = 0;   // this thread's entry: first pair of the next window to stage
  auto take_row = [&]() {   // the next row's inputs -> staging registers (their loads have landed)
    cid = id1;
    cna = na1;
    cav = av1;
    bq = wb1.y;   // first pair of the entry's B row in the padded pair array
    cl0 = wa1.y;
    cl1 = wa1.z;
    cl2 = wa1.w;
    cl3 = wb1.x;
    if (lane <= nwin) suo[lane] = uo1;   // read after the stage's scan barrier
  };

  // ---- the staged unit ------------------------------------------------------
  int srow = me, sq = 0;
  int sTC = 0, snr = 0, sclo = 0, swant = 0;
  int64_t soff = 0;
  bool sskip = false;
  bm_v4u xb[RL];
  uint32_t okm = 0;     // bit s: product slot s (round s / 2, pair s % 2) is in its segment
  bool dirty = false;   // the bitmap holds a formed unit's columns

  // Stage unit (srow, sq): scan, descriptors, offsets.  An empty or
  // oversized unit is staged like any other with sskip set (no loop in
  // here); the main loop runs no passes for it.  The scan's barrier also ends
  // the previous unit's pass 2 (every rank lookup and slot write done).
  auto stage = [&]() {
    const int q = sq;
    int len = 0, nch = 0;
    if (tid < cna) {
      len = (int)((cl0 >> (16 * (q & 1))) & 0xffffu);
      nch = (len + Gc - 1) >> lgc;
    }
    if (q & 1) {   // uniform
      cl0 = cl1;
      cl1 = cl2;
      cl2 = cl3;
    }
    const uint32_t b0 = bq;
    bq += (uint32_t)(((len + (1 << kPadLg) - 1) >> kPadLg) << kPadLg);
    int pre, plen, TCv, Pv;
    bm_scan2<NT>(nch, len, wscan, pre, plen, TCv, Pv);
    const int TC = __builtin_amdgcn_readfirstlane(TCv), P = __builtin_amdgcn_readfirstlane(Pv);
    const int u = srow * nwin + q;
    const bool too_big = cna > NT || P > PCAP || TC > CCAP || TC > RL * ngrp;
    sskip = P == 0 || too_big;
    if (too_big && P != 0 && tid == 0) {   // the reload kernel forms it
      const uint32_t at = atomicAdd(p.novf, 1u);
      if ((int64_t)at < p.ovf_cap) p.ovf[at] = u;
      else atomicOr(p.err, 4);
    }
    if (dirty) {   // the previous unit's rank lookups are done (scan barrier)
      for (int i = tid; i < NWORD / 2; i += NT) reinterpret_cast<uint4*>(bm)[i] = make_uint4(0, 0, 0, 0);
      dirty = false;
    }
    if (!sskip)
      for (int kk = 0; kk < nch; ++kk) {
        const int rem = len - (kk << lgc);
        desc[pre + kk] = make_uint2(b0 + ((uint32_t)kk << lgc), (uint32_t)(rem < Gc ? rem : Gc));
        dval[pre + kk] = cav;
      }
    {   // this unit's offset in C and its count (the count kernel's)
      const int64_t o0 = suo[q], o1 = suo[q + 1];
      soff = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)o0 >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)o0));
      swant = __builtin_amdgcn_readfirstlane((int)(o1 - o0));
    }
    sTC = TC;
    snr = sskip ? 0 : (TC + ngrp - 1) / ngrp;
    sclo = q << LGW;
    __syncthreads();   // descriptors written, bitmap clear, wscan / suo read
  };
  // descriptor reads and B gathers of the staged unit (rounds past its chunks load nothing)
  auto issue_loads = [&]() {
    const int TC = sTC;
    uint2 ds[RL];
#pragma unroll
    for (int d = 0; d < RL; ++d) {
      const int t = gid + d * ngrp;
      ds[d] = desc[t < TC ? t : TC - 1];
    }
    okm = 0;
    uint32_t f[RL];
#pragma unroll
    for (int d = 0; d < RL; ++d) {
      const int t = gid + d * ngrp;
      const int nv = (int)ds[d].y - 2 * gl;
      const bool ok = (t < TC) & (nv > 0);
      okm |= (ok ? 1u : 0u) << (2 * d);
      okm |= ((ok & (nv > 1)) ? 1u : 0u) << (2 * d + 1);
      f[d] = ds[d].x + (ok ? (uint32_t)(2 * gl) : 0u);
    }
#pragma unroll
    for (int d = 0; d < RL; ++d) {
      xb[d] = bm_v4u{0u, 0u, 0u, 0u};
      if (d < snr) xb[d] = __builtin_amdgcn_raw_buffer_load_b128(rsb, (int)(f[d] * 8u), 0, 0);   // wave-uniform guard
    }
  };
  // a unit's slots to C: NWR rounds of four entries per lane, 16-byte stores
  // through descriptors of lim entries (lanes past the unit dropped)
  auto write_out = [&](int64_t off, int lim) {
    const int nb = __builtin_amdgcn_readfirstlane(lim * 4);
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(p.Cci + off, 0, nb, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc(p.Cv + off, 0, nb, 0x00020000);
#pragma unroll
    for (int rd = 0; rd < NWR; ++rd) {
      const int e = (rd * NT + tid) * 4;
      const ulonglong2 i01 = *reinterpret_cast<const ulonglong2*>(&items[e]);
      const ulonglong2 i23 = *reinterpret_cast<const ulonglong2*>(&items[e + 2]);
      const bm_v4u cc{(uint32_t)i01.x, (uint32_t)i01.y, (uint32_t)i23.x, (uint32_t)i23.y};
      const bm_v4u vv{(uint32_t)(i01.x >> 32), (uint32_t)(i01.y >> 32), (uint32_t)(i23.x >> 32),
                      (uint32_t)(i23.y >> 32)};
      __builtin_amdgcn_raw_buffer_store_b128(cc, rc, e * 4, 0, 2);   // aux 2: nt
      __builtin_amdgcn_raw_buffer_store_b128(vv, rv, e * 4, 0, 2);
    }
  };

  take_row();     // staging registers: row me
  row_block(me + 3 * NG);   // next-row registers: row me + NG's bounds; A entries of me + 2 NG; Arp of me + 3 NG
  stage();
  issue_loads();
  // the loop is entered with the same stores behind the first unit's B
  // loads as every later unit has (all dropped: zero records), so the
  // compiler's wait at pass 1 is vmcnt(#stores) on every path, not vmcnt(0)
  write_out(0, 0);
  int c[RR];
  float v[RR];
  // one unit of row `row`, window q; LAST: the row's last window (the row
  // inputs move one row along, and the next unit staged is the next row's first)
  auto unit = [&](auto last_tag, int row, int q) {
    constexpr bool LAST = decltype(last_tag)::value;
      const int TC = sTC, nr = snr, clo = sclo, want = swant;
      const int64_t off = soff;
      int lim = 0;
      int tk = 0;
      if constexpr (LAST && SPMM_BM_TICKETS)
        if (tid == 0) tk = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rtk, tkz, 0, 0);   // (to LDS at the unit's end)
      BM_STAMP(4);   // (the previous unit's write-out)
      if (sskip) {   // uniform
        if constexpr (LAST) {
          take_row();
          row_block(next_row());
        }
      } else {
        // ---- pass 1: the landed products, columns into the bitmap --------
        // (a(i, j) from dval: rewritten only by the stage after this unit's pass 2)
#pragma unroll
        for (int d = 0; d < RL; ++d) {
          const int t = gid + d * ngrp;
          const float a = dval[t < TC ? t : TC - 1];
          c[2 * d] = ((okm >> (2 * d)) & 1u) ? (int)xb[d].x - clo : -1;
          c[2 * d + 1] = ((okm >> (2 * d + 1)) & 1u) ? (int)xb[d].z - clo : -1;
          v[2 * d] = a * __uint_as_float(xb[d].y);
          v[2 * d + 1] = a * __uint_as_float(xb[d].w);
        }
        uint32_t dupm = 0;
        {
          uint32_t old[RR];
#pragma unroll
          for (int d = 0; d < RR; ++d) {
            old[d] = 0u;
            if (c[d] >= 0) old[d] = atomicOr(bm32 + (c[d] >> 5), 1u << (c[d] & 31));
          }
#pragma unroll
          for (int d = 0; d < RR; ++d) dupm |= (c[d] >= 0 ? (old[d] >> (c[d] & 31)) & 1u : 0u) << d;
        }
        dirty = true;
        if (dupm) sdup = 1;
        __syncthreads();
        if constexpr (LAST) {   // the next row into the staging registers; the row inputs move along
          take_row();
          row_block(next_row());
        }
        BM_STAMP(1);
        // ---- rank prefix per 64-bit word ---------------------------------
        int run[WPT];
        int wtot = 0;
        if constexpr (PAIRS) {
#pragma unroll
          for (int kk = 0; kk < WPT / SG; ++kk) {
            const ulonglong2* src = reinterpret_cast<const ulonglong2*>(&bm[w * WPW + kk * 64 * SG + SG * lane]);
            int cw[SG];
#pragma unroll
            for (int h = 0; h < SG / 2; ++h) {
              const ulonglong2 x = src[h];
              cw[2 * h] = __popcll(x.x);
              cw[2 * h + 1] = __popcll(x.y);
            }
            int sum = 0;
#pragma unroll
            for (int i = 0; i < SG; ++i) {
              if (i > 0) run[SG * kk + i] = sum;
              sum += cw[i];
            }
            const int incl = bm_wave_incl(sum);
            run[SG * kk] = wtot + incl - sum;
            wtot += __builtin_amdgcn_readlane(incl, 63);
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < WPT; ++kk) {
            const int cnt = __popcll(bm[w * WPW + kk * 64 + lane]);
            const int incl = bm_wave_incl(cnt);
            run[kk] = wtot + incl - cnt;
            wtot += __builtin_amdgcn_readlane(incl, 63);
          }
        }
        const int any_dup = sdup;
        if (lane == 0) wsum[w] = wtot;
        __syncthreads();
        int base = 0, total = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
          const int sw = wsum[i];
          base += (i < w) ? sw : 0;
          total += sw;
        }
        total = __builtin_amdgcn_readfirstlane(total);
        if constexpr (PAIRS) {
#pragma unroll
          for (int kk = 0; kk < WPT / SG; ++kk) {
            const uint32_t g0 = (uint32_t)(base + run[SG * kk]);
            uint32_t pk[SG / 2];
#pragma unroll
            for (int h = 0; h < SG / 2; ++h) {
              const uint32_t lo = g0 + (h > 0 ? (uint32_t)run[SG * kk + 2 * h] : 0u);
              const uint32_t hi = g0 + (uint32_t)run[SG * kk + 2 * h + 1];
              pk[h] = (lo & 0xffffu) | (hi << 16);
            }
            uint16_t* dst = &pre16[w * WPW + kk * 64 * SG + SG * lane];
            if constexpr (SG == 2) {
              *reinterpret_cast<uint32_t*>(dst) = pk[0];
            } else if constexpr (SG == 4) {
              *reinterpret_cast<uint2*>(dst) = make_uint2(pk[0], pk[1]);
            } else {
              static_assert(SG == 8, "sweep group of 2, 4 or 8 words");
              *reinterpret_cast<uint4*>(dst) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            }
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < WPT; ++kk) pre16[w * WPW + kk * 64 + lane] = (uint16_t)(base + run[kk]);
        }
        if (tid == 0) sdup = 0;
        __syncthreads();
        BM_STAMP(2);
        // ---- pass 2: rank -> slot; owners store, duplicates add after a barrier
        auto rank = [&](int cc) {
          const int wd = cc >> 6;
          return (int)pre16[wd] + __popcll(bm[wd] & ((1ull << (cc & 63)) - 1ull));
        };
#pragma unroll
        for (int d0 = 0; d0 < RR; d0 += 4) {
          if (d0 >= nr * 2) break;   // uniform: slots past the unit's chunks hold no product
          int r[4];
#pragma unroll
          for (int dd = 0; dd < 4 && d0 + dd < RR; ++dd) r[dd] = rank(c[d0 + dd] >= 0 ? c[d0 + dd] : 0);
#pragma unroll
          for (int dd = 0; dd < 4 && d0 + dd < RR; ++dd) {
            const int d = d0 + dd;
            if (c[d] >= 0 && !((dupm >> d) & 1u))
              items[r[dd]] = ((unsigned long long)__float_as_uint(v[d]) << 32) | (uint32_t)(c[d] + clo);
          }
        }
        if (any_dup) {   // uniform
          __syncthreads();
#pragma unroll
          for (int d = 0; d < RR; ++d)
            if ((dupm >> d) & 1u) atomicAdd(reinterpret_cast<float*>(&items[rank(c[d])]) + 1, v[d]);
        }
        lim = total;
        if (want != total || off < 0 || off + total > p.cap) {   // never write outside the unit or C
          if (tid == 0) atomicOr(p.err, 2);
          lim = (off < 0 || off + total > p.cap) ? 0 : (total < want ? total : want);
        }
      }
      BM_STAMP(3);
      // ---- stage the next unit and issue its B gathers; then this unit's write-out
      bool more = true;
      if constexpr (LAST) {
        srow = cid;   // (taken in this unit)
        sq = 0;
        more = srow < m;
      } else {
        sq = q + 1;
      }
      if (more) {
        SPMM_BM_PRIO_HI();
        stage();
        issue_loads();
        SPMM_BM_PRIO_LO();
      } else {
        __syncthreads();   // this unit's pass 2 done before its slots are read
      }
      BM_STAMP(0);
      BM_STAMP_UNIT();
      write_out(off, lim);
      if constexpr (LAST && SPMM_BM_TICKETS) {
        if (tid == 0) s_tk[kl & 1] = 6 * NG + tk;   // (read in row kl + 2's last unit, barriers between)
        ++kl;
      }
      };
  for (int row = me; row < m; row = srow) {   // (srow: the next row, staged by the row's last unit)
    for (int q = 0; q + 1 < nwin; ++q) unit(std::false_type{}, row, q);
    unit(std::true_type{}, row, nwin - 1);
  }
  BM_STAMP_FLUSH();
  BM_WG_FLUSH();
}

// ---- row-major count kernel (nwin <= 8, A rows <= NT entries) -------------
// The count kernel of the same row pipeline: one window's bitmap (16 KB at
// W = 2^17) per workgroup, so eight 256-thread workgroups share a CU and
// hide each other's B-load latency (the 8-window, 128 KB-bitmap count kernel
// runs one workgroup per CU).  Every unit: ORs (no return), popcount of the
// wave's own bitmap rows, clear of the same rows, one barrier.
template <int LGW, int NSUB, int NT, int RR, int CCAP, bool PADC>
#ifndef SPMM_BM_COUNT_WPS   // row count kernel: waves per SIMD its registers are sized for (8: <= 64 VGPRs)
#define SPMM_BM_COUNT_WPS 8   // (64k: 8 = 1.547-1.551 ms with 2 spills, 7 = 1.547-1.565, 6 = 1.641)
#endif
__global__ __launch_bounds__(NT, SPMM_BM_COUNT_WPS) void spgemm_bm_rows_count(BmRowArgs ra) {
  const BmArgs& p = ra.a;
  constexpr int NW = NT / 64;
  constexpr int NWORD = (NSUB << LGW) / 64, WPW = NWORD / NW, WPT = WPW / 64;
  constexpr int WORDS_PER_WIN = NWORD / NSUB;
  static_assert(WPW % 64 == 0 && WORDS_PER_WIN % WPW == 0, "a wave's bitmap block inside one window");
  // log2 columns per lane and load: padded columns are read 4 at a time
  // (16-byte loads: the gathers are bound by their load-instruction count,
  // 1M count 16.5 -> 15.3 ms vs 8-byte loads, PERF_LOG round 4), the host's
  // lane groups halved to keep a chunk at one 128-byte line
  constexpr bool WIDE = PADC;
  constexpr int SH = PADC ? 2 : 0;
  constexpr int CPL = 1 << SH;

  __shared__ __attribute__((aligned(16))) unsigned long long bm[NWORD];
  __shared__ __attribute__((aligned(16))) uint2 desc[CCAP];
  __shared__ int wsum[2 * NW];
  __shared__ int csum[NW];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = p.lg - (WIDE ? 1 : 0);
  const int Gl = 1 << lg;
  const int ngrp = NW << (6 - lg);
  const int gid = (w << (6 - lg)) + (lane >> lg);
  const int gl = lane & (Gl - 1);
  const int nwin = p.nwin;
  uint32_t* const bm32 = reinterpret_cast<uint32_t*>(bm);
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  if (*p.err & 8) return;   // ws8 lengths truncated: the host re-counts with spgemm_bm (uniform exit)

  for (int i = tid; i < NWORD / 2; i += NT) reinterpret_cast<uint4*>(bm)[i] = make_uint4(0, 0, 0, 0);

  // 32-bit row / unit indices: the host takes this path only for m * nwin < 2^31
  const int NG = (int)gridDim.x;
  const int me = (NG % 8 == 0) ? (int)(blockIdx.x % 8) * (NG / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
  const int m = (int)p.m;
  // chunked grid (ra.a.chunk > 0): rows b * chunk .. + chunk a workgroup, as the per-unit
  // numeric kernel's chunked schedule; else persistent (me, me + NG, ...)
  const int CR = ra.a.chunk;
  const int S = CR > 0 ? 1 : NG;
  int row = CR > 0 ? (int)blockIdx.x * CR : me;
  const int lim = CR > 0 ? min(m, row + CR) : m;
  int cna = 0;
  uint4 cwa = make_uint4(0, 0, 0, 0);
  uint32_t cwb = 0;
  int n1a = 0, n1b = 0, n2a = 0, n2b = 0, njj = 0;
  uint4 nwa = make_uint4(0, 0, 0, 0);
  uint32_t nwb = 0;
  auto ld_arp = [&](int r, int& a, int& b) {
    if (r < m) {
      a = (int)p.Arp[r + vz];
      b = (int)p.Arp[r + 1 + vz];
    }
  };
  auto ld_entries = [&](int r) {
    if (r < m) {
      const int a0 = __builtin_amdgcn_readfirstlane(n1a), na = __builtin_amdgcn_readfirstlane(n1b) - a0;
      if (tid < na) njj = p.Aci[a0 + tid];
    }
  };
  auto ld_bounds = [&](int r) {
    if (r < m) {
      const int na = __builtin_amdgcn_readfirstlane(n1b) - __builtin_amdgcn_readfirstlane(n1a);
      if (tid < na) {
        nwa = ra.ws8[2 * (int64_t)njj];
        const uint4 x = ra.ws8[2 * (int64_t)njj + 1];
        nwb = x.x;
        if constexpr (PADC) nwa.x = x.z;   // the row's first column in the padded column array
      }
    }
  };
  auto take_next = [&]() {
    cna = __builtin_amdgcn_readfirstlane(n1b) - __builtin_amdgcn_readfirstlane(n1a);
    cwa = nwa;
    cwb = nwb;
    n1a = n2a;
    n1b = n2b;
  };
  ld_arp(row, n1a, n1b);
  ld_entries(row);
  ld_bounds(row);
  ld_arp(row + S, n2a, n2b);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  take_next();
  __syncthreads();

  for (; row < lim; row += S) {
    const int na = cna;
    uint32_t bq = cwa.x;
    for (int q = 0; q < nwin; q += NSUB) {   // a unit: windows [q, q + NSUB) of the row
      const bool last = q + NSUB >= nwin;
      if (q == 0) {
        ld_entries(row + S);
        ld_arp(row + 2 * S, n2a, n2b);
      }
      if (last) ld_bounds(row + S);
      const uint32_t wl = q < 2 ? cwa.y : q < 4 ? cwa.z : q < 6 ? cwa.w : cwb;
      int len = 0, nch = 0;
      if (tid < na && tid < NT) {
        if constexpr (NSUB == 1) {
          len = (int)((wl >> (16 * (q & 1))) & 0xffffu);
        } else if constexpr (NSUB == 2) {   // q even: windows q and q + 1 share one 32-bit word of lengths
          len = (int)(wl & 0xffffu) + (int)(wl >> 16);   // (lengths past nwin are packed as 0)
        } else {   // q a multiple of NSUB: the unit's lengths are whole 32-bit words of ws8
          static_assert(NSUB == 4 || NSUB == 8, "count units of 1, 2, 4 or 8 windows");
          const uint32_t wq[4] = {cwa.y, cwa.z, cwa.w, cwb};
#pragma unroll
          for (int k = 0; k < NSUB / 2; ++k) {
            const uint32_t x = wq[(q >> 1) + k < 4 ? (q >> 1) + k : 3];
            len += (int)(x & 0xffffu) + (int)(x >> 16);
          }
        }
        nch = (len + (Gl << SH) - 1) >> (lg + SH);
      }
      const uint32_t b0 = bq;
      bq += PADC ? (uint32_t)(((len + (1 << kPadCLg) - 1) >> kPadCLg) << kPadCLg) : (uint32_t)len;
      const int clo = q << LGW;
      const int u = row * nwin + q;
      int pre, plen, TC, P;
      bm_scan2<NT>(nch, len, wsum, pre, plen, TC, P);
      for (int cb = 0; cb < TC; cb += CCAP) {
        const int TCb = TC - cb < CCAP ? TC - cb : CCAP;
        const int k0 = max(cb - pre, 0), k1 = min(cb + CCAP - pre, nch);
        for (int kk = k0; kk < k1; ++kk) {
          const int rem = len - (kk << (lg + SH));
          desc[pre + kk - cb] =
              make_uint2(b0 + ((uint32_t)kk << (lg + SH)), (uint32_t)(rem < (Gl << SH) ? rem : (Gl << SH)));
        }
        __syncthreads();
        const int nr = (TCb + ngrp - 1) / ngrp;
        for (int i0 = 0; i0 < nr; i0 += RR) {
          uint2 ds[RR];
#pragma unroll
          for (int d = 0; d < RR; ++d) {
            const int t = gid + (i0 + d) * ngrp;
            ds[d] = desc[t < TCb ? t : TCb - 1];
          }
          if constexpr (PADC) {
            // four columns per lane: one 16-byte load (aligned: chunks start on
            // 32-column boundaries of the padded array); the later columns
            // may be past the segment (padding)
            static_assert(RR * CPL <= 32, "one bit per loaded column");
            uint32_t x[RR][CPL];
            uint32_t okb = 0;   // bit d * CPL + i: column i of round d is in its segment
#pragma unroll
            for (int d = 0; d < RR; ++d) {
              const int t = gid + (i0 + d) * ngrp;
              const int nv = (int)ds[d].y - CPL * gl;
              const bool ok = (t < TCb) & (nv > 0);
              okb |= (ok ? ((nv >= CPL) ? (1u << CPL) - 1u : (1u << nv) - 1u) : 0u) << (d * CPL);
#pragma unroll
              for (int i = 0; i < CPL; ++i) x[d][i] = 0u;
              if (i0 + d < nr) {   // wave-uniform guard
                const uint4 v = *reinterpret_cast<const uint4*>(p.Bci + ds[d].x + (ok ? (uint32_t)(CPL * gl) : 0u));
                x[d][0] = v.x; x[d][1] = v.y; x[d][2] = v.z; x[d][3] = v.w;
              }
            }
#pragma unroll
            for (int d = 0; d < RR; ++d) {
#pragma unroll
              for (int i = 0; i < CPL; ++i) {
                if ((okb >> (d * CPL + i)) & 1u) {
                  const int cc = (int)x[d][i] - clo;
                  atomicOr(bm32 + (cc >> 5), 1u << (cc & 31));
                }
              }
            }
          } else {
            int x[RR];
            uint32_t okm = 0;
#pragma unroll
            for (int d = 0; d < RR; ++d) {
              const int t = gid + (i0 + d) * ngrp;
              const bool ok = (t < TCb) & ((uint32_t)gl < ds[d].y);
              okm |= (ok ? 1u : 0u) << d;
              x[d] = 0;
              if (i0 + d < nr) x[d] = p.Bci[ds[d].x + (ok ? (uint32_t)gl : 0u)];   // wave-uniform guard
            }
#pragma unroll
            for (int d = 0; d < RR; ++d) {
              if ((okm >> d) & 1u) {
                const int cc = x[d] - clo;
                atomicOr(bm32 + (cc >> 5), 1u << (cc & 31));
              }
            }
          }
        }
        __syncthreads();   // descriptors consumed before they are rewritten; every OR in place
      }
      if (last) take_next();   // after this unit's B loads: every older load has landed
      if (P == 0) {   // uniform: nothing was ORed
        if constexpr (NSUB == 1) {
          if (tid == 0) p.ucnt[u] = 0;
        } else if (tid < NSUB && q + tid < nwin) {
          p.ucnt[u + tid] = 0;
        }
        __syncthreads();   // wsum reads done before the next scan
        continue;
      }
      // popcount of this wave's bitmap rows, clearing them as they are read
      int cnt = 0;
#pragma unroll
      for (int kk = 0; kk < WPT; ++kk) {
        const int wd = w * WPW + kk * 64 + lane;
        cnt += __popcll(bm[wd]);
        bm[wd] = 0ull;
      }
      cnt = bm_wave_sum(cnt);
      if (lane == 0) csum[w] = cnt;
      __syncthreads();
      if constexpr (NSUB == 1) {
        if (tid == 0) {
          int t = 0;
#pragma unroll
          for (int i = 0; i < NW; ++i) t += csum[i];
          p.ucnt[u] = t;
        }
      } else if (tid < NSUB && q + tid < nwin) {   // window tid of the unit: the waves whose blocks lie in it
        constexpr int WAVES_PER_WIN = WORDS_PER_WIN / WPW;
        int t = 0;
#pragma unroll
        for (int i = 0; i < WAVES_PER_WIN; ++i) t += csum[tid * WAVES_PER_WIN + i];
        p.ucnt[u + tid] = t;
      }
    }
  }
}

// ---- pipelined row-major count kernel (two-window units, padded columns) ---
// spgemm_bm_rows_count<..., NSUB = 2, PADC> in the pipelined form of
// spgemm_bm_rows_pipe: unit k+1's scan rides unit k's OR phase (its
// per-wave sums are written before that phase's barrier), its descriptors
// are written after it and its B loads issued BEFORE unit k's popcount and
// clear, so the gathers travel while unit k's bitmap is counted and
// cleared.  Three barriers per unit instead of four; column loads through a
// buffer descriptor (32-bit offsets); the row inputs are loaded once per row
// at the top of the row loop from values that landed during the previous
// row (as in spgemm_bm_rows_pipe).  Chunks past the RR load rounds (rare:
// units of > RR * ngrp chunks) are loaded and ORed in the same phase,
// synchronously.
struct BmCountPipeArgs {
  BmRowArgs r;
  uint32_t colp_bytes;   // bytes of the padded column array (< 2^32: checked by the host)
  int64_t annz;          // nnz(A) > 0
};

template <int LGW, int NT, int RR, int CCAP>
__global__ __launch_bounds__(NT, 4) void spgemm_bm_rows_count_pipe(BmCountPipeArgs pa) {
  const BmRowArgs& ra = pa.r;
  const BmArgs& p = ra.a;
  constexpr int NSUB = 2;
  constexpr int NW = NT / 64;
  constexpr int NWORD = (NSUB << LGW) / 64, WPW = NWORD / NW, WPT = WPW / 64;
  constexpr int WORDS_PER_WIN = NWORD / NSUB;
  constexpr int WAVES_PER_WIN = WORDS_PER_WIN / WPW;
  static_assert(WPW % 64 == 0 && WORDS_PER_WIN % WPW == 0, "a wave's bitmap block inside one window");
  static_assert(RR * 4 <= 32, "one bit per loaded column");

  __shared__ __attribute__((aligned(16))) unsigned long long bm[NWORD];
  __shared__ __attribute__((aligned(16))) uint2 desc[CCAP];
  __shared__ int wscan[2 * NW];
  __shared__ int csum[NW];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = p.lg - 1;       // log2 lanes per chunk (four columns per lane)
  const int Gl = 1 << lg;
  const int Gc = Gl << 2;        // columns per chunk
  const int ngrp = NW << (6 - lg);
  const int gid = (w << (6 - lg)) + (lane >> lg);
  const int gl = lane & (Gl - 1);
  const int nwin = p.nwin;
  uint32_t* const bm32 = reinterpret_cast<uint32_t*>(bm);
  BM_STAMP_DECL
  if (*p.err & 8) return;   // ws8 lengths truncated: the host re-counts with spgemm_bm (uniform exit)
  const auto rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(p.Bci), 0, (int)pa.colp_bytes, 0x00020000);
  const auto rsu = __builtin_amdgcn_make_buffer_rsrc(p.ucnt, 0, (int)((uint32_t)p.m * (uint32_t)nwin * 4u), 0x00020000);

  for (int i = tid; i < NWORD / 2; i += NT) reinterpret_cast<uint4*>(bm)[i] = make_uint4(0, 0, 0, 0);

  const int NG = (int)gridDim.x;
  const int me = (NG % 8 == 0) ? (int)(blockIdx.x % 8) * (NG / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
  const int m = (int)p.m;
  const int annz = (int)pa.annz;
  const int ngc = (nwin + 1) / 2;   // units per row
  // static row schedule (me, me + NG, ...): ticket rows as in spgemm_bm_rows_pipe measured
  // slower here (1M 55.8 vs 54.1 ms, 65536^2 1.86 vs 1.36 ms, PERF_LOG round 6)
  int id1 = me, id2 = me + NG, id3 = me + 2 * NG;
  auto next_row = [&]() { return id3 + NG; };

  // ---- row pipeline (as spgemm_bm_rows_pipe) --------------------------------
  auto arp2 = [&](int r, int& a, int& b) {   // (low words: nnz(A) < 2^31)
    const int rr = r < m ? r : m - 1;
    const int* lo = reinterpret_cast<const int*>(p.Arp);
    a = lo[2 * rr];
    b = lo[2 * rr + 2];
  };
  auto entry = [&](int a, int b) {
    const int a0 = __builtin_amdgcn_readfirstlane(a), na = __builtin_amdgcn_readfirstlane(b) - a0;
    const int e = a0 + (tid < na ? tid : 0);
    return e < annz ? e : annz - 1;
  };
  int a1 = 0, b1 = 0, a2 = 0, b2 = 0, a3 = 0, b3 = 0;
  arp2(id1, a1, b1);
  uint32_t jj1 = (uint32_t)p.Aci[entry(a1, b1)];
  uint4 wa1 = ra.ws8[2 * (int64_t)jj1];       // {., lengths of windows 0-1, 2-3, 4-5}
  uint4 wb1 = ra.ws8[2 * (int64_t)jj1 + 1];   // {lengths 6-7, ., first padded column, .}
  int na1 = __builtin_amdgcn_readfirstlane(b1 - a1);
  arp2(id2, a2, b2);
  uint32_t jj2 = (uint32_t)p.Aci[entry(a2, b2)];
  int na2 = b2 - a2;
  arp2(id3, a3, b3);
  // once per row, at the top of the row's last unit (after take_row took the
  // next row): the row after's bounds, the third row's A columns, the fourth
  // row's row pointers (as spgemm_bm_rows_pipe's row_block)
  auto row_block = [&](int next_id) {
    id1 = id2;
    id2 = id3;
    id3 = next_id;
    wa1 = ra.ws8[2 * (int64_t)jj2];
    wb1 = ra.ws8[2 * (int64_t)jj2 + 1];
    na1 = __builtin_amdgcn_readfirstlane(na2);
    jj2 = (uint32_t)p.Aci[entry(a3, b3)];
    na2 = b3 - a3;
    arp2(id3, a3, b3);
  };

  int cna = 0, cid = me;   // (cid: the staged row's id)
  uint32_t cl0 = 0, cl1 = 0, cl2 = 0, cl3 = 0;   // a unit's two 16-bit lengths: cl0 (shifted down per unit)
  uint32_t bq = 0;
  auto take_row = [&]() {
    cid = id1;
    cna = na1;
    bq = wb1.z;
    cl0 = wa1.y;
    cl1 = wa1.z;
    cl2 = wa1.w;
    cl3 = wb1.x;
  };

  // ---- the staged unit ------------------------------------------------------
  int su = 0, sq = 0, sTC = 0, snr = 0, sclo = 0, sP = 0;
  uint2 xb[RR][2];     // four columns per round (two 8-byte halves)
  uint32_t okb = 0;    // bit 4 d + i: column i of round d is in its segment
  // per-thread scan inputs of the next unit (computed in the OR phase)
  int nlen = 0, nch = 0;
  uint32_t nb0 = 0;
  auto next_inputs = [&]() {   // lengths of the next unit of the staged row (cl0), advance
    nlen = 0;
    nch = 0;
    if (tid < cna) {
      nlen = (int)(cl0 & 0xffffu) + (int)(cl0 >> 16);   // (lengths past nwin are packed as 0)
      nch = (nlen + Gc - 1) / Gc;
    }
    nb0 = bq;
    bq += (uint32_t)(((nlen + (1 << kPadCLg) - 1) >> kPadCLg) << kPadCLg);
    cl0 = cl1;
    cl1 = cl2;
    cl2 = cl3;
  };
  int pre = 0;
  // the scan's per-wave sums (before a barrier) ...
  auto scan_begin = [&]() {
    const int xa = bm_wave_incl(nch), xc = bm_wave_incl(nlen);
    if (lane == 63) {
      wscan[w] = xa;
      wscan[NW + w] = xc;
    }
    pre = xa - nch;
  };
  // ... and after it: totals, descriptors of the staged unit
  auto scan_end = [&](int u, int q0) {
    int qa = 0, ta = 0, tc = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int sa = wscan[i], sc = wscan[NW + i];
      qa += (i < w) ? sa : 0;
      ta += sa;
      tc += sc;
    }
    pre += qa;
    sTC = __builtin_amdgcn_readfirstlane(ta);
    sP = __builtin_amdgcn_readfirstlane(tc);
    su = u;
    sq = q0;
    sclo = q0 << LGW;
    snr = (sTC + ngrp - 1) / ngrp;
    for (int kk = 0; kk < nch; ++kk) {
      const int rem = nlen - kk * Gc;
      if (pre + kk < CCAP) desc[pre + kk] = make_uint2(nb0 + (uint32_t)(kk * Gc), (uint32_t)(rem < Gc ? rem : Gc));
    }
  };
  auto ld_round = [&](int d, int i0, int TC, uint2 (&x)[2], uint32_t& ok4) {   // chunk round i0 + d of this lane group
    const int t = gid + (i0 + d) * ngrp;
    const uint2 ds = desc[t < TC ? t : TC - 1];
    const int nv = (int)ds.y - 4 * gl;
    const bool ok = (t < TC) & (nv > 0);
    ok4 = ok ? ((nv >= 4) ? 15u : (1u << nv) - 1u) : 0u;
    const bm_v4u v = __builtin_amdgcn_raw_buffer_load_b128(rsb, (int)((ds.x + (ok ? (uint32_t)(4 * gl) : 0u)) * 4u), 0, 0);
    x[0] = make_uint2(v.x, v.y);
    x[1] = make_uint2(v.z, v.w);
  };
  auto issue_loads = [&]() {
    okb = 0;
    const int TC = sTC < CCAP ? sTC : CCAP;
#pragma unroll
    for (int d = 0; d < RR; ++d) {
      xb[d][0] = make_uint2(0u, 0u);
      xb[d][1] = make_uint2(0u, 0u);
      if (d < snr) {   // wave-uniform guard
        uint32_t ok4;
        ld_round(d, 0, TC, xb[d], ok4);
        okb |= ok4 << (4 * d);
      }
    }
  };
  auto or_cols = [&](const uint2 (&x)[2], uint32_t ok4, int clo) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if ((ok4 >> i) & 1u) {
        const int cc = (int)(i < 2 ? (i == 0 ? x[0].x : x[0].y) : (i == 2 ? x[1].x : x[1].y)) - clo;
        atomicOr(bm32 + (cc >> 5), 1u << (cc & 31));
      }
    }
  };

  // prologue: the first unit staged and its loads issued
  take_row();
  row_block(me + 3 * NG);
  next_inputs();
  scan_begin();
  __syncthreads();
  scan_end(me * nwin, 0);
  __syncthreads();
  issue_loads();
  // (one store per wave behind every unit's loads: the ucnt store; dropped here)
  __builtin_amdgcn_raw_buffer_store_b32(0u, rsu, -1, 0, 0);

  auto unit = [&](auto last_tag, int row, int g) {
    constexpr bool LAST = decltype(last_tag)::value;
    const int u = su, q0 = sq, TC = sTC, nr = snr, clo = sclo, P = sP;
    if constexpr (LAST) {   // the next row into the staging registers; the row inputs move along
      take_row();
      row_block(next_row());
    }
    // ---- ORs of unit k (its loads landed) --------------------------------
#pragma unroll
    for (int d = 0; d < RR; ++d) or_cols(xb[d], (okb >> (4 * d)) & 15u, clo);
    for (int i0 = RR; i0 < nr; ++i0) {   // rare: chunks past the register rounds, synchronously
      uint2 x[2];
      uint32_t ok4;
      ld_round(0, i0, TC < CCAP ? TC : CCAP, x, ok4);
      or_cols(x, ok4, clo);
    }
    // the next unit's scan inputs
    const bool more = !LAST || cid < m;
    next_inputs();
    scan_begin();
    __syncthreads();   // A: every OR of unit k done; the next scan's wave sums written
    BM_STAMP(5);
    if (more) scan_end(LAST ? cid * nwin : row * nwin + 2 * (g + 1), LAST ? 0 : 2 * (g + 1));
    __syncthreads();   // E: the next unit's descriptors written
    if (more) {
      SPMM_BM_PRIO_HI();
      issue_loads();
      SPMM_BM_PRIO_LO();
    }
    // ---- popcount of this wave's bitmap rows (unit k), clearing them ------
    int cnt = 0;
    if (P != 0) {   // uniform (an empty unit left the bitmap clean)
#pragma unroll
      for (int kk = 0; kk < WPT; ++kk) {
        const int wd = w * WPW + kk * 64 + lane;
        cnt += __popcll(bm[wd]);
        bm[wd] = 0ull;
      }
      cnt = __builtin_amdgcn_readlane(bm_wave_incl(cnt), 63);
    }
    if (lane == 0) csum[w] = cnt;
    // a unit of more chunks than the descriptor buffer (long two-window segments under a
    // 256-entry A row): its count is short -> err bit 6, the host recounts the product on
    // the per-unit kernels, which take descriptors in batches (a batch loop here changes
    // hipcc's schedule of the ORs above: every OR became its own branch)
    if (TC > CCAP && tid == 0) atomicOr(p.err, 64);
    __syncthreads();   // F: bitmap clear for the next ORs, csum written
    // ucnt of unit k's windows: one buffer store per wave (lanes past NSUB, other waves: dropped)
    int t = 0;
#pragma unroll
    for (int i = 0; i < WAVES_PER_WIN; ++i) t += csum[(lane & 1) * WAVES_PER_WIN + i];
    const bool wr = w == 0 && lane < NSUB && q0 + lane < nwin;
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)t, rsu, wr ? (u + lane) * 4 : -1, 0, 0);
    BM_STAMP(6);
  };
  for (int row = me; row < m; row = cid) {   // (cid: the next row, taken by the row's last unit)
    for (int g = 0; g + 1 < ngc; ++g) unit(std::false_type{}, row, g);
    unit(std::true_type{}, row, ngc - 1);
  }
  BM_STAMP_FLUSH();
}

// ---- configurations -------------------------------------------------------
// Every fast kernel: 256 threads and <= 40 KB of LDS, so four workgroups
// (16 waves, 128 VGPRs each) share a CU; count and reload kernels take most
// of a CU's LDS.
//   cfg 0: W = 2^17 (1M columns at ~105 nnz per row: ~1.4k products per window)
//          count 8 windows per unit (128 KB bitmap, 1024 threads)
//          fast  <= 2048 products, 12 register rounds
//   cfg 1: W = 2^15 (65536 columns at ~65 nnz per row: ~2.1k per window)
//          count 2 windows (8 KB, 512 threads); fast <= 3840 products, SPMM_BM_CFG1_R (14) rounds
//   cfg 2: W = 2^16: count 4 windows (32 KB, 1024 threads); fast <= 3072, 16 rounds
// Reload (deferred units): min(1024, W / 64) threads, <= 12288 products, 2048 chunks.
// (A W = 2^18 configuration with a 512-thread row kernel -- longer, better
// aligned segments -- measured 82 vs 76 ms on the 1M step and was removed:
// its units are latency-bound at 2 workgroups per CU, PERF_LOG round 4.)
// Wider windows mean longer contiguous B segments per (A entry, unit): random
// segment gathers run at ~7 TB/s of 128-byte LINES, so 100-byte segments
// deliver ~3.2 TB/s of useful bytes and 200-byte ones ~4.4
// (tools/probes/seg_gather.hip, profiles/r4/seg_gather.md).
struct BmCfg {
  int lgw, nsub_count, pcap_fast, rounds_fast, rows_nt, rows_r;
};
#ifndef SPMM_BM_CFG1_R   // register rounds of cfg 1's per-unit fast kernel (the 65536^2 config)
#define SPMM_BM_CFG1_R 14   // 65536^2: 16 rounds spill 5 VGPRs; 14 = 1.64 -> 1.56 ms (384 of 131072 units deferred), 13: 1.61-1.67, 12: 1.82
#endif
// cfg 1's pipelined row kernel (65536^2): the per-unit kernel's 14 rounds, so its units fit as
// they did there (at 10 rounds 74k of 131k units were deferred: 3.45 ms a step); 14 rounds and
// four 4096-entry write-out rounds need 158 VGPRs, so 3 waves per SIMD (at 4: 49 spill ops).
// 65536^2 step 1.202-1.205 vs 1.250-1.253 ms on the per-unit kernel (12 rounds: 1.56; r6g27;
// 512 threads at 8 / 10 rounds, 4 waves per SIMD: 1.40 / 1.46, r6g35)
#ifndef SPMM_BM_CFG1_ROWS_R
#define SPMM_BM_CFG1_ROWS_R 14
#endif
#ifndef SPMM_BM_CFG1_ROWS_WPE
#define SPMM_BM_CFG1_ROWS_WPE 3
#endif
constexpr BmCfg kCfgs[] = {{17, 8, 2048, 12, 256, SPMM_BM_ROWS_R},
                           {15, 2, 3840, SPMM_BM_CFG1_R, 256, SPMM_BM_CFG1_ROWS_R},
                           {16, 4, 3072, 16, 256, SPMM_BM_ROWS_R}};
constexpr int kNumCfgs = 3;
constexpr int kFastNT = 256, kReloadCcap = 2048;
// reload product slots: 96 KB of items
constexpr int reload_pcap(int) { return 12288; }
// reload workgroup: up to 1024 threads (the longest A row it can stage), at
// most one wave per 64 bitmap words
constexpr int reload_nt(int lgw) { return ((1 << lgw) / 64) < 1024 ? ((1 << lgw) / 64) : 1024; }

template <int C>
struct BmKernels {
  static constexpr BmCfg K = kCfgs[C];
  static constexpr int kCountNT = (K.nsub_count << K.lgw) >= (1 << 19) ? 1024 : 512;
  static constexpr auto count = spgemm_bm<K.lgw, K.nsub_count, kCountNT, 2, 1, 2048, 0>;
  static constexpr auto fast = spgemm_bm<K.lgw, 1, kFastNT, K.pcap_fast, K.rounds_fast,
                                         K.rounds_fast * (kFastNT / 16), 1>;
  // the wide kernel reads two padded pairs per lane: it exists only for an even
  // round count; otherwise bm_numeric takes the plain kernel (B read through
  // ws / Bci / Bv, never the padded pair array at unpadded offsets)
  static constexpr bool kWide = K.rounds_fast % 2 == 0;
  static constexpr auto fast_wide = spgemm_bm<K.lgw, 1, kFastNT, K.pcap_fast, K.rounds_fast,
                                              K.rounds_fast * (kFastNT / 16), 1, false, kWide, kWide>;
  static constexpr int kReloadNT = reload_nt(K.lgw);
  static constexpr auto reload = spgemm_bm<K.lgw, 1, kReloadNT, reload_pcap(K.lgw), 8, kReloadCcap, 2>;
  // the reload kernel on the padded pairs (two a lane; the row numeric kernel's deferred
  // units): reads B only through ws8 + the pairs, so B's plain arrays need not exist
  static constexpr auto reload_wide = spgemm_bm<K.lgw, 1, kReloadNT, reload_pcap(K.lgw), 8, kReloadCcap, 2, false, true,
                                                true>;
  static constexpr auto fast_det = spgemm_bm<K.lgw, 1, kFastNT, K.pcap_fast, K.rounds_fast,
                                             K.rounds_fast * (kFastNT / 16), 1, true>;
  static constexpr auto reload_det = spgemm_bm<K.lgw, 1, kReloadNT, reload_pcap(K.lgw), 8, kReloadCcap, 2, true>;
};

template <typename K>
int launch_bm(K kernel, int nt, int64_t work, const BmArgs& a, hipStream_t s) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (int)hipErrorInvalidDevice;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, nt, 0) != hipSuccess || per <= 0) per = 1;
  int64_t g = (int64_t)per * ncu;
  if (work < g) g = work < 1 ? 1 : work;
  hipLaunchKernelGGL(kernel, dim3((unsigned)g), dim3(nt), 0, s, a);
  SPMM_LAUNCH_CHECK();
  return 0;
}

template <int C>
int bm_count(int64_t work, const BmArgs& a, hipStream_t s) {
  return launch_bm(BmKernels<C>::count, BmKernels<C>::kCountNT, work, a, s);
}

// row-major fast kernel of configuration C (same geometry as its fast kernel)
template <int C>
struct BmRowKernel {
  static constexpr BmCfg K = kCfgs[C];
  static constexpr int NT = K.rows_nt;
  // register rounds (the row pipeline's registers cost rounds)
  static constexpr int R = K.rounds_fast > K.rows_r ? K.rows_r : K.rounds_fast;
  static constexpr int RP = R & ~1;   // the pipelined kernel loads two pairs per lane and round
  static constexpr auto kpipe = spgemm_bm_rows_pipe<K.lgw, NT, K.pcap_fast, RP, RP * (NT / 16), C == 1 ? SPMM_BM_CFG1_ROWS_WPE : 4>;
};


template <typename Kern, typename Args>
int launch_rows(Kern kernel, const Args& args, int64_t m, hipStream_t s, int nt = kFastNT) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (int)hipErrorInvalidDevice;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, nt, 0) != hipSuccess || per <= 0) per = 1;
  int64_t g = (int64_t)per * ncu;
  if (m < g) g = m;
  hipLaunchKernelGGL(kernel, dim3((unsigned)g), dim3(nt), 0, s, args);
  SPMM_LAUNCH_CHECK();
  return 0;
}
template <typename Kern>
int launch_rows(Kern kernel, const BmRowArgs& ra, hipStream_t s, int nt = kFastNT) {
  return launch_rows(kernel, ra, ra.a.m, s, nt);
}
// a grid of exactly g workgroups (chunked schedules)
template <typename Kern>
int launch_rows_grid(Kern kernel, const BmRowArgs& ra, int64_t g, hipStream_t s, int nt) {
  if (g < 1 || g > (int64_t)INT32_MAX) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kernel, dim3((unsigned)g), dim3(nt), 0, s, ra);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// count: one window (16 KB at W = 2^17, 8 workgroups per CU) or two windows
// per unit (32 KB, 4 per CU: a B row's column segment read once for both)
#ifndef SPMM_BM_COUNT_RR   // B loads in flight per thread (diagnostic builds: tools/bm_variants.py)
#define SPMM_BM_COUNT_RR 8
#endif
#ifndef SPMM_BM_COUNT_NT   // threads per count workgroup (the host gates A rows <= this)
#define SPMM_BM_COUNT_NT 256
#endif
// workgroup size by bitmap bytes: 32 KB -> 256 threads (4 per CU), 64 KB -> 512 (2 per CU)
constexpr int count_nt(int lgw, int nsub) {
  return ((nsub << lgw) / 8) > (64 << 10) ? 1024 : ((nsub << lgw) / 8) > (32 << 10) ? 512 : SPMM_BM_COUNT_NT;
}
template <int C, int NSUB>
struct BmRowCountKernel {
  static constexpr int NT = count_nt(kCfgs[C].lgw, NSUB);
  static constexpr auto k = spgemm_bm_rows_count<kCfgs[C].lgw, NSUB, NT, SPMM_BM_COUNT_RR, 256, false>;
  static constexpr auto kp = spgemm_bm_rows_count<kCfgs[C].lgw, NSUB, NT, SPMM_BM_COUNT_RR / 2, 256, true>;
};
// pipelined (two-window units, padded columns; 32 KB bitmap + 6 KB descriptors: 4 workgroups per CU)
template <int C>
struct BmRowCountPipe {
  static constexpr int NT = 256;
  static constexpr auto k = spgemm_bm_rows_count_pipe<kCfgs[C].lgw, NT, SPMM_BM_COUNT_RR / 2, 768>;
};

#ifndef SPMM_BM_ROWCOUNT_CHUNK   // flat row count kernel: rows a workgroup (0: persistent grid)
#define SPMM_BM_ROWCOUNT_CHUNK 4
#endif

template <int C>
int bm_count_rows(BmRowArgs ra, int nsub, int pipe, int64_t annz, hipStream_t s) {
  using K1 = BmRowCountKernel<C, 1>;
  using K2 = BmRowCountKernel<C, 2>;
  const int64_t colp_bytes = ra.a.cap * 4;
  // (pipelined from two units per row up: with one, every unit is a row's last and the
  // pipeline only adds work -- 65536^2 count 1.32 -> 1.36 ms step, PERF_LOG round 5)
  if (ra.pad && pipe && nsub == 2 && ra.a.nwin >= 3 && K2::NT == BmRowCountPipe<C>::NT && annz > 0 &&
      colp_bytes < (int64_t(1) << 32) && ra.a.m * ra.a.nwin < (int64_t(1) << 30))
    return launch_rows(BmRowCountPipe<C>::k, BmCountPipeArgs{ra, (uint32_t)colp_bytes, annz}, ra.a.m, s,
                       BmRowCountPipe<C>::NT);
  constexpr int CR = SPMM_BM_ROWCOUNT_CHUNK;
  if (CR > 0) {   // chunked grid: CR rows a workgroup (spgemm_bm_rows_count)
    ra.a.chunk = CR;
    const int64_t g = (ra.a.m + CR - 1) / CR;
    if (ra.pad)
      return nsub == 2 ? launch_rows_grid(K2::kp, ra, g, s, K2::NT) : launch_rows_grid(K1::kp, ra, g, s, K1::NT);
    return nsub == 2 ? launch_rows_grid(K2::k, ra, g, s, K2::NT) : launch_rows_grid(K1::k, ra, g, s, K1::NT);
  }
  if (ra.pad)
    return nsub == 2 ? launch_rows(K2::kp, ra, s, K2::NT) : launch_rows(K1::kp, ra, s, K1::NT);
  return nsub == 2 ? launch_rows(K2::k, ra, s, K2::NT) : launch_rows(K1::k, ra, s, K1::NT);
}

// The pipelined row numeric kernel (2 pairs per lane and 16-byte loads on the
// padded pairs, 32-bit buffer offsets), then the reload kernel over the
// deferred units; same conditions as the planner's `rows`.
template <int C>
int bm_numeric_rows(BmRowArgs ra, int det, int64_t nbcv, int pipe, int64_t annz, hipStream_t s) {
  using K = BmRowKernel<C>;
  if (!(ra.a.Bcv && ra.pad && ra.a.lg >= 1 && !det && pipe && annz > 0 && nbcv > 0 && nbcv * 8 < (int64_t(1) << 32)))
    return (int)hipErrorInvalidValue;
  const int rc = launch_rows(K::kpipe, BmPipeArgs{ra, (uint32_t)(nbcv * 8), annz, ra.a.err + 2}, ra.a.m, s, K::NT);
  if (rc) return rc;
  BmArgs ar = ra.a;   // (the padded pairs and their bounds: ws8)
  ar.ws8 = ra.ws8;
  return launch_bm(BmKernels<C>::reload_wide, BmKernels<C>::kReloadNT, int64_t(1) << 30, ar, s);
}

#ifndef SPMM_BM_UNIT_CHUNK   // per-unit fast numeric: units a workgroup (0: persistent grid)
#define SPMM_BM_UNIT_CHUNK 8
#endif

// the fast numeric kernel on a grid of `chunk`-unit workgroups (see spgemm_bm's unit schedule)
template <typename K>
int launch_bm_chunked(K kernel, int nt, int64_t work, BmArgs a, int chunk, hipStream_t s) {
  const int64_t g = (work + chunk - 1) / chunk;
  if (g > (int64_t)INT32_MAX) return (int)hipErrorInvalidValue;
  a.chunk = chunk;
  hipLaunchKernelGGL(kernel, dim3((unsigned)(g < 1 ? 1 : g)), dim3(nt), 0, s, a);
  SPMM_LAUNCH_CHECK();
  return 0;
}

template <int C>
int bm_numeric(int64_t work, const BmArgs& a, int det, hipStream_t s) {
  using K = BmKernels<C>;
  const bool wide = K::kWide && a.ws8 != nullptr && a.Bcv != nullptr && a.lg >= 1;   // padded pairs given
  constexpr int CH = SPMM_BM_UNIT_CHUNK;
  const int rc = det ? launch_bm(K::fast_det, kFastNT, work, a, s)
               : CH > 0 ? (wide ? launch_bm_chunked(K::fast_wide, kFastNT, work, a, CH, s)
                                : launch_bm_chunked(K::fast, kFastNT, work, a, CH, s))
                        : (wide ? launch_bm(K::fast_wide, kFastNT, work, a, s) : launch_bm(K::fast, kFastNT, work, a, s));
  if (rc) return rc;
  return det ? launch_bm(K::reload_det, K::kReloadNT, int64_t(1) << 30, a, s)
             : launch_bm(K::reload, K::kReloadNT, int64_t(1) << 30, a, s);
}


}  // namespace

// Host planning: window log2, windows per count unit, fast-kernel product
// capacity and register rounds of configuration cfg, and the longest A row
// the reload kernel can stage.
SPMM_EXPORT int spmm_spgemm_bm_config(int cfg, int* lgw, int* nsub_count, int* pcap_fast, int* rounds_fast,
                                      int* reload_rows) {
  if (cfg < 0 || cfg >= kNumCfgs) return (int)hipErrorInvalidValue;
  *reload_rows = reload_nt(kCfgs[cfg].lgw);
  *lgw = kCfgs[cfg].lgw;
  *nsub_count = kCfgs[cfg].nsub_count;
  *pcap_fast = kCfgs[cfg].pcap_fast;
  *rounds_fast = kCfgs[cfg].rounds_fast;
  return 0;
}

// Count kernel: ucnt[m * nwin] = exact nnz of every (row, window) unit.
SPMM_EXPORT int spmm_spgemm_bm_count(int cfg, const int64_t* Arp, const int32_t* Aci, const uint32_t* ws,
                                     const int32_t* Bci, int64_t m, int nwin, int lg, int32_t* ucnt, int32_t* err,
                                     void* stream) {
  if (m <= 0) return 0;
  if (lg < 4 || lg > 6 || cfg < 0 || cfg >= kNumCfgs || nwin < 1) return (int)hipErrorInvalidValue;
  BmArgs a{Arp, Aci, nullptr, ws, Bci, nullptr, m, nwin, lg, ucnt, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0,
           nullptr, err};
  hipStream_t s = (hipStream_t)stream;
  const int64_t work = m * ((nwin + kCfgs[cfg].nsub_count - 1) / kCfgs[cfg].nsub_count);
  switch (cfg) {
    case 0: return bm_count<0>(work, a, s);
    case 1: return bm_count<1>(work, a, s);
    default: return bm_count<2>(work, a, s);
  }
}

// Numeric: the fast kernel over every unit, then the reload kernel over the
// units it deferred (novf must be zero; ovf has room for ovf_cap units).
// det: fixed summation order (see "deterministic mode"); err bit 4 then
// means a unit needs the CPU engine.
SPMM_EXPORT int spmm_spgemm_bm_numeric(int cfg, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                       const uint32_t* ws, const int32_t* Bci, const float* Bv, int64_t m, int nwin,
                                       int lg, const int64_t* uoff, int64_t cap, int32_t* Cci, float* Cv,
                                       int32_t* ovf, uint32_t* novf, int64_t ovf_cap, int32_t* err, int det,
                                       const void* ws8, const void* bcv_padded, void* stream) {
  if (m <= 0) return 0;
  if (lg < 4 || lg > 6 || cfg < 0 || cfg >= kNumCfgs || nwin < 1) return (int)hipErrorInvalidValue;
  if ((ws8 != nullptr) != (bcv_padded != nullptr) || (ws8 != nullptr && nwin > 8)) return (int)hipErrorInvalidValue;
  BmArgs a{Arp, Aci, Av, ws, Bci, Bv, m, nwin, lg, nullptr, uoff, Cci, Cv, ovf, novf, ovf_cap, cap,
           (const uint2*)bcv_padded, err, (const uint4*)ws8};
  hipStream_t s = (hipStream_t)stream;
  const int64_t work = m * nwin;
  switch (cfg) {
    case 0: return bm_numeric<0>(work, a, det, s);
    case 1: return bm_numeric<1>(work, a, det, s);
    default: return bm_numeric<2>(work, a, det, s);
  }
}

// Diagnostics: on >= 0 resets the stamp accumulators and enables (1) or
// disables (0) them; on < 0 synchronises and reads the eight accumulators:
// numeric [0] staging [1] pass 1 [2] rank scan [3] pass 2 [4] write-out,
// count [5] staging + ORs [6] popcount + clear, [7] numeric units.
SPMM_EXPORT int spmm_spgemm_bm_stamps(int on, unsigned long long* out8) {
  if (on >= 0) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_bm_stamps), z, sizeof z);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_bm_stamp_on), &on, sizeof on);
    return (int)e;
  }
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_bm_stamps), 8 * sizeof(unsigned long long));
  return (int)e;
}

// Diagnostics (stamps build): per-workgroup {start, end, xcd << 32 | units} of the last
// pipelined numeric launch, n <= kBmWgMax workgroups; on = 1 clears them first.
SPMM_EXPORT int spmm_spgemm_bm_wg_times(int on, unsigned long long* out, int n) {
  if (n < 0 || n > kBmWgMax) return (int)hipErrorInvalidValue;
  if (on) {
    static unsigned long long z[3 * kBmWgMax];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_bm_wg), z, sizeof z);
  }
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bm_wg), 3 * (size_t)n * sizeof(unsigned long long));
  return (int)e;
}

// Row-major numeric (nwin <= 8, ws8 from spmm_spgemm_bm_pack_ws8), then the
// reload kernel over the deferred units; same contract as spmm_spgemm_bm_numeric.
// Bcv: optional [nnz(B)] (column, value bits) pairs read by the row-major kernel.
// nbcv: pairs in Bcv; pipe: the software-pipelined kernel (padded pairs, unordered
// sum, nbcv * 8 < 2^32, annz = nnz(A) > 0; err then int32[4]: err[2] is its row-ticket
// counter, zero at launch), else the flat one.
SPMM_EXPORT int spmm_spgemm_bm_numeric_rows(int cfg, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                            const void* ws8, const uint32_t* ws, const int32_t* Bci, const float* Bv,
                                            const void* Bcv,
                                            int64_t m, int nwin, int lg, const int64_t* uoff, int64_t cap,
                                            int32_t* Cci, float* Cv, int32_t* ovf, uint32_t* novf, int64_t ovf_cap,
                                            int32_t* err, int det, int pad, int64_t nbcv, int pipe, int64_t annz,
                                            void* stream) {
  if (m <= 0) return 0;
  if (lg < 4 || lg > 6 || cfg < 0 || cfg >= kNumCfgs || nwin < 1 || nwin > 8) return (int)hipErrorInvalidValue;
  if (pad && !Bcv) return (int)hipErrorInvalidValue;
  BmRowArgs ra{BmArgs{Arp, Aci, Av, ws, Bci, Bv, m, nwin, lg, nullptr, uoff, Cci, Cv, ovf, novf, ovf_cap, cap,
                      (const uint2*)Bcv, err},
               (const uint4*)ws8, pad ? 1 : 0};
  hipStream_t s = (hipStream_t)stream;
  switch (cfg) {
    case 0: return bm_numeric_rows<0>(ra, det, nbcv, pipe, annz, s);
    case 1: return bm_numeric_rows<1>(ra, det, nbcv, pipe, annz, s);
    default: return bm_numeric_rows<2>(ra, det, nbcv, pipe, annz, s);
  }
}

// Row-major count (nwin <= 8, every A row <= 256 entries, ws8 packed): same
// output as spmm_spgemm_bm_count.  Returns without counting when err bit 3
// is set (ws8 lengths truncated); the host then uses spmm_spgemm_bm_count.
// pad: Bci is the padded column array of spmm_spgemm_bm_pad_pairs (gc = nsub).
// pipe: the pipelined kernel (pad, nsub 2, nnzb * 4 < 2^32, annz = nnz(A) > 0; err then
// int32[4]).
SPMM_EXPORT int spmm_spgemm_bm_count_rows(int cfg, const int64_t* Arp, const int32_t* Aci, const void* ws8,
                                          const int32_t* Bci, int64_t m, int nwin, int lg, int nsub, int32_t* ucnt,
                                          int32_t* err, int64_t nnzb, int pad, int pipe, int64_t annz, void* stream) {
  if (m <= 0) return 0;
  if (lg < 4 || lg > 6 || cfg < 0 || cfg >= kNumCfgs || nwin < 1 || nwin > 8) return (int)hipErrorInvalidValue;
  BmRowArgs ra{BmArgs{Arp, Aci, nullptr, nullptr, Bci, nullptr, m, nwin, lg, ucnt, nullptr, nullptr, nullptr, nullptr,
                      nullptr, 0, nnzb, nullptr, err},
               (const uint4*)ws8, pad ? 1 : 0};
  hipStream_t s = (hipStream_t)stream;
  if (nsub != 1 && nsub != 2) return (int)hipErrorInvalidValue;
  switch (cfg) {
    case 0: return bm_count_rows<0>(ra, nsub, pipe, annz, s);
    case 1: return bm_count_rows<1>(ra, nsub, pipe, annz, s);
    default: return bm_count_rows<2>(ra, nsub, pipe, annz, s);
  }
}
