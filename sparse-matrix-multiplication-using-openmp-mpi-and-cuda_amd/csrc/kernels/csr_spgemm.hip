// CSR x CSR SpGEMM (fp32) for gfx950: row-binned accumulation in LDS.
//
// North-star engine (BASELINE.json configs 2, 4, 5).  The reference has no CSR
// path at all; its tile-level analogue is the host join + per-tile kernel of
// sparse_matrix_mult.cu:140-253.
//
// Gustavson row by row.  Rows are binned by their intermediate-product count;
// each bin gets a kernel instantiation sized for it (every LDS footprint
// <= 80 KB so two 512-thread workgroups share a CU):
//   symbolic (exact nnz per row, two-phase mode): CAS-probing hash tables of
//            128 .. 16384 keys, long rows over 1/2/4/8 column slices
//   numeric  short rows: ordered linear probing (sorted table, output is a
//            compaction); long rows: bucketed ESC (histogram, scatter, per-
//            bucket register sort + fold, compaction) over 1/2/4/8 slices
//   longest  rows (R-MAT hubs, > 8 ESC slices): column-chunked dense
//            accumulation through an HBM scratch ("long rows" below)
// Both LDS schemes use a MONOTONE hash / bucket function of the column,
// h(c) = floor((c - c_lo) * S / width), so slot order is column order and
// rows come out sorted without a sort pass.
// One-pass mode (ops/spgemm.py) skips the symbolic phase: numeric writes at
// product-count offsets and spgemm_compact packs the result.
#include "common.hpp"

namespace {

constexpr int EMPTY = -1;

// Diagnostic phase stamps (off unless the host sets g_stamp_on): thread 0 of
// every workgroup adds the shader-clock cycles of each phase, measured between
// the workgroup barriers that delimit it.  Read with spmm_spgemm_stamps().
__device__ int g_stamp_on = 0;
__device__ unsigned long long g_stamps[8];
// Diagnostic only (never set by the library): the ordered ESC publishes its
// prefix without waiting for predecessors (wrong offsets) — an upper bound on
// what any look-back redesign could gain.  tools/lookback_bound.py.
__device__ int g_nowait = 0;
#define SPMM_STAMP(i)                                                              \
  do {                                                                             \
    if (stamp_on && threadIdx.x == 0) {                                            \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();                  \
      atomicAdd(&g_stamps[i], _t - t_prev);                                        \
      t_prev = _t;                                                                 \
    }                                                                              \
  } while (0)

// Block-wide exclusive scan (+ total); ends with the block synchronised and
// wsum still live: a second scan needs a barrier before it reuses wsum.
template <int NT, typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* wsum, T* total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    T s = wsum[i];
    pre += (i < w) ? s : 0;
    tot += s;
  }
  *total = tot;
  return pre + x - v;
}

__device__ __forceinline__ uint32_t hash_mult(int64_t S, int ncols) {
  return (S >= ncols) ? 0u : (uint32_t)(((uint64_t)S << 32) / (uint64_t)ncols);
}
__device__ __forceinline__ int hash_home(int c, uint32_t mult) {
  return mult ? (int)__umulhi((uint32_t)c, mult) : c;
}

// ---------------------------------------------------------------------------
// LDS-resident tables.  S = hash range, TS = S + NT slots (the overflow tail
// lets probes run forward without wrapping).
//
// Product stream (both phases): the row's A entries (<= NT per batch) are
// staged in LDS (B-row segment start, A value) and cut into chunks of
// G = 1 << lg products (16, 32 or 64, chosen by the host from the mean B-row
// segment length).  A block scan lays the chunk descriptors (entry, chunk
// index, valid lanes) out in LDS; lanes form groups of G and group g takes
// chunks g, g + #groups, ... so a lane's product is b0 + G*k + lane: no
// per-product search, coalesced B reads, a wave-uniform trip count.  D chunks
// per lane are fetched per batch and the next batch's loads are in flight
// while the current one is inserted (register double buffer; loads are never
// predicated off, so the compiler keeps counted vmcnt waits).
//
// Symbolic: 32-bit keys, CAS-only linear probing in rounds (a CAS of
// EMPTY -> key both claims a free slot and reports the occupant); every lane
// issues all of its CASes of a round before looking at any result.
//
// Numeric: ORDERED linear probing over 64-bit slots (key | value bits).  An
// insert walks forward from its home slot; at an occupant with a larger key it
// swaps itself in (one 64-bit CAS) and carries the displaced pair onward, at
// an equal key it adds its value (CAS), at a smaller key it moves on.  With
// the monotone hash every cluster stays sorted and clusters are ordered, so
// the table read in slot order IS the sorted row: the output position is just
// the number of occupied slots before the slot (ballot + mbcnt + one block
// scan over 64-slot windows).  A cheap adjacency check (DPP) flags any row
// whose slots are not increasing (only possible after a wrap-around), and the
// host re-sorts those rows.

// Smallest lg >= 4 whose worst-case chunk count fits the descriptor buffer
// (chunks <= products / G + entries and products <= TS are both enforced).
constexpr int lds_lg_min(int TS, int NT, int CCAP) {
  int lg = 4;
  while (lg < 6 && ((TS + (1 << lg) - 1) >> lg) + NT > CCAP) ++lg;
  return lg;
}

template <int S, int NT>
struct LdsGeom {
  static constexpr int TS = S + NT;        // multiple of 64
  static constexpr int NW = NT / 64;
  static constexpr int ACAP = NT;          // A entries per batch
  static constexpr int CCAP = (S / NT >= 32) ? 3 * NT : 2 * NT;   // chunk descriptors per batch
  static constexpr int LG_MIN = lds_lg_min(TS, NT, CCAP);
  static constexpr int NWIN = TS / 64;
  static_assert(((TS + 63) >> 6) + NT <= CCAP, "descriptor buffer too small even for 64-lane chunks");
  static_assert(NWIN <= CCAP, "window counts reuse the descriptor buffer");
  static_assert(NT <= 1024, "entry index is 10 bits in a chunk descriptor");
};

// Chunk count of this thread's entry and one block scan giving the chunk
// offsets (low word) and the product total (high word).
template <int NT>
__device__ __forceinline__ void scan_chunks(int len, int lgE, int64_t* wsum, int& nch, int& pre, int& TC,
                                            int64_t& tot) {
  nch = (len + (1 << lgE) - 1) >> lgE;
  int64_t both;
  const int64_t pk = block_excl_scan<NT, int64_t>(((int64_t)len << 32) | nch, wsum, &both);
  pre = (int)(pk & 0xffffffff);
  TC = (int)(both & 0xffffffff);
  tot = (int64_t)((uint64_t)both >> 32);
}

// Stage one batch of A entries of a row slice: B-row segment starts (abeg) and
// A values (aval) in LDS, one block scan for the chunk offsets and the product
// total.  Ends synchronised.  The caller checks the capacities, then calls
// write_chunks().
template <int NT, int NP, bool VALUES>
__device__ __forceinline__ void stage_batch(const int32_t* __restrict__ Aci, const float* __restrict__ Av,
                                            const int64_t* __restrict__ Brp, const int64_t* __restrict__ bsplit,
                                            int64_t abase, int nb, int q0, int q1, int lgE, int64_t* abeg,
                                            float* aval, int64_t* wsum, int& len, int& nch, int& pre, int& TC,
                                            int64_t& tot) {
  const int tid = threadIdx.x;
  len = 0;
  if (tid < nb) {
    const int j = Aci[abase + tid];
    const int64_t rb = Brp[j], re = Brp[j + 1];
    const int64_t b0 = (NP == 1 || q0 == 0) ? rb : bsplit[(int64_t)j * 7 + q0 - 1];
    const int64_t b1 = (NP == 1 || q1 == 8) ? re : bsplit[(int64_t)j * 7 + q1 - 1];
    len = (int)(b1 - b0);
    abeg[tid] = b0;
    if constexpr (VALUES) aval[tid] = Av[abase + tid];
  }
  scan_chunks<NT>(len, lgE, wsum, nch, pre, TC, tot);
}


// A chunk descriptor: entry index (bits 0-9: workgroups of up to 1024 threads), lanes
// (10-16), chunk of the entry (17-30).
__device__ __forceinline__ void write_chunks(int* clist, int len, int nch, int pre, int lgE) {
  const int G = 1 << lgE;
  for (int k = 0; k < nch; ++k) {
    const int lim = (len - (k << lgE)) < G ? (len - (k << lgE)) : G;
    clist[pre + k] = threadIdx.x | (lim << 10) | (k << 17);
  }
}

// Chunk round i of a lane group = descriptor gid + i * ngrp.  Fills D products
// per lane: column, B value, A value, valid flag.
template <int D, bool VALUES>
__device__ __forceinline__ void fetch_chunks(int i0, int gid, int ngrp, int gl, int lgE, int TC, const int* clist,
                                             const int64_t* abeg, const float* aval, const int32_t* __restrict__ Bci,
                                             const float* __restrict__ Bv, int (&c)[D], float (&bv)[D],
                                             float (&av)[D], bool (&v)[D]) {
  int d[D], t[D];
#pragma unroll
  for (int u = 0; u < D; ++u) {
    t[u] = gid + (i0 + u) * ngrp;
    d[u] = clist[t[u] < TC ? t[u] : TC - 1];   // clamped: every LDS read issues, one wait
  }
  int64_t eb[D];
#pragma unroll
  for (int u = 0; u < D; ++u) {
    eb[u] = abeg[d[u] & 1023];
    if constexpr (VALUES) av[u] = aval[d[u] & 1023];
  }
  int64_t f[D];
#pragma unroll
  for (int u = 0; u < D; ++u) {
    const int lim = (d[u] >> 10) & 127, k = d[u] >> 17;
    v[u] = (t[u] < TC) & (gl < lim);
    f[u] = v[u] ? eb[u] + (k << lgE) + gl : 0;   // 0: a valid B index (TC > 0); loads never predicated off
  }
#pragma unroll
  for (int u = 0; u < D; ++u) {
    c[u] = Bci[f[u]];
    if constexpr (VALUES) bv[u] = Bv[f[u]];
  }
}

// ------------------------------------------------------------- symbolic ----
template <int S, int NT, int NP>
__global__ __launch_bounds__(NT, 4) void spgemm_lds_sym(
    const int64_t* __restrict__ Arp, const int32_t* __restrict__ Aci, const int64_t* __restrict__ Brp,
    const int32_t* __restrict__ Bci, const int64_t* __restrict__ bsplit, const int32_t* __restrict__ rows,
    int ncols, int lg, int32_t* __restrict__ row_nnz, int32_t* __restrict__ flags) {
  using Gm = LdsGeom<S, NT>;
  constexpr int TS = Gm::TS, NW = Gm::NW, ACAP = Gm::ACAP, CCAP = Gm::CCAP;
  constexpr int QSTEP = 8 / NP;
  constexpr int D = (S >= 16384) ? 8 : 4;   // deeper where LDS caps occupancy anyway
  __shared__ __attribute__((aligned(16))) int keys[TS];
  __shared__ int64_t abeg[ACAP];
  __shared__ int clist[CCAP];
  __shared__ int64_t wsum[NW];
  __shared__ int s_count;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform
  const int row = rows[blockIdx.x];
  const int64_t a0 = Arp[row], na = Arp[row + 1] - a0;
  const int lgE = lg > Gm::LG_MIN ? lg : Gm::LG_MIN;
  const int ngrp = NW << (6 - lgE);                         // lane groups in the workgroup
  const int gid = (w << (6 - lgE)) + (lane >> lgE);
  const int gl = lane & ((1 << lgE) - 1);
  const int stamp_on = g_stamp_on;
  unsigned long long t_prev = stamp_on ? __builtin_amdgcn_s_memtime() : 0ull;
  int row_count = 0;

  for (int sl = 0; sl < NP; ++sl) {
    const int q0 = sl * QSTEP, q1 = q0 + QSTEP;
    const int clo = (int)(((int64_t)q0 * ncols) >> 3), chi = (int)(((int64_t)q1 * ncols) >> 3);
    const uint32_t mult = hash_mult(S, chi - clo);
    for (int i = tid; i < TS / 4; i += NT) reinterpret_cast<int4*>(keys)[i] = make_int4(EMPTY, EMPTY, EMPTY, EMPTY);
    if (tid == 0) s_count = 0;
    int mine = 0;
    int64_t slice_products = 0;
    bool overflow = false;
    for (int64_t bat = 0; bat < na; bat += ACAP) {
      const int nb = (int)((na - bat) < ACAP ? (na - bat) : ACAP);
      __syncthreads();  // init done / previous batch consumed
      int len, nch, pre, TC;
      int64_t tot;
      stage_batch<NT, NP, false>(Aci, nullptr, Brp, bsplit, a0 + bat, nb, q0, q1, lgE, abeg, nullptr, wsum, len,
                                 nch, pre, TC, tot);
      SPMM_STAMP(0);
      // distinct keys <= products: a slice that could overfill the table goes to the HBM path
      slice_products += tot;
      if (slice_products > TS - 8 || TC > CCAP) { overflow = true; break; }
      if (TC == 0) continue;
      write_chunks(clist, len, nch, pre, lgE);
      __syncthreads();

      int cA[D], cB[D];
      float dummy[D];
      bool vA[D], vB[D];
      auto consume = [&](const int (&c)[D], const bool (&v)[D]) {
        int h[D];
        bool st[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
          h[u] = hash_home(c[u] - clo, mult);
          st[u] = v[u];
        }
        while (true) {
          int old[D];
#pragma unroll
          for (int u = 0; u < D; ++u) old[u] = st[u] ? atomicCAS(&keys[h[u]], EMPTY, c[u]) : c[u];
          bool more = false;
#pragma unroll
          for (int u = 0; u < D; ++u) {
            mine += (st[u] & (old[u] == EMPTY)) ? 1 : 0;
            const bool again = st[u] & (old[u] != EMPTY) & (old[u] != c[u]);
            h[u] += again ? 1 : 0;
            if (again && h[u] >= TS) h[u] = 0;   // wrap: only counts matter here
            st[u] = again;
            more |= again;
          }
          if (!__any(more)) break;
        }
      };
      const int nit = (TC + ngrp - 1) / ngrp;   // chunk rounds of the busiest group (wave-uniform)
      fetch_chunks<D, false>(0, gid, ngrp, gl, lgE, TC, clist, abeg, nullptr, Bci, nullptr, cA, dummy, dummy, vA);
      for (int i = 0; i < nit; i += 2 * D) {
        fetch_chunks<D, false>(i + D, gid, ngrp, gl, lgE, TC, clist, abeg, nullptr, Bci, nullptr, cB, dummy, dummy,
                               vB);
        consume(cA, vA);
        fetch_chunks<D, false>(i + 2 * D, gid, ngrp, gl, lgE, TC, clist, abeg, nullptr, Bci, nullptr, cA, dummy,
                               dummy, vA);
        consume(cB, vB);
      }
    }
    if (overflow) {
      if (tid == 0) flags[row] |= 2;
      return;   // uniform: every thread saw the same totals
    }
    SPMM_STAMP(1);
    if (mine) atomicAdd(&s_count, mine);
    __syncthreads();
    row_count += s_count;
    __syncthreads();   // s_count read before the next slice resets it
  }
  if (stamp_on && tid == 0) atomicAdd(&g_stamps[7], 1ull);
  if (tid == 0) row_nnz[row] = row_count;
}

// -------------------------------------------------------------- numeric ----
constexpr unsigned long long EMPTY64 = 0x00000000FFFFFFFFull;   // key EMPTY, value +0

template <int S, int NT, int NP>
__global__ __launch_bounds__(NT, 4) void spgemm_lds_num(
    const int64_t* __restrict__ Arp, const int32_t* __restrict__ Aci, const float* __restrict__ Av,
    const int64_t* __restrict__ Brp, const int32_t* __restrict__ Bci, const float* __restrict__ Bv,
    const int64_t* __restrict__ bsplit, const int32_t* __restrict__ rows, int ncols, int lg,
    const int32_t* __restrict__ row_cap, int32_t* __restrict__ out_nnz, const int64_t* __restrict__ Crp,
    int32_t* __restrict__ Cci, float* __restrict__ Cv, int32_t* __restrict__ flags) {
  using Gm = LdsGeom<S, NT>;
  constexpr int TS = Gm::TS, NW = Gm::NW, ACAP = Gm::ACAP, CCAP = Gm::CCAP, NWIN = Gm::NWIN;
  constexpr int QSTEP = 8 / NP;
  constexpr int D = 4;
  __shared__ __attribute__((aligned(16))) unsigned long long tab[TS + 2];   // key (low word) | value bits (high)
  __shared__ int64_t abeg[ACAP];
  __shared__ int clist[CCAP];           // chunk descriptors; later the per-window counts
  __shared__ float aval[ACAP];
  __shared__ int64_t wsum[NW];
  __shared__ int s_wrapped;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row = rows[blockIdx.x];
  const int64_t a0 = Arp[row], na = Arp[row + 1] - a0;
  const int lgE = lg > Gm::LG_MIN ? lg : Gm::LG_MIN;
  const int ngrp = NW << (6 - lgE);
  const int gid = (w << (6 - lgE)) + (lane >> lgE);
  const int gl = lane & ((1 << lgE) - 1);
  const int stamp_on = g_stamp_on;
  unsigned long long t_prev = stamp_on ? __builtin_amdgcn_s_memtime() : 0ull;
  int written = 0;   // entries of earlier slices already stored
  bool unsorted = false;

  for (int sl = 0; sl < NP; ++sl) {
    const int q0 = sl * QSTEP, q1 = q0 + QSTEP;
    const int clo = (int)(((int64_t)q0 * ncols) >> 3), chi = (int)(((int64_t)q1 * ncols) >> 3);
    const uint32_t mult = hash_mult(S, chi - clo);
    for (int i = tid; i < (TS + 2) / 2; i += NT)
      reinterpret_cast<ulonglong2*>(tab)[i] = make_ulonglong2(EMPTY64, EMPTY64);
    if (tid == 0) s_wrapped = 0;
    int64_t slice_products = 0;
    bool overflow = false;
    for (int64_t bat = 0; bat < na; bat += ACAP) {
      const int nb = (int)((na - bat) < ACAP ? (na - bat) : ACAP);
      __syncthreads();
      int len, nch, pre, TC;
      int64_t tot;
      stage_batch<NT, NP, true>(Aci, Av, Brp, bsplit, a0 + bat, nb, q0, q1, lgE, abeg, aval, wsum, len, nch, pre,
                                TC, tot);
      SPMM_STAMP(0);
      slice_products += tot;
      if (slice_products > TS - 8 || TC > CCAP) { overflow = true; break; }
      if (TC == 0) continue;
      write_chunks(clist, len, nch, pre, lgE);
      __syncthreads();

      int cA[D], cB[D];
      float bA[D], bB[D], aA[D], aB[D];
      bool vA[D], vB[D];
      auto consume = [&](const int (&c)[D], const float (&bv)[D], const float (&av)[D], const bool (&v)[D]) {
        int h[D];
        uint32_t ck[D];
        float cv[D];
        unsigned long long cur[D];
        bool st[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
          h[u] = hash_home(c[u] - clo, mult);
          ck[u] = (uint32_t)c[u];
          cv[u] = av[u] * bv[u];
          cur[u] = EMPTY64;   // belief about tab[h]
          st[u] = v[u];
        }
        while (true) {
          unsigned long long old[D];
#pragma unroll
          for (int u = 0; u < D; ++u) {
            const uint32_t k = (uint32_t)cur[u];
            const float nv = (k == ck[u]) ? __uint_as_float((uint32_t)(cur[u] >> 32)) + cv[u] : cv[u];
            const unsigned long long want = ((unsigned long long)__float_as_uint(nv) << 32) | ck[u];
            old[u] = st[u] ? atomicCAS(&tab[h[u]], cur[u], want) : cur[u];
          }
          bool more = false;
#pragma unroll
          for (int u = 0; u < D; ++u) {
            if (st[u]) {
              const uint32_t k = (uint32_t)cur[u];
              if (old[u] == cur[u]) {             // our CAS landed
                if (k == (uint32_t)EMPTY || k == ck[u]) {
                  st[u] = false;                  // placed / merged
                } else {                          // displaced a larger key: carry it on
                  ck[u] = k;
                  cv[u] = __uint_as_float((uint32_t)(cur[u] >> 32));
                  ++h[u];
                  cur[u] = EMPTY64;
                }
              } else if ((uint32_t)old[u] < ck[u]) {   // smaller key (EMPTY is the largest): move on
                ++h[u];
                cur[u] = EMPTY64;
              } else {
                cur[u] = old[u];                  // retry this slot with what is there
              }
              if (st[u] && h[u] >= TS) { h[u] = 0; s_wrapped = 1; }
              more |= st[u];
            }
          }
          if (!__any(more)) break;
        }
      };
      const int nit = (TC + ngrp - 1) / ngrp;
      fetch_chunks<D, true>(0, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cA, bA, aA, vA);
      for (int i = 0; i < nit; i += 2 * D) {
        fetch_chunks<D, true>(i + D, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cB, bB, aB, vB);
        consume(cA, bA, aA, vA);
        fetch_chunks<D, true>(i + 2 * D, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cA, bA, aA, vA);
        consume(cB, bB, aB, vB);
      }
    }
    if (overflow) {
      if (tid == 0) flags[row] |= 2;
      return;
    }
    __syncthreads();
    SPMM_STAMP(1);
    // Output = the table in slot order: position = occupied slots before it.
    constexpr int WPW = (NWIN + NW - 1) / NW;
    unsigned long long q[WPW];
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int W = w + j * NW;
      q[j] = (W < NWIN) ? tab[W * 64 + lane] : EMPTY64;
      const unsigned long long M = __ballot((uint32_t)q[j] != (uint32_t)EMPTY);
      if (lane == 0 && W < NWIN) clist[W] = __popcll(M);
    }
    __syncthreads();
    int total;
    {
      const int cw = (tid < NWIN) ? clist[tid] : 0;
      const int bw = block_excl_scan<NT, int>(cw, reinterpret_cast<int*>(wsum), &total);
      __syncthreads();
      if (tid < NWIN) clist[tid] = bw;
    }
    __syncthreads();
    const int64_t base = Crp[row] + written;
    // the row's space (exact size from symbolic, or the product count in
    // one-pass mode): never store past it whatever happened here
    const int room = row_cap[row] - written;
    const int lim = total < room ? total : room;
    if (tid == 0 && total > room) atomicOr(&flags[row], 4);
    bool bad = false;
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int W = w + j * NW;
      if (W < NWIN) {
        const uint32_t key = (uint32_t)q[j];
        const bool occ = key != (uint32_t)EMPTY;
        const unsigned long long M = __ballot(occ);
        // adjacency check: the next slot's key must be larger (EMPTY is the largest)
        uint32_t nk = (uint32_t)__builtin_amdgcn_update_dpp((int)EMPTY, (int)key, 0x130, 0xF, 0xF, false);   // wave_shl:1
        if (lane == 63) nk = (W * 64 + 64 < TS) ? (uint32_t)tab[W * 64 + 64] : (uint32_t)EMPTY;
        bad |= occ & (nk <= key);
        if (occ) {
          const int pos = clist[W] + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
          if (pos < lim) {
            Cci[base + pos] = (int)key;
            Cv[base + pos] = __uint_as_float((uint32_t)(q[j] >> 32));
          } else {
            atomicOr(&flags[row], 4);   // internal error: never write outside the row
          }
        }
      }
    }
    unsorted |= bad | (s_wrapped != 0);
    SPMM_STAMP(2);
    written += total;
    __syncthreads();   // slice done before the next slice re-initialises the table
  }
  if (__any(unsorted) && lane == 0) atomicOr(&flags[row], 1);
  if (out_nnz != nullptr && tid == 0) out_nnz[row] = written;
  if (stamp_on && tid == 0) atomicAdd(&g_stamps[7], 1ull);
}

// ---------------------------------------------------------------- ESC -----
// Numeric kernel for long rows: bucketed expand-sort-compress in LDS.
//
// The CAS-probing tables above spend most of their time in dependent LDS
// atomic rounds (every probe step is a round trip, and a wave keeps looping
// until its slowest lane is placed).  Here every product costs a fixed,
// round-free sequence:
//   pass H: bucket histogram (ds_add without return: fire and forget)
//   scan:   bucket offsets (16-bit counters, two per word)
//   pass S: one ds_add_rtn for the slot + one 8-byte write of (column, a*b)
//   sort:   one lane per bucket sorts its few items in registers (sorting
//           network sized by the wave's largest bucket) and folds duplicate
//           columns into their first occurrence (the rest become holes)
//   write:  compaction of the non-hole items in slot order (ballot + mbcnt)
// Buckets are a monotone function of the column, so slot order is column
// order.  Each product is read from B twice (histogram + scatter); the second
// read mostly hits L2 / MALL.
constexpr int ESC_NB = 4096;   // buckets per slice

// max over the 64 lanes without LDS: DPP within each 16-lane row, then 4 readlanes
__device__ __forceinline__ int wave_max(int x) {
  x = max(x, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));    // quad_perm [1,0,3,2]
  x = max(x, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));    // quad_perm [2,3,0,1]
  x = max(x, __builtin_amdgcn_update_dpp(x, x, 0x141, 0xF, 0xF, false));   // row_half_mirror
  x = max(x, __builtin_amdgcn_update_dpp(x, x, 0x140, 0xF, 0xF, false));   // row_mirror
  const int a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 16);
  const int c = __builtin_amdgcn_readlane(x, 32), d = __builtin_amdgcn_readlane(x, 48);
  return max(max(a, b), max(c, d));
}

// Ordered mode (one-pass without the compaction copy): the grid walks
// "units" = (row, column-eighth range) in row order; a workgroup takes the
// next unit from a ticket counter (so every earlier unit is already running
// or done), and its output position comes from a decoupled look-back over
// the units' published counts.  Rows land directly at their final CSR
// offsets: no staging buffer, no compaction pass.
struct EscOrd {
  const int32_t* unit_row;
  const uint8_t* unit_q;            // q0 | q1 << 4 (column eighths [q0, q1))
  uint32_t* ticket;
  unsigned long long* status;       // per unit: flag (2 bits) | count or inclusive prefix (62 bits)
  int64_t cap;                      // entries allocated for C
  int32_t* err;                     // bit 0: a unit overflowed its LDS slice, bit 1: C capacity
};

// Publish this unit's count, sum the predecessors back to the first
// inclusive prefix, publish the inclusive prefix; returns the exclusive one.
// Run by one whole wave: the 64 nearest predecessors' status words are loaded
// at once (one memory round trip instead of one per predecessor), and the
// window slides back only while all 64 are counts without a prefix.
__device__ __forceinline__ int64_t ord_lookback(unsigned long long* status, int64_t u, int64_t count, int lane) {
  constexpr unsigned long long AGG = 1ull << 62, INC = 2ull << 62, VM = (1ull << 62) - 1;
  if (u == 0 || g_nowait) {
    if (lane == 0)
      __hip_atomic_store(&status[u], INC | (unsigned long long)count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(&status[u], AGG | (unsigned long long)count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int64_t pre = 0;
  for (int64_t end = u;;) {
    const int64_t j = end - 1 - lane;   // lane 0 = nearest predecessor
    const unsigned long long st =
        j >= 0 ? __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : INC;
    const unsigned f = (unsigned)(st >> 62);
    const unsigned long long inc = __ballot(f == 2), notready = __ballot(f == 0);
    const int first = inc ? __ffsll((long long)inc) - 1 : 64;
    const unsigned long long need = first >= 63 ? ~0ull : ((2ull << first) - 1);   // lanes 0..first
    if (notready & need) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    int64_t v = lane <= first ? (int64_t)(st & VM) : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    pre += v;
    if (first < 64) break;
    end -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(&status[u], INC | (unsigned long long)(pre + count), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return pre;
}

template <int PCAP, int NT, int NP, bool ORD = false, int NBT = ESC_NB>
__global__ __launch_bounds__(NT, NT >= 1024 ? 1 : 4) void spgemm_esc(
    const int64_t* __restrict__ Arp, const int32_t* __restrict__ Aci, const float* __restrict__ Av,
    const int64_t* __restrict__ Brp, const int32_t* __restrict__ Bci, const float* __restrict__ Bv,
    const int64_t* __restrict__ bsplit, const int32_t* __restrict__ rows, int ncols, int lg,
    const int32_t* __restrict__ row_cap, int32_t* __restrict__ out_nnz, const int64_t* __restrict__ Crp,
    int32_t* __restrict__ Cci, float* __restrict__ Cv, int32_t* __restrict__ flags, EscOrd ord) {
  constexpr int NW = NT / 64, ACAP = NT, CCAP = 2 * NT, NB = NBT;
  constexpr int BPT = NB / NT;                 // buckets per thread in the scan / sort
  constexpr int QSTEP = 8 / NP;
  constexpr int D = 4;
  constexpr int NWIN = PCAP / 64;
  constexpr int WPW = (NWIN + NW - 1) / NW;
  constexpr int LG_MIN = lds_lg_min(PCAP, NT, CCAP);
  static_assert(PCAP % 64 == 0 && PCAP < 65536, "16-bit bucket counters");
  static_assert(BPT % 2 == 0 && BPT <= 8, "a thread owns whole counter words, at most 8 buckets");
  static_assert(NWIN <= CCAP, "window counts reuse the descriptor buffer");
  static_assert(NT <= 1024, "entry index is 10 bits in a chunk descriptor");
  __shared__ __attribute__((aligned(16))) unsigned long long items[PCAP];   // key (low) | value bits (high)
  __shared__ __attribute__((aligned(16))) uint32_t hist[NB / 2];            // two 16-bit counters per word
  __shared__ int64_t abeg[ACAP];
  __shared__ int clist[CCAP];
  __shared__ float aval[ACAP];
  __shared__ int64_t wsum[NW];
  __shared__ int64_t ord_sh;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int row, uq0 = 0, uq1 = 8;
  int64_t unit = 0;
  if constexpr (ORD) {
    if (tid == 0) ord_sh = (int64_t)atomicAdd(ord.ticket, 1u);
    __syncthreads();
    unit = ord_sh;
    row = ord.unit_row[unit];
    const int q = ord.unit_q[unit];
    uq0 = q & 15;
    uq1 = q >> 4;
  } else {
    row = rows[blockIdx.x];
  }
  const int64_t a0 = Arp[row], na = Arp[row + 1] - a0;
  const int lgE = lg > LG_MIN ? lg : LG_MIN;
  const int ngrp = NW << (6 - lgE);
  const int gid = (w << (6 - lgE)) + (lane >> lgE);
  const int gl = lane & ((1 << lgE) - 1);
  const int stamp_on = g_stamp_on;
  unsigned long long t_prev = stamp_on ? __builtin_amdgcn_s_memtime() : 0ull;
  int written = 0;
  int tc_keep = 0;   // chunk count of a single-batch row, reused by the second pass
  // Single-batch rows (na <= ACAP, the common case) keep their entry in
  // registers across slices: the column j, a(i,j), the current segment start
  // and the NEXT slice boundary, loaded one slice ahead so that only slice 0
  // waits for global memory during staging.
  const bool single = na <= ACAP;
  int ej = 0;
  float eav = 0.f;
  int64_t eb0 = 0, eb1 = 0;
  if (single && tid < na) {
    ej = Aci[a0 + tid];
    eav = Av[a0 + tid];
    if constexpr (ORD) {
      eb0 = uq0 == 0 ? Brp[ej] : bsplit[(int64_t)ej * 7 + uq0 - 1];
      eb1 = uq1 == 8 ? Brp[ej + 1] : bsplit[(int64_t)ej * 7 + uq1 - 1];
    } else {
      eb0 = Brp[ej];
      eb1 = (NP == 1) ? Brp[ej + 1] : bsplit[(int64_t)ej * 7 + QSTEP - 1];
    }
  }

  constexpr int NSL = ORD ? 1 : NP;
  for (int sl = 0; sl < NSL; ++sl) {
    const int q0 = ORD ? uq0 : sl * QSTEP, q1 = ORD ? uq1 : q0 + QSTEP;
    const int clo = (int)(((int64_t)q0 * ncols) >> 3), chi = (int)(((int64_t)q1 * ncols) >> 3);
    const uint32_t mult = hash_mult(NB, chi - clo);
    for (int i = tid; i < NB / 8; i += NT) reinterpret_cast<uint4*>(hist)[i] = make_uint4(0, 0, 0, 0);
    int64_t slice_products = 0;
    bool overflow = false;
    for (int pass = 0; pass < 2 && !overflow; ++pass) {
      for (int64_t bat = 0; bat < na; bat += ACAP) {
        const int nb = (int)((na - bat) < ACAP ? (na - bat) : ACAP);
        int TC;
        if (pass == 0 || !single) {   // single-batch rows keep their staging for the second pass
          __syncthreads();
          int len, nch, pre;
          int64_t tot;
          if (single) {
            len = 0;
            if (tid < nb) {
              len = (int)(eb1 - eb0);
              abeg[tid] = eb0;
              aval[tid] = eav;
              eb0 = eb1;   // next slice starts where this one ends
              if (!ORD && sl + 1 < NP)   // prefetch the next slice's end
                eb1 = (sl + 2 == NP) ? Brp[ej + 1] : bsplit[(int64_t)ej * 7 + (sl + 2) * QSTEP - 1];
            }
            scan_chunks<NT>(len, lgE, wsum, nch, pre, TC, tot);
          } else {
            stage_batch<NT, (ORD ? 2 : NP), true>(Aci, Av, Brp, bsplit, a0 + bat, nb, q0, q1, lgE, abeg, aval, wsum,
                                                  len, nch, pre, TC, tot);
          }
          if (pass == 0) {
            slice_products += tot;
            if (slice_products > PCAP || TC > CCAP) { overflow = true; break; }
          }
          tc_keep = TC;
          if (TC == 0) continue;
          write_chunks(clist, len, nch, pre, lgE);
          __syncthreads();
        } else {
          TC = tc_keep;
          if (TC == 0) continue;
        }
        SPMM_STAMP(0);
        int cA[D], cB[D];
        float bA[D], bB[D], aA[D], aB[D];
        bool vA[D], vB[D];
        auto bucket = [&](int c) { return hash_home(c - clo, mult); };
        auto consume = [&](const int (&c)[D], const float (&bv)[D], const float (&av)[D], const bool (&v)[D]) {
          if (pass == 0) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
              const int b = bucket(c[u]);
              if (v[u]) atomicAdd(&hist[b >> 1], (b & 1) ? 0x10000u : 1u);
            }
          } else {
            uint32_t old[D];
#pragma unroll
            for (int u = 0; u < D; ++u) {
              const int b = bucket(c[u]);
              old[u] = v[u] ? atomicAdd(&hist[b >> 1], (b & 1) ? 0x10000u : 1u) : 0u;
            }
#pragma unroll
            for (int u = 0; u < D; ++u) {
              const int b = bucket(c[u]);
              const int pos = (b & 1) ? (int)(old[u] >> 16) : (int)(old[u] & 0xffff);
              if (v[u])
                items[pos] = ((unsigned long long)__float_as_uint(av[u] * bv[u]) << 32) | (uint32_t)c[u];
            }
          }
        };
        const int nit = (TC + ngrp - 1) / ngrp;
        if (pass == 0) {
          fetch_chunks<D, false>(0, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cA, bA, aA, vA);
          for (int i = 0; i < nit; i += 2 * D) {
            fetch_chunks<D, false>(i + D, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cB, bB, aB, vB);
            consume(cA, bA, aA, vA);
            fetch_chunks<D, false>(i + 2 * D, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cA, bA, aA, vA);
            consume(cB, bB, aB, vB);
          }
        } else {
          fetch_chunks<D, true>(0, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cA, bA, aA, vA);
          for (int i = 0; i < nit; i += 2 * D) {
            fetch_chunks<D, true>(i + D, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cB, bB, aB, vB);
            consume(cA, bA, aA, vA);
            fetch_chunks<D, true>(i + 2 * D, gid, ngrp, gl, lgE, TC, clist, abeg, aval, Bci, Bv, cA, bA, aA, vA);
            consume(cB, bB, aB, vB);
          }
        }
        SPMM_STAMP(1);
      }
      if (overflow) break;
      __syncthreads();   // all counts (pass 0) / all items (pass 1) in place
      if (pass == 0) {
        // exclusive bucket offsets; thread t owns buckets [BPT*t, BPT*t + BPT)
        uint32_t cw[BPT / 2];
        int run = 0;
#pragma unroll
        for (int i = 0; i < BPT / 2; ++i) {
          cw[i] = hist[tid * (BPT / 2) + i];
          run += (int)(cw[i] & 0xffff) + (int)(cw[i] >> 16);
        }
        int total;
        __syncthreads();
        int off = block_excl_scan<NT, int>(run, reinterpret_cast<int*>(wsum), &total);
#pragma unroll
        for (int i = 0; i < BPT / 2; ++i) {
          const int lo = off, hi = off + (int)(cw[i] & 0xffff);
          off = hi + (int)(cw[i] >> 16);
          hist[tid * (BPT / 2) + i] = (uint32_t)lo | ((uint32_t)hi << 16);
        }
        __syncthreads();
      }
    }
    if (overflow) {
      if (tid == 0) atomicOr(&flags[row], 2);
      if constexpr (ORD) {   // successors still need this unit's count: publish 0, the host recomputes
        if (tid == 0) atomicOr(ord.err, 1);
        if (w == 0) ord_lookback(ord.status, unit, 0, lane);
      }
      return;   // uniform: every thread saw the same totals
    }
    // hist[b] now holds the END offset of bucket b.  Sort + fold each bucket.
    const int P = (int)slice_products;
    {
      int e[BPT];
#pragma unroll
      for (int i = 0; i < BPT / 2; ++i) {
        const uint32_t x = hist[tid * (BPT / 2) + i];
        e[2 * i] = (int)(x & 0xffff);
        e[2 * i + 1] = (int)(x >> 16);
      }
      const int s0 = tid ? (int)(hist[tid * (BPT / 2) - 1] >> 16) : 0;
      auto sb = [&](int i) { return i ? e[i - 1] : s0; };
      auto kb = [&](int i) { return e[i] - sb(i); };
      int km[BPT];   // wave-uniform (SGPRs)
#pragma unroll
      for (int i = 0; i < BPT; ++i) km[i] = wave_max(kb(i));   // DPP + readlane: no LDS round trips
      // software pipeline: bucket i+1's items are read while bucket i sorts
      auto load = [&](int i, uint32_t (&key)[8], float (&val)[8]) {
        const int s = sb(i), k = kb(i);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          key[j] = (uint32_t)EMPTY;
          val[j] = 0.f;
          if (j < km[i] && km[i] >= 2) {   // wave-uniform
            const unsigned long long x = items[(j < k) ? s + j : min(s, PCAP - 1)];   // clamped, unpredicated
            key[j] = (j < k) ? (uint32_t)x : (uint32_t)EMPTY;
            val[j] = __uint_as_float((uint32_t)(x >> 32));
          }
        }
      };
      auto process = [&](int i, uint32_t (&key)[8], float (&val)[8]) {
        const int s = sb(i), k = kb(i), kmax = km[i];
        if (kmax < 2) return;
        auto ce = [&](int a, int b) {
          const bool sw = key[b] < key[a];
          const uint32_t ka = sw ? key[b] : key[a], kb2 = sw ? key[a] : key[b];
          const float va = sw ? val[b] : val[a], vb = sw ? val[a] : val[b];
          key[a] = ka; key[b] = kb2; val[a] = va; val[b] = vb;
        };
        // small sorting networks sized by the wave's largest bucket
        if (kmax == 2) {
          ce(0, 1);
        } else if (kmax <= 4) {
          ce(0, 1); ce(2, 3); ce(0, 2); ce(1, 3); ce(1, 2);
        } else if (kmax <= 6) {
          ce(0, 5); ce(1, 3); ce(2, 4); ce(1, 2); ce(3, 4); ce(0, 3); ce(2, 5); ce(0, 1); ce(2, 3);
          ce(4, 5); ce(1, 2); ce(3, 4);
        } else {
          ce(0, 1); ce(2, 3); ce(4, 5); ce(6, 7);
          ce(0, 2); ce(1, 3); ce(4, 6); ce(5, 7);
          ce(1, 2); ce(5, 6);
          ce(0, 4); ce(1, 5); ce(2, 6); ce(3, 7);
          ce(2, 4); ce(3, 5);
          ce(1, 2); ce(3, 4); ce(5, 6);
        }
#pragma unroll
        for (int j = 7; j >= 1; --j) {   // fold equal columns into the first occurrence
          if (j >= kmax) continue;   // wave-uniform
          const bool dup = key[j] != (uint32_t)EMPTY && key[j] == key[j - 1];
          val[j - 1] += dup ? val[j] : 0.f;
          key[j] = dup ? (uint32_t)EMPTY : key[j];
        }
        if (k <= 8) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < k) items[s + j] = ((unsigned long long)__float_as_uint(val[j]) << 32) | key[j];
        } else {
          // rare oversized bucket: insertion sort + fold in LDS by this lane
          for (int a = s + 1; a < s + k; ++a) {
            const unsigned long long x = items[a];
            int b = a - 1;
            while (b >= s && (uint32_t)items[b] > (uint32_t)x) { items[b + 1] = items[b]; --b; }
            items[b + 1] = x;
          }
          for (int a = s + k - 1; a > s; --a) {
            const unsigned long long x = items[a], y = items[a - 1];
            if ((uint32_t)x == (uint32_t)y && (uint32_t)x != (uint32_t)EMPTY) {
              const float sum = __uint_as_float((uint32_t)(y >> 32)) + __uint_as_float((uint32_t)(x >> 32));
              items[a - 1] = ((unsigned long long)__float_as_uint(sum) << 32) | (uint32_t)y;
              items[a] = EMPTY64;
            }
          }
        }
      };
      uint32_t kX[8];   // (a register double buffer across buckets spills: measured slower)
      float vX[8];
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        load(i, kX, vX);
        process(i, kX, vX);
      }
    }
    __syncthreads();
    SPMM_STAMP(2);
    // compaction of the non-hole items [0, P) in slot order
    unsigned long long q[WPW];
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int W = w + j * NW;
      const int slot = W * 64 + lane;
      q[j] = (W < NWIN && slot < P) ? items[slot] : EMPTY64;
      const unsigned long long M = __ballot((uint32_t)q[j] != (uint32_t)EMPTY);
      if (lane == 0 && W < NWIN) clist[W] = __popcll(M);
    }
    __syncthreads();
    int total;
    {
      const int cw = (tid < NWIN) ? clist[tid] : 0;
      const int bw = block_excl_scan<NT, int>(cw, reinterpret_cast<int*>(wsum), &total);
      __syncthreads();
      if (tid < NWIN) clist[tid] = bw;
    }
    __syncthreads();
    int64_t base;
    int lim;
    if constexpr (ORD) {
      if (w == 0) {
        const int64_t b = ord_lookback(ord.status, unit, total, lane);
        if (lane == 0) ord_sh = b;
      }
      __syncthreads();
      base = ord_sh;
      SPMM_STAMP(4);   // unit count scan + look-back
      const int64_t room = ord.cap - base;
      lim = total <= room ? total : (int)(room > 0 ? room : 0);
      if (tid == 0 && total > room) atomicOr(ord.err, 2);
    } else {
      base = Crp[row] + written;
      const int room = row_cap[row] - written;
      lim = total < room ? total : room;
      if (tid == 0 && total > room) atomicOr(&flags[row], 4);
    }
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int W = w + j * NW;
      if (W < NWIN) {
        const uint32_t key = (uint32_t)q[j];
        const bool occ = key != (uint32_t)EMPTY;
        const unsigned long long M = __ballot(occ);
        if (occ) {
          const int pos = clist[W] + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
          if (pos < lim) {
            Cci[base + pos] = (int)key;
            Cv[base + pos] = __uint_as_float((uint32_t)(q[j] >> 32));
          } else {
            atomicOr(&flags[row], 4);   // internal error: never write outside the row
          }
        }
      }
    }
    SPMM_STAMP(3);
    written += total;
    __syncthreads();   // slice done before the next slice reuses the buffers
  }
  if (out_nnz != nullptr && tid == 0) {
    if constexpr (ORD) atomicAdd(&out_nnz[row], written);   // several units per row
    else out_nnz[row] = written;
  }
  if (stamp_on && tid == 0) atomicAdd(&g_stamps[7], 1ull);
}

// Eighth split points of every B row (rows column-sorted): bsplit[j*7 + q-1] =
// first index of row j whose column >= floor(q * ncols / 8), q = 1..7.
// Eight lanes per row, lane q searches split q: seven short independent
// binary searches instead of one thread chaining all seven (the searches
// are latency bound: ~log2(row length) dependent loads each).
__global__ __launch_bounds__(256) void spgemm_row_splits(const int64_t* __restrict__ Brp,
                                                         const int32_t* __restrict__ Bci, int64_t mb, int ncols,
                                                         int64_t* __restrict__ bsplit) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t j = t >> 3;
  const int q = (int)(t & 7);
  if (j >= mb || q == 0) return;
  const int bound = (int)(((int64_t)q * ncols) >> 3);
  int64_t lo = Brp[j], hi = Brp[j + 1];   // first index with col >= bound
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (Bci[mid] < bound) lo = mid + 1; else hi = mid;
  }
  bsplit[j * 7 + q - 1] = lo;
}

// One-pass mode: rows were written at their product-count offsets (src_off);
// copy each row's n[i] entries to the final CSR (dst_off).  One wave per row.
// src_off < 0: the row is placed by another kernel (long rows, long_place).
__global__ __launch_bounds__(256) void spgemm_compact(const int64_t* __restrict__ src_off,
                                                      const int64_t* __restrict__ dst_off, int64_t m,
                                                      const int32_t* __restrict__ sci, const float* __restrict__ sv,
                                                      int32_t* __restrict__ dci, float* __restrict__ dv) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= m) return;
  const int64_t s0 = src_off[row], d0 = dst_off[row], n = dst_off[row + 1] - d0;
  if (s0 < 0) return;
  int64_t i = lane;
  for (; i + 192 < n; i += 256) {   // 4 loads in flight per lane
    const int c0 = sci[s0 + i], c1 = sci[s0 + i + 64], c2 = sci[s0 + i + 128], c3 = sci[s0 + i + 192];
    const float v0 = sv[s0 + i], v1 = sv[s0 + i + 64], v2 = sv[s0 + i + 128], v3 = sv[s0 + i + 192];
    dci[d0 + i] = c0; dci[d0 + i + 64] = c1; dci[d0 + i + 128] = c2; dci[d0 + i + 192] = c3;
    dv[d0 + i] = v0; dv[d0 + i + 64] = v1; dv[d0 + i + 128] = v2; dv[d0 + i + 192] = v3;
  }
  for (; i < n; i += 64) {
    dci[d0 + i] = sci[s0 + i];
    dv[d0 + i] = sv[s0 + i];
  }
}

// ------------------------------------------------------------ long rows ---
// Rows beyond the LDS bins (R-MAT hubs: up to ~10^7 products, ~5*10^5
// outputs) go through a column-chunked dense pipeline with an HBM scratch:
//   route  (pass 1) every workgroup takes <= LONG_EPW A entries of ONE row and
//          histograms its products by column chunk (W columns) in LDS
//   scan   (host/torch) per-(row, chunk) regions in the scratch and each
//          workgroup's slot range inside them: no global atomics
//   route  (pass 2) the same products are scattered into their (row, chunk)
//          region as (column | a*b bits), slots from LDS cursors
//   dense  one workgroup per (row, chunk): LDS dense accumulator (W floats +
//          occupancy bits), then the occupied columns are written back in
//          column order over the chunk's region, count in rt_nnz
//   place  chunk results copied to their final CSR positions
// Traffic per product: 4 + 8 B of B reads, 8 B scratch write + 8 B read.
//
// Direct products (hub B rows, long_btab): an item of more than LR_CAP
// products takes the products of the row's LONG B rows (>= LONG_BTAB_MIN
// entries per chunk; R-MAT 24: ~85 % of the long-row products) straight from
// B in long_dense, through their chunk segments in long_btab: no scratch
// write, no scratch read.  The route passes histogram them apart (dhist),
// skip them in the scatter, and list the row's long entries (dl) instead;
// items of <= LR_CAP products still route them (long_rank reads the scratch).
#ifndef SPMM_LONG_EPW                   // (diagnostic builds: tools/bm_variants.py)
#define SPMM_LONG_EPW 64
#endif
#ifndef SPMM_LONG_FRESH
#define SPMM_LONG_FRESH 1
#endif
#ifndef SPMM_LONG_DLOADS
#define SPMM_LONG_DLOADS 4
#endif
constexpr int LONG_NT = 512;
constexpr int LONG_EPW = SPMM_LONG_EPW; // A entries per routing workgroup
constexpr int LONG_DL = SPMM_LONG_DLOADS;   // scratch loads in flight per lane (long_dense)
#ifndef SPMM_LONG_XCD
#define SPMM_LONG_XCD 1
#endif
#ifndef SPMM_LONG_LGW
#define SPMM_LONG_LGW 15
#endif
constexpr int LONG_LGW = SPMM_LONG_LGW; // W = 32768 columns per chunk (2^14: 3 % slower at R-MAT 24)
constexpr int LONG_W = 1 << LONG_LGW;
constexpr int LONG_DNT = LONG_W / 32;  // long_dense: one occupancy word per thread
constexpr int LONG_MAXCH = 4096;        // chunks per row (ncols <= 2^26)

// 64-lane inclusive prefix sum on the DPP network (VALU; no LDS traffic):
// row_shr 1/2/4/8 inside 16-lane rows, then row_bcast:15 / row_bcast:31.
__device__ __forceinline__ int wave_incl_scan_dpp(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
  return x;
}

// 64-lane inclusive max scan on the DPP network (identity -1).
__device__ __forceinline__ int wave_incl_max_dpp(int x) {
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false));
  return x;
}

#ifndef SPMM_LR_R   // long_rank: register rounds per lane (items of <= 64 * LR_R products; larger ones go to long_dense)
#define SPMM_LR_R 16   // (8: 4 workgroups/CU instead of 3, but R-MAT 22 2.11-2.15 vs 1.99-2.01 s/step)
#endif
constexpr int LR_R = SPMM_LR_R, LR_CAP = LR_R * 64, LR_WAVES = 4;
constexpr int LR_WORDS = LONG_W / 64;   // 64-bit bitmap words per chunk
static_assert(LR_WORDS % 64 == 0, "whole bitmap rows per lane");

__device__ __forceinline__ void lr_wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-level expansion of 64 sources (lane = source, exclusive prefix `pre`
// of the lengths `len`) into slots: the owner of slot qw + lane, the window
// [qw, qw + 64) of the concatenated sources (any window, in any order).
// `own` = 64 ints of this wave's LDS.  A source starting inside the window
// marks its first slot; a max scan over the marks gives every slot the last
// source starting at or before it, the sources starting before the window
// (one ballot) the slots before the first mark.
__device__ __forceinline__ int wave_slot_owner(int pre, int len, int qw, int lane, int* own) {
  const unsigned long long before = __ballot(len > 0 && pre < qw);
  const int carry = before ? 63 - __clzll((long long)before) : -1;
  own[lane] = -1;
  lr_wave_fence();
  if (len > 0 && pre >= qw && pre < qw + 64) own[pre - qw] = lane;
  lr_wave_fence();
  const int o = max(wave_incl_max_dpp(own[lane]), carry);
  lr_wave_fence();
  return o;
}

// SCATTER: wg_hist holds each workgroup's offset inside its (row, chunk)
// regions (long_wg_scan), row_off[row * nch + t] the regions' scratch bases.
// Direct mode (wg_dhist / dl given; lidx / btab required):
//   histogram  the long B rows' chunk counts go to wg_dhist (not wg_hist),
//              wg_nlong = the workgroup's long entries
//   scatter    rt_mode[row * nch + t] (long_wg_scan): 0 = the item routes its
//              long products too (same cursor), 1 = direct (skipped), 2 = no
//              long products; every long entry is listed in dl at
//              dl_off[wg] + i as {B row start, btab row, a bits, 0}
template <bool SCATTER, bool DIRECT>
__global__ __launch_bounds__(LONG_NT) void long_route(
    const int32_t* __restrict__ Aci, const float* __restrict__ Av, const int64_t* __restrict__ Brp,
    const int32_t* __restrict__ Bci, const float* __restrict__ Bv, const int64_t* __restrict__ wg_e0,
    const int64_t* __restrict__ wg_e1, int nch, int32_t* __restrict__ wg_hist,
    const int32_t* __restrict__ wg_row, const int64_t* __restrict__ row_off,
    unsigned long long* __restrict__ scratch, const int32_t* __restrict__ lidx, const uint32_t* __restrict__ btab,
    int32_t* __restrict__ wg_dhist, int32_t* __restrict__ wg_nlong, const uint8_t* __restrict__ rt_mode,
    uint4* __restrict__ dl, const int64_t* __restrict__ dl_off) {
  constexpr int NWV = LONG_NT / 64;
  constexpr bool DS = SCATTER && DIRECT;
  __shared__ unsigned long long cur[SCATTER ? LONG_MAXCH : 1];
  __shared__ int hist[SCATTER ? 1 : LONG_MAXCH];
  __shared__ int dhist[!SCATTER && DIRECT ? LONG_MAXCH : 1];
  __shared__ int own_all[DS ? NWV : 1][64];
  __shared__ uint2 seg_all[DS ? NWV : 1][64];                 // {first B index (low 32 bits), slot prefix}
  __shared__ unsigned long long dst_all[DS ? NWV : 1][64];    // scratch slot of each chunk's first product
  __shared__ int16_t m0list[DS ? LONG_MAXCH : 1];             // the row's mode-0 chunks
  __shared__ int nlong, nm0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // Neighbouring workgroups own neighbouring scratch runs of every chunk, so
  // they share cache lines: give them one XCD (one L2) so the partial lines
  // merge there instead of reaching the fabric as masked partial writes.
#if SPMM_LONG_XCD
  const int64_t wg = spmm::xcd_remap(blockIdx.x, gridDim.x);
#else
  const int64_t wg = blockIdx.x;
#endif
  const int64_t ro = SCATTER ? (int64_t)wg_row[wg] * nch : 0;
  if (tid == 0) {
    nlong = 0;
    nm0 = 0;
  }
  __syncthreads();
  for (int t = tid; t < nch; t += LONG_NT) {
    if constexpr (SCATTER) {
      cur[t] = (unsigned long long)(row_off[ro + t] + wg_hist[wg * nch + t]);
      if constexpr (DS)
        if (rt_mode[ro + t] == 0) m0list[atomicAdd(&nm0, 1)] = (int16_t)t;   // (any order)
    } else {
      hist[t] = 0;
      if constexpr (DIRECT) dhist[t] = 0;
    }
  }
  __syncthreads();
  const int64_t e1 = wg_e1[wg];
  for (int64_t e = wg_e0[wg] + w; e < e1; e += NWV) {
    const int j = Aci[e];
    const float a = SCATTER ? Av[e] : 0.f;
    const int k = lidx != nullptr ? lidx[j] : -1;
    if constexpr (!SCATTER) {
      // a long B row (long_btab): its chunk histogram is the difference of
      // its chunk offsets, nch + 1 words instead of its whole column list
      if (k >= 0) {   // wave-uniform
        const uint32_t* tk = btab + (int64_t)k * (nch + 1);
        int* hh = DIRECT ? dhist : hist;
        for (int t = lane; t < nch; t += 64) {
          const int n = (int)(tk[t + 1] - tk[t]);
          if (n) atomicAdd(&hh[t], n);
        }
        if (DIRECT && lane == 0) atomicAdd(&nlong, 1);
        continue;
      }
    } else {
      if (DIRECT && k >= 0) {   // wave-uniform: listed for long_dense; routed only into mode-0 items
        const int64_t b0 = Brp[j];
        if (lane == 0) {
          const int at = atomicAdd(&nlong, 1);
          dl[dl_off[wg] + at] = make_uint4((uint32_t)b0, (uint32_t)k, __float_as_uint(a), 0u);
        }
        const int n0 = nm0;
        if (n0 == 0) continue;   // uniform: every long product of this row is direct
        const uint32_t* tk = btab + (int64_t)k * (nch + 1);
        int* own = own_all[w];
        uint2* sg = seg_all[w];
        unsigned long long* dst = dst_all[w];
        for (int t0 = 0; t0 < n0; t0 += 64) {   // lane = a mode-0 chunk: its segment of this B row
          int len = 0, t = 0;
          uint32_t s0 = 0;
          if (t0 + lane < n0) {
            t = m0list[t0 + lane];
            s0 = tk[t];
            len = (int)(tk[t + 1] - s0);
          }
          const int incl = wave_incl_scan_dpp(len);
          const int tot = __builtin_amdgcn_readlane(incl, 63);
          if (tot == 0) continue;   // uniform
          const int pre = incl - len;
          sg[lane] = make_uint2((uint32_t)b0 + s0, (uint32_t)pre);
          dst[lane] = len ? atomicAdd(&cur[t], (unsigned long long)len) : 0ull;
          for (int qw = 0; qw < tot; qw += 64) {
            const int o = wave_slot_owner(pre, len, qw, lane, own);
            const int q = qw + lane;
            if (q < tot) {
              const uint2 g = sg[o];
              const uint32_t f = g.x + (uint32_t)(q - (int)g.y);
              const int c = Bci[f];
              scratch[dst[o] + (uint32_t)(q - (int)g.y)] = ((unsigned long long)__float_as_uint(a * Bv[f]) << 32) |
                                                           (uint32_t)c;
            }
          }
          lr_wave_fence();   // seg / dst reads done before the next block's writes
        }
        continue;
      }
    }
    const int64_t b0 = Brp[j], b1 = Brp[j + 1];
    for (int64_t f0 = b0; f0 < b1; f0 += 256) {   // 4 loads in flight per lane
      int c[4];
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t f = f0 + u * 64 + lane;
        const bool ok = f < b1;
        c[u] = ok ? Bci[f] : -1;
        if constexpr (SCATTER) v[u] = ok ? Bv[f] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        // Lanes holding the same chunk form runs (a sorted B row puts ~64
        // consecutive columns in a handful of chunks): one LDS atomic per
        // run instead of 64 same-address atomics, which serialise.
        const int t = c[u] < 0 ? -1 : c[u] >> LONG_LGW;
        const int tp = __shfl_up(t, 1);
        const unsigned long long heads = __ballot(lane == 0 || t != tp);
        const unsigned long long below = heads & (~0ull >> (63 - lane));   // heads at lanes <= lane
        const int head = 63 - __clzll((long long)below);
        const unsigned long long after = heads & ~(~0ull >> (63 - lane));  // heads at lanes > lane
        const int next = after ? __ffsll((long long)after) - 1 : 64;
        if constexpr (SCATTER) {
          unsigned long long base = 0;
          if (head == lane && t >= 0) base = atomicAdd(&cur[t], (unsigned long long)(next - lane));
          base = __shfl(base, head);
          if (t >= 0)
            scratch[base + (lane - head)] = ((unsigned long long)__float_as_uint(a * v[u]) << 32) | (uint32_t)c[u];
        } else {
          if (head == lane && t >= 0) atomicAdd(&hist[t], next - lane);
        }
      }
    }
  }
  if constexpr (!SCATTER) {
    __syncthreads();
    for (int t = tid; t < nch; t += LONG_NT) {
      wg_hist[wg * nch + t] = hist[t];
      if constexpr (DIRECT) wg_dhist[wg * nch + t] = dhist[t];
    }
    if (DIRECT && tid == 0) wg_nlong[wg] = nlong;
  }
}

// Product-parallel scatter (default; SPMM_LONG_ROUTE_PP=0 selects long_route<true, false>).
// The workgroup's <= LONG_EPW A entries (one row) are expanded jointly: lane e of every wave
// holds entry e's B-row length, a DPP prefix gives each entry's first product slot, and the
// waves take 64-product windows of the concatenation round-robin, LONG_PPU windows per step
// with all their B loads in flight.  long_route<true, false> walks one A entry per wave, so a
// wave holding a hub entry (~14k products at R-MAT 24) runs on while its workgroup's other
// waves sit idle, and every entry pays four dependent load latencies (A, B row pointer, B)
// before its first product: PMC at R-MAT 24 averaged ~9 resident waves per CU and ~2000
// cycles per 256-product step.  Same slots (per-chunk LDS cursors from long_wg_scan, one
// cursor atomic per run of a chunk), same scratch records; only the order inside a
// (workgroup, chunk) run changes, which long_dense and long_rank do not depend on.
#ifndef SPMM_LONG_PPU
#define SPMM_LONG_PPU 4
#endif
constexpr int LONG_PPU = SPMM_LONG_PPU;
#ifndef SPMM_LONG_PPG
#define SPMM_LONG_PPG 64
#endif
constexpr int LONG_PPG = SPMM_LONG_PPG;   // chunks per phase of a long B row
static_assert(LONG_EPW <= 64, "one A entry per lane");

__global__ __launch_bounds__(LONG_NT) void long_route_pp(
    const int32_t* __restrict__ Aci, const float* __restrict__ Av, const int64_t* __restrict__ Brp,
    const int32_t* __restrict__ Bci, const float* __restrict__ Bv, const int64_t* __restrict__ wg_e0,
    const int64_t* __restrict__ wg_e1, int nch, int32_t* __restrict__ wg_hist,
    const int32_t* __restrict__ wg_row, const int64_t* __restrict__ row_off,
    unsigned long long* __restrict__ scratch, const int32_t* __restrict__ lidx, const uint32_t* __restrict__ btab,
    int ph_lo, int ph_hi) {
  constexpr int NWV = LONG_NT / 64;
  __shared__ unsigned long long cur[LONG_MAXCH];
  __shared__ int own_all[NWV][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#if SPMM_LONG_XCD
  const int64_t wg = spmm::xcd_remap(blockIdx.x, gridDim.x);
#else
  const int64_t wg = blockIdx.x;
#endif
  const int64_t ro = (int64_t)wg_row[wg] * nch;
  // [ph_lo, ph_hi): the phases of this launch.  One launch per phase puts every workgroup
  // on the same column group, so the B rows' segments of that group (1/8 of B at R-MAT 24,
  // ~64 MB of hub rows) stay in the MALL across rows instead of streaming from HBM per row.
  // A launch touches the cursors of its phases' chunks only and hands them to the next
  // launch through wg_hist (offsets inside the (row, chunk) regions).
  const int ngrp = lidx != nullptr ? (nch + LONG_PPG - 1) / LONG_PPG : 0;
  const int ph_end = min(ph_hi, ngrp + 1);
  const int tlo = ph_lo == 0 ? 0 : (ph_lo - 1) * LONG_PPG;
  const int thi = ph_lo == 0 ? nch : min(nch, (ph_end - 1) * LONG_PPG);
  const bool handoff = !(ph_lo == 0 && ph_end == ngrp + 1);
  for (int t = tlo + tid; t < thi; t += LONG_NT) cur[t] = (unsigned long long)(row_off[ro + t] + wg_hist[wg * nch + t]);
  const int64_t e0 = wg_e0[wg];
  const int ne = (int)(wg_e1[wg] - e0);
  int blen = 0, k = -1;
  int64_t b0 = 0;
  float a = 0.f;
  if (lane < ne) {
    const int j = Aci[e0 + lane];
    a = Av[e0 + lane];
    b0 = Brp[j];
    blen = (int)(Brp[j + 1] - b0);
    if (lidx != nullptr) k = lidx[j];
  }
  __syncthreads();
  int* own = own_all[w];
  // phase 0: entries on short B rows, whole rows; phases 1..: entries on long B rows (chunk
  // offset table), LONG_PPG chunks at a time, so a workgroup keeps ~LONG_PPG scratch runs
  // open instead of nch and their partly written lines complete in L2 (entry-major order
  // left ~nch partial lines per workgroup, 8 MB per XCD: 1.3x the bytes written at R-MAT 24)
  for (int ph = ph_lo; ph < ph_end; ++ph) {
    int64_t st = b0;
    int len = 0;
    if (ph == 0) {
      len = k < 0 ? blen : 0;
    } else if (k >= 0) {
      const uint32_t* tk = btab + (int64_t)k * (nch + 1);
      const int t0 = (ph - 1) * LONG_PPG;
      const uint32_t s0 = tk[t0];
      len = (int)(tk[min(t0 + LONG_PPG, nch)] - s0);
      st = b0 + s0;
    }
    const int incl = wave_incl_scan_dpp(len);
    const int tot = __builtin_amdgcn_readlane(incl, 63);
    if (tot == 0) continue;   // uniform
    const int pre = incl - len;
    const int nwin = (tot + 63) >> 6;
    for (int j0 = w; j0 < nwin; j0 += NWV * LONG_PPU) {
      int c[LONG_PPU];
      float v[LONG_PPU];
#pragma unroll
      for (int u = 0; u < LONG_PPU; ++u) {
        const int qw = (j0 + u * NWV) << 6;
        c[u] = -1;
        v[u] = 0.f;
        if (qw < tot) {   // uniform
          const int o = wave_slot_owner(pre, len, qw, lane, own);
          const int q = qw + lane;
          const int64_t so = ((int64_t)__shfl((int)(st >> 32), o) << 32) | (uint32_t)__shfl((int)st, o);
          const int po = __shfl(pre, o);
          const float ao = __shfl(a, o);
          if (q < tot) {
            const int64_t f = so + (q - po);
            c[u] = Bci[f];
            v[u] = ao * Bv[f];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < LONG_PPU; ++u) {
        // lanes of one chunk form runs (consecutive products of a sorted B row): one cursor
        // atomic per run
        const int t = c[u] < 0 ? -1 : c[u] >> LONG_LGW;
        const int tp = __shfl_up(t, 1);
        const unsigned long long heads = __ballot(lane == 0 || t != tp);
        const unsigned long long below = heads & (~0ull >> (63 - lane));
        const int head = 63 - __clzll((long long)below);
        const unsigned long long after = heads & ~(~0ull >> (63 - lane));
        const int next = after ? __ffsll((long long)after) - 1 : 64;
        unsigned long long base = 0;
        if (head == lane && t >= 0) base = atomicAdd(&cur[t], (unsigned long long)(next - lane));
        base = __shfl(base, head);
        if (t >= 0) scratch[base + (lane - head)] = ((unsigned long long)__float_as_uint(v[u]) << 32) | (uint32_t)c[u];
      }
    }
  }
  if (handoff) {
    __syncthreads();
    for (int t = tlo + tid; t < thi; t += LONG_NT) wg_hist[wg * nch + t] = (int32_t)(cur[t] - (unsigned long long)row_off[ro + t]);
  }
}

// Routing plan on the device (replaces a chain of torch ops over the
// [workgroups x chunks] histogram: widening copies, a transpose, cumsums,
// gathers; ~10 passes over arrays of ~2e9 entries per R-MAT 24 batch).  Per
// (row, chunk): the histogram counts of the row's workgroups (consecutive:
// wg0[r] .. wg0[r] + nwg[r]) become each workgroup's offset inside the
// (row, chunk) scratch region, in place; the routed counts go to cnt.
// Direct mode (dhist given): T = short-row products, D = long-row products;
// an item of more than LR_CAP products with D > 0 takes D directly (mode 1:
// dcnt = D, cnt = T); otherwise its long products are routed with the short
// ones under the same per-workgroup offsets (mode 0: cnt = T + D; mode 2
// when D = 0).
__global__ __launch_bounds__(256) void long_wg_scan(int32_t* __restrict__ hist, const int64_t* __restrict__ wg0,
                                                   const int64_t* __restrict__ nwg, int nch,
                                                   int64_t* __restrict__ cnt, const int32_t* __restrict__ dhist,
                                                   int64_t* __restrict__ dcnt, uint8_t* __restrict__ mode,
                                                   int64_t dmin) {
  const int64_t r = blockIdx.x;
  const int k = blockIdx.y * 256 + threadIdx.x;
  if (k >= nch) return;
  const int64_t w0 = wg0[r], w1 = w0 + nwg[r];
  bool with_long = false;
  if (dhist != nullptr) {
    int64_t T = 0, D = 0;
    for (int64_t w = w0; w < w1; ++w) {
      T += hist[w * nch + k];
      D += dhist[w * nch + k];
    }
    const uint8_t md = D == 0 ? 2 : (T + D > dmin ? 1 : 0);
    mode[r * nch + k] = md;
    dcnt[r * nch + k] = md == 1 ? D : 0;
    with_long = md == 0;
  }
  int64_t run = 0;
  for (int64_t w = w0; w < w1; ++w) {   // consecutive threads: consecutive chunks of one row (coalesced)
    const int32_t v = hist[w * nch + k] + (with_long ? dhist[w * nch + k] : 0);
    hist[w * nch + k] = (int32_t)run;
    run += v;
  }
  cnt[r * nch + k] = run;
}

// Chunk offsets of the long rows of B (the routing histogram's shortcut):
// tab[k * (nch + 1) + c] = first entry of B row lrows[k] whose column is
// >= c * W, relative to the row start (c = nch: the row length).  One thread
// per (row, chunk boundary), a binary search each.  Built once per right
// operand; a hub row of B (R-MAT: up to ~10^6 entries, referenced by as many
// A entries) then costs nch + 1 words per A entry in the histogram pass.
__global__ __launch_bounds__(256) void long_btab(const int64_t* __restrict__ Brp, const int32_t* __restrict__ Bci,
                                                 const int32_t* __restrict__ lrows, int64_t nlong, int nch,
                                                 uint32_t* __restrict__ tab) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nlong * (nch + 1)) return;
  const int64_t k = t / (nch + 1);
  const int c = (int)(t - k * (nch + 1));
  const int j = lrows[k];
  const int64_t r0 = Brp[j], r1 = Brp[j + 1];
  int64_t lo = c < nch ? r0 : r1, hi = r1;   // boundary nch: the row end
  if (c < nch) {
    const int bound = c << LONG_LGW;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (Bci[mid] < bound) lo = mid + 1; else hi = mid;
    }
  }
  tab[t] = (uint32_t)(lo - r0);
}

// Persistent: a workgroup walks (row, chunk) items rt = blockIdx.x,
// + gridDim.x, ...  At R-MAT scale 24 (2^24 columns = 1024 chunks per hub
// row) an item averages ~500 products, so the fixed per-item LDS work of a
// one-item-per-workgroup kernel (clear 64 KB, scan 512 occupancy words)
// outweighed the product atomics ~10:1.  Here the accumulator is cleared by
// the write-back itself (only occupied columns are non-zero; the 64 KB clear
// runs once per workgroup), the block scan runs on DPP instead of LDS
// permutes, empty items cost nothing, and the next item's counts and first
// scratch loads are in flight during the current write-back.
// Direct products (dt_cnt given): after an item's routed products, the row's
// long entries (dl[dl_rp[r] .. dl_rp[r + 1]) are taken in blocks of 64 (lane
// = entry: its B segment in this chunk from btab) and expanded into
// 64-product windows (wave_slot_owner); DU windows at a time are folded into
// the accumulator, their B loads in flight together.  A row of >= NW blocks
// gives each wave whole blocks; a row of fewer spreads every block's windows
// over all the waves (one hub B row can hold all of an item's products).
constexpr int LONG_DU = 4;
// long_dense item schedule: tickets (1, the default) or static items (0, diagnostic builds)
#ifndef SPMM_LONG_TICKETS
#define SPMM_LONG_TICKETS 1
#endif

template <bool VALUES, bool DIRECT>
__global__ __launch_bounds__(LONG_DNT, 2) void long_dense(const int32_t* __restrict__ list,
                                                         const int32_t* __restrict__ nlist,
                                                         const int64_t* __restrict__ rt_off,
                                                         const int64_t* __restrict__ rt_cnt, int nch,
                                                         unsigned long long* __restrict__ scratch,
                                                         int64_t* __restrict__ rt_nnz,
                                                         const int64_t* __restrict__ dt_cnt,
                                                         const uint4* __restrict__ dl,
                                                         const int64_t* __restrict__ dl_rp,
                                                         const uint32_t* __restrict__ btab,
                                                         const int32_t* __restrict__ Bci,
                                                         const float* __restrict__ Bv,
                                                         int32_t* __restrict__ ticket) {
  constexpr int NW = LONG_DNT / 64;
  __shared__ float vals[VALUES ? LONG_W : 1];
  __shared__ uint32_t bits[LONG_W / 32];
  __shared__ int wsum[LONG_DNT / 64];
  __shared__ int own_all[DIRECT ? NW : 1][64];
  __shared__ uint2 seg_all[DIRECT ? NW : 1][64];
  __shared__ float sa_all[DIRECT ? NW : 1][64];
  __shared__ int s_tk[2];
  static_assert(LONG_W / 32 == LONG_DNT, "one occupancy word per thread");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bits[tid] = 0u;
  if constexpr (VALUES)
    for (int i = tid; i < LONG_W / 4; i += LONG_DNT) reinterpret_cast<float4*>(vals)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  // the items of this kernel (long_partition: more than LR_CAP products)
  const int64_t nl = *nlist;
  // Item schedule: the first two items static (blockIdx.x, + gridDim.x), then tickets (2 G + a
  // global counter).  Items span 10^3 .. 10^7 products (R-MAT hub rows), so equal item counts
  // per workgroup are far from equal work.  Thread 0 fetches a ticket at the top of an item and
  // publishes it to LDS before the item's last barrier; it names the item after next.
  // (A zero hipcc cannot see through makes the atomic's offset look divergent: the atomic
  // optimizer would otherwise wait for it on the spot.)
  int tkz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(tkz));
  const auto rtk = __builtin_amdgcn_make_buffer_rsrc(ticket, 0, 4, 0x00020000);
  const int64_t G = gridDim.x;
  int kd = 0;   // items done by this workgroup
  int64_t it = blockIdx.x;   // position in the list
  int64_t rt = it < nl ? list[it] : -1;
  int64_t n = 0, base = 0;
  if (rt >= 0) { n = rt_cnt[rt]; base = rt_off[rt]; }
  unsigned long long x[LONG_DL];
#pragma unroll
  for (int u = 0; u < LONG_DL; ++u) {
    const int64_t i = tid + u * LONG_DNT;
    x[u] = i < n ? scratch[base + i] : ~0ull;
  }
  __syncthreads();
  while (it < nl) {
    int tk = 0;
    if (tid == 0) tk = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rtk, tkz, 0, 0);
    const int64_t it2 = (kd == 0 || !SPMM_LONG_TICKETS) ? it + G : 2 * G + __builtin_amdgcn_readfirstlane(s_tk[(kd + 1) & 1]);
    const int64_t rt2 = it2 < nl ? list[it2] : -1;   // in flight during the atomics
    const int c0 = (int)(rt % nch) << LONG_LGW;
    for (int64_t i0 = tid;;) {
      int ci[LONG_DL];
      float cv[LONG_DL];
      bool fresh[LONG_DL];
#pragma unroll
      for (int u = 0; u < LONG_DL; ++u) {
        ci[u] = x[u] == ~0ull ? -1 : (int)(uint32_t)x[u] - c0;
        cv[u] = __uint_as_float((uint32_t)(x[u] >> 32));
        fresh[u] = false;
        if (ci[u] >= 0) {
          const uint32_t bit = 1u << (ci[u] & 31);
#if SPMM_LONG_FRESH   // the first product of a column skips the slot read (the slot is +0.0)
          fresh[u] = !(atomicOr(&bits[ci[u] >> 5], bit) & bit);
#else
          atomicOr(&bits[ci[u] >> 5], bit);
#endif
        }
      }
      if constexpr (VALUES) spmm::lds_fadd_n(vals, ci, cv, fresh);
      i0 += LONG_DL * LONG_DNT;
      if (i0 >= n) break;
      // LONG_DL scratch loads in flight per lane before the LDS updates
#pragma unroll
      for (int u = 0; u < LONG_DL; ++u) {
        const int64_t i = i0 + u * LONG_DNT;
        x[u] = i < n ? scratch[base + i] : ~0ull;
      }
    }
    if (DIRECT && dt_cnt[rt] > 0) {   // uniform: direct products
      const int64_t r = rt / nch;
      const int t = (int)(rt % nch);
      const int64_t d0 = dl_rp[r], d1 = dl_rp[r + 1];
      const int nb = (int)((d1 - d0 + 63) >> 6);
      // >= NW blocks of 64 long entries: a wave per block; fewer: every wave
      // expands every block and takes every NW-th of its 64-product windows
      const bool share = nb < NW;
      int* own = own_all[w];
      uint2* sg = seg_all[w];
      float* sa = sa_all[w];
      int gwin = 0;   // (share) windows of the blocks before this one
      for (int b = share ? 0 : w; b < nb; b += share ? 1 : NW) {
        const int64_t i = d0 + ((int64_t)b << 6) + lane;
        int len = 0;
        uint32_t st = 0;
        float a = 0.f;
        if (i < d1) {
          const uint4 e = dl[i];
          const uint32_t* tk = btab + (int64_t)e.y * (nch + 1);
          const uint32_t s0 = tk[t];
          len = (int)(tk[t + 1] - s0);
          st = e.x + s0;
          a = __uint_as_float(e.z);
        }
        const int incl = wave_incl_scan_dpp(len);
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        if (tot == 0) continue;   // uniform
        const int pre = incl - len;
        const int nwin = (tot + 63) >> 6;
        sg[lane] = make_uint2(st, (uint32_t)pre);
        sa[lane] = a;
        // this wave's windows: j0, j0 + js, ... (all of them unless shared)
        const int j0 = share ? (w - gwin % NW + NW) % NW : 0;
        const int js = share ? NW : 1;
        gwin += nwin;
        for (int j = j0; j < nwin; j += js * LONG_DU) {
          uint32_t f[LONG_DU];
          float av[LONG_DU];
          bool ok[LONG_DU];
#pragma unroll
          for (int u = 0; u < LONG_DU; ++u) {
            const int q0 = (j + u * js) << 6;
            ok[u] = false;
            f[u] = 0u;
            av[u] = 0.f;
            if (q0 < tot) {   // uniform
              const int o = wave_slot_owner(pre, len, q0, lane, own);
              const int q = q0 + lane;
              if (q < tot) {
                const uint2 g = sg[o];
                f[u] = g.x + (uint32_t)(q - (int)g.y);
                av[u] = sa[o];
                ok[u] = true;
              }
            }
          }
          int cc[LONG_DU];
          float vv[LONG_DU];
#pragma unroll
          for (int u = 0; u < LONG_DU; ++u) {
            cc[u] = ok[u] ? Bci[f[u]] : -1;
            vv[u] = 0.f;
            if constexpr (VALUES) vv[u] = ok[u] ? Bv[f[u]] : 0.f;
          }
          int ci[LONG_DU];
          float cv[LONG_DU];
          bool fresh[LONG_DU];
#pragma unroll
          for (int u = 0; u < LONG_DU; ++u) {
            ci[u] = cc[u] < 0 ? -1 : cc[u] - c0;
            cv[u] = av[u] * vv[u];
            fresh[u] = false;
            if (ci[u] >= 0) atomicOr(&bits[ci[u] >> 5], 1u << (ci[u] & 31));
          }
          if constexpr (VALUES) spmm::lds_fadd_n(vals, ci, cv, fresh);
        }
        lr_wave_fence();   // seg / sa reads done before the next block's writes
      }
    }
    __syncthreads();
    // (the products' loads are all consumed here: waiting for the ticket costs nothing; it is
    // read as the item after next, after this item's last barrier)
    if (tid == 0) s_tk[kd & 1] = tk;
    int64_t n2 = 0, base2 = 0;
    if (rt2 >= 0) { n2 = rt_cnt[rt2]; base2 = rt_off[rt2]; }
    // one occupancy word per thread: its columns in order; the write-back
    // clears what it reads
    const uint32_t word = bits[tid];
    bits[tid] = 0u;
    const int cnt = __popc(word);
    const int incl = wave_incl_scan_dpp(cnt);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int pre = 0, total = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int sw = wsum[i];
      pre += (i < w) ? sw : 0;
      total += sw;
    }
    const int pos = pre + incl - cnt;
    int k = 0;
    for (uint32_t m = word; m; m &= m - 1, ++k) {
      const int b = __ffs(m) - 1;
      const int cl = tid * 32 + b;
      float v = 0.f;
      if constexpr (VALUES) { v = vals[cl]; vals[cl] = 0.f; }
      scratch[base + pos + k] = ((unsigned long long)__float_as_uint(v) << 32) | (uint32_t)(c0 + cl);
    }
    if (tid == 0) rt_nnz[rt] = total;
#pragma unroll
    for (int u = 0; u < LONG_DL; ++u) {
      const int64_t i = tid + u * LONG_DNT;
      x[u] = i < n2 ? scratch[base2 + i] : ~0ull;
    }
    it = it2; rt = rt2; n = n2; base = base2;
    ++kd;
    __syncthreads();   // write-back clears and wsum reads done before the next item's atomics / wsum writes
  }
}

// Wave-per-item long rows: most (row, chunk) items of an R-MAT hub row hold
// a few hundred products, where long_dense's fixed per-item cost (three
// workgroup barriers, a 512-word scan and write-back by 512 threads) dominates.
// Here ONE WAVE owns an item of <= LR_CAP products and runs the bitmap-rank
// scheme of csr_spgemm_bitmap.hip on it with no workgroup barrier:
//   load the item's (column | a*b) words into registers (16 per lane);
//   OR each column into the wave's 2 KB chunk bitmap (ds_or_rtn: the return
//   marks duplicates); 16-bit rank prefix per 64-bit word (4 DPP scans);
//   slot = prefix + popcount of the bits below; owners store their item,
//   duplicates add after; write-back over the item's own scratch region
//   (all its words are in registers by then), count to rt_nnz; the wave clears
//   its bitmap and takes the next item (rt += waves in the grid).
// LDS ops of one wave complete in issue order, so the phases only need the
// compiler not to move LDS accesses across them (wave-scope fences).
template <bool VALUES>
__global__ __launch_bounds__(LR_WAVES * 64) void long_rank(const int32_t* __restrict__ list,
                                                           const int32_t* __restrict__ nlist,
                                                           const int64_t* __restrict__ rt_off,
                                                           const int64_t* __restrict__ rt_cnt, int nch,
                                                           unsigned long long* __restrict__ scratch,
                                                           int64_t* __restrict__ rt_nnz) {
  __shared__ __attribute__((aligned(16))) unsigned long long bm_all[LR_WAVES][LR_WORDS];
  __shared__ __attribute__((aligned(16))) uint16_t pre_all[LR_WAVES][LR_WORDS];
  __shared__ __attribute__((aligned(16))) unsigned long long it_all[VALUES ? LR_WAVES : 1][VALUES ? LR_CAP : 1];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  unsigned long long* const bm = bm_all[w];
  uint32_t* const bm32 = reinterpret_cast<uint32_t*>(bm);
  uint16_t* const pre = pre_all[w];
  unsigned long long* const it = it_all[VALUES ? w : 0];
#pragma unroll
  for (int k = 0; k < LR_WORDS / 64; ++k) bm[k * 64 + lane] = 0ull;
  lr_wave_fence();
  const int64_t nwv = (int64_t)gridDim.x * LR_WAVES;
  const int64_t nl = *nlist;   // items of 1..LR_CAP products (long_partition)
  for (int64_t li = (int64_t)blockIdx.x * LR_WAVES + w; li < nl; li += nwv) {
    const int64_t rt = list[li];
    const int64_t n = rt_cnt[rt];
    const int64_t base = rt_off[rt];
    const uint32_t c0 = (uint32_t)(rt % nch) << LONG_LGW;
    const int nu = (int)((n + 63) >> 6);   // wave-uniform rounds
    unsigned long long x[LR_R];
#pragma unroll
    for (int u = 0; u < LR_R; ++u) {   // unconditional issue: no per-load branch
      const int64_t i = u * 64 + lane;
      x[u] = ~0ull;
      if (u < nu && i < n) x[u] = scratch[base + i];
    }
    uint32_t dupm = 0;
    {
      uint32_t old[LR_R];
#pragma unroll
      for (int u = 0; u < LR_R; ++u) {
        old[u] = 0u;
        if (x[u] != ~0ull) {
          const uint32_t c = (uint32_t)x[u] - c0;
          old[u] = atomicOr(bm32 + (c >> 5), 1u << (c & 31));
        }
      }
#pragma unroll
      for (int u = 0; u < LR_R; ++u)
        if (x[u] != ~0ull) dupm |= ((old[u] >> (((uint32_t)x[u] - c0) & 31)) & 1u) << u;
    }
    lr_wave_fence();
    int run = 0;
#pragma unroll
    for (int k = 0; k < LR_WORDS / 64; ++k) {
      const int cnt = __popcll(bm[k * 64 + lane]);
      const int incl = wave_incl_scan_dpp(cnt);
      pre[k * 64 + lane] = (uint16_t)(run + incl - cnt);
      run += __builtin_amdgcn_readlane(incl, 63);
    }
    lr_wave_fence();
    const int total = run;
    if constexpr (VALUES) {
      auto rank = [&](uint32_t c) {
        const uint32_t wd = c >> 6;
        return (int)pre[wd] + (int)__popcll(bm[wd] & ((1ull << (c & 63)) - 1ull));
      };
#pragma unroll
      for (int u = 0; u < LR_R; ++u)
        if (x[u] != ~0ull && !((dupm >> u) & 1u)) it[rank((uint32_t)x[u] - c0)] = x[u];
      if (__ballot(dupm != 0)) {   // uniform
        lr_wave_fence();
#pragma unroll
        for (int u = 0; u < LR_R; ++u)
          if ((dupm >> u) & 1u)
            atomicAdd(reinterpret_cast<float*>(&it[rank((uint32_t)x[u] - c0)]) + 1, __uint_as_float((uint32_t)(x[u] >> 32)));
      }
      lr_wave_fence();
      for (int i = lane; i < total; i += 64) scratch[base + i] = it[i];
    }
    if (lane == 0) rt_nnz[rt] = total;
#pragma unroll
    for (int k = 0; k < LR_WORDS / 64; ++k) bm[k * 64 + lane] = 0ull;
    lr_wave_fence();
  }
}

// (row, chunk) items -> the work lists of long_rank (1..small products) and
// long_dense (more); nl[0], nl[1] = their lengths (zeroed by the caller).
// Empty items get their zero count here.  The persistent kernels then walk
// only their own items: a walk over all items costs a dependent count load
// per skipped item (R-MAT 24: 82 % of the items are long_rank's).
// Items with direct products (dt_cnt > 0) always go to long_dense.
__global__ __launch_bounds__(256) void long_partition(const int64_t* __restrict__ rt_cnt, int64_t nrt, int64_t small,
                                                      int32_t* __restrict__ rank_list,
                                                      int32_t* __restrict__ dense_list, int32_t* __restrict__ nl,
                                                      int64_t* __restrict__ rt_nnz,
                                                      const int64_t* __restrict__ dt_cnt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t n = i < nrt ? rt_cnt[i] : 0;
  const int64_t dn = (i < nrt && dt_cnt != nullptr) ? dt_cnt[i] : 0;
  if (i < nrt && n == 0 && dn == 0) rt_nnz[i] = 0;
  const bool r = dn == 0 && n > 0 && n <= small;
  const bool d = dn > 0 || n > small;
  const unsigned long long mr = __ballot(r), md = __ballot(d);
  int br = 0, bd = 0;
  if (lane == 0) {
    if (mr) br = atomicAdd(&nl[0], __popcll(mr));
    if (md) bd = atomicAdd(&nl[1], __popcll(md));
  }
  br = __shfl(br, 0);
  bd = __shfl(bd, 0);
  const unsigned long long below = (1ull << lane) - 1ull;
  if (r) rank_list[br + __popcll(mr & below)] = (int32_t)i;
  if (d) dense_list[bd + __popcll(md & below)] = (int32_t)i;
}

// chunk results -> final CSR positions (one wave per (row, chunk))
__global__ __launch_bounds__(256) void long_place(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                  const int64_t* __restrict__ cnt, int64_t nrt,
                                                  const unsigned long long* __restrict__ scratch,
                                                  int32_t* __restrict__ Cci, float* __restrict__ Cv) {
  const int64_t rt = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (rt >= nrt) return;
  const int64_t s = src[rt], d = dst[rt], n = cnt[rt];
  for (int64_t i = lane; i < n; i += 64) {
    const unsigned long long x = scratch[s + i];
    Cci[d + i] = (int32_t)(uint32_t)x;
    Cv[d + i] = __uint_as_float((uint32_t)(x >> 32));
  }
}

// nprod[i] = sum over A(i,:) of nnz(B(j,:)); one wave per row.
__global__ __launch_bounds__(256) void spgemm_row_nprod(const int64_t* __restrict__ Arp,
                                                        const int32_t* __restrict__ Aci,
                                                        const int64_t* __restrict__ Brp, int64_t m,
                                                        int64_t* __restrict__ nprod) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= m) return;
  int64_t s = 0;
  for (int64_t e = Arp[row] + lane; e < Arp[row + 1]; e += 64) {
    const int j = Aci[e];
    s += Brp[j + 1] - Brp[j];
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
  if (lane == 0) nprod[row] = s;
}

// Dispatcher plan in one pass over A (replaces ~40 small PyTorch launches per
// SpGEMM call): nprod[i] as above, the ordered one-pass unit count nsl[i]
// (0 for an empty row, else 1 / 2 / 4 / 8 by the caps, torch.bucketize
// semantics: nprod <= cap1 -> 1), and per-workgroup partial statistics
// part[blockIdx][16] = {sum, max, nonempty, light (0 < nprod <= esc_min),
// #nsl==1, #nsl==2, #nsl==4, #nsl==8, max nnz of an A row, 0 x 7}, folded by
// spgemm_plan_finish (max for slots 1 and 8, sum otherwise).
constexpr int kPlanStats = 16;
__device__ __forceinline__ bool plan_is_max(int i) { return i == 1 || i == 8; }
constexpr int kPlanBlocks = 1024;

__global__ __launch_bounds__(256) void spgemm_row_plan(const int64_t* __restrict__ Arp,
                                                       const int32_t* __restrict__ Aci,
                                                       const int64_t* __restrict__ Brp, int64_t m, int64_t cap1,
                                                       int64_t cap2, int64_t cap4, int64_t esc_min,
                                                       int64_t* __restrict__ nprod, int64_t* __restrict__ nsl,
                                                       int64_t* __restrict__ part) {
  __shared__ int64_t red[4][kPlanStats];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t acc[kPlanStats] = {};
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < m; row += (int64_t)gridDim.x * 4) {
    int64_t s = 0;
    for (int64_t e = Arp[row] + lane; e < Arp[row + 1]; e += 64) {
      const int j = Aci[e];
      s += Brp[j + 1] - Brp[j];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);   // every lane holds the row total
    const int k = s == 0 ? 0 : s <= cap1 ? 1 : s <= cap2 ? 2 : s <= cap4 ? 4 : 8;
    if (lane == 0) {
      nprod[row] = s;
      nsl[row] = k;
    }
    acc[0] += s;
    acc[1] = s > acc[1] ? s : acc[1];
    acc[2] += s > 0;
    acc[3] += (s > 0) & (s <= esc_min);
    acc[4] += k == 1;
    acc[5] += k == 2;
    acc[6] += k == 4;
    acc[7] += k == 8;
    const int64_t na = Arp[row + 1] - Arp[row];
    acc[8] = na > acc[8] ? na : acc[8];
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < kPlanStats; ++i) red[wave][i] = acc[i];
  __syncthreads();
  if (threadIdx.x < kPlanStats) {
    const int i = threadIdx.x;
    int64_t v = red[0][i];
    for (int w = 1; w < 4; ++w) v = plan_is_max(i) ? (red[w][i] > v ? red[w][i] : v) : v + red[w][i];
    part[(int64_t)blockIdx.x * kPlanStats + i] = v;
  }
}

// stats[i] = fold of part[0..nb)[i] (max for i == 1, sum otherwise); one workgroup.
__global__ __launch_bounds__(256) void spgemm_plan_finish(const int64_t* __restrict__ part, int nb,
                                                          int64_t* __restrict__ stats) {
  __shared__ int64_t red[256];
  const int i = threadIdx.x & (kPlanStats - 1), r0 = threadIdx.x / kPlanStats;
  int64_t v = 0;
  for (int r = r0; r < nb; r += 256 / kPlanStats) {
    const int64_t x = part[(int64_t)r * kPlanStats + i];
    v = plan_is_max(i) ? (x > v ? x : v) : v + x;
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int h = 128; h >= kPlanStats; h >>= 1) {
    if ((int)threadIdx.x < h) {
      const int64_t x = red[threadIdx.x + h];
      red[threadIdx.x] = plan_is_max(i) ? (x > red[threadIdx.x] ? x : red[threadIdx.x]) : red[threadIdx.x] + x;
    }
    __syncthreads();
  }
  if (threadIdx.x < kPlanStats) stats[threadIdx.x] = red[threadIdx.x];
}

// Ordered one-pass units from the inclusive scan of nsl: row i owns units
// [incl[i] - nsl[i], incl[i]); unit k of s covers column eighths
// [k * 8 / s, (k + 1) * 8 / s), stored as q0 | q1 << 4.
__global__ __launch_bounds__(256) void spgemm_ordered_units(const int64_t* __restrict__ nsl,
                                                            const int64_t* __restrict__ incl, int64_t m,
                                                            int32_t* __restrict__ unit_row,
                                                            uint8_t* __restrict__ unit_q) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= m) return;
  const int s = (int)nsl[row];
  const int64_t first = incl[row] - s;
  for (int k = 0; k < s; ++k) {
    unit_row[first + k] = (int32_t)row;
    unit_q[first + k] = (uint8_t)((k * 8 / s) | (((k + 1) * 8 / s) << 4));
  }
}

template <int S, int NT, int NP>
int launch_sym(const int64_t* Arp, const int32_t* Aci, const int64_t* Brp, const int32_t* Bci, const int64_t* bsplit,
               const int32_t* rows, int64_t nrows, int ncols, int lg, int32_t* row_nnz, int32_t* flags,
               hipStream_t s) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL((spgemm_lds_sym<S, NT, NP>), dim3((unsigned)nrows), dim3(NT), 0, s, Arp, Aci, Brp, Bci, bsplit,
                     rows, ncols, lg, row_nnz, flags);
  SPMM_LAUNCH_CHECK();
  return 0;
}

template <int PCAP, int NT, int NP>
int launch_esc(const int64_t* Arp, const int32_t* Aci, const float* Av, const int64_t* Brp, const int32_t* Bci,
               const float* Bv, const int64_t* bsplit, const int32_t* rows, int64_t nrows, int ncols, int lg,
               const int32_t* row_cap, int32_t* out_nnz, const int64_t* Crp, int32_t* Cci, float* Cv,
               int32_t* flags, hipStream_t s) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL((spgemm_esc<PCAP, NT, NP>), dim3((unsigned)nrows), dim3(NT), 0, s, Arp, Aci, Av, Brp, Bci, Bv,
                     bsplit, rows, ncols, lg, row_cap, out_nnz, Crp, Cci, Cv, flags, EscOrd{});
  SPMM_LAUNCH_CHECK();
  return 0;
}

template <int S, int NT, int NP>
int launch_num(const int64_t* Arp, const int32_t* Aci, const float* Av, const int64_t* Brp, const int32_t* Bci,
               const float* Bv, const int64_t* bsplit, const int32_t* rows, int64_t nrows, int ncols, int lg,
               const int32_t* row_cap, int32_t* out_nnz, const int64_t* Crp, int32_t* Cci, float* Cv,
               int32_t* flags, hipStream_t s) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL((spgemm_lds_num<S, NT, NP>), dim3((unsigned)nrows), dim3(NT), 0, s, Arp, Aci, Av, Brp, Bci, Bv,
                     bsplit, rows, ncols, lg, row_cap, out_nnz, Crp, Cci, Cv, flags);
  SPMM_LAUNCH_CHECK();
  return 0;
}

}  // namespace

SPMM_EXPORT int spmm_spgemm_row_nprod(const int64_t* Arp, const int32_t* Aci, const int64_t* Brp, int64_t m,
                                      int64_t* nprod, void* stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(spgemm_row_nprod, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, Arp, Aci,
                     Brp, m, nprod);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Row-binning table of the binned two-phase path, the one copy for ops/spgemm.py (_bins) and
// the native engine (csr_engine.cpp): caps[b] = the most products (numeric) or the most
// distinct-key bound (symbolic) a row of bin b may have; bins 0..6 are single-pass LDS tables
// of 128 << b slots at load <= load, symbolic 7..10 the 16384-slot table over 1/2/4/8 column
// slices at load <= load_sliced, numeric 7..10 the bucketed ESC kernels (kEscPcap products
// per slice, esc_load per-slice margin from 2 slices up); beyond caps[10]: the long-row path.
// Numeric rows of more than esc_min products skip the single-pass tables.
constexpr int64_t kEscPcap = 7680;   // launch_esc<7680, ...>
// (A 15360-product top bin on 1024-thread workgroups, which keeps R-MAT rows of 55K-110K
// products off the long-row pipeline, measured slower: R-MAT 24 13.41 / 13.45 s vs 13.03 /
// 12.95 s a step, PERF_LOG round 5; removed.)
constexpr double kEscLoad = 0.9;
SPMM_EXPORT int spmm_spgemm_bin_caps(int numeric, double load, double load_sliced, int64_t esc_min, int64_t* caps) {
  for (int b = 0; b < 7; ++b) {
    const int64_t c = (int64_t)(load * (double)(128 << b));
    caps[b] = numeric ? std::min(c, esc_min) : c;
  }
  for (int k = 0; k < 4; ++k)
    caps[7 + k] = numeric ? (k == 0 ? kEscPcap : (int64_t)(kEscLoad * kEscPcap) * (1 << k))
                          : (int64_t)(load_sliced * 16384) * (1 << k);
  return 0;
}

// Constants the host planners size their buffers from: the row-plan partials
// (kPlanBlocks x kPlanStats) and the ordered one-pass caps' ESC margin.
SPMM_EXPORT int spmm_spgemm_plan_params(int* plan_blocks, int* plan_stats, double* esc_load) {
  *plan_blocks = kPlanBlocks;
  *plan_stats = kPlanStats;
  *esc_load = kEscLoad;
  return 0;
}

// nprod / nsl: [m]; part: [1024 * 16] scratch; stats: [16] (see spgemm_row_plan).
SPMM_EXPORT int spmm_spgemm_row_plan(const int64_t* Arp, const int32_t* Aci, const int64_t* Brp, int64_t m,
                                     int64_t cap1, int64_t cap2, int64_t cap4, int64_t esc_min, int64_t* nprod,
                                     int64_t* nsl, int64_t* part, int64_t* stats, void* stream) {
  if (m < 0 || !(cap1 <= cap2 && cap2 <= cap4)) return (int)hipErrorInvalidValue;
  const int64_t want = (m + 3) / 4;
  const int nb = (int)(want < kPlanBlocks ? (want > 0 ? want : 1) : kPlanBlocks);
  hipLaunchKernelGGL(spgemm_row_plan, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, Arp, Aci, Brp, m, cap1,
                     cap2, cap4, esc_min, nprod, nsl, part);
  SPMM_LAUNCH_CHECK();
  hipLaunchKernelGGL(spgemm_plan_finish, dim3(1), dim3(256), 0, (hipStream_t)stream, part, nb, stats);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// unit_row / unit_q: [incl[m - 1]] (the host sizes them from the plan's stats).
SPMM_EXPORT int spmm_spgemm_ordered_units(const int64_t* nsl, const int64_t* incl, int64_t m, int32_t* unit_row,
                                          uint8_t* unit_q, void* stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(spgemm_ordered_units, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, nsl,
                     incl, m, unit_row, unit_q);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_compact(const int64_t* src_off, const int64_t* dst_off, int64_t m, const int32_t* sci,
                                    const float* sv, int32_t* dci, float* dv, void* stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(spgemm_compact, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, src_off,
                     dst_off, m, sci, sv, dci, dv);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_row_splits(const int64_t* Brp, const int32_t* Bci, int64_t mb, int ncols,
                                       int64_t* bsplit, void* stream) {
  if (mb <= 0) return 0;
  // 8 lanes per row, one grid: gridDim.x * 256 work-items must stay below 2^32
  if (mb > ((int64_t)UINT32_MAX - 255) / 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(spgemm_row_splits, dim3((unsigned)((mb * 8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     Brp, Bci, mb, ncols, bsplit);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// LDS bins.  Every table is sized so that at least two workgroups fit a CU
// (<= 80 KB of LDS): a workgroup's phases (staging, inserts, ranking) are
// separated by barriers and their latencies only overlap with ANOTHER
// workgroup's work.  Long rows are cut into 2 / 4 / 8 column slices instead of
// using bigger tables.
//   symbolic bins 0..6: 128 << b keys, one pass; 7..10: 16384 keys x 1/2/4/8 slices
//   numeric  bins 0..6: 128 << b key/value slots, one pass (ordered hash);
//            7..10: bucketed ESC, 7680 products per slice x 1/2/4/8 slices
SPMM_EXPORT int spmm_spgemm_lds(int bin, int numeric, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                const int64_t* Brp, const int32_t* Bci, const float* Bv, const int64_t* bsplit,
                                const int32_t* rows, int64_t nrows, int ncols, int lg, int32_t* row_nnz,
                                int32_t* out_nnz, const int64_t* Crp, int32_t* Cci, float* Cv, int32_t* flags,
                                void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (lg < 4 || lg > 6) return (int)hipErrorInvalidValue;
#define SPMM_NARGS Arp, Aci, Av, Brp, Bci, Bv, bsplit, rows, nrows, ncols, lg, row_nnz, out_nnz, Crp, Cci, Cv, flags, s
#define SPMM_SARGS Arp, Aci, Brp, Bci, bsplit, rows, nrows, ncols, lg, row_nnz, flags, s
#define SPMM_BIN(B, S, NT)                                                                   \
  case B:                                                                                     \
    return numeric ? launch_num<S, NT, 1>(SPMM_NARGS) : launch_sym<S, NT, 1>(SPMM_SARGS);
  if (numeric) {
    if (bin == 7) return launch_esc<7680, 512, 1>(SPMM_NARGS);
    if (bin == 8) return launch_esc<7680, 512, 2>(SPMM_NARGS);
    if (bin == 9) return launch_esc<7680, 512, 4>(SPMM_NARGS);
    if (bin == 10) return launch_esc<7680, 512, 8>(SPMM_NARGS);
  } else {
    if (bin == 7) return launch_sym<16384, 512, 1>(SPMM_SARGS);
    if (bin == 8) return launch_sym<16384, 512, 2>(SPMM_SARGS);
    if (bin == 9) return launch_sym<16384, 512, 4>(SPMM_SARGS);
    if (bin == 10) return launch_sym<16384, 512, 8>(SPMM_SARGS);
  }
  switch (bin) {
    SPMM_BIN(0, 128, 64)
    SPMM_BIN(1, 256, 64)
    SPMM_BIN(2, 512, 128)
    SPMM_BIN(3, 1024, 128)
    SPMM_BIN(4, 2048, 256)
    SPMM_BIN(5, 4096, 256)
    SPMM_BIN(6, 8192, 512)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef SPMM_BIN
#undef SPMM_NARGS
#undef SPMM_SARGS
}


// Ordered one-pass ESC over units (see EscOrd).  ticket / status / err /
// out_nnz must be zero; unit_q holds q0 | q1 << 4.
SPMM_EXPORT int spmm_spgemm_esc_ordered(const int64_t* Arp, const int32_t* Aci, const float* Av, const int64_t* Brp,
                                        const int32_t* Bci, const float* Bv, const int64_t* bsplit,
                                        const int32_t* unit_row, const uint8_t* unit_q, int64_t nunits, int ncols,
                                        int lg, uint32_t* ticket, unsigned long long* status, int64_t cap,
                                        int32_t* err, int32_t* out_nnz, int32_t* Cci, float* Cv, int32_t* flags,
                                        int pcap, void* stream) {
  if (nunits <= 0) return 0;
  if (lg < 4 || lg > 6 || nunits > 0xffffffffll) return (int)hipErrorInvalidValue;
  EscOrd o{unit_row, unit_q, ticket, status, cap, err};
  // pcap 7680: 512-thread workgroups, 80 KB of LDS (2 per CU); pcap 3840:
  // 256 threads, 40 KB (4 per CU: twice the independent units per CU to hide
  // the staging latency and the look-back waits, same bucket density)
  if (pcap == 7680)
    hipLaunchKernelGGL((spgemm_esc<7680, 512, 2, true>), dim3((unsigned)nunits), dim3(512), 0, (hipStream_t)stream,
                       Arp, Aci, Av, Brp, Bci, Bv, bsplit, nullptr, ncols, lg, nullptr, out_nnz, nullptr, Cci, Cv,
                       flags, o);
  else if (pcap == 3840)
    hipLaunchKernelGGL((spgemm_esc<3840, 256, 2, true, 2048>), dim3((unsigned)nunits), dim3(256), 0,
                       (hipStream_t)stream, Arp, Aci, Av, Brp, Bci, Bv, bsplit, nullptr, ncols, lg, nullptr, out_nnz,
                       nullptr, Cci, Cv, flags, o);
  else
    return (int)hipErrorInvalidValue;
  SPMM_LAUNCH_CHECK();
  return 0;
}

// ---- long rows (see the kernels' comment) -----------------------------------
// Diagnostic (SPMM_LONG_ROUTE_LDS_PAD = bytes of dynamic LDS): fewer scatter
// workgroups per CU, so fewer (workgroup, chunk) write runs are open in an
// XCD's L2 at once.
static size_t route_lds_pad() {
  static const size_t pad = [] {
    const char* e = getenv("SPMM_LONG_ROUTE_LDS_PAD");
    return e ? (size_t)atoll(e) : (size_t)0;
  }();
  return pad;
}

static int route_pp() {   // 0: long_route<true, false>; 1: long_route_pp, a launch per phase; 2: one launch
  static const int on = [] {
    const char* e = getenv("SPMM_LONG_ROUTE_PP");
    return e ? atoi(e) : 1;
  }();
  return on;
}

SPMM_EXPORT int spmm_spgemm_long_route(int scatter, const int32_t* Aci, const float* Av, const int64_t* Brp,
                                       const int32_t* Bci, const float* Bv, const int64_t* wg_e0,
                                       const int64_t* wg_e1, int64_t nwg, int nch, int32_t* wg_hist,
                                       const int32_t* wg_row, const int64_t* row_off, void* scratch,
                                       const int32_t* lidx, const uint32_t* btab, int32_t* wg_dhist,
                                       int32_t* wg_nlong, const uint8_t* rt_mode, void* dl, const int64_t* dl_off,
                                       void* stream) {
  // histogram pass: wg_hist out; lidx / btab (optional): B row -> long-row
  // index or -1, and the long rows' chunk offsets (spmm_spgemm_long_btab).
  // Direct mode: wg_dhist / wg_nlong out (the long rows' counts apart).
  // scatter pass: wg_hist = per-workgroup offsets (spmm_spgemm_long_wg_scan),
  // wg_row = each workgroup's row in the batch, row_off = region bases;
  // direct mode: lidx, btab, rt_mode, dl, dl_off (see long_route).
  if (nwg <= 0) return 0;
  if (nch > LONG_MAXCH) return (int)hipErrorInvalidValue;
  if ((lidx == nullptr) != (btab == nullptr)) return (int)hipErrorInvalidValue;
  if (scatter && (wg_row == nullptr || row_off == nullptr)) return (int)hipErrorInvalidValue;
  if (!scatter && (wg_dhist != nullptr) && (lidx == nullptr || wg_nlong == nullptr)) return (int)hipErrorInvalidValue;
  if (scatter && dl != nullptr && (lidx == nullptr || rt_mode == nullptr || dl_off == nullptr))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (scatter && dl != nullptr)
    hipLaunchKernelGGL((long_route<true, true>), dim3((unsigned)nwg), dim3(LONG_NT), 0, s, Aci, Av, Brp, Bci, Bv, wg_e0,
                       wg_e1, nch, wg_hist, wg_row, row_off, (unsigned long long*)scratch, lidx, btab, nullptr, nullptr,
                       rt_mode, (uint4*)dl, dl_off);
  else if (scatter && route_pp()) {
    const int nph = lidx != nullptr ? (nch + LONG_PPG - 1) / LONG_PPG + 1 : 1;
    const int per = route_pp() == 1 ? 1 : nph;   // SPMM_LONG_ROUTE_PP=2: every phase in one launch
    for (int p0 = 0; p0 < nph; p0 += per)
      hipLaunchKernelGGL(long_route_pp, dim3((unsigned)nwg), dim3(LONG_NT), route_lds_pad(), s, Aci, Av, Brp, Bci, Bv,
                         wg_e0, wg_e1, nch, wg_hist, wg_row, row_off, (unsigned long long*)scratch, lidx, btab, p0,
                         p0 + per);
  }
  else if (scatter)
    hipLaunchKernelGGL((long_route<true, false>), dim3((unsigned)nwg), dim3(LONG_NT), route_lds_pad(), s, Aci, Av, Brp, Bci, Bv,
                       wg_e0, wg_e1, nch, wg_hist, wg_row, row_off, (unsigned long long*)scratch, nullptr, nullptr,
                       nullptr, nullptr, nullptr, nullptr, nullptr);
  else if (wg_dhist != nullptr)
    hipLaunchKernelGGL((long_route<false, true>), dim3((unsigned)nwg), dim3(LONG_NT), 0, s, Aci, Av, Brp, Bci, Bv,
                       wg_e0, wg_e1, nch, wg_hist, nullptr, nullptr, (unsigned long long*)scratch, lidx, btab,
                       wg_dhist, wg_nlong, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL((long_route<false, false>), dim3((unsigned)nwg), dim3(LONG_NT), 0, s, Aci, Av, Brp, Bci, Bv,
                       wg_e0, wg_e1, nch, wg_hist, nullptr, nullptr, (unsigned long long*)scratch, lidx, btab,
                       nullptr, nullptr, nullptr, nullptr, nullptr);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// In place: routing histogram -> per-workgroup offsets inside each (row,
// chunk) region; cnt[r * nch + k] = routed counts.  wg0 / nwg: int64 [R].
// Direct mode (dhist): dcnt = direct counts, mode = item modes (long_wg_scan).
SPMM_EXPORT int spmm_spgemm_long_wg_scan(int32_t* wg_hist, const int64_t* wg0, const int64_t* nwg, int64_t R,
                                         int nch, int64_t* cnt, const int32_t* dhist, int64_t* dcnt, uint8_t* mode,
                                         void* stream) {
  if (R <= 0) return 0;
  if (nch > LONG_MAXCH || R > (int64_t)UINT32_MAX) return (int)hipErrorInvalidValue;
  if (dhist != nullptr && (dcnt == nullptr || mode == nullptr)) return (int)hipErrorInvalidValue;
  // items of more than dmin products take their long products directly
  // (SPMM_LONG_DIRECT_MIN, default LR_CAP: the smaller ones are long_rank's)
  static const int64_t dmin = [] {
    const char* e = getenv("SPMM_LONG_DIRECT_MIN");
    return e ? (int64_t)atoll(e) : (int64_t)LR_CAP;
  }();
  hipLaunchKernelGGL(long_wg_scan, dim3((unsigned)R, (unsigned)((nch + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, wg_hist, wg0, nwg, nch, cnt, dhist, dcnt, mode, dmin);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_long_btab(const int64_t* Brp, const int32_t* Bci, const int32_t* lrows, int64_t nlong,
                                      int nch, uint32_t* tab, void* stream) {
  if (nlong <= 0) return 0;
  if (nch > LONG_MAXCH) return (int)hipErrorInvalidValue;
  const int64_t n = nlong * (nch + 1);
  hipLaunchKernelGGL(long_btab, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Brp, Bci, lrows,
                     nlong, nch, tab);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_long_dense(int values, const int64_t* rt_off, const int64_t* rt_cnt, int64_t nrt, int nch,
                                       void* scratch, int64_t* rt_nnz, int32_t* ws, const int64_t* dt_cnt,
                                       const void* dl, const int64_t* dl_rp, const uint32_t* btab, const int32_t* Bci,
                                       const float* Bv, int grid_pct, void* stream) {
  // ws: 2 * nrt + 4 int32 (the two work lists, their lengths and long_dense's item ticket counter)
  // grid_pct: share (percent) of the resident capacity the two persistent grids take -- less than
  // all when another stream's kernels (the next batch's routing) run beside them (R-MAT 24:
  // 75 % = 11.46-11.48 s, 100 % = 11.94, 50 % = 13.13; PERF_LOG round 6)
  // direct products (optional): dt_cnt per item, dl / dl_rp the batch rows'
  // long entries (long_route), btab, B
  if (nrt <= 0) return 0;
  if (nrt >= (int64_t(1) << 31)) return (int)hipErrorInvalidValue;
  if (dt_cnt != nullptr && (dl == nullptr || dl_rp == nullptr || btab == nullptr || Bci == nullptr || Bv == nullptr))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  // items of <= LR_CAP products: one wave each (long_rank); the rest: long_dense
  // (SPMM_LONG_RANK=0: every item on long_dense, for A/B runs)
  static const int use_rank = [] {
    const char* e = getenv("SPMM_LONG_RANK");
    return e && e[0] == '0' ? 0 : 1;
  }();
  const int64_t gpct = grid_pct < 1 || grid_pct > 100 ? 100 : grid_pct;
  int32_t* nl = ws;
  int32_t* ticket = ws + 2;
  int32_t* rank_list = ws + 4;
  int32_t* dense_list = ws + 4 + nrt;
  hipError_t e = hipMemsetAsync(nl, 0, 4 * sizeof(int32_t), s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(long_partition, dim3((unsigned)((nrt + 255) / 256)), dim3(256), 0, s, rt_cnt, nrt,
                     use_rank ? (int64_t)LR_CAP : int64_t(0), rank_list, dense_list, nl, rt_nnz, dt_cnt);
  SPMM_LAUNCH_CHECK();
  // persistent grids at the resident capacity (list lengths are device-side)
  if (use_rank) {
    const unsigned rgrid = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((nrt + LR_WAVES - 1) / LR_WAVES, (values ? 3 : 8) * (int64_t)ncu * gpct / 100));
    if (values)
      hipLaunchKernelGGL(long_rank<true>, dim3(rgrid), dim3(LR_WAVES * 64), 0, s, rank_list, nl, rt_off, rt_cnt, nch,
                         (unsigned long long*)scratch, rt_nnz);
    else
      hipLaunchKernelGGL(long_rank<false>, dim3(rgrid), dim3(LR_WAVES * 64), 0, s, rank_list, nl, rt_off, rt_cnt, nch,
                         (unsigned long long*)scratch, rt_nnz);
    SPMM_LAUNCH_CHECK();
  }
  auto launch = [&](auto kern) {
    int per = 0;   // resident workgroups per CU (LDS-bound with values: 132 KB at W = 2^15)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, LONG_DNT, 0) != hipSuccess || per <= 0) per = 1;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nrt, (int64_t)per * ncu * gpct / 100));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(LONG_DNT), 0, s, dense_list, nl + 1, rt_off, rt_cnt, nch,
                       (unsigned long long*)scratch, rt_nnz, dt_cnt, (const uint4*)dl, dl_rp, btab, Bci, Bv, ticket);
  };
  if (dt_cnt != nullptr) {
    if (values) launch(long_dense<true, true>);
    else launch(long_dense<false, true>);
  } else {
    if (values) launch(long_dense<true, false>);
    else launch(long_dense<false, false>);
  }
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_long_place(const int64_t* src, const int64_t* dst, const int64_t* cnt, int64_t nrt,
                                       const void* scratch, int32_t* Cci, float* Cv, void* stream) {
  if (nrt <= 0) return 0;
  hipLaunchKernelGGL(long_place, dim3((unsigned)((nrt + 3) / 4)), dim3(256), 0, (hipStream_t)stream, src, dst, cnt,
                     nrt, (const unsigned long long*)scratch, Cci, Cv);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_long_params(int* lgw, int* epw, int* maxch) {
  *lgw = LONG_LGW;
  *epw = LONG_EPW;
  *maxch = LONG_MAXCH;
  return 0;
}

// Diagnostics: enable/reset (on >= 0; bit 0 stamps, bit 1 g_nowait) or read the phase-cycle accumulators of
// spgemm_lds: [0] init+A staging, [1] product inserts, [2] rank computation,
// [3] output writes, [7] rows.
SPMM_EXPORT int spmm_spgemm_stamps(int on, unsigned long long* out8) {
  if (on >= 0) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int st = on & 1, nw = (on >> 1) & 1;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_on), &st, sizeof st);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_nowait), &nw, sizeof nw);
    return (int)e;
  }
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_stamps), 8 * sizeof(unsigned long long));
  return (int)e;
}
