// CSR x CSR SpGEMM (fp32) for gfx950: row-binned hash accumulation.
//
// North-star engine (BASELINE.json configs 2, 4, 5).  The reference has no CSR
// path at all; its tile-level analogue is the host join + per-tile kernel of
// sparse_matrix_mult.cu:140-253.
//
// Gustavson row by row, two phases:
//   symbolic: |union of B rows selected by A(i,:)| per row -> row pointer
//   numeric:  accumulate a(i,j) * b(j,c) per distinct c, write sorted columns
// Rows are binned by their intermediate-product count (symbolic) or their
// exact output count (numeric); each bin gets a kernel instantiation whose
// per-row hash table lives in LDS (up to 16K key/value slots = 128 KiB, one
// 1024-thread workgroup per CU).  Rows too long for LDS (R-MAT hubs) use the
// same algorithm with the table in an HBM workspace.
//
// Sorted output without a sort: the hash is MONOTONE in the column,
// h(c) = floor(c * S / ncols), with forward linear probing into an overflow
// tail.  A key can only land in a cluster (run of occupied slots) that starts
// at or after its home slot, so every key of an earlier cluster is smaller:
// a key's output position is (#occupied slots before its cluster) + (#smaller
// keys inside its cluster), computed independently per slot.  A probe that
// wraps past the table end sets a per-row flag; the row is then emitted in
// slot order and re-sorted by the host (not observed at the bin load factors,
// but correctness does not depend on it).
#include "common.hpp"

namespace {

constexpr int EMPTY = -1;

// Diagnostic phase stamps (off unless the host sets g_stamp_on): thread 0 of
// every workgroup adds the shader-clock cycles of each phase, measured between
// the workgroup barriers that delimit it.  Read with spmm_spgemm_stamps().
__device__ int g_stamp_on = 0;
__device__ int g_diag_mode = 0;   // diagnostics only: 1 = skip inserts, 2 = synthetic keys (no B loads)
__device__ unsigned long long g_stamps[8];
#define SPMM_STAMP(i)                                                              \
  do {                                                                             \
    if (stamp_on && threadIdx.x == 0) {                                            \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();                  \
      atomicAdd(&g_stamps[i], _t - t_prev);                                        \
      t_prev = _t;                                                                 \
    }                                                                              \
  } while (0)

template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* wsum, int* total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    int s = wsum[i];
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
// LDS-resident table.  S = hash range, TS = S + NT slots (the overflow tail lets
// probes run forward without wrapping) + 4 EMPTY sentinels so cluster scans can
// read 4 keys per step unguarded.
//
// Product stream: the row's A entries (<= NT per batch) are staged in LDS with
// their B row start and an exclusive prefix of B row lengths; the row's
// intermediate products are then split into one contiguous range per wave and
// walked 64 at a time (lane = product), so every lane is busy whatever the B
// row lengths, B reads are coalesced, and D products per lane are fetched per
// batch with the next batch's loads in flight while the current one is
// inserted (register double buffer) to cover HBM latency.
//
// Sorted output (numeric): position of the key in slot s = (#occupied slots
// before its cluster) + (#keys of its cluster that are smaller) — the monotone
// hash guarantees keys of earlier clusters are smaller.  Every occupied slot
// computes its rank independently (no serial per-cluster sort).

__device__ __forceinline__ int advance(const int* apre, int nb, int e, int p) {
  // largest e' >= e with apre[e'] <= p  (apre[nb] > p)
  if (apre[e + 1] > p) return e;
  int lo = e + 1, step = 1, hi;
  while (true) {
    const int nx = lo + step;
    if (nx >= nb || apre[nx] > p) { hi = nx < nb ? nx : nb; break; }
    lo = nx;
    step <<= 1;
  }
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (apre[mid] <= p) lo = mid; else hi = mid;
  }
  return lo;
}

template <int S, int NT, bool NUMERIC, int NP>
__global__ __launch_bounds__(NT) void spgemm_lds(
    const int64_t* __restrict__ Arp, const int32_t* __restrict__ Aci, const float* __restrict__ Av,
    const int64_t* __restrict__ Brp, const int32_t* __restrict__ Bci, const float* __restrict__ Bv,
    const int64_t* __restrict__ bsplit, const int32_t* __restrict__ rows, int ncols,
    int32_t* __restrict__ row_nnz, const int64_t* __restrict__ Crp, int32_t* __restrict__ Cci,
    float* __restrict__ Cv, int32_t* __restrict__ flags) {
  constexpr int TS = S + NT;            // multiple of 4 (S, NT powers of two >= 64)
  constexpr int PER = TS / NT;
  constexpr int NW = NT / 64;
  constexpr int ACAP = NT;
  constexpr int QSTEP = 8 / NP;         // eighths of the column space per slice
  // products per lane per fetch batch: deep where LDS already caps occupancy at
  // one workgroup per CU, shallow (fewer VGPRs, more waves) for small tables
  constexpr int D = NUMERIC ? 4 : ((NT >= 512) ? 8 : 4);
  __shared__ __attribute__((aligned(16))) int keys[TS + 4];
  __shared__ __attribute__((aligned(16))) float vals[NUMERIC ? TS : 4];
  __shared__ int64_t abeg[ACAP];
  __shared__ int apre[ACAP + 1];
  __shared__ float aval[NUMERIC ? ACAP : 1];
  __shared__ int wsum[NW];
  __shared__ int s_count, s_wrapped;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform
  const int row = rows[blockIdx.x];
  const int64_t a0 = Arp[row], na = Arp[row + 1] - a0;
  const int stamp_on = g_stamp_on;
  const int diag = g_diag_mode;
  unsigned long long t_prev = stamp_on ? __builtin_amdgcn_s_memtime() : 0ull;
  int written = 0;      // numeric: entries of earlier slices already stored
  int row_count = 0;    // symbolic: distinct columns over all slices

  for (int sl = 0; sl < NP; ++sl) {
    // column slice [clo, chi) and its monotone hash
    const int q0 = sl * QSTEP, q1 = q0 + QSTEP;
    const int clo = (int)(((int64_t)q0 * ncols) >> 3), chi = (int)(((int64_t)q1 * ncols) >> 3);
    const uint32_t mult = hash_mult(S, chi - clo);
    for (int i = tid; i < (TS + 4) / 4; i += NT) reinterpret_cast<int4*>(keys)[i] = make_int4(EMPTY, EMPTY, EMPTY, EMPTY);
    if constexpr (NUMERIC) {
      for (int i = tid; i < TS / 4; i += NT) reinterpret_cast<float4*>(vals)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid == 0) { s_count = 0; s_wrapped = 0; }
    int mine = 0;
    int64_t slice_products = 0;
    bool overflow = false;

    for (int64_t bat = 0; bat < na; bat += ACAP) {
      const int nb = (int)((na - bat) < ACAP ? (na - bat) : ACAP);
      __syncthreads();  // init done / previous batch consumed
      int len = 0;
      if (tid < nb) {
        const int j = Aci[a0 + bat + tid];
        const int64_t rb = Brp[j], re = Brp[j + 1];
        const int64_t b0 = (NP == 1 || q0 == 0) ? rb : bsplit[(int64_t)j * 7 + q0 - 1];
        const int64_t b1 = (NP == 1 || q1 == 8) ? re : bsplit[(int64_t)j * 7 + q1 - 1];
        len = (int)(b1 - b0);
        abeg[tid] = b0;
        if constexpr (NUMERIC) aval[tid] = Av[a0 + bat + tid];
      }
      int tot;
      const int pre = block_excl_scan<NT>(len, wsum, &tot);
      if (tid < nb) apre[tid] = pre;
      if (tid == 0) apre[nb] = tot;
      __syncthreads();
      SPMM_STAMP(0);
      // Distinct keys <= products: a slice whose products could exceed the
      // table is handed to the HBM path instead (a full table would never
      // terminate a probe).
      slice_products += tot;
      if (slice_products > TS - 8) { overflow = true; break; }

      // This wave's contiguous share of the products; lane takes D consecutive
      // products per batch with its current A entry cached in registers.
      int nlog = 0;
      while ((1 << nlog) < nb) ++nlog;   // binary-search depth over nb entries (uniform)
      const int Q = (tot + NW - 1) / NW;
      const int pbeg = w * Q;
      const int pend = (pbeg + Q < tot) ? pbeg + Q : tot;
      const int nbat = (pend > pbeg) ? (pend - pbeg + 64 * D - 1) / (64 * D) : 0;
      if (nbat > 0) {
        int cA[D], cB[D];
        float bA[D], bB[D], aA[D], aB[D];
        auto fetch = [&](int bt, int (&c)[D], float (&bv)[D], float (&av)[D]) {
          // entry of each product: D independent binary searches over apre with a
          // wave-uniform trip count (no divergent per-lane advance loops)
          int64_t f[D];
          int lo[D], hi[D], pp[D];
          const int p0 = pbeg + (bt * 64 + lane) * D;
#pragma unroll
          for (int u = 0; u < D; ++u) {
            pp[u] = (p0 + u < pend) ? p0 + u : pend - 1;   // clamp: always a valid product
            lo[u] = 0;
            hi[u] = nb;
          }
          for (int it = 0; it < nlog; ++it) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
              const int mid = (lo[u] + hi[u]) >> 1;
              if (apre[mid] <= pp[u]) lo[u] = mid; else hi[u] = mid;
            }
          }
#pragma unroll
          for (int u = 0; u < D; ++u) {
            f[u] = abeg[lo[u]] + (pp[u] - apre[lo[u]]);
            if constexpr (NUMERIC) av[u] = aval[lo[u]];
          }
          if (diag == 2) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
              c[u] = clo + (int)__umulhi((uint32_t)(f[u] * 2654435761ull), (uint32_t)(chi - clo));
              if constexpr (NUMERIC) bv[u] = 1.f;
            }
            return;
          }
#pragma unroll
          for (int u = 0; u < D; ++u) {
            c[u] = Bci[f[u]];
            if constexpr (NUMERIC) bv[u] = Bv[f[u]];
          }
        };
        auto consume = [&](int bt, const int (&c)[D], const float (&bv)[D], const float (&av)[D]) {
          const int p0 = pbeg + (bt * 64 + lane) * D;
          if (diag == 1) {   // keep the loaded values live, skip the table
#pragma unroll
            for (int u = 0; u < D; ++u) mine ^= (p0 + u < pend) ? (c[u] & 1) : 0;
            return;
          }
          // CAS-only linear probing in rounds over the lane's D keys: a CAS of
          // EMPTY -> key both claims a free slot and reports the occupant
          // (one LDS op per probe step; ds_cmpst costs ~11 cycles per
          // wave-instruction on gfx950, a read + CAS pair ~17).  A key u is
          // only touched while some lane still has it pending.
          int h[D], st[D];
#pragma unroll
          for (int u = 0; u < D; ++u) {
            const int hk = c[u] - clo;
            h[u] = mult ? (int)__umulhi((uint32_t)hk, mult) : hk;
            st[u] = (p0 + u < pend) ? 1 : 0;   // 1 = pending
          }
          while (true) {
            bool more = false;
#pragma unroll
            for (int u = 0; u < D; ++u) {
              if (__any(st[u] != 0)) {
                if (st[u]) {
                  const int old = atomicCAS(&keys[h[u]], EMPTY, c[u]);
                  if (old == EMPTY) { ++mine; st[u] = 0; }
                  else if (old == c[u]) st[u] = 0;
                  else if (++h[u] >= TS) { h[u] = 0; s_wrapped = 1; }
                }
                more |= st[u] != 0;
              }
            }
            if (!__any(more)) break;
          }
          if constexpr (NUMERIC) {
            // float accumulate by read + CAS (ds_add_f32 serialises lanes: ~192
            // cycles per wave-instruction measured on gfx950)
            int ob[D];
            bool pendv[D];
#pragma unroll
            for (int u = 0; u < D; ++u) {
              pendv[u] = p0 + u < pend;
              ob[u] = pendv[u] ? __hip_atomic_load(reinterpret_cast<int*>(&vals[h[u]]), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
            }
            while (true) {
              bool again = false;
#pragma unroll
              for (int u = 0; u < D; ++u) {
                if (pendv[u]) {
                  const int nv = __float_as_int(__int_as_float(ob[u]) + av[u] * bv[u]);
                  const int o = atomicCAS(reinterpret_cast<int*>(&vals[h[u]]), ob[u], nv);
                  if (o == ob[u]) pendv[u] = false;
                  else { ob[u] = o; again = true; }
                }
              }
              if (!__any(again)) break;
            }
          }
        };
        fetch(0, cA, bA, aA);
        for (int bt = 0; bt < nbat; bt += 2) {
          fetch(bt + 1, cB, bB, aB);
          consume(bt, cA, bA, aA);
          fetch(bt + 2, cA, bA, aA);
          consume(bt + 1, cB, bB, aB);
        }
      }
    }
    if (overflow) {
      if (tid == 0) flags[row] |= 2;
      return;   // uniform: every thread saw the same slice_products
    }
    __syncthreads();
    SPMM_STAMP(1);
    if (mine) atomicAdd(&s_count, mine);
    if constexpr (!NUMERIC) {
      __syncthreads();
      row_count += s_count;
      continue;
    } else {
      // Sorted positions.  Windows of 64 slots (one wave-instruction each):
      // occupancy ballots give per-window counts (scanned into apre, free now)
      // and each key's cluster start without walking; the rank inside the
      // cluster is a scan of the cluster (lanes of one cluster read the same
      // addresses: LDS broadcast).
      constexpr int NWIN = TS / 64;
      constexpr int WPW = (NWIN + NW - 1) / NW;   // windows per wave, kept in registers
      int kq[WPW];
      float vq[WPW];
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        const int W = w + j * NW;
        kq[j] = (W < NWIN) ? keys[W * 64 + lane] : EMPTY;
        vq[j] = (W < NWIN) ? vals[W * 64 + lane] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        const int W = w + j * NW;
        const unsigned long long M = __ballot(kq[j] != EMPTY);
        if (lane == 0 && W < NWIN) apre[W] = __popcll(M);
      }
      __syncthreads();
      int total;
      {
        const int cw = (tid < NWIN) ? apre[tid] : 0;
        const int bw = block_excl_scan<NT>(cw, wsum, &total);
        __syncthreads();
        if (tid < NWIN) apre[tid] = bw;
      }
      __syncthreads();
      const bool wrapped = s_wrapped != 0;
      const int64_t base = Crp[row] + written;
      // symbolic fixed the row's size; never store past it whatever happened here
      const int room = row_nnz[row] - written;
      const int lim = total < room ? total : room;
      if (tid == 0 && total > room) flags[row] |= 4;
      const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
      const int rlo = lane & ~15;   // first lane of this lane's 16-lane DPP row
#pragma unroll
      for (int j = 0; j < WPW; ++j) {
        const int W = w + j * NW;
        if (W < NWIN) {
          const int key = kq[j];
          const unsigned long long M = __ballot(key != EMPTY);
          // neighbours inside the 16-lane row (DPP row shifts, no LDS traffic)
          const int m1 = __builtin_amdgcn_update_dpp(EMPTY, key, 0x111, 0xF, 0xF, false);
          const int m2 = __builtin_amdgcn_update_dpp(EMPTY, key, 0x112, 0xF, 0xF, false);
          const int m3 = __builtin_amdgcn_update_dpp(EMPTY, key, 0x113, 0xF, 0xF, false);
          const int p1 = __builtin_amdgcn_update_dpp(EMPTY, key, 0x101, 0xF, 0xF, false);
          const int p2 = __builtin_amdgcn_update_dpp(EMPTY, key, 0x102, 0xF, 0xF, false);
          const int p3 = __builtin_amdgcn_update_dpp(EMPTY, key, 0x103, 0xF, 0xF, false);
          if (key != EMPTY) {
            int pos;
            if (wrapped) {
              pos = apre[W] + __popcll(M & below);
            } else {
              const unsigned long long zb = ~M & below;                       // empty slots below me
              const unsigned long long za = ~M & ~(below | (1ull << lane));   // empty slots above me
              const int ci = zb ? 64 - __builtin_clzll(zb) : -1;              // cluster start lane (-1: before window)
              const int ce = za ? __builtin_ctzll(za) : 64;                   // cluster end lane (64: past window)
              int Pcs, cs;
              if (ci >= 0) {
                cs = W * 64 + ci;
                Pcs = apre[W] + __popcll(M & (ci ? (~0ull >> (64 - ci)) : 0ull));
              } else {
                cs = W * 64;
                while (cs > 0 && keys[cs - 1] != EMPTY) --cs;
                Pcs = apre[W] - (W * 64 - cs);
              }
              int r = 0;
              if (ci >= rlo && ce < 64 && ce <= rlo + 16 && ce - ci <= 4) {   // whole cluster within 3 lanes, same row
                r += (lane - 1 >= ci) & (m1 < key);
                r += (lane - 2 >= ci) & (m2 < key);
                r += (lane - 3 >= ci) & (m3 < key);
                r += (lane + 1 < ce) & (p1 < key);
                r += (lane + 2 < ce) & (p2 < key);
                r += (lane + 3 < ce) & (p3 < key);
              } else {   // long or boundary-crossing cluster: scan it in LDS
                int x = cs;
                while (true) {
                  const int k0 = keys[x], k1 = keys[x + 1], k2 = keys[x + 2], k3 = keys[x + 3];
                  if (k0 == EMPTY) break;
                  r += k0 < key;
                  if (k1 == EMPTY) break;
                  r += k1 < key;
                  if (k2 == EMPTY) break;
                  r += k2 < key;
                  if (k3 == EMPTY) break;
                  r += k3 < key;
                  x += 4;
                }
              }
              pos = Pcs + r;
            }
            if (pos >= 0 && pos < lim) {
              Cci[base + pos] = key;
              Cv[base + pos] = vq[j];
            } else {
              flags[row] |= 4;   // internal error: never write outside the row
            }
          }
        }
      }
      SPMM_STAMP(2);
      written += total;
      if (tid == 0 && wrapped) flags[row] |= 1;
      SPMM_STAMP(3);
      __syncthreads();   // copy-out done before the next slice re-initialises the table
    }
  }
  if (stamp_on && tid == 0) atomicAdd(&g_stamps[7], 1ull);
  if constexpr (!NUMERIC) {
    if (tid == 0) row_nnz[row] = row_count;
  }
}

// Eighth split points of every B row (rows column-sorted): bsplit[j*7 + q-1] =
// first index of row j whose column >= floor(q * ncols / 8), q = 1..7.
__global__ __launch_bounds__(256) void spgemm_row_splits(const int64_t* __restrict__ Brp,
                                                         const int32_t* __restrict__ Bci, int64_t mb, int ncols,
                                                         int64_t* __restrict__ bsplit) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= mb) return;
  const int64_t lo0 = Brp[j], hi0 = Brp[j + 1];
  int64_t lo = lo0;
#pragma unroll
  for (int q = 1; q <= 7; ++q) {
    const int bound = (int)(((int64_t)q * ncols) >> 3);
    int64_t hi = hi0;   // first index with col >= bound (search starts at the previous split)
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (Bci[mid] < bound) lo = mid + 1; else hi = mid;
    }
    bsplit[j * 7 + q - 1] = lo;
  }
}

// ---------------------------------------------------------------------------
// HBM-resident table for rows beyond the LDS bins.  One 1024-thread workgroup
// per row; table (keys + vals, TS slots each) at ws_off[b] in the workspace,
// pre-filled with EMPTY / 0 by the host.  Every table access is an atomic or
// an agent-scope relaxed load, so no L1 staleness can creep in.
constexpr int GNT = 1024;

template <bool NUMERIC>
__global__ __launch_bounds__(GNT) void spgemm_global(
    const int64_t* __restrict__ Arp, const int32_t* __restrict__ Aci, const float* __restrict__ Av,
    const int64_t* __restrict__ Brp, const int32_t* __restrict__ Bci, const float* __restrict__ Bv,
    const int32_t* __restrict__ rows, const int64_t* __restrict__ ws_off, const int64_t* __restrict__ ws_size,
    int32_t* __restrict__ ws_keys, float* __restrict__ ws_vals, int ncols, int32_t* __restrict__ row_nnz,
    const int64_t* __restrict__ Crp, int32_t* __restrict__ Cci, float* __restrict__ Cv,
    int32_t* __restrict__ unsorted) {
  constexpr int NW = GNT / 64;
  __shared__ int wsum[NW];
  __shared__ int s_count, s_wrapped;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row = rows[blockIdx.x];
  const int64_t TS = ws_size[blockIdx.x];
  const int64_t S = TS - GNT;
  int32_t* keys = ws_keys + ws_off[blockIdx.x];
  float* vals = ws_vals + ws_off[blockIdx.x];
  if (tid == 0) { s_count = 0; s_wrapped = 0; }
  __syncthreads();
  const uint32_t mult = hash_mult(S, ncols);
  int mine = 0;
  const int64_t a0 = Arp[row], a1 = Arp[row + 1];
  for (int64_t e = a0 + w; e < a1; e += NW) {
    const int j = Aci[e];
    const float a = NUMERIC ? Av[e] : 0.f;
    for (int64_t f = Brp[j] + lane; f < Brp[j + 1]; f += 64) {
      const int c = Bci[f];
      int64_t h = hash_home(c, mult);
      while (true) {
        int k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == c) break;
        if (k == EMPTY) {
          int old = atomicCAS(&keys[h], EMPTY, c);
          if (old == EMPTY) { ++mine; break; }
          if (old == c) break;
        }
        if (++h == TS) { h = 0; s_wrapped = 1; }
      }
      if (NUMERIC) atomicAdd(&vals[h], a * Bv[f]);
    }
  }
  if (!NUMERIC) {
    if (mine) atomicAdd(&s_count, mine);
    __syncthreads();
    if (tid == 0) row_nnz[row] = s_count;
    return;
  }
  __syncthreads();
  auto ld = [](const int32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto ldf = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto st = [](int32_t* p, int32_t x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto stf = [](float* p, float x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int64_t s = tid; s < TS; s += GNT) {
    if (ld(&keys[s]) != EMPTY && (s == 0 || ld(&keys[s - 1]) == EMPTY)) {
      int64_t e = s;
      while (e + 1 < TS && ld(&keys[e + 1]) != EMPTY) ++e;
      for (int64_t i = s + 1; i <= e; ++i) {
        const int kk = ld(&keys[i]);
        const float vv = ldf(&vals[i]);
        int64_t q = i - 1;
        while (q >= s && ld(&keys[q]) > kk) { st(&keys[q + 1], ld(&keys[q])); stf(&vals[q + 1], ldf(&vals[q])); --q; }
        st(&keys[q + 1], kk);
        stf(&vals[q + 1], vv);
      }
    }
  }
  __syncthreads();
  const int64_t per = (TS + GNT - 1) / GNT;
  const int64_t s0 = tid * per, s1 = (s0 + per < TS) ? s0 + per : TS;
  int cnt = 0;
  for (int64_t s = s0; s < s1; ++s) cnt += ld(&keys[s]) != EMPTY;
  int total;
  int o = block_excl_scan<GNT>(cnt, wsum, &total);
  const int64_t base = Crp[row] + o;
  int64_t q = 0;
  for (int64_t s = s0; s < s1; ++s) {
    const int k = ld(&keys[s]);
    if (k != EMPTY) { Cci[base + q] = k; Cv[base + q] = ldf(&vals[s]); ++q; }
  }
  if (tid == 0 && s_wrapped) unsorted[row] = 1;
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

template <int S, int NT, bool NUMERIC, int NP>
int launch_lds(const int64_t* Arp, const int32_t* Aci, const float* Av, const int64_t* Brp, const int32_t* Bci,
               const float* Bv, const int64_t* bsplit, const int32_t* rows, int64_t nrows, int ncols,
               int32_t* row_nnz, const int64_t* Crp, int32_t* Cci, float* Cv, int32_t* flags, hipStream_t s) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL((spgemm_lds<S, NT, NUMERIC, NP>), dim3((unsigned)nrows), dim3(NT), 0, s, Arp, Aci, Av, Brp,
                     Bci, Bv, bsplit, rows, ncols, row_nnz, Crp, Cci, Cv, flags);
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

SPMM_EXPORT int spmm_spgemm_row_splits(const int64_t* Brp, const int32_t* Bci, int64_t mb, int ncols,
                                       int64_t* bsplit, void* stream) {
  if (mb <= 0) return 0;
  hipLaunchKernelGGL(spgemm_row_splits, dim3((unsigned)((mb + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Brp,
                     Bci, mb, ncols, bsplit);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// LDS bins.  Every table is sized so that at least two workgroups fit a CU
// (<= 80 KB of LDS): a workgroup's phases (staging, inserts, ranking) are
// separated by barriers and their latencies only overlap with ANOTHER
// workgroup's work.  Long rows are cut into 2 / 4 / 8 column slices instead of
// using bigger tables.
//   symbolic bins 0..6: 128 << b keys, one pass; 7..10: 16384 keys x 1/2/4/8 slices
//   numeric  bins 0..6: 128 << b key/value slots, one pass; 7..9: 8192 slots x 2/4/8 slices
SPMM_EXPORT int spmm_spgemm_lds(int bin, int numeric, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                const int64_t* Brp, const int32_t* Bci, const float* Bv, const int64_t* bsplit,
                                const int32_t* rows, int64_t nrows, int ncols, int32_t* row_nnz, const int64_t* Crp,
                                int32_t* Cci, float* Cv, int32_t* flags, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define SPMM_ARGS Arp, Aci, Av, Brp, Bci, Bv, bsplit, rows, nrows, ncols, row_nnz, Crp, Cci, Cv, flags, s
#define SPMM_BIN(B, S, NT)                                                                   \
  case B:                                                                                     \
    return numeric ? launch_lds<S, NT, true, 1>(SPMM_ARGS) : launch_lds<S, NT, false, 1>(SPMM_ARGS);
  if (numeric) {
    if (bin == 7) return launch_lds<8192, 512, true, 2>(SPMM_ARGS);
    if (bin == 8) return launch_lds<8192, 512, true, 4>(SPMM_ARGS);
    if (bin == 9) return launch_lds<8192, 512, true, 8>(SPMM_ARGS);
  } else {
    if (bin == 7) return launch_lds<16384, 512, false, 1>(SPMM_ARGS);
    if (bin == 8) return launch_lds<16384, 512, false, 2>(SPMM_ARGS);
    if (bin == 9) return launch_lds<16384, 512, false, 4>(SPMM_ARGS);
    if (bin == 10) return launch_lds<16384, 512, false, 8>(SPMM_ARGS);
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
#undef SPMM_ARGS
}

SPMM_EXPORT int spmm_spgemm_global(int numeric, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                   const int64_t* Brp, const int32_t* Bci, const float* Bv, const int32_t* rows,
                                   int64_t nrows, const int64_t* ws_off, const int64_t* ws_size, int32_t* ws_keys,
                                   float* ws_vals, int ncols, int32_t* row_nnz, const int64_t* Crp, int32_t* Cci,
                                   float* Cv, int32_t* unsorted, void* stream) {
  if (nrows <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (numeric)
    hipLaunchKernelGGL(spgemm_global<true>, dim3((unsigned)nrows), dim3(GNT), 0, s, Arp, Aci, Av, Brp, Bci, Bv,
                       rows, ws_off, ws_size, ws_keys, ws_vals, ncols, row_nnz, Crp, Cci, Cv, unsorted);
  else
    hipLaunchKernelGGL(spgemm_global<false>, dim3((unsigned)nrows), dim3(GNT), 0, s, Arp, Aci, Av, Brp, Bci, Bv,
                       rows, ws_off, ws_size, ws_keys, ws_vals, ncols, row_nnz, Crp, Cci, Cv, unsorted);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Diagnostics: enable/reset (on >= 0) or read the phase-cycle accumulators of
// spgemm_lds: [0] init+A staging, [1] product inserts, [2] rank computation,
// [3] output writes, [7] rows.
SPMM_EXPORT int spmm_spgemm_stamps(int on, unsigned long long* out8) {
  if (on >= 0) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int st = on & 1, mode = on >> 1;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_on), &st, sizeof st);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_diag_mode), &mode, sizeof mode);
    return (int)e;
  }
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_stamps), 8 * sizeof(unsigned long long));
  return (int)e;
}
