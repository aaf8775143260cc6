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

template <int S, int NT, bool NUMERIC>
__global__ __launch_bounds__(NT) void spgemm_lds(
    const int64_t* __restrict__ Arp, const int32_t* __restrict__ Aci, const float* __restrict__ Av,
    const int64_t* __restrict__ Brp, const int32_t* __restrict__ Bci, const float* __restrict__ Bv,
    const int32_t* __restrict__ rows, int ncols, int32_t* __restrict__ row_nnz,
    const int64_t* __restrict__ Crp, int32_t* __restrict__ Cci, float* __restrict__ Cv,
    int32_t* __restrict__ unsorted) {
  constexpr int TS = S + NT;
  constexpr int PER = TS / NT;
  constexpr int NW = NT / 64;
  constexpr int ACAP = NT;
  // products per lane per fetch batch: deep where LDS already caps occupancy at
  // one workgroup per CU, shallow (fewer VGPRs, more waves) for small tables
  constexpr int D = (NT >= 512) ? (NUMERIC ? 6 : 8) : 4;
  __shared__ int keys[TS + 4];
  __shared__ float vals[NUMERIC ? TS : 1];
  __shared__ int64_t abeg[ACAP];
  __shared__ int apre[ACAP + 1];
  __shared__ float aval[NUMERIC ? ACAP : 1];
  __shared__ int wsum[NW];
  __shared__ int s_count, s_wrapped;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform
  const int row = rows[blockIdx.x];
  for (int s = tid; s < TS + 4; s += NT) keys[s] = EMPTY;
  if constexpr (NUMERIC) {
    for (int s = tid; s < TS; s += NT) vals[s] = 0.f;
  }
  if (tid == 0) { s_count = 0; s_wrapped = 0; }

  const uint32_t mult = hash_mult(S, ncols);
  int mine = 0;
  const int64_t a0 = Arp[row], na = Arp[row + 1] - a0;

  for (int64_t bat = 0; bat < na; bat += ACAP) {
    const int nb = (int)((na - bat) < ACAP ? (na - bat) : ACAP);
    __syncthreads();  // init done / previous batch consumed
    int len = 0;
    if (tid < nb) {
      const int j = Aci[a0 + bat + tid];
      const int64_t b0 = Brp[j];
      len = (int)(Brp[j + 1] - b0);
      abeg[tid] = b0;
      if constexpr (NUMERIC) aval[tid] = Av[a0 + bat + tid];
    }
    int tot;
    const int pre = block_excl_scan<NT>(len, wsum, &tot);
    if (tid < nb) apre[tid] = pre;
    if (tid == 0) apre[nb] = tot;
    __syncthreads();

    const int Q = (((tot + NW - 1) / NW) + 63) & ~63;
    const int pbeg = w * Q;
    const int pend = (pbeg + Q < tot) ? pbeg + Q : tot;
    // Batches of D products per lane (lane-strided by 64: coalesced B reads),
    // double-buffered: the loads of batch t+1 are issued before batch t is
    // inserted.  All loads are unconditional (addresses clamped to a valid
    // product) and all branches around them wave-uniform, so the compiler
    // emits a counted vmcnt instead of draining per load.
    const int nbat = (pend > pbeg) ? (pend - pbeg + 64 * D - 1) / (64 * D) : 0;
    if (nbat > 0) {
      int e_is = 0;
      int cA[D], cB[D];
      float bA[D], bB[D], aA[D], aB[D];
      auto fetch = [&](int bt, int (&c)[D], float (&bv)[D], float (&av)[D]) {
        int64_t f[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
          int pp = pbeg + (bt * D + u) * 64 + lane;
          pp = pp < pend ? pp : pend - 1;
          e_is = advance(apre, nb, e_is, pp);
          f[u] = abeg[e_is] + (pp - apre[e_is]);
          if constexpr (NUMERIC) av[u] = aval[e_is];
        }
#pragma unroll
        for (int u = 0; u < D; ++u) {
          c[u] = Bci[f[u]];
          if constexpr (NUMERIC) bv[u] = Bv[f[u]];
        }
      };
      auto consume = [&](int bt, const int (&c)[D], const float (&bv)[D], const float (&av)[D]) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          if (pbeg + (bt * D + u) * 64 + lane < pend) {
            const int key = c[u];
            int h = hash_home(key, mult);
            while (true) {
              // LDS-typed relaxed load (a volatile generic pointer would become a
              // flat_load, whose vmcnt(0) drains the prefetched B loads)
              const int kv = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (kv == key) break;
              if (kv == EMPTY) {
                const int old = atomicCAS(&keys[h], EMPTY, key);
                if (old == EMPTY) { ++mine; break; }
                if (old == key) break;
              }
              if (++h == TS) { h = 0; s_wrapped = 1; }
            }
            if constexpr (NUMERIC) atomicAdd(&vals[h], av[u] * bv[u]);
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
  __syncthreads();
  if constexpr (!NUMERIC) {
    if (mine) atomicAdd(&s_count, mine);
    __syncthreads();
    if (tid == 0) row_nnz[row] = s_count;
  } else {
    const int s0 = tid * PER;
    int kb[PER], pos[PER];
    float vb[PER];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      kb[q] = keys[s0 + q];
      vb[q] = vals[s0 + q];
      cnt += kb[q] != EMPTY;
    }
    int total;
    const int P0 = block_excl_scan<NT>(cnt, wsum, &total);
    const bool wrapped = s_wrapped != 0;
    if (!wrapped) {
      int cs = s0, Pcs = P0;
      if (kb[0] != EMPTY) {
        while (cs > 0 && keys[cs - 1] != EMPTY) --cs;
        Pcs = P0 - (s0 - cs);
      }
      int lp = 0;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        pos[q] = -1;
        if (kb[q] != EMPTY) {
          if (q > 0 && kb[q - 1] == EMPTY) { cs = s0 + q; Pcs = P0 + lp; }
          const int key = kb[q];
          int r = 0, i = cs;
          while (true) {
            const int k0 = keys[i], k1 = keys[i + 1], k2 = keys[i + 2], k3 = keys[i + 3];
            if (k0 == EMPTY) break;
            r += k0 < key;
            if (k1 == EMPTY) break;
            r += k1 < key;
            if (k2 == EMPTY) break;
            r += k2 < key;
            if (k3 == EMPTY) break;
            r += k3 < key;
            i += 4;
          }
          pos[q] = Pcs + r;
          ++lp;
        }
      }
    } else {  // a probe wrapped: emit slot order, the host re-sorts this row
      int lp = 0;
#pragma unroll
      for (int q = 0; q < PER; ++q) pos[q] = (kb[q] != EMPTY) ? P0 + lp++ : -1;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (pos[q] >= 0) { keys[pos[q]] = kb[q]; vals[pos[q]] = vb[q]; }
    }
    __syncthreads();
    const int64_t base = Crp[row];
    for (int i = tid; i < total; i += NT) {
      Cci[base + i] = keys[i];
      Cv[base + i] = vals[i];
    }
    if (tid == 0 && wrapped) unsorted[row] = 1;
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

template <int S, int NT, bool NUMERIC>
int launch_lds(const int64_t* Arp, const int32_t* Aci, const float* Av, const int64_t* Brp, const int32_t* Bci,
               const float* Bv, const int32_t* rows, int64_t nrows, int ncols, int32_t* row_nnz,
               const int64_t* Crp, int32_t* Cci, float* Cv, int32_t* unsorted, hipStream_t s) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL((spgemm_lds<S, NT, NUMERIC>), dim3((unsigned)nrows), dim3(NT), 0, s, Arp, Aci, Av, Brp, Bci,
                     Bv, rows, ncols, row_nnz, Crp, Cci, Cv, unsorted);
  SPMM_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// Bin b uses table range S = 128 << b (b = 0..8 symbolic, 0..7 numeric).
SPMM_EXPORT int spmm_spgemm_lds_max_bin(int numeric) { return numeric ? 7 : 8; }

SPMM_EXPORT int spmm_spgemm_row_nprod(const int64_t* Arp, const int32_t* Aci, const int64_t* Brp, int64_t m,
                                      int64_t* nprod, void* stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(spgemm_row_nprod, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, Arp, Aci,
                     Brp, m, nprod);
  SPMM_LAUNCH_CHECK();
  return 0;
}

SPMM_EXPORT int spmm_spgemm_lds(int bin, int numeric, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                const int64_t* Brp, const int32_t* Bci, const float* Bv, const int32_t* rows,
                                int64_t nrows, int ncols, int32_t* row_nnz, const int64_t* Crp, int32_t* Cci,
                                float* Cv, int32_t* unsorted, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define SPMM_BIN(B, S, NT)                                                                                    \
  case B:                                                                                                      \
    return numeric ? launch_lds<S, NT, true>(Arp, Aci, Av, Brp, Bci, Bv, rows, nrows, ncols, row_nnz, Crp,     \
                                             Cci, Cv, unsorted, s)                                             \
                   : launch_lds<S, NT, false>(Arp, Aci, Av, Brp, Bci, Bv, rows, nrows, ncols, row_nnz, Crp,    \
                                              Cci, Cv, unsorted, s);
  switch (bin) {
    SPMM_BIN(0, 128, 64)
    SPMM_BIN(1, 256, 64)
    SPMM_BIN(2, 512, 128)
    SPMM_BIN(3, 1024, 128)
    SPMM_BIN(4, 2048, 256)
    SPMM_BIN(5, 4096, 256)
    SPMM_BIN(6, 8192, 512)
    SPMM_BIN(7, 16384, 1024)
    case 8:
      if (numeric) return (int)hipErrorInvalidValue;
      return launch_lds<32768, 1024, false>(Arp, Aci, Av, Brp, Bci, Bv, rows, nrows, ncols, row_nnz, Crp, Cci, Cv,
                                            unsorted, s);
    default:
      return (int)hipErrorInvalidValue;
  }
#undef SPMM_BIN
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
