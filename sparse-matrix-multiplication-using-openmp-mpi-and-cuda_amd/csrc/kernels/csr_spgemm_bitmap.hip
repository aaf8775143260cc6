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
// row come from one binary-search kernel (bm_window_splits), uint32 indices.
#include "common.hpp"

#include <type_traits>

namespace {

// 64-lane inclusive prefix sum on the DPP network (VALU only; no LDS
// traffic): row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15 / 31.
__device__ __forceinline__ int bm_wave_incl(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
  return x;
}

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

__device__ __forceinline__ int bm_wave_sum(int x) {
  return __builtin_amdgcn_readlane(bm_wave_incl(x), 63);
}

__device__ __forceinline__ int64_t bm_rfl64(int64_t x) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
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
  int32_t* err;            // bit 0: a deferred unit exceeds the reload budget (host falls back)
                           // bit 1: count / numeric disagree (kernel invariant)
                           // bit 2: deferred list full (host falls back)
};

template <int LGW, int NSUB, int NT, int PCAP, int R, int CCAP, int MODE>
__global__ __launch_bounds__(NT, 4) void spgemm_bm(BmArgs p) {
  using Gm = BmGeom<LGW, NSUB, NT, PCAP, R, CCAP, MODE>;
  constexpr int NW = NT / 64;
  constexpr bool VALUES = MODE != 0;
  constexpr int NWORD = Gm::NWORD, WPW = Gm::WPW, WPT = Gm::WPT;
  constexpr int RR = MODE == 1 ? R : (MODE == 0 ? 16 : 8);   // rounds of loads in flight per block

  // LDS.  bm: the window's column bitmap.  pre16: exclusive rank prefix of
  // every 64-bit word.  items: (column, value) of every output slot.
  // desc: chunk descriptors {first B index, valid lanes, a(i, j) bits}.
  __shared__ __attribute__((aligned(16))) unsigned long long bm[NWORD];
  __shared__ __attribute__((aligned(16))) uint16_t pre16[VALUES ? NWORD : 1];
  __shared__ __attribute__((aligned(16))) unsigned long long items[VALUES ? PCAP : 1];
  using Desc = typename std::conditional<VALUES, uint4, uint2>::type;
  __shared__ __attribute__((aligned(16))) Desc desc[CCAP];
  __shared__ int wsum[NW];
  __shared__ int scnt[NSUB];
  __shared__ int sdup;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = p.lg;
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

  // bitmap clear: 16-byte stores, consecutive lanes on consecutive slots (conflict-free)
  auto clear_bm = [&]() {
    for (int i = tid; i < Gm::NCLR; i += NT) reinterpret_cast<uint4*>(bm)[i] = make_uint4(0, 0, 0, 0);
  };
  clear_bm();
  if (tid < NSUB) scnt[tid] = 0;
  if (tid == 0) sdup = 0;

  // Unit schedule.  Count / numeric: static and persistent; iteration k of
  // workgroup g takes unit k * gridDim + perm(g), perm putting consecutive
  // units (the windows of one row: same A row, neighbouring B lines) on one
  // XCD (blocks b and b + 8 share one; speed only).  Reload: the deferred list.
  const int64_t nsw = MODE == 0 ? (nwin + NSUB - 1) / NSUB : nwin;   // units per row
  int64_t nunits = MODE == 2 ? (int64_t)__hip_atomic_load(p.novf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : p.m * nsw;
  if (MODE == 2 && nunits > p.ovf_cap) nunits = p.ovf_cap;
  const int64_t NG = gridDim.x;
  const int64_t me = (MODE != 2 && NG % 8 == 0) ? (int64_t)(blockIdx.x % 8) * (NG / 8) + blockIdx.x / 8
                                                : (int64_t)blockIdx.x;
  // (row, window) of consecutive slots by carries, not divisions
  const int64_t step_row = NG / nsw;
  const int step_q = (int)(NG - step_row * nsw);

  // ---- software pipeline over this workgroup's units ----------------------
  // Unit k+2: row pointer loads (s1) at the top of unit k.  Unit k+1: its A
  // entries and output offsets (s2) at the top of unit k, its window bounds
  // (s3) after unit k's first B pass.  So unit k+1's staging finds every
  // input in registers; each link of the Arp -> Aci -> ws chain has a whole
  // phase to land.
  struct Head {   // wave-uniform identity of a unit
    int64_t slot, u, row;
    int qi;       // unit index inside its row
  };
  auto first_head = [&](int64_t slot) {
    Head h{slot, 0, 0, 0};
    if (slot < nunits) {
      h.u = MODE == 2 ? (int64_t)p.ovf[slot] : slot;
      h.row = h.u / nsw;
      h.qi = (int)(h.u - h.row * nsw);
    }
    return h;
  };
  auto next_head = [&](const Head& h) {
    if constexpr (MODE == 2) return first_head(h.slot + NG);
    Head n{h.slot + NG, h.u + NG, h.row + step_row, h.qi + step_q};
    if (n.qi >= nsw) {
      n.qi -= (int)nsw;
      ++n.row;
    }
    return n;
  };
  Head h1 = first_head(me);
  Head h2 = next_head(h1);   // units k+1 and k+2
  auto q0_of = [&](const Head& h) { return h.qi * (MODE == 0 ? NSUB : 1); };
  auto q1_of = [&](const Head& h) { return MODE == 0 ? min(h.qi * NSUB + NSUB, nwin) : h.qi + 1; };
  int64_t r1a = 0, r1b = 0, r2a = 0, r2b = 0;   // Arp[row], Arp[row + 1] (vector registers)
  int64_t o1a = 0, o1b = 0;                     // uoff[u], uoff[u + 1] of unit k+1
  int j1 = 0;
  float av1 = 0.f;
  uint32_t b01 = 0, b11 = 0;
  auto s1 = [&](const Head& h, int64_t& ra, int64_t& rb) {
    if (h.slot < nunits) {
      ra = p.Arp[h.row + vz];
      rb = p.Arp[h.row + 1 + vz];
    }
  };
  auto s2 = [&]() {
    if (h1.slot < nunits) {
      const int64_t a0 = bm_rfl64(r1a), na = bm_rfl64(r1b) - a0;
      if (tid < na) {
        j1 = p.Aci[a0 + tid];
        if constexpr (VALUES) av1 = p.Av[a0 + tid];
      }
      if constexpr (VALUES) {
        o1a = p.uoff[h1.u + vz];
        o1b = p.uoff[h1.u + 1 + vz];
      }
    }
  };
  auto s3 = [&]() {
    if (h1.slot < nunits) {
      const int64_t a0 = bm_rfl64(r1a), na = bm_rfl64(r1b) - a0;
      if (tid < na) {
        const uint32_t* wr = p.ws + (int64_t)j1 * nw1;
        b01 = wr[q0_of(h1)];
        b11 = wr[q1_of(h1)];
      }
    }
  };
  s1(h1, r1a, r1b);
  s1(h2, r2a, r2b);
  s2();
  s3();
  __syncthreads();

  // Products of chunk rounds [i0, i0 + RR) of this lane group: one 16-byte
  // descriptor read (a broadcast inside the group) and the B loads of the
  // rounds that exist (wave-uniform guards), every load before any use.
  int c[RR];
  float v[RR];
  auto fetch = [&](int i0, int nr, int TC, int clo) {
    uint32_t f[RR];
    float a[RR];
    uint32_t okm = 0;
#pragma unroll
    for (int d = 0; d < RR; ++d) {
      f[d] = 0;
      a[d] = 0.f;
      if (i0 + d < nr) {   // wave-uniform
        const int t = gid + (i0 + d) * ngrp;
        const Desc ds = desc[t < TC ? t : TC - 1];
        const bool ok = (t < TC) & ((uint32_t)gl < ds.y);
        okm |= (ok ? 1u : 0u) << d;
        f[d] = ds.x + (ok ? (uint32_t)gl : 0u);
        if constexpr (VALUES) a[d] = __uint_as_float(reinterpret_cast<const uint4&>(ds).z);
      }
    }
    int x[RR];
    float b[RR];
#pragma unroll
    for (int d = 0; d < RR; ++d) {
      x[d] = 0;
      b[d] = 0.f;
      if (i0 + d < nr) {   // wave-uniform
        x[d] = p.Bci[f[d]];
        if constexpr (VALUES) b[d] = p.Bv[f[d]];
      }
    }
#pragma unroll
    for (int d = 0; d < RR; ++d) {
      c[d] = ((okm >> d) & 1u) ? x[d] - clo : -1;
      if constexpr (VALUES) v[d] = a[d] * b[d];
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

  while (h1.slot < nunits) {
    // ---- take unit k from the pipeline registers; start k+1 / k+2 loads ----
    const Head h = h1;
    const int64_t a0 = bm_rfl64(r1a), na = bm_rfl64(r1b) - a0;
    const int64_t off = bm_rfl64(o1a), want = bm_rfl64(o1b) - off;
    const float av0 = av1;
    const uint32_t b00 = b01, b10 = b11;
    h1 = h2;
    r1a = r2a;
    r1b = r2b;
    h2 = next_head(h2);
    s1(h2, r2a, r2b);
    s2();
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
            b0 = b00;
            len = (int)(b10 - b00);
          } else {
            const uint32_t* wr = p.ws + (int64_t)p.Aci[a0 + bat + tid] * nw1;
            b0 = wr[q0];
            len = (int)(wr[q1] - b0);
          }
          nch = (len + Gl - 1) >> lg;
        }
        int TCall, Pb;
        const int pre = bm_scan<NT>(nch, wsum, &TCall);
        __syncthreads();
        bm_scan<NT>(len, wsum, &Pb);
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
      s3();
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
    } else {
      // ---- numeric staging: the whole row in one batch, from registers -----
      int len = 0, nch = 0;
      if (tid < na && tid < NT) {
        len = (int)(b10 - b00);
        nch = (len + Gl - 1) >> lg;
      }
      // one scan of (products, chunks): len < 2^16 is checked below through P
      const bool big = len >= 65536;
      int both;
      const int pk = bm_scan<NT>(big ? 0 : ((len << 16) | nch), wsum, &both);
      const int pre = pk & 0xffff;
      const int TC = both & 0xffff;
      const int P = (int)((uint32_t)both >> 16);
      const bool any_big = __syncthreads_or(big);
      if (P == 0 && !any_big) {   // uniform; the count kernel wrote 0 for this unit
        s3();
        continue;
      }
      const bool too_big = any_big || na > NT || P > PCAP || TC > CCAP || (MODE == 1 && TC > R * ngrp);
      if (too_big) {   // uniform
        if (tid == 0) {
          if (MODE == 1) {
            const uint32_t at = atomicAdd(p.novf, 1u);
            if ((int64_t)at < p.ovf_cap) p.ovf[at] = (int32_t)h.u;
            else atomicOr(p.err, 4);
          } else {
            atomicOr(p.err, 1);
          }
        }
        s3();
        continue;
      }
      for (int kk = 0; kk < nch; ++kk) {
        const int rem = len - (kk << lg);
        Desc dd{};
        dd.x = b00 + ((uint32_t)kk << lg);
        dd.y = (uint32_t)(rem < Gl ? rem : Gl);
        reinterpret_cast<uint4&>(dd).z = __float_as_uint(av0);
        desc[pre + kk] = dd;
      }
      __syncthreads();
      // ---- pass 1: products into registers, columns into the bitmap -------
      const int nr = (TC + ngrp - 1) / ngrp;
      uint32_t dupm = 0;
      if constexpr (MODE == 1) {
        fetch(0, nr, TC, clo);
        s3();
        dupm = or_all();
      } else {
        for (int i0 = 0; i0 < nr; i0 += RR) {
          fetch(i0, nr, TC, clo);
          or_all();
        }
        s3();
      }
      if (dupm) sdup = 1;
      __syncthreads();
      // ---- rank prefix per 64-bit word: wave w owns words [w*WPW, (w+1)*WPW)
      int run[WPT];
      int wtot = 0;
#pragma unroll
      for (int kk = 0; kk < WPT; ++kk) {
        const int cnt = __popcll(bm[w * WPW + kk * 64 + lane]);
        const int incl = bm_wave_incl(cnt);
        run[kk] = wtot + incl - cnt;
        wtot += __builtin_amdgcn_readlane(incl, 63);
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
#pragma unroll
      for (int kk = 0; kk < WPT; ++kk) pre16[w * WPW + kk * 64 + lane] = (uint16_t)(base + run[kk]);
      if (tid == 0) sdup = 0;
      __syncthreads();
      // ---- pass 2: rank -> slot; owners store (column, value), duplicates
      // add their value after a barrier (bit set by an earlier product)
      auto rank = [&](int cc) {
        const int wd = cc >> 6;
        return (int)pre16[wd] + __popcll(bm[wd] & ((1ull << (cc & 63)) - 1ull));
      };
      if constexpr (MODE == 1) {
        // ranks of 4 rounds at a time (their LDS reads in flight together)
#pragma unroll
        for (int d0 = 0; d0 < RR; d0 += 4) {
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
      } else {
        // reload: B re-read; every product adds into a zeroed slot
        for (int i = tid; i < total; i += NT) items[i] = 0ull;
        __syncthreads();
        for (int i0 = 0; i0 < nr; i0 += RR) {
          fetch(i0, nr, TC, clo);
#pragma unroll
          for (int d = 0; d < RR; ++d) {
            if (c[d] >= 0) {
              const int rr = rank(c[d]);
              reinterpret_cast<uint32_t*>(&items[rr])[0] = (uint32_t)(c[d] + clo);
              atomicAdd(reinterpret_cast<float*>(&items[rr]) + 1, v[d]);
            }
          }
        }
      }
      __syncthreads();
      // ---- the unit's slots to C at its final offset; clear the bitmap -----
      int lim = total;
      if (want != total) {   // count and numeric disagree: never write outside the unit
        if (tid == 0) atomicOr(p.err, 2);
        lim = total < want ? total : (int)want;
      }
      for (int i = tid; i < lim; i += NT) {
        const unsigned long long it = items[i];
        p.Cci[off + i] = (int32_t)(uint32_t)it;
        p.Cv[off + i] = __uint_as_float((uint32_t)(it >> 32));
      }
      clear_bm();
      __syncthreads();   // cleared (and items read) before the next unit's pass 1
    }
  }
}

// ws[j * (nwin + 1) + q] = first index of B row j whose column >= q * 2^lgw
// (q = 0: row start, q = nwin: row end).  One thread per (row, q).
__global__ __launch_bounds__(256) void bm_window_splits(const int64_t* __restrict__ Brp,
                                                        const int32_t* __restrict__ Bci, int64_t mb, int lgw,
                                                        int nwin, uint32_t* __restrict__ ws) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nw1 = nwin + 1;
  if (t >= mb * nw1) return;
  const int64_t j = t / nw1;
  const int q = (int)(t - j * nw1);
  int64_t lo = Brp[j], hi = Brp[j + 1];
  if (q == 0) {
    hi = lo;
  } else if (q == nwin) {
    lo = hi;
  } else {
    const int64_t bound = (int64_t)q << lgw;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)Bci[mid] < bound) lo = mid + 1; else hi = mid;
    }
  }
  ws[t] = (uint32_t)lo;
}

// ---- configurations -------------------------------------------------------
// Every fast kernel: 256 threads and <= 40 KB of LDS, so four workgroups
// (16 waves, 128 VGPRs each) share a CU; count and reload kernels take most
// of a CU's LDS.
//   cfg 0: W = 2^17 (1M columns at ~105 nnz per row: ~1.4k products per window)
//          count 8 windows per unit (128 KB bitmap, 1024 threads)
//          fast  <= 2048 products, 12 register rounds
//   cfg 1: W = 2^15 (65536 columns at ~65 nnz per row: ~2.1k per window)
//          count 2 windows (8 KB, 512 threads); fast <= 3840 products, 16 rounds
//   cfg 2: W = 2^16: count 4 windows (32 KB, 1024 threads); fast <= 3072, 16 rounds
// Reload (deferred units): min(1024, W / 64) threads, <= 12288 products, 2048 chunks.
struct BmCfg {
  int lgw, nsub_count, pcap_fast, rounds_fast;
};
constexpr BmCfg kCfgs[] = {{17, 8, 2048, 12}, {15, 2, 3840, 16}, {16, 4, 3072, 16}};
constexpr int kNumCfgs = 3;
constexpr int kFastNT = 256, kReloadPcap = 12288, kReloadCcap = 2048;
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
  static constexpr int kReloadNT = reload_nt(K.lgw);
  static constexpr auto reload = spgemm_bm<K.lgw, 1, kReloadNT, kReloadPcap, 8, kReloadCcap, 2>;
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

template <int C>
int bm_numeric(int64_t work, const BmArgs& a, hipStream_t s) {
  const int rc = launch_bm(BmKernels<C>::fast, kFastNT, work, a, s);
  return rc ? rc : launch_bm(BmKernels<C>::reload, BmKernels<C>::kReloadNT, int64_t(1) << 30, a, s);
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

SPMM_EXPORT int spmm_spgemm_bm_splits(const int64_t* Brp, const int32_t* Bci, int64_t mb, int lgw, int nwin,
                                      uint32_t* ws, void* stream) {
  if (mb <= 0) return 0;
  const int64_t n = mb * (nwin + 1);
  if (nwin < 1 || lgw < 6 || lgw > 30 || n > (int64_t)UINT32_MAX - 255) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_window_splits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Brp, Bci,
                     mb, lgw, nwin, ws);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Count kernel: ucnt[m * nwin] = exact nnz of every (row, window) unit.
SPMM_EXPORT int spmm_spgemm_bm_count(int cfg, const int64_t* Arp, const int32_t* Aci, const uint32_t* ws,
                                     const int32_t* Bci, int64_t m, int nwin, int lg, int32_t* ucnt, int32_t* err,
                                     void* stream) {
  if (m <= 0) return 0;
  if (lg < 4 || lg > 6 || cfg < 0 || cfg >= kNumCfgs || nwin < 1) return (int)hipErrorInvalidValue;
  BmArgs a{Arp, Aci, nullptr, ws, Bci, nullptr, m, nwin, lg, ucnt, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
           err};
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
SPMM_EXPORT int spmm_spgemm_bm_numeric(int cfg, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                       const uint32_t* ws, const int32_t* Bci, const float* Bv, int64_t m, int nwin,
                                       int lg, const int64_t* uoff, int32_t* Cci, float* Cv, int32_t* ovf,
                                       uint32_t* novf, int64_t ovf_cap, int32_t* err, void* stream) {
  if (m <= 0) return 0;
  if (lg < 4 || lg > 6 || cfg < 0 || cfg >= kNumCfgs || nwin < 1) return (int)hipErrorInvalidValue;
  BmArgs a{Arp, Aci, Av, ws, Bci, Bv, m, nwin, lg, nullptr, uoff, Cci, Cv, ovf, novf, ovf_cap, err};
  hipStream_t s = (hipStream_t)stream;
  const int64_t work = m * nwin;
  switch (cfg) {
    case 0: return bm_numeric<0>(work, a, s);
    case 1: return bm_numeric<1>(work, a, s);
    default: return bm_numeric<2>(work, a, s);
  }
}
