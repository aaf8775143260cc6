// Layout kernels for the right operand B of the bitmap-rank SpGEMM
// (csr_spgemm_bitmap.hip): window bounds inside every B row (binary search),
// the packed 16-bit window lengths (ws8) of the row kernels, B's padded
// layouts (every (row, window) pair segment and every (row, count group)
// column segment starting on a 128-byte line, so the kernels gather them 16
// bytes per lane), and the pack / unpack of an all-gathered operand payload
// (models/spgemm.py).
#include "bitmap_common.hpp"
#include "bitmap_plan.hpp"
#include "common.hpp"

using namespace spmm_bitmap;

namespace {

// B entry access for the layout kernels: the contiguous arrays, or the gathered
// panels in place (SpmmBmGathered).  begin(j) fixes the panel of row j (a loop
// over the W panel bounds); col(e) / val(e) then take B's global entry index.
struct BView {
  const int32_t* col;
  const uint32_t* val;
  SpmmBmGathered g;
  const uint32_t* pc = nullptr;   // row's panel: its column / value words, its first entry
  const uint32_t* pv = nullptr;
  int64_t e0 = 0;
  __device__ void begin(int64_t j) {
    if (!g.gc) return;
    int r = 0;
    while (r + 1 < g.W && g.rbase[r + 1] <= j) ++r;
    pc = g.gc + (int64_t)r * g.cstride;
    pv = g.gv ? g.gv + (int64_t)r * g.vstride : nullptr;
    e0 = g.ebase[r];
  }
  __device__ uint32_t c(int64_t e) const {
    if (!g.gc) return (uint32_t)col[e];
    const int64_t i = e - e0;
    if (g.bits >= 32) return pc[i];
    const int64_t o = i * g.bits;   // two aligned words hold the entry (the sender pads one word)
    const uint64_t two = (uint64_t)pc[(o >> 5) + 1] << 32 | pc[o >> 5];
    return (uint32_t)(two >> (o & 31)) & ((1u << g.bits) - 1u);
  }
  __device__ uint32_t v(int64_t e) const { return g.gc ? pv[e - e0] : val[e]; }
};

// ws8[j] from ws (nwin <= 8): first index + 16-bit window lengths; err bit 3
// if a window segment of some B row is 65536 entries or longer.  plen (if
// given): the row's length in the padded pair array (segments rounded up to
// 2^kPadLg pairs).
__global__ __launch_bounds__(256) void bm_pack_ws8(const uint32_t* __restrict__ ws, int64_t mb, int nwin,
                                                   uint4* __restrict__ ws8, int32_t* __restrict__ err,
                                                   int64_t* __restrict__ plen, int64_t* __restrict__ plen_c, int gc) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= mb) return;
  const uint32_t* wr = ws + j * (nwin + 1);
  uint32_t l[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool bad = false;
  int64_t pl = 0, pc = 0;
  for (int q = 0; q < nwin; ++q) {
    const uint32_t d = wr[q + 1] - wr[q];
    bad |= d > 0xffffu;
    l[q] = d & 0xffffu;
    pl += (((int64_t)d + (1 << kPadLg) - 1) >> kPadLg) << kPadLg;
  }
  for (int q = 0; q < nwin; q += gc) {   // count groups of gc windows
    const int64_t d = (int64_t)wr[q + gc < nwin ? q + gc : nwin] - wr[q];
    pc += ((d + (1 << kPadCLg) - 1) >> kPadCLg) << kPadCLg;
  }
  if (bad) atomicOr(err, 8);
  ws8[2 * j] = make_uint4(wr[0], l[0] | (l[1] << 16), l[2] | (l[3] << 16), l[4] | (l[5] << 16));
  ws8[2 * j + 1] = make_uint4(l[6] | (l[7] << 16), 0u, 0u, 0u);
  if (plen) plen[j] = pl;
  if (plen_c) plen_c[j] = pc;
}

// Padded pair array: one wave per B row copies its (column, value) pairs to
// row base pbase[j] + the padded start of each window (padding slots are left
// as they are: the kernels never read a padded slot as a product), and stores
// the base in ws8[2j + 1].y.
__global__ __launch_bounds__(256) void bm_pad_pairs(const uint32_t* __restrict__ ws, BView B, int64_t mb, int nwin,
                                                    int lgw, const int64_t* __restrict__ pbase, uint4* __restrict__ ws8,
                                                    uint2* __restrict__ out, const int64_t* __restrict__ cbase,
                                                    int gc, int32_t* __restrict__ outc, int64_t cap, int64_t cap_c,
                                                    int32_t* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (j >= mb) return;
  B.begin(j);
  const uint32_t* wr = ws + j * (nwin + 1);
  const uint32_t w = lane <= nwin ? wr[lane] : 0u;   // lane q: first index of window q (q = nwin: row end)
  const int64_t base = out ? pbase[j] : 0, cb = outc ? cbase[j] : 0;
  if (lane == 0) {
    uint32_t* x = reinterpret_cast<uint32_t*>(&ws8[2 * j + 1]);
    if (out) x[1] = (uint32_t)base;
    if (outc) x[2] = (uint32_t)cb;
  }
  // padded start of window q (lane q): exclusive scan of the rounded lengths;
  // an entry of window q goes to e + dp[q] (dp = padded start - first index)
  const uint32_t wn = __shfl_down(w, 1);
  const uint32_t rl = lane < nwin ? ((wn - w + (1u << kPadLg) - 1) >> kPadLg) << kPadLg : 0u;
  const uint32_t ps = (uint32_t)bm_wave_incl((int)rl) - rl;
  const uint32_t dp = ps - w;
  // padded start of count group g (lane g): windows [g gc, (g + 1) gc)
  const int ng = (nwin + gc - 1) / gc;
  const uint32_t g0 = (uint32_t)__shfl(w, lane * gc < nwin ? lane * gc : nwin);
  const uint32_t g1 = (uint32_t)__shfl(w, (lane + 1) * gc < nwin ? (lane + 1) * gc : nwin);
  const uint32_t rc = lane < ng ? ((g1 - g0 + (1u << kPadCLg) - 1) >> kPadCLg) << kPadCLg : 0u;
  const uint32_t pc = (uint32_t)bm_wave_incl((int)rc) - rc;
  const uint32_t dc = pc - g0;
  // entry loop with a wave-uniform trip count; an entry's window is its
  // column >> lgw (B's rows are column-sorted), so its destination needs ONE
  // lane shuffle per layout (round 4: seven window-bound compares and two
  // shuffles per layout)
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)w);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)w, nwin);
  for (uint32_t e0 = r0; e0 < r1; e0 += 64) {
    const uint32_t e = e0 + lane;
    const bool ok = e < r1;
    const uint32_t c = ok ? B.c(e) : 0u;
    const int q = (int)(c >> lgw);
    if (out) {
      const int64_t d = base + (uint32_t)(e + (uint32_t)__shfl((int)dp, q));
      if (ok) {
        if (d < cap) out[d] = make_uint2(c, B.v(e));
        else atomicOr(err, 32);   // (a layout bug, never a write out of bounds)
      }
    }
    if (outc) {
      const int64_t d = cb + (uint32_t)(e + (uint32_t)__shfl((int)dc, q / gc));
      if (ok) {
        if (d < cap_c) outc[d] = (int32_t)c;
        else atomicOr(err, 32);
      }
    }
  }
}

// ws[j * (nwin + 1) + q] = first index of B row j whose column >= q * 2^lgw
// (q = 0: row start, q = nwin: row end).  One thread per (row, q).
__global__ __launch_bounds__(256) void bm_window_splits(const int64_t* __restrict__ Brp, BView B, int64_t mb, int lgw,
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
    B.begin(j);
    const int64_t bound = (int64_t)q << lgw;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)B.c(mid) < bound) lo = mid + 1; else hi = mid;
    }
  }
  ws[t] = (uint32_t)lo;
}

// The all-gathered right operand of a row-block SpGEMM -> contiguous arrays
// in one pass (replaces concatenations and an interleave copy).  Rank r's
// columns are at gc + r * cstride (bits < 32: packed by bm_pack_bits, entry i
// at bit i * bits; else one word each), its value bits gv[r * gstride + i],
// i < base[r + 1] - base[r] (base[r] = first output index of rank r).  Any of
// col / val / cv may be null; with gc null the columns are read back from
// col (already unpacked: the two-stage gather, columns first).
// A workgroup takes kUnpackPer x 256 consecutive entries of one rank (strided
// by 256: coalesced), so the grid is small enough that workgroup dispatch does
// not bound the pass (one entry a thread ran at ~2 TB/s).
constexpr int kUnpackPer = 8;
__global__ __launch_bounds__(256) void bm_unpack_gathered(const uint32_t* __restrict__ gc, const uint32_t* __restrict__ gv,
                                                         int64_t gstride, int64_t cstride, int bits,
                                                         const int64_t* __restrict__ base,
                                                         int32_t* __restrict__ col, uint32_t* __restrict__ val,
                                                         uint2* __restrict__ cv) {
  const int r = blockIdx.y;
  const int64_t b0 = base[r], n = base[r + 1] - b0;
  const uint32_t* g = gc + (int64_t)r * cstride;
  const uint32_t msk = bits < 32 ? (1u << bits) - 1u : ~0u;
#pragma unroll
  for (int k = 0; k < kUnpackPer; ++k) {
    const int64_t i = ((int64_t)blockIdx.x * kUnpackPer + k) * 256 + threadIdx.x;
    if (i >= n) break;
    uint32_t c;
    if (!gc) {
      c = (uint32_t)col[b0 + i];
    } else if (bits < 32) {   // two aligned words hold the entry (the sender pads one word)
      const int64_t o = i * bits;
      const uint64_t two = (uint64_t)g[(o >> 5) + 1] << 32 | g[o >> 5];
      c = (uint32_t)(two >> (o & 31)) & msk;
    } else {
      c = g[i];
    }
    if (gc && col) col[b0 + i] = (int32_t)c;
    if (gv) {
      const uint32_t v = gv[(int64_t)r * gstride + i];
      if (val) val[b0 + i] = v;
      if (cv) cv[b0 + i] = make_uint2(c, v);
    }
  }
}

// Column indices of an operand panel packed to `bits` (< 32) bits each for the
// all-gather: entry i at bit i * bits of a little-endian word stream, one
// thread per output word (no atomics), words past the entries zero.  Columns
// < 2^bits (the caller's bits = ceil(log2 n)); 1M columns cross xGMI in 20 bits.
__global__ __launch_bounds__(256) void bm_pack_bits(const uint32_t* __restrict__ src, int64_t n, int bits,
                                                   uint32_t* __restrict__ dst, int64_t words) {
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= words) return;
  const int64_t lo = w * 32;
  const int64_t iend = min((lo + 32 + bits - 1) / bits, n);
  uint64_t acc = 0;
  for (int64_t i = lo / bits; i < iend; ++i) {
    const int64_t o = i * bits - lo;   // < 32; negative: the entry began in the previous word
    const uint64_t v = src[i];
    acc |= o >= 0 ? v << o : v >> -o;
  }
  dst[w] = (uint32_t)acc;
}

}  // namespace

namespace {
// (a null or column-less gathered view: the contiguous arrays)
BView bview(const int32_t* col, const void* val, const SpmmBmGathered* g) {
  BView v{col, (const uint32_t*)val, SpmmBmGathered{}};
  if (g && g->gc) v.g = *g;
  return v;
}
bool bview_ok(const SpmmBmGathered* g, bool values) {
  return !g || !g->gc || (g->W >= 1 && g->bits >= 1 && g->bits <= 32 && g->ebase && g->rbase && (!values || g->gv));
}
}  // namespace

// g (may be null): B read in place from its gathered panels (SpmmBmGathered), Bci unused.
SPMM_EXPORT int spmm_spgemm_bm_splits(const int64_t* Brp, const int32_t* Bci, int64_t mb, int lgw, int nwin,
                                      uint32_t* ws, const SpmmBmGathered* g, void* stream) {
  if (mb <= 0) return 0;
  const int64_t n = mb * (nwin + 1);
  if (nwin < 1 || lgw < 6 || lgw > 30 || n > (int64_t)UINT32_MAX - 255 || !bview_ok(g, false))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_window_splits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Brp,
                     bview(Bci, nullptr, g), mb, lgw, nwin, ws);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// ws8 for the row-major numeric kernel (nwin <= 8); err bit 3: a window
// segment too long for 16 bits (use spmm_spgemm_bm_numeric instead).
SPMM_EXPORT int spmm_spgemm_bm_pack_ws8(const uint32_t* ws, int64_t mb, int nwin, void* ws8, int32_t* err,
                                        int64_t* plen, int64_t* plen_c, int gc, void* stream) {
  if (mb <= 0) return 0;
  if (nwin < 1 || nwin > 8 || gc < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_pack_ws8, dim3((unsigned)((mb + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ws, mb, nwin,
                     (uint4*)ws8, err, plen, plen_c, gc);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Padded arrays of B (either may be null): the (column, value) pair array of
// the row-major numeric kernel (pass pad = 1 to it; pbase = exclusive scan of
// the plen from spmm_spgemm_bm_pack_ws8) and the column array of the row
// count kernel with count groups of gc windows padded to 32 columns (pad = 1
// to it; cbase = exclusive scan of plen_c); totals < 2^32.  Also stores each
// row's bases in ws8.
// cap / cap_c: entries allocated for out / outc; err bit 5 if a row would
// not fit (a layout invariant; nothing is written out of bounds).
SPMM_EXPORT int spmm_spgemm_bm_pad_pairs(const uint32_t* ws, const int32_t* col, const float* val, int64_t mb,
                                         int nwin, int lgw, const int64_t* pbase, void* ws8, void* out, const int64_t* cbase,
                                         int gc, int32_t* outc, int64_t cap, int64_t cap_c, int32_t* err,
                                         const SpmmBmGathered* g, void* stream) {
  if (mb <= 0) return 0;
  if (nwin < 1 || nwin > 8 || gc < 1 || gc > 8 || lgw < 1 || lgw > 30 || (mb * 64 + 255) / 256 > (int64_t)UINT32_MAX ||
      !bview_ok(g, out != nullptr))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_pad_pairs, dim3((unsigned)((mb * 64 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ws,
                     bview(col, val, g), mb, nwin, lgw, pbase, (uint4*)ws8, (uint2*)out, cbase, gc, outc, cap, cap_c,
                     err);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Unpack an all-gathered operand payload: rank r's columns at gc + r *
// cstride (packed to `bits` bits when bits < 32), its value bits at gv + r *
// gstride (either may be null, see the kernel); base: device int64[world + 1]
// output offsets.
SPMM_EXPORT int spmm_spgemm_bm_unpack_gathered(const void* gc, const void* gv, int world, int64_t gstride,
                                               int64_t cstride, int bits, const int64_t* base, int64_t max_n,
                                               int32_t* col, float* val, void* cv, void* stream) {
  if (world <= 0 || max_n <= 0) return 0;
  if (world > 65535 || (max_n + 255) / 256 > (int64_t)UINT32_MAX || bits < 1 || bits > 32) return (int)hipErrorInvalidValue;
  if (!gc && !col) return (int)hipErrorInvalidValue;
  if (gc && bits < 32 && cstride < (max_n * bits + 31) / 32 + 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_unpack_gathered, dim3((unsigned)((max_n + 256 * kUnpackPer - 1) / (256 * kUnpackPer)), (unsigned)world), dim3(256), 0,
                     (hipStream_t)stream, (const uint32_t*)gc, (const uint32_t*)gv, gstride, cstride, bits, base, col,
                     (uint32_t*)val, (uint2*)cv);
  SPMM_LAUNCH_CHECK();
  return 0;
}

// Pack n column indices (each < 2^bits, 1 <= bits < 32) into `words` words
// (>= (n * bits + 31) / 32 + 1: the unpacker reads two words an entry).
SPMM_EXPORT int spmm_pack_bits(const int32_t* src, int64_t n, int bits, uint32_t* dst, int64_t words, void* stream) {
  if (words <= 0) return 0;
  if (n < 0 || bits < 1 || bits > 31 || words < (n * bits + 31) / 32 + 1 || (words + 255) / 256 > (int64_t)UINT32_MAX)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_pack_bits, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint32_t*)src, n, bits, dst, words);
  SPMM_LAUNCH_CHECK();
  return 0;
}
