// Host orchestration of one bitmap-rank SpGEMM (csr_spgemm_bitmap.hip): the path decision,
// the plan (window configuration, lane groups, which kernels, padded-layout capacities,
// one workspace layout) and the launch sequence.  The single copy of this logic: the
// Python front end (ops/spgemm.py _bitmap_ok / _bitmap_plan / _bitmap_launch) and the
// native Matrix-Market chain (csrc/runtime/csr_engine.cpp) both call it, so thresholds
// and kernel order cannot drift apart (round 4 kept two copies).
//
// front = B layouts (window splits, ws8, padded column / pair arrays) + count kernel +
//         unit-offset scan; back = padded pairs (if B's values came late) + numeric kernel.
// Launches only, no allocation and no host synchronisation: capturable into a HIP graph.
// The reference sizes its device rounds from host counts instead
// (sparse_matrix_mult.cu:181-270).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "bitmap_plan.hpp"

#define SPMM_EXPORT extern "C" __attribute__((visibility("default")))

extern "C" {
int spmm_spgemm_bm_config(int cfg, int* lgw, int* nsub_count, int* pcap_fast, int* rounds_fast, int* reload_rows);
int spmm_spgemm_bm_splits(const int64_t* Brp, const int32_t* Bci, int64_t mb, int lgw, int nwin, uint32_t* ws,
                          const SpmmBmGathered* g, void* stream);
int spmm_spgemm_bm_pack_ws8(const uint32_t* ws, int64_t mb, int nwin, void* ws8, int32_t* err, int64_t* plen,
                            int64_t* plen_c, int gc, void* stream);
int spmm_spgemm_bm_pad_pairs(const uint32_t* ws, const int32_t* col, const float* val, int64_t mb, int nwin, int lgw,
                             const int64_t* pbase, void* ws8, void* out, const int64_t* cbase, int gc, int32_t* outc,
                             int64_t cap, int64_t cap_c, int32_t* err, const SpmmBmGathered* g, void* stream);
int spmm_spgemm_bm_count(int cfg, const int64_t* Arp, const int32_t* Aci, const uint32_t* ws, const int32_t* Bci,
                         int64_t m, int nwin, int lg, int32_t* ucnt, int32_t* err, void* stream);
int spmm_spgemm_bm_count_rows(int cfg, const int64_t* Arp, const int32_t* Aci, const void* ws8, const int32_t* Bci,
                              int64_t m, int nwin, int lg, int nsub, int32_t* ucnt, int32_t* err, int64_t nnzb, int pad,
                              int pipe, int64_t annz, void* stream);
int spmm_spgemm_bm_numeric(int cfg, const int64_t* Arp, const int32_t* Aci, const float* Av, const uint32_t* ws,
                           const int32_t* Bci, const float* Bv, int64_t m, int nwin, int lg, const int64_t* uoff,
                           int64_t cap, int32_t* Cci, float* Cv, int32_t* ovf, uint32_t* novf, int64_t ovf_cap,
                           int32_t* err, int det, const void* ws8, const void* bcv_padded, void* stream);
int spmm_spgemm_bm_numeric_rows(int cfg, const int64_t* Arp, const int32_t* Aci, const float* Av, const void* ws8,
                                const uint32_t* ws, const int32_t* Bci, const float* Bv, const void* Bcv, int64_t m,
                                int nwin, int lg, const int64_t* uoff, int64_t cap, int32_t* Cci, float* Cv,
                                int32_t* ovf, uint32_t* novf, int64_t ovf_cap, int32_t* err, int det, int pad,
                                int64_t nbcv, int pipe, int64_t annz, void* stream);
size_t spmm_prim_scan_ws(int64_t n);
int spmm_prim_scan(const void* in, int in_bytes, int64_t n, int64_t* out, int inclusive, void* ws, void* stream);
}

namespace {

constexpr double kFill = 0.7;          // mean products per window <= kFill * fast capacity
constexpr int kPadPairs = 16;          // padded pair segments: multiples of 16 pairs (bitmap_common.hpp kPadLg)
constexpr int kPadCols = 32;           // padded count segments: multiples of 32 columns (kPadCLg)
constexpr int64_t kOvfCap = 1 << 20;   // deferred-unit list capacity

struct Cfg {
  int lgw, nsub, pcap, rounds, reload_rows;
};

Cfg cfg_of(int c) {
  Cfg r{};
  spmm_spgemm_bm_config(c, &r.lgw, &r.nsub, &r.pcap, &r.rounds, &r.reload_rows);
  return r;
}

// widest window whose mean products per window fit kFill of its fast capacity
int pick(double mean_row_products, int64_t ncols) {
  for (int c : {0, 2, 1}) {
    const Cfg k = cfg_of(c);
    const double W = (double)((int64_t)1 << k.lgw);
    const double per_window = mean_row_products * std::min(W, (double)ncols) / (double)std::max<int64_t>(ncols, 1);
    if (per_window <= kFill * k.pcap) return c;
  }
  return -1;
}

int group_log2(double seg) { return seg >= 40 ? 6 : (seg >= 16 ? 5 : 4); }

int64_t al(int64_t b) { return (b + 255) & ~(int64_t)255; }

template <typename T>
T* at(void* ws, int64_t off) {
  return off >= 0 ? reinterpret_cast<T*>(static_cast<char*>(ws) + off) : nullptr;
}

}  // namespace

// Options from the environment, with the defaults of utils/config.py (the same variables:
// SPMM_SPGEMM_BITMAP, _CFG, _ROWS, _PAD, _CV, _PIPE, SPMM_SPGEMM_DETERMINISTIC;
// tests/test_spgemm.py checks the two sets of defaults agree).  For the native engine.
SPMM_EXPORT int spmm_spgemm_bm_env_opts(SpmmBmOpts* o) {
  auto num = [](const char* k, int d) {
    const char* e = getenv(k);
    return e && *e ? atoi(e) : d;
  };
  auto tri = [](const char* k) {
    const char* e = getenv(k);
    if (!e || !*e) return 1;
    return strcmp(e, "off") == 0 ? 0 : (strcmp(e, "on") == 0 ? 2 : 1);
  };
  o->mode = tri("SPMM_SPGEMM_BITMAP");
  o->cfg = num("SPMM_SPGEMM_BITMAP_CFG", -1);
  o->rows_mode = tri("SPMM_SPGEMM_BITMAP_ROWS");
  o->det = num("SPMM_SPGEMM_DETERMINISTIC", 0) > 0;
  o->pad = num("SPMM_SPGEMM_BITMAP_PAD", 1) > 0;
  o->cv = num("SPMM_SPGEMM_BITMAP_CV", 1) != 0;
  o->pipe = num("SPMM_SPGEMM_BITMAP_PIPE", 1) > 0;
  o->use_ws8 = 1;
  return 0;
}

// The bitmap gate (ops/spgemm.py _bitmap_ok without its free-memory check, which each
// caller makes with its own allocator): the configuration to use, or -1.
SPMM_EXPORT int spmm_spgemm_bm_choose(const SpmmBmOpts* o, int64_t m, int64_t annz, int64_t bn, int64_t bnnz,
                                      int64_t tot, int64_t nonempty, int64_t pmax, int64_t amax) {
  if (o->mode == 0 || tot == 0 || bnnz >= ((int64_t)1 << 31) || bn >= ((int64_t)1 << 30) || annz >= ((int64_t)1 << 31))
    return -1;
  const int64_t nz = std::max<int64_t>(nonempty, 1);
  const double mean = (double)tot / (double)nz;
  int cfg = o->cfg >= 0 ? o->cfg : pick(mean, bn);
  if (cfg < 0) cfg = o->mode == 2 ? 1 : -1;
  if (cfg < 0 || amax > cfg_of(cfg).reload_rows) return -1;
  if (o->mode == 2) return cfg;
  if ((double)pmax > 4 * mean || (double)nz < 0.5 * (double)m) return -1;
  return cfg;
}

// The plan of one product (ops/spgemm.py _bitmap_plan + the layout decisions of
// _bitmap_launch) and its workspace layout.  amax < 0: A's longest row unknown.
// mean_seg <= 0: B's mean row length stands in.  Returns 1 when the units do not fit int32.
SPMM_EXPORT int spmm_spgemm_bm_make_plan(const SpmmBmOpts* o, int64_t m, int64_t annz, int64_t mb, int64_t bn,
                                         int64_t bnnz, int64_t tot, int64_t nonempty, int64_t amax, double mean_seg,
                                         SpmmBmPlan* p) {
  *p = SpmmBmPlan{};
  const int64_t nz = std::max<int64_t>(nonempty, 1);
  int cfg = o->cfg >= 0 ? o->cfg : pick((double)tot / (double)nz, bn);
  if (cfg < 0) cfg = 1;
  const Cfg k = cfg_of(cfg);
  const int nwin = (int)std::max<int64_t>(1, (bn + ((int64_t)1 << k.lgw) - 1) >> k.lgw);
  if (m * nwin >= ((int64_t)1 << 31)) return 1;
  const double seg = mean_seg > 0 ? mean_seg : (double)bnnz / (double)std::max<int64_t>(mb, 1);
  const bool ws8_ok = nwin <= 8 && o->rows_mode != 0;
  // windows per row-count unit: two (a B row's two-window segment read once for both; units of
  // 1 / 4 windows measured slower, PERF_LOG rounds 4-5), one when the row has one window
  const int nsub_c = nwin >= 2 ? 2 : 1;
  const double sl = seg * nsub_c / nwin;   // B-segment length per row-count unit
  p->cfg = cfg;
  p->lgw = k.lgw;
  p->nwin = nwin;
  p->nsub = k.nsub;
  p->lg_count = group_log2(seg * std::min(k.nsub, nwin) / nwin);
  p->lg_c = sl < 48 ? 4 : (sl < 96 ? 5 : 6);
  p->nsub_c = nsub_c;
  p->lg_num = seg / nwin < 48 ? 4 : (seg / nwin < 96 ? 5 : 6);
  p->det = o->det != 0;
  p->pipe = o->pipe != 0;
  // the row numeric kernel exists only in its pipelined form (padded pairs, 32-bit buffer
  // offsets, unordered sums); every other product takes the per-unit numeric kernels
  const bool pad = o->pad != 0 && o->use_ws8 != 0;
  const int64_t ngc = (nwin + nsub_c - 1) / nsub_c;
  const int64_t cap_bcv = bnnz + (kPadPairs - 1) * (int64_t)nwin * mb;
  const int64_t cap_colp = bnnz + (kPadCols - 1) * ngc * mb;
  p->count_rows = ws8_ok && amax >= 0 && amax <= 256;
  // (cfg 2 keeps the per-unit kernels unless forced: not measured on the row kernel)
  p->rows = ws8_ok && (o->rows_mode == 2 || cfg <= 1) && pad && o->cv != 0 && !p->det && p->pipe && annz > 0 &&
            cap_bcv * 8 < ((int64_t)1 << 32);
  p->m = m;
  p->annz = annz;
  p->mb = mb;
  p->nnzb = bnnz;
  p->tot = tot;
  p->nunits = m * nwin;
  p->ngc = (nwin + nsub_c - 1) / nsub_c;
  p->pad_num = pad && (p->rows || !p->det) && o->cv != 0 && cap_bcv < ((int64_t)1 << 32);
  p->pad_cnt = pad && p->count_rows && cap_colp < ((int64_t)1 << 32);
  p->ws8 = o->use_ws8 != 0 && ws8_ok && (p->count_rows || p->rows || p->pad_num);
  if (!p->ws8) p->pad_num = p->pad_cnt = p->rows = p->count_rows = 0;
  p->cap_bcv = p->pad_num ? cap_bcv : 0;
  p->cap_colp = p->pad_cnt ? cap_colp : 0;
  p->ovf_cap = std::max<int64_t>(1, std::min<int64_t>(p->nunits, kOvfCap));
  int64_t off = 0;
  auto take = [&](int64_t bytes, bool on) -> int64_t {
    if (!on) return -1;
    const int64_t r = off;
    off += al(std::max<int64_t>(bytes, 8));
    return r;
  };
  p->o_split = take(mb * (nwin + 1) * 4, true);
  p->o_ucnt = take(p->nunits * 4, true);
  p->o_ws8 = take(mb * 32, p->ws8);
  p->o_plen = take(mb * 8, p->pad_num);
  p->o_plenc = take(mb * 8, p->pad_cnt && p->count_rows);
  p->o_pbase = take(mb * 8, p->pad_num);
  p->o_cbase = take(mb * 8, p->pad_cnt && p->count_rows);
  p->o_colp = take(p->cap_colp * 4, p->cap_colp > 0);
  p->o_bcv = take(p->cap_bcv * 8, p->cap_bcv > 0);
  p->o_ovf = take(p->ovf_cap * 4, true);
  p->o_scan = take((int64_t)spmm_prim_scan_ws(std::max<int64_t>(p->nunits, mb)), true);
  p->ws_bytes = off;
  return 0;
}

// Whether the plan's kernels read B only through the layouts built by the splits / pad
// passes (so B may stay in its gathered panels): pipelined row count on the padded count
// columns, pipelined row numeric + the reload kernel on the padded pairs.
SPMM_EXPORT int spmm_spgemm_bm_gathered_ok(const SpmmBmPlan* p) {
  return p->ws8 && p->count_rows && p->pad_cnt && p->rows && p->pad_num && p->pipe && !p->det && p->nsub_c == 2 &&
         p->nwin >= 2;
}

// The front's reset of z (int32[4]) and uoff[0], as a kernel: a 16-byte hipMemsetAsync captured
// into the row-block step's first graph wrote device-address-like garbage into z on replay
// (ROCm 7.x; tools/r6/diag_rows_graph4.py): deferred count and row ticket garbage, so the
// numeric kernel took rows past the matrix.  Vector stores, one lane each.
namespace {
__global__ __launch_bounds__(64) void bm_front_reset(int32_t* __restrict__ z, int64_t* __restrict__ uoff) {
  const int t = threadIdx.x;
  if (t < 4) z[t] = 0;
  if (t == 4) uoff[t - 4] = 0;
}
}  // namespace

#define BM_TRY(x)               \
  do {                          \
    const int _rc = (x);        \
    if (_rc != 0) return _rc;   \
  } while (0)

// Layouts + count kernel + unit offsets.  Bv may be null (B's values still in flight:
// the padded pairs are then built by spmm_spgemm_bm_back).  g (may be null): B read in
// place from its all-gathered panels (SpmmBmGathered; Bci / Bv unused): only for plans
// whose kernels read B through the padded layouts alone (spmm_spgemm_bm_gathered_ok).
// uoff: nunits + 1 entries;
// z: int32[4] {error bits, deferred units, numeric row ticket, 0} (zeroed here).  *pairs_built: whether the padded
// pairs exist after this call (pass it to spmm_spgemm_bm_back).
SPMM_EXPORT int spmm_spgemm_bm_front(const SpmmBmPlan* p, const int64_t* Arp, const int32_t* Aci, const int64_t* Brp,
                                     const int32_t* Bci, const float* Bv, void* ws, int64_t* uoff, int32_t* z,
                                     int* pairs_built, const SpmmBmGathered* g, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  *pairs_built = 0;
  const bool gath = g != nullptr && g->gc != nullptr;
  if (gath && !spmm_spgemm_bm_gathered_ok(p)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bm_front_reset, dim3(1), dim3(64), 0, s, z, uoff);
  if (hipGetLastError() != hipSuccess) return (int)hipErrorUnknown;
  uint32_t* split = at<uint32_t>(ws, p->o_split);
  int32_t* ucnt = at<int32_t>(ws, p->o_ucnt);
  void* ws8 = at<void>(ws, p->o_ws8);
  int64_t* plen = at<int64_t>(ws, p->o_plen);
  int64_t* plenc = at<int64_t>(ws, p->o_plenc);
  int64_t* pbase = at<int64_t>(ws, p->o_pbase);
  int64_t* cbase = at<int64_t>(ws, p->o_cbase);
  int32_t* colp = at<int32_t>(ws, p->o_colp);
  void* bcv = at<void>(ws, p->o_bcv);
  void* scan = at<void>(ws, p->o_scan);
  BM_TRY(spmm_spgemm_bm_splits(Brp, Bci, p->mb, p->lgw, p->nwin, split, g, s));
  if (p->ws8) BM_TRY(spmm_spgemm_bm_pack_ws8(split, p->mb, p->nwin, ws8, z, plen, plenc, p->nsub_c, s));
  if (p->ws8 && p->count_rows) {
    if (colp != nullptr) {
      BM_TRY(spmm_prim_scan(plenc, 8, p->mb, cbase, 0, scan, s));
      const bool both = p->pad_num && (gath ? g->gv != nullptr : Bv != nullptr);   // values here: both layouts, one pass
      if (both) BM_TRY(spmm_prim_scan(plen, 8, p->mb, pbase, 0, scan, s));
      BM_TRY(spmm_spgemm_bm_pad_pairs(split, Bci, both ? Bv : nullptr, p->mb, p->nwin, p->lgw, both ? pbase : nullptr,
                                      ws8, both ? bcv : nullptr, cbase, p->nsub_c, colp, both ? p->cap_bcv : 0,
                                      p->cap_colp, z, g, s));
      *pairs_built = both ? 1 : 0;
    }
    BM_TRY(spmm_spgemm_bm_count_rows(p->cfg, Arp, Aci, ws8, colp != nullptr ? colp : Bci, p->m, p->nwin, p->lg_c,
                                     p->nsub_c, ucnt, z, colp != nullptr ? p->cap_colp : p->nnzb,
                                     colp != nullptr ? 1 : 0, p->pipe, p->annz, s));
  } else {
    BM_TRY(spmm_spgemm_bm_count(p->cfg, Arp, Aci, split, Bci, p->m, p->nwin, p->lg_count, ucnt, z, s));
  }
  return spmm_prim_scan(ucnt, 4, p->nunits, uoff + 1, 1, scan, s);
}

// Padded pairs (unless built by the front) + numeric kernel into C (cap entries).
SPMM_EXPORT int spmm_spgemm_bm_back(const SpmmBmPlan* p, const int64_t* Arp, const int32_t* Aci, const float* Av,
                                    const int32_t* Bci, const float* Bv, int pairs_built, void* ws,
                                    const int64_t* uoff, int32_t* z, int64_t cap, int32_t* Cci, float* Cv,
                                    const SpmmBmGathered* g, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (g != nullptr && g->gc != nullptr && (!spmm_spgemm_bm_gathered_ok(p) || g->gv == nullptr))
    return (int)hipErrorInvalidValue;
  uint32_t* split = at<uint32_t>(ws, p->o_split);
  void* ws8 = at<void>(ws, p->o_ws8);
  int64_t* plen = at<int64_t>(ws, p->o_plen);
  int64_t* pbase = at<int64_t>(ws, p->o_pbase);
  void* bcv = at<void>(ws, p->o_bcv);
  int32_t* ovf = at<int32_t>(ws, p->o_ovf);
  void* scan = at<void>(ws, p->o_scan);
  uint32_t* novf = reinterpret_cast<uint32_t*>(z + 1);
  if (p->pad_num && !pairs_built) {
    BM_TRY(spmm_prim_scan(plen, 8, p->mb, pbase, 0, scan, s));
    BM_TRY(spmm_spgemm_bm_pad_pairs(split, Bci, Bv, p->mb, p->nwin, p->lgw, pbase, ws8, bcv, nullptr, 1, nullptr,
                                    p->cap_bcv, 0, z, g, s));
  }
  if (p->ws8 && p->rows) {
    return spmm_spgemm_bm_numeric_rows(p->cfg, Arp, Aci, Av, ws8, split, Bci, Bv, bcv, p->m, p->nwin, p->lg_num, uoff,
                                       cap, Cci, Cv, ovf, novf, p->ovf_cap, z, p->det, p->pad_num, p->cap_bcv,
                                       p->pipe, p->annz, s);
  }
  const bool wide = p->pad_num && !p->det;
  return spmm_spgemm_bm_numeric(p->cfg, Arp, Aci, Av, split, Bci, Bv, p->m, p->nwin, p->lg_num, uoff, cap, Cci, Cv,
                                ovf, novf, p->ovf_cap, z, p->det, wide ? ws8 : nullptr, wide ? bcv : nullptr, s);
}
