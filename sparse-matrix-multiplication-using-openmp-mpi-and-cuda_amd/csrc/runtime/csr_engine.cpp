// Device-resident CSR SpGEMM for the native Matrix-Market chain (see
// csr_engine.hpp).  Host orchestration of the gfx950 kernels, mirroring
// ops/spgemm.py: the row plan (one 16-word read-back) picks the bitmap-rank
// path for uniform products; everything else takes the binned two-phase path
// (LDS tables by product count, hub rows through the long-row pipeline), so
// no product falls back to the CPU.  Per-row host arrays (product counts,
// flags, the long rows' chunk counts) are the only device->host traffic.
#include "csr_engine.hpp"
#include "../kernels/bitmap_plan.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>

extern "C" {
// csr_spgemm.hip
int spmm_spgemm_row_plan(const int64_t* Arp, const int32_t* Aci, const int64_t* Brp, int64_t m, int64_t cap1,
                         int64_t cap2, int64_t cap4, int64_t esc_min, int64_t* nprod, int64_t* nsl, int64_t* part,
                         int64_t* stats, void* stream);
int spmm_spgemm_row_splits(const int64_t* Brp, const int32_t* Bci, int64_t mb, int ncols, int64_t* bsplit,
                           void* stream);
int spmm_spgemm_lds(int bin, int numeric, const int64_t* Arp, const int32_t* Aci, const float* Av, const int64_t* Brp,
                    const int32_t* Bci, const float* Bv, const int64_t* bsplit, const int32_t* rows, int64_t nrows,
                    int ncols, int lg, int32_t* row_nnz, int32_t* out_nnz, const int64_t* Crp, int32_t* Cci, float* Cv,
                    int32_t* flags, void* stream);
int spmm_spgemm_long_route(int scatter, const int32_t* Aci, const float* Av, const int64_t* Brp, const int32_t* Bci,
                           const float* Bv, const int64_t* wg_e0, const int64_t* wg_e1, int64_t nwg, int nch,
                           int32_t* wg_hist, const int32_t* wg_row, const int64_t* row_off, void* scratch,
                           const int32_t* lidx, const uint32_t* btab, int32_t* wg_dhist, int32_t* wg_nlong,
                           const uint8_t* rt_mode, void* dl, const int64_t* dl_off, void* stream);
int spmm_spgemm_long_wg_scan(int32_t* wg_hist, const int64_t* wg0, const int64_t* nwg, int64_t R, int nch,
                             int64_t* cnt, const int32_t* dhist, int64_t* dcnt, uint8_t* mode, void* stream);
int spmm_spgemm_long_dense(int values, const int64_t* rt_off, const int64_t* rt_cnt, int64_t nrt, int nch,
                           void* scratch, int64_t* rt_nnz, int32_t* ws, const int64_t* dt_cnt, const void* dl,
                           const int64_t* dl_rp, const uint32_t* btab, const int32_t* Bci, const float* Bv,
                           int grid_pct, void* stream);
int spmm_spgemm_long_place(const int64_t* src, const int64_t* dst, const int64_t* cnt, int64_t nrt,
                           const void* scratch, int32_t* Cci, float* Cv, void* stream);
int spmm_spgemm_long_params(int* lgw, int* epw, int* maxch);
int spmm_spgemm_plan_params(int* plan_blocks, int* plan_stats, double* esc_load);
// csr_rowsort.hip
size_t spmm_spgemm_bin_rows_ws(int64_t m);
int spmm_spgemm_bin_rows(const int64_t* nprod, int64_t m, int numeric, double load, double load_sliced,
                         int64_t esc_min, int32_t* order, int64_t* hist, void* ws, void* stream);
int spmm_rows_with_flag(const int32_t* flags, int64_t m, int mask, int32_t* out, int64_t* count, void* stream);
size_t spmm_csr_sort_rows_ws(int64_t nrows, int64_t total, int64_t maxlen);
int spmm_csr_sort_rows(const int64_t* rp, const int64_t* rows, int64_t nrows, int64_t total, int64_t maxlen,
                       int32_t* ci, float* v, void* ws, void* stream);
// csr_bitmap_plan.hip (SpmmBmOpts / SpmmBmPlan: bitmap_plan.hpp)
int spmm_spgemm_bm_env_opts(SpmmBmOpts* o);
int spmm_spgemm_bm_choose(const SpmmBmOpts* o, int64_t m, int64_t annz, int64_t bn, int64_t bnnz, int64_t tot,
                          int64_t nonempty, int64_t pmax, int64_t amax);
int spmm_spgemm_bm_make_plan(const SpmmBmOpts* o, int64_t m, int64_t annz, int64_t mb, int64_t bn, int64_t bnnz,
                             int64_t tot, int64_t nonempty, int64_t amax, double mean_seg, SpmmBmPlan* p);
int spmm_spgemm_bm_front(const SpmmBmPlan* p, const int64_t* Arp, const int32_t* Aci, const int64_t* Brp,
                         const int32_t* Bci, const float* Bv, void* ws, int64_t* uoff, int32_t* z, int* pairs_built,
                         const SpmmBmGathered* g, void* stream);
int spmm_spgemm_bm_back(const SpmmBmPlan* p, const int64_t* Arp, const int32_t* Aci, const float* Av,
                        const int32_t* Bci, const float* Bv, int pairs_built, void* ws, const int64_t* uoff,
                        int32_t* z, int64_t cap, int32_t* Cci, float* Cv, const SpmmBmGathered* g, void* stream);
}

namespace a4 {

namespace {

// Knobs shared with ops/spgemm.py through the same environment variables and defaults
// (utils/config.py: SPMM_SPGEMM_LOAD, _LOAD_SLICED, _ESC_MIN, SPMM_GLOBAL_WS_GB); the bin
// table itself and the planner constants come from the kernel library.
double env_f(const char* k, double d) {
  const char* e = getenv(k);
  return e && *e ? atof(e) : d;
}
struct Knobs {
  double load = env_f("SPMM_SPGEMM_LOAD", 0.5), load_sliced = env_f("SPMM_SPGEMM_LOAD_SLICED", 0.5);
  int64_t esc_min = (int64_t)env_f("SPMM_SPGEMM_ESC_MIN", 2048);
  int64_t ws_products = (int64_t)(env_f("SPMM_GLOBAL_WS_GB", 8.0) * (double)(int64_t(1) << 30)) / 8;
  int64_t ordered_pcap = (int64_t)env_f("SPMM_SPGEMM_ORDERED_PCAP", 7680);
  int plan_blocks = 0, plan_stats = 0;
  double esc_load = 0;
  Knobs() { spmm_spgemm_plan_params(&plan_blocks, &plan_stats, &esc_load); }
};
const Knobs& knobs() {
  static const Knobs k;
  return k;
}

template <typename T>
DevBuf<T> up(const std::vector<T>& h, hipStream_t s) {
  DevBuf<T> d(std::max<size_t>(h.size(), 1), s);
  if (!h.empty()) A4_HIP(hipMemcpyAsync(d.get(), h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return d;
}

template <typename T>
std::vector<T> down(const T* d, size_t n, hipStream_t s) {
  std::vector<T> h(n);
  if (n) A4_HIP(hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
  A4_HIP(hipStreamSynchronize(s));
  return h;
}

int group_log2(double seg) { return seg >= 40 ? 6 : (seg >= 16 ? 5 : 4); }   // ops/spgemm.py _group_log2

struct Plan {
  int64_t tot = 0, mx = 0, nz = 0, amax = 0;
  DevBuf<int64_t> nprod;
};

Plan row_plan(const DCsr& A, const DCsr& B, hipStream_t s) {
  Plan p;
  p.nprod = DevBuf<int64_t>(std::max<int64_t>(A.m, 1), s);
  const Knobs& k = knobs();
  DevBuf<int64_t> nsl(std::max<int64_t>(A.m, 1), s), part((size_t)(k.plan_blocks + 1) * k.plan_stats, s);
  const int64_t c1 = (int64_t)(k.esc_load * k.ordered_pcap);
  const int64_t nst = (int64_t)k.plan_blocks * k.plan_stats;
  A4_HIP((hipError_t)spmm_spgemm_row_plan(A.rp.get(), A.ci.get(), B.rp.get(), A.m, c1, 2 * c1, 4 * c1, k.esc_min,
                                          p.nprod.get(), nsl.get(), part.get(), part.get() + nst, s));
  const std::vector<int64_t> st = down(part.get() + nst, k.plan_stats, s);
  p.tot = st[0];
  p.mx = st[1];
  p.nz = st[2];
  p.amax = st[8];
  return p;
}

DCsr empty_product(const DCsr& A, const DCsr& B, hipStream_t s) {
  DCsr C;
  C.m = A.m;
  C.n = B.n;
  C.rp = DevBuf<int64_t>(A.m + 1, s);
  A4_HIP(hipMemsetAsync(C.rp.get(), 0, (A.m + 1) * sizeof(int64_t), s));
  C.ci = DevBuf<int32_t>(1, s);
  C.v = DevBuf<float>(1, s);
  return C;
}

// ---- bitmap-rank path: the shared native planner (csr_bitmap_plan.hip), the same
// decisions, layouts and kernels as ops/spgemm.py onepass_bitmap (eager flow) ------------
bool bitmap_product(const DCsr& A, const DCsr& B, const Plan& pl, hipStream_t s, DCsr* out) {
  SpmmBmOpts o{};
  spmm_spgemm_bm_env_opts(&o);
  if (spmm_spgemm_bm_choose(&o, A.m, A.nnz, B.n, B.nnz, pl.tot, pl.nz, pl.mx, pl.amax) < 0) return false;
  const double seg = (double)pl.tot / (double)std::max<int64_t>(A.nnz, 1);   // B-segment length per A entry
  for (int use_ws8 = 1; use_ws8 >= 0; --use_ws8) {
    o.use_ws8 = use_ws8;
    SpmmBmPlan p{};
    if (spmm_spgemm_bm_make_plan(&o, A.m, A.nnz, B.m, B.n, B.nnz, pl.tot, pl.nz, pl.amax, seg, &p)) return false;
    DevBuf<uint8_t> ws((size_t)std::max<int64_t>(p.ws_bytes, 1), s);
    DevBuf<int32_t> z(4, s);   // err, deferred units, row tickets (csr_bitmap_plan.hip front)
    DevBuf<int64_t> uoff((size_t)p.nunits + 1, s);
    int built = 0;
    A4_HIP((hipError_t)spmm_spgemm_bm_front(&p, A.rp.get(), A.ci.get(), B.rp.get(), B.ci.get(), B.v.get(), ws.get(),
                                            uoff.get(), z.get(), &built, nullptr, s));
    const int64_t nnz = down(uoff.get() + p.nunits, 1, s)[0];   // the one sizing read-back
    const int e0 = down(z.get(), 1, s)[0];
    A4_CHECK((e0 & 32) == 0, "spgemm bitmap: padded B layout overflow");
    // a window segment of >= 65536 entries (bit 3), or a count unit of more chunks than the
    // pipelined count kernel's descriptors (bit 6): per-unit kernels
    if (e0 & (8 | 64)) continue;
    if (e0 != 0) return false;
    A4_HIP(hipMemsetAsync(z.get(), 0, 4, s));
    DCsr C;
    C.m = A.m;
    C.n = B.n;
    C.nnz = nnz;
    C.ci = DevBuf<int32_t>((size_t)std::max<int64_t>(nnz, 1), s);
    C.v = DevBuf<float>((size_t)std::max<int64_t>(nnz, 1), s);
    A4_HIP((hipError_t)spmm_spgemm_bm_back(&p, A.rp.get(), A.ci.get(), A.v.get(), B.ci.get(), B.v.get(), built,
                                           ws.get(), uoff.get(), z.get(), nnz, C.ci.get(), C.v.get(), nullptr, s));
    const int e = down(z.get(), 1, s)[0];
    A4_CHECK((e & 2) == 0, "spgemm bitmap: numeric and count kernels disagree");
    // a unit beyond the reload kernel's budget (bits 0 / 2), or, deterministic, a unit no
    // deterministic kernel could form (bit 4: nothing was written for it): the binned path
    // redoes the product (correct C; its fp32 sums are not in the fixed order)
    if (e & (p.det ? 21 : 5)) return false;
    // row pointer: every nwin-th unit offset, gathered on the device
    C.rp = DevBuf<int64_t>((size_t)A.m + 1, s);
    A4_HIP(hipMemcpy2DAsync(C.rp.get(), sizeof(int64_t), uoff.get(), sizeof(int64_t) * p.nwin, sizeof(int64_t),
                            (size_t)A.m + 1, hipMemcpyDeviceToDevice, s));
    *out = std::move(C);
    return true;
  }
  return false;
}

// ---- long rows (ops/spgemm.py _long_rows, routed mode) -----------------------
// values = 0: per-row nnz into cnt_out; 1: the rows written at Crp_h[row].
void long_rows(int values, const DCsr& A, const DCsr& B, const std::vector<int32_t>& rows,
               const std::vector<int64_t>& nprod_h, const std::vector<int64_t>& Arp_h, hipStream_t s,
               std::vector<int64_t>* cnt_out, const std::vector<int64_t>* Crp_h, int32_t* Cci, float* Cv) {
  if (rows.empty()) return;
  int lgw = 0, epw = 0, maxch = 0;
  A4_HIP((hipError_t)spmm_spgemm_long_params(&lgw, &epw, &maxch));
  const int nch = (int)((B.n + (int64_t(1) << lgw) - 1) >> lgw);
  A4_CHECK(nch <= maxch, "long-row path: too many columns");
  const int64_t nrows = (int64_t)rows.size();
  int64_t maxp = 0;
  for (int32_t r : rows) maxp = std::max(maxp, nprod_h[r]);
  const int64_t cap = std::max(knobs().ws_products, maxp);
  for (int64_t start = 0; start < nrows;) {
    int64_t end = start, acc = 0;   // batch: the longest run of rows whose products fit cap (at least one row)
    while (end < nrows && (end == start || acc + nprod_h[rows[end]] <= cap)) acc += nprod_h[rows[end++]];
    const int64_t R = end - start;
    std::vector<int64_t> first(R), nwg_r(R), e0, e1;
    std::vector<int32_t> wrow;
    for (int64_t i = 0; i < R; ++i) {
      const int32_t r = rows[start + i];
      const int64_t a0 = Arp_h[r], na = Arp_h[r + 1] - a0;
      nwg_r[i] = std::max<int64_t>(1, (na + epw - 1) / epw);
      first[i] = (int64_t)e0.size();
      for (int64_t k = 0; k < nwg_r[i]; ++k) {
        e0.push_back(a0 + k * epw);
        e1.push_back(std::min(a0 + (k + 1) * epw, a0 + na));
        wrow.push_back((int32_t)i);
      }
    }
    const int64_t nwg = (int64_t)e0.size();
    DevBuf<int64_t> de0 = up(e0, s), de1 = up(e1, s), dfirst = up(first, s), dnwg = up(nwg_r, s);
    DevBuf<int32_t> dwrow = up(wrow, s);
    DevBuf<int32_t> hist((size_t)nwg * nch, s);
    A4_HIP((hipError_t)spmm_spgemm_long_route(0, A.ci.get(), A.v.get(), B.rp.get(), B.ci.get(), B.v.get(), de0.get(),
                                              de1.get(), nwg, nch, hist.get(), nullptr, nullptr, nullptr, nullptr,
                                              nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, s));
    DevBuf<int64_t> T((size_t)R * nch, s);
    A4_HIP((hipError_t)spmm_spgemm_long_wg_scan(hist.get(), dfirst.get(), dnwg.get(), R, nch, T.get(), nullptr, nullptr,
                                                nullptr, s));
    const std::vector<int64_t> Th = down(T.get(), (size_t)R * nch, s);
    std::vector<int64_t> rt_off((size_t)R * nch);
    int64_t base = 0;
    for (int64_t i = 0; i < R; ++i) {
      int64_t rowtot = 0;
      for (int t = 0; t < nch; ++t) {
        rt_off[i * nch + t] = base + rowtot;
        rowtot += Th[i * nch + t];
      }
      A4_CHECK(rowtot == nprod_h[rows[start + i]], "long rows: routing histogram disagrees with the product counts");
      base += rowtot;
    }
    DevBuf<int64_t> drt_off = up(rt_off, s);
    DevBuf<unsigned long long> scratch((size_t)std::max<int64_t>(base, 1), s);
    A4_HIP((hipError_t)spmm_spgemm_long_route(1, A.ci.get(), A.v.get(), B.rp.get(), B.ci.get(), B.v.get(), de0.get(),
                                              de1.get(), nwg, nch, hist.get(), dwrow.get(), drt_off.get(),
                                              scratch.get(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                              nullptr, s));
    DevBuf<int64_t> rt_nnz((size_t)R * nch, s);
    DevBuf<int32_t> lists((size_t)2 * R * nch + 4, s);
    A4_HIP((hipError_t)spmm_spgemm_long_dense(values, drt_off.get(), T.get(), R * nch, nch, scratch.get(), rt_nnz.get(),
                                              lists.get(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 100, s));
    const std::vector<int64_t> nz = down(rt_nnz.get(), (size_t)R * nch, s);
    if (!values) {
      for (int64_t i = 0; i < R; ++i) {
        int64_t t = 0;
        for (int c = 0; c < nch; ++c) t += nz[i * nch + c];
        (*cnt_out)[start + i] = t;
      }
    } else {
      std::vector<int64_t> dst((size_t)R * nch);
      for (int64_t i = 0; i < R; ++i) {
        int64_t at = (*Crp_h)[rows[start + i]];
        for (int c = 0; c < nch; ++c) {
          dst[i * nch + c] = at;
          at += nz[i * nch + c];
        }
        A4_CHECK(at == (*Crp_h)[rows[start + i] + 1], "long rows: numeric count disagrees with the symbolic count");
      }
      DevBuf<int64_t> ddst = up(dst, s);
      A4_HIP((hipError_t)spmm_spgemm_long_place(drt_off.get(), ddst.get(), rt_nnz.get(), R * nch, scratch.get(), Cci,
                                                Cv, s));
      A4_HIP(hipStreamSynchronize(s));
    }
    start = end;
  }
}

// ---- binned two-phase path (ops/spgemm.py symbolic + numeric) -----------------
// Rows binned on the device by their product count (bins 0..10: LDS kernels; 11: long rows).
DCsr binned_product(const DCsr& A, const DCsr& B, const Plan& pl, hipStream_t s, EngineStats* st) {
  const std::vector<int64_t> nprod_h = down(pl.nprod.get(), A.m, s);
  const std::vector<int64_t> Arp_h = down(A.rp.get(), A.m + 1, s);
  const double seg = (double)pl.tot / (double)std::max<int64_t>(A.nnz, 1);
  DevBuf<int64_t> bsplit;
  auto splits = [&]() -> const int64_t* {
    if (!bsplit.get()) {
      bsplit = DevBuf<int64_t>((size_t)B.m * 7, s);
      A4_HIP((hipError_t)spmm_spgemm_row_splits(B.rp.get(), B.ci.get(), B.m, (int)B.n, bsplit.get(), s));
    }
    return bsplit.get();
  };
  auto slices = [](int b) { return b == 8 ? 2 : (b == 9 ? 4 : (b == 10 ? 8 : 1)); };
  DevBuf<int32_t> flags((size_t)std::max<int64_t>(A.m, 1), s);
  DevBuf<int64_t> d64(1, s);
  DevBuf<int32_t> d32(1, s);
  DevBuf<float> df(1, s);
  // rows ordered by bin on the device (csr_rowsort.hip spmm_spgemm_bin_rows, the bin table of
  // ops/spgemm.py _bins): one 13-word read-back per phase instead of a host pass over the rows
  DevBuf<int32_t> order((size_t)std::max<int64_t>(A.m, 1), s), sel((size_t)std::max<int64_t>(A.m, 1), s);
  DevBuf<int64_t> hist(13, s), nsel(1, s);
  DevBuf<uint8_t> bws(std::max<size_t>(spmm_spgemm_bin_rows_ws(A.m), 1), s);
  const Knobs& kn = knobs();
  // rows whose flag word has a bit of mask (device selection, the small list read back, sorted)
  auto flagged = [&](int mask) {
    A4_HIP((hipError_t)spmm_rows_with_flag(flags.get(), A.m, mask, sel.get(), nsel.get(), s));
    const int64_t n = down(nsel.get(), 1, s)[0];
    std::vector<int32_t> r = down(sel.get(), (size_t)n, s);
    std::sort(r.begin(), r.end());
    return r;
  };
  // run the LDS bins of one phase; returns the rows for the long-row path
  auto run_bins = [&](int numeric, int32_t* row_nnz, const int64_t* Crp, int32_t* Cci, float* Cv) {
    A4_HIP((hipError_t)spmm_spgemm_bin_rows(pl.nprod.get(), A.m, numeric, kn.load, kn.load_sliced, kn.esc_min,
                                            order.get(), hist.get(), bws.get(), s));
    const std::vector<int64_t> hh = down(hist.get(), 13, s);
    A4_HIP(hipMemsetAsync(flags.get(), 0, std::max<int64_t>(A.m, 1) * sizeof(int32_t), s));
    int64_t off = hh[0];   // (empty rows first)
    for (int b = 0; b <= 10; ++b) {
      const int64_t cnt = hh[b + 1];
      if (cnt) {
        const bool multi = b >= 8;
        A4_HIP((hipError_t)spmm_spgemm_lds(b, numeric, A.rp.get(), A.ci.get(), A.v.get(), B.rp.get(), B.ci.get(),
                                           B.v.get(), multi ? splits() : nullptr, order.get() + off, cnt, (int)B.n,
                                           group_log2(seg / slices(b)), row_nnz, nullptr, Crp ? Crp : d64.get(),
                                           Cci ? Cci : d32.get(), Cv ? Cv : df.get(), flags.get(), s));
      }
      off += cnt;
    }
    std::vector<int32_t> lr = down(order.get() + off, (size_t)hh[12], s);   // bin 11: the long-row path
    A4_CHECK(flagged(4).empty(), "spgemm: output position out of range (kernel invariant violated)");
    const std::vector<int32_t> ovf = flagged(2);   // a slice could overflow its LDS table
    lr.insert(lr.end(), ovf.begin(), ovf.end());
    std::sort(lr.begin(), lr.end());
    return lr;
  };
  // symbolic: exact nnz per row
  DevBuf<int32_t> row_nnz((size_t)std::max<int64_t>(A.m, 1), s);
  A4_HIP(hipMemsetAsync(row_nnz.get(), 0, std::max<int64_t>(A.m, 1) * sizeof(int32_t), s));
  const std::vector<int32_t> sym = run_bins(0, row_nnz.get(), nullptr, nullptr, nullptr);
  std::vector<int32_t> nnz_h = down(row_nnz.get(), A.m, s);
  std::vector<int64_t> lcnt(sym.size());
  long_rows(0, A, B, sym, nprod_h, Arp_h, s, &lcnt, nullptr, nullptr, nullptr);
  for (size_t i = 0; i < sym.size(); ++i) {
    A4_CHECK(lcnt[i] < INT32_MAX, "a row of the product has 2^31 or more entries");
    nnz_h[sym[i]] = (int32_t)lcnt[i];
  }
  std::vector<int64_t> Crp_h(A.m + 1, 0);
  for (int64_t r = 0; r < A.m; ++r) Crp_h[r + 1] = Crp_h[r] + nnz_h[r];
  DCsr C;
  C.m = A.m;
  C.n = B.n;
  C.nnz = Crp_h[A.m];
  C.rp = up(Crp_h, s);
  C.ci = DevBuf<int32_t>((size_t)std::max<int64_t>(C.nnz, 1), s);
  C.v = DevBuf<float>((size_t)std::max<int64_t>(C.nnz, 1), s);
  row_nnz = up(nnz_h, s);   // the numeric kernels' per-row capacities (exact)
  // numeric: values into the layout fixed by the symbolic phase
  const std::vector<int32_t> num = run_bins(1, row_nnz.get(), C.rp.get(), C.ci.get(), C.v.get());
  long_rows(1, A, B, num, nprod_h, Arp_h, s, nullptr, &Crp_h, C.ci.get(), C.v.get());
  st->long_rows += (int64_t)num.size();
  // rows the ordered LDS tables could not keep sorted (flag 1): re-sorted here
  const std::vector<int32_t> bad = flagged(1);
  // ... on the device (csr_rowsort.hip, the kernels ops/csr.py sort_rows uses): the row
  // lengths are host values here, so no read-back at all
  if (!bad.empty()) {
    std::vector<int64_t> rows_h(bad.begin(), bad.end());
    int64_t total = 0, maxlen = 0;
    for (int32_t r : bad) {
      const int64_t n = Crp_h[r + 1] - Crp_h[r];
      total += n;
      maxlen = std::max(maxlen, n);
    }
    DevBuf<int64_t> rows_d = up(rows_h, s);
    DevBuf<uint8_t> ws(std::max<size_t>(spmm_csr_sort_rows_ws((int64_t)rows_h.size(), total, maxlen), 1), s);
    A4_HIP((hipError_t)spmm_csr_sort_rows(C.rp.get(), rows_d.get(), (int64_t)rows_h.size(), total, maxlen, C.ci.get(),
                                          C.v.get(), ws.get(), s));
    st->device_sorted_rows += (int64_t)bad.size();
  }
  return C;
}

}  // namespace

DCsr dcsr_upload(const Csr& H, hipStream_t s) {
  DCsr D;
  D.m = H.m;
  D.n = H.n;
  D.nnz = H.nnz();
  D.rp = up(H.rp, s);
  D.ci = up(H.ci, s);
  D.v = up(H.v, s);
  return D;
}

Csr dcsr_download(const DCsr& D, hipStream_t s) {
  Csr H;
  H.m = D.m;
  H.n = D.n;
  H.rp = down(D.rp.get(), D.m + 1, s);
  H.ci = down(D.ci.get(), D.nnz, s);
  H.v = down(D.v.get(), D.nnz, s);
  return H;
}

DCsr dev_spgemm(const DCsr& A, const DCsr& B, hipStream_t s, EngineStats* st, int64_t* products) {
  A4_CHECK(A.n == B.m, "inner dimensions differ");
  if (A.m == 0 || A.nnz == 0 || B.nnz == 0) {
    *products = 0;
    return empty_product(A, B, s);
  }
  const Plan pl = row_plan(A, B, s);
  *products = pl.tot;
  if (pl.tot == 0) return empty_product(A, B, s);
  A4_CHECK(pl.mx < (int64_t(1) << 31), "a row of the product has 2^31 or more intermediate products");
  DCsr C;
  if (bitmap_product(A, B, pl, s, &C)) {
    ++st->bitmap;
    return C;
  }
  ++st->binned;
  return binned_product(A, B, pl, s, st);
}

}  // namespace a4
