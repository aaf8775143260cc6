// Plan of one bitmap-rank SpGEMM (csr_bitmap_plan.hip): plain C structs shared by the HIP
// library, the native engine (csrc/runtime/csr_engine.cpp) and ops/spgemm.py (ctypes mirror
// _BmOpts / _BmPlan: keep the field order in step).
#pragma once
#include <cstdint>

extern "C" {

struct SpmmBmOpts {
  int32_t mode;            // 0 off, 1 auto, 2 on (SPMM_SPGEMM_BITMAP)
  int32_t cfg;             // window configuration, -1 = pick from the mean row products
  int32_t rows_mode;       // row-major kernels: 0 off, 1 auto, 2 on
  int32_t det;             // deterministic summation order
  int32_t pad;             // padded 128-byte B segments
  int32_t cv;              // interleaved (column, value) pairs for the numeric kernels
  int32_t pipe;            // software-pipelined row kernels
  int32_t use_ws8;         // 0: per-unit kernels only (a B window segment of >= 65536 entries)
};

struct SpmmBmPlan {
  int32_t cfg, lgw, nwin, nsub, lg_count, lg_c, nsub_c, lg_num;
  int32_t count_rows, rows, det, pipe, ws8, pad_num, pad_cnt;
  int64_t m, annz, mb, nnzb, tot, nunits, ngc, cap_bcv, cap_colp, ovf_cap;
  // workspace byte offsets (-1: not used) and size
  int64_t o_split, o_ucnt, o_ws8, o_plen, o_plenc, o_pbase, o_cbase, o_colp, o_bcv, o_ovf, o_scan, ws_bytes;
};

// B as it lands from the row-block all-gathers (models/spgemm.py RowblockGraph), read in
// place by the layout kernels instead of being unpacked into contiguous arrays first.
// Panel r (B rows rbase[r] .. rbase[r + 1], entries ebase[r] .. ebase[r + 1]) has its
// columns at gc + r * cstride (packed to `bits` bits when bits < 32) and its value bits at
// gv + r * vstride.  gc == nullptr: B is contiguous (the plain arrays).
struct SpmmBmGathered {
  const uint32_t* gc;
  const uint32_t* gv;
  const int64_t* ebase;   // device [W + 1]
  const int64_t* rbase;   // device [W + 1]
  int64_t cstride, vstride;
  int32_t W, bits;
};

}
