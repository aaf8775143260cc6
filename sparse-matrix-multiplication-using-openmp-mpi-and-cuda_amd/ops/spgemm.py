"""CSR x CSR SpGEMM (fp32): C = A . B.

GPU path (gfx950, ``csrc/kernels/csr_spgemm.hip``):
  1. ``nprod``: intermediate products per row (one wave per row).
  2. Symbolic: rows binned by nprod into LDS hash kernels (128 .. 8192 keys
     single pass at load <= LOAD, 16384 keys over 1/2/4/8 column slices at load
     <= LOAD_SLICED); longer rows go to the HBM-workspace kernel.  Output:
     exact nnz per row.
  3. Row pointer by a device scan; C allocated once.
  4. Numeric: short rows in ordered-linear-probing LDS tables (a monotone
     hash keeps every table sorted: the output is a compaction of the table),
     long rows in the bucketed ESC kernel over 1/2/4/8 column slices, hub rows
     through the HBM column-chunked path.
  One-pass mode (default when memory allows) skips 2-3: rows are written at
  product-count offsets and compacted ("plain"), or, when that staging does
  not fit, processed in row chunks with two chunk-sized staging buffers and
  the compaction overlapped on a side stream ("pipelined").
CPU path: OpenMP Gustavson (``libspmm_host.so``), identical output layout.

FLOPs are counted as 2 * sum(nprod) (one multiply + one add per intermediate
product), the convention of BASELINE.md.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import _native
from .._native import c_vp
from ..utils.config import CONFIG
from .csr import CSR, sort_rows
import ctypes as C
import threading

C_I64 = C.c_int64
C_INT = C.c_int

_native.register_hip("spmm_spgemm_row_nprod", c_vp, c_vp, c_vp, C_I64, c_vp, c_vp)
_native.register_hip("spmm_spgemm_row_plan", c_vp, c_vp, c_vp, C_I64, C_I64, C_I64, C_I64, C_I64, c_vp, c_vp, c_vp,
                     c_vp, c_vp)
_native.register_hip("spmm_spgemm_ordered_units", c_vp, c_vp, C_I64, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_row_splits", c_vp, c_vp, C_I64, C_INT, c_vp, c_vp)
_native.register_hip("spmm_spgemm_lds", C_INT, C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT,
                     C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_compact", c_vp, c_vp, C_I64, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_long_route", C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT, c_vp,
                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_long_wg_scan", c_vp, c_vp, c_vp, C_I64, C_INT, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_long_btab", c_vp, c_vp, c_vp, C_I64, C_INT, c_vp, c_vp)
_native.register_hip("spmm_spgemm_long_dense", C_INT, c_vp, c_vp, C_I64, C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                     c_vp, c_vp, C_INT, c_vp)
_native.register_hip("spmm_spgemm_long_place", c_vp, c_vp, c_vp, C_I64, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_long_params", c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_esc_ordered", c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT,
                     C_INT, c_vp, c_vp, C_I64, c_vp, c_vp, c_vp, c_vp, c_vp, C_INT, c_vp)
_native.register_hip("spmm_spgemm_stamps", C_INT, c_vp)
_native.register_hip("spmm_spgemm_bm_config", C_INT, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_bm_stamps", C_INT, c_vp)
_native.register_hip("spmm_spgemm_bm_pack_ws8", c_vp, C_I64, C_INT, c_vp, c_vp, c_vp, c_vp, C_INT, c_vp)
_native.register_hip("spmm_spgemm_bm_count_rows", C_INT, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT, C_INT, C_INT, c_vp, c_vp,
                     C_I64, C_INT, C_INT, C_I64, c_vp)
_native.register_hip("spmm_spgemm_bm_numeric_rows", C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT,
                     C_INT, c_vp, C_I64, c_vp, c_vp, c_vp, c_vp, C_I64, c_vp, C_INT, C_INT, C_I64, C_INT, C_I64, c_vp)
_native.register_hip("spmm_spgemm_bm_pad_pairs", c_vp, c_vp, c_vp, C_I64, C_INT, C_INT, c_vp, c_vp, c_vp, c_vp, C_INT, c_vp,
                     C_I64, C_I64, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_bm_splits", c_vp, c_vp, C_I64, C_INT, C_INT, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_bm_unpack_gathered", c_vp, c_vp, C_INT, C_I64, C_I64, C_INT, c_vp, C_I64, c_vp,
                     c_vp, c_vp, c_vp)
_native.register_hip("spmm_pack_bits", c_vp, C_I64, C_INT, c_vp, C_I64, c_vp)
_native.register_hip("spmm_spgemm_bm_count", C_INT, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT, C_INT, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_bm_numeric", C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT, C_INT, c_vp,
                     C_I64, c_vp, c_vp, c_vp, c_vp, C_I64, c_vp, C_INT, c_vp, c_vp, c_vp)

# LDS bins (csr_spgemm.hip: every table <= 80 KB so two workgroups share a CU).
# Symbolic: b = 0..6 single pass (128 << b keys), 7..10 = 16384 keys over
# 1 / 2 / 4 / 8 column slices.  Numeric: b = 0..6 single pass (128 << b ordered
# key/value slots) for rows of <= ESC_MIN products, 7..10 = bucketed ESC with
# 7680 products per slice over 1 / 2 / 4 / 8 slices (bin_caps).  Then the HBM path.
# Numeric rows are binned by their PRODUCT count (the ESC capacity is in
# products, and it bounds the distinct count for the hash bins).
SYM_SINGLE_TOP = 6
NUM_SINGLE_TOP = 6
SYM_SLICED = (7, 8, 9, 10)
NUM_SLICED = (8, 9, 10)
SYM_GLOBAL = 11
NUM_GLOBAL = 11
LOAD = CONFIG.spgemm_load              # max load factor of a single-pass LDS table
LOAD_SLICED = CONFIG.spgemm_load_sliced   # ... of the big (column-sliced) tables
ESC_MIN = CONFIG.spgemm_esc_min        # numeric rows with more products use the ESC kernel
GLOBAL_WS_BYTES = int(CONFIG.spgemm_global_ws_gb * (1 << 30))   # HBM scratch budget per batch of long rows


@dataclass
class SpgemmInfo:
    flops: int = 0
    nnz: int = 0
    rows_per_bin_sym: Dict[int, int] = field(default_factory=dict)
    rows_per_bin_num: Dict[int, int] = field(default_factory=dict)
    resorted_rows: int = 0
    partial_nnz: int = 0      # innerdim_spgemm: nnz of this rank's full-height partial before the merge
    deterministic: bool = False   # C's fp32 sums were formed in a fixed (Gustavson) order
    mean_seg: float = 0.0     # mean B-row length per A entry (products / nnz(A)); picks the LDS lane groups


_native.register_hip("spmm_spgemm_bin_caps", C_INT, C.c_double, C.c_double, C_I64, c_vp)
_native.register_hip("spmm_spgemm_plan_params", c_vp, c_vp, c_vp)
_CAPS: Dict[tuple, List[int]] = {}
_PARAMS: List = []


def bin_caps(numeric: int) -> List[int]:
    """Capacities of LDS bins 0..10 (csr_spgemm.hip spmm_spgemm_bin_caps, the
    table the native engine bins with too); a row beyond caps[10] takes the
    long-row path."""
    key = (int(numeric), LOAD, LOAD_SLICED, ESC_MIN)
    if key not in _CAPS:
        caps = (C.c_int64 * 11)()
        _native.check(_native.hip().spmm_spgemm_bin_caps(int(numeric), float(LOAD), float(LOAD_SLICED), int(ESC_MIN),
                                                         caps), "spgemm_bin_caps")
        _CAPS[key] = list(caps)
    return _CAPS[key]


def plan_params():
    """(row-plan workgroups, statistics per workgroup, ESC per-slice margin) of
    csr_spgemm.hip (spmm_spgemm_plan_params)."""
    if not _PARAMS:
        pb, ps, el = C.c_int(), C.c_int(), C.c_double()
        _native.check(_native.hip().spmm_spgemm_plan_params(C.byref(pb), C.byref(ps), C.byref(el)), "plan_params")
        _PARAMS.append((pb.value, ps.value, el.value))
    return _PARAMS[0]


def _bins(counts: torch.Tensor, numeric: int) -> torch.Tensor:
    """Bin per row: the smallest single-pass table with counts <= LOAD * S, then
    the sliced passes (slice capacity LOAD * S_top * slices), then the HBM path;
    -1 for empty rows."""
    caps = bin_caps(numeric)
    b = torch.bucketize(counts, torch.tensor(caps, device=counts.device, dtype=counts.dtype))
    return torch.where(counts == 0, torch.full_like(b, -1), b)


def _group(bins: torch.Tensor, nbins: int):
    """rows ordered by bin + host list of (bin, offset, count) for bins 0..nbins-1."""
    order = torch.argsort(bins, stable=True).to(torch.int32)
    hist = torch.bincount(bins + 1, minlength=nbins + 1).tolist()
    groups, off = [], hist[0]
    for b in range(nbins):
        cnt = hist[b + 1]
        if cnt:
            groups.append((b, off, cnt))
        off += cnt
    return order, groups




def row_plan(A: CSR, B: CSR):
    """Device row plan (``spgemm_row_plan`` + ``spgemm_plan_finish``): per-row
    product counts, ordered one-pass unit counts (``_ordered_slices``), and an
    int64[16] of {sum, max, non-empty rows, light rows, #rows with 1 / 2 / 4 / 8
    units, max nnz of an A row, 0 ...}.  GPU only."""
    dev = A.device
    nprod = torch.empty(A.m, dtype=torch.int64, device=dev)
    nsl = torch.empty(A.m, dtype=torch.int64, device=dev)
    nblk, nst, esc_load = plan_params()
    part = torch.empty((nblk + 1) * nst, dtype=torch.int64, device=dev)
    stats = part[nblk * nst:]
    c1 = int(esc_load * CONFIG.spgemm_ordered_pcap)
    P = _native.ptr
    _native.check(_native.hip().spmm_spgemm_row_plan(P(A.rowptr), P(A.col), P(B.rowptr), A.m, c1, 2 * c1, 4 * c1,
                                                      ESC_MIN, P(nprod), P(nsl), P(part), P(stats),
                                                      _native.stream_ptr(dev)), "spgemm_row_plan")
    return nprod, nsl, stats


def row_nprod(A: CSR, B: CSR) -> torch.Tensor:
    nprod = torch.empty(A.m, dtype=torch.int64, device=A.device)
    P = _native.ptr
    if A.device.type == "cuda":
        _native.check(_native.hip().spmm_spgemm_row_nprod(P(A.rowptr), P(A.col), P(B.rowptr), A.m, P(nprod),
                                                           _native.stream_ptr(A.device)), "spgemm_row_nprod")
    else:
        _native.host().spmm_cpu_csr_nprod(A.m, P(A.rowptr), P(A.col), P(B.rowptr), P(nprod), 0)
    return nprod


class _FreeMem:
    """Device bytes free to this process, asked lazily: the driver's free
    memory (hipMemGetInfo, ~2 us) answers most questions; the caching
    allocator's spare (reserved - allocated: ~70 us, it builds the full
    allocator statistics) is added only when the driver figure alone is too
    small, e.g. when an earlier product's C is still cached in the pool."""

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.driver = torch.cuda.mem_get_info(dev)[0]
        self.spare = None

    def fits(self, nbytes: float, frac: float = 0.8) -> bool:
        if nbytes <= frac * self.driver:
            return True
        if self.spare is None:
            self.spare = torch.cuda.memory_reserved(self.dev) - torch.cuda.memory_allocated(self.dev)
        return nbytes <= frac * (self.driver + self.spare)


def _onepass_mode(total_products: int, dev: torch.device, allow_pipeline: bool = True,
                  pre_free: Optional[_FreeMem] = None) -> Optional[str]:
    """"plain": a product-count-sized staging buffer next to C (fastest);
    "pipelined": C at its product-count bound plus two chunk-sized staging
    buffers (~half the memory, ~3 % slower: the overlapped compaction and
    the numeric kernels compete for HBM); None: symbolic + numeric."""
    mode = CONFIG.spgemm_onepass
    if mode == "off":
        return None
    pipe_ok = allow_pipeline and total_products >= PIPE_MIN_PRODUCTS and CONFIG.spgemm_pipeline != "off"
    if CONFIG.spgemm_pipeline == "on" and pipe_ok:
        return "pipelined"
    if mode == "on":
        return "plain"
    free = pre_free if pre_free is not None else _FreeMem(dev)
    if free.fits(2 * total_products * 8):
        return "plain"
    if pipe_ok and free.fits((total_products + 2 * PIPE_CHUNK_PRODUCTS) * 8):
        return "pipelined"
    return None


_LONG = None
LONG_STATS: Optional[dict] = None   # diagnostics (tools/long_items.py): item-size histogram of the long-row path


def _long_stats(rt_cnt: torch.Tensor) -> None:
    """Accumulate (items, products) per log2 item-size bucket into LONG_STATS."""
    b = torch.floor(torch.log2(rt_cnt.double() + 1)).long()
    items = torch.bincount(b, minlength=40).tolist()
    prods = torch.bincount(b, weights=rt_cnt.double(), minlength=40).tolist()
    for k in range(40):
        if items[k]:
            it, pr = LONG_STATS.get(k, (0, 0.0))
            LONG_STATS[k] = (it + items[k], pr + prods[k])


def _long_params():
    global _LONG
    if _LONG is None:
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        _native.hip().spmm_spgemm_long_params(C.byref(a), C.byref(b), C.byref(c))
        _LONG = (a.value, b.value, c.value)
    return _LONG


LONG_BTAB_MIN = 4   # B rows of >= this many entries per column chunk get a chunk-offset table


def _long_btab(B: CSR, nch: int):
    """(lidx, btab) of B for the routing histogram (csr_spgemm.hip long_btab):
    lidx[j] = index of B row j among the rows of >= LONG_BTAB_MIN * nch
    entries (else -1), btab = those rows' nch + 1 chunk offsets.  Memoised on
    the operand like :func:`_splits` (a streamed product routes many A row
    panels against one B).  (None, None) when B has no such row."""
    key = (B.rowptr.data_ptr(), B.col.data_ptr(), B.m, B.n, B.nnz, nch)
    hit = getattr(B, "_btab_memo", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    lens = B.rowptr[1:] - B.rowptr[:-1]
    lrows = (lens >= LONG_BTAB_MIN * nch).nonzero().flatten().to(torch.int32)
    nlong = lrows.numel()
    out = (None, None)
    if nlong:
        lidx = torch.full((B.m,), -1, dtype=torch.int32, device=B.device)
        lidx[lrows.long()] = torch.arange(nlong, dtype=torch.int32, device=B.device)
        btab = torch.empty(nlong * (nch + 1), dtype=torch.int32, device=B.device)
        _native.check(_native.hip().spmm_spgemm_long_btab(_native.ptr(B.rowptr), _native.ptr(B.col), _native.ptr(lrows),
                                                           nlong, nch, _native.ptr(btab), _native.stream_ptr(B.device)),
                      "spgemm_long_btab")
        out = (lidx, btab)
    B._btab_memo = (key, out)
    return out


# long_dense / long_rank grids on the side stream, beside the next batch's routing: this share
# (percent) of their resident capacity (R-MAT 24: 75 -> 11.46-11.48 s, 70 -> 11.59, 80 -> 11.89,
# 100 -> 11.94, 50 -> 13.13; PERF_LOG round 6)
LONG_SIDE_GRID_PCT = 75


def _long_rows(values: int, A: CSR, B: CSR, rows: torch.Tensor, nprod_rows: torch.Tensor, stream,
               out_nnz: Optional[torch.Tensor] = None, Crp=None, Cci=None, Cv=None,
               expect_nnz: Optional[torch.Tensor] = None, defer: Optional[list] = None) -> None:
    """Rows beyond the LDS bins: column-chunked dense accumulation through an
    HBM scratch (csr_spgemm.hip "long rows").  ``values=0`` only counts
    (writes ``out_nnz[rows]``); ``values=1`` also writes each row at
    ``Crp[row]`` (and its count to ``out_nnz`` when given).  Rows are
    processed in batches whose products fit the scratch budget.

    Direct mode (``CONFIG.spgemm_long_direct``, B with long rows): items of
    more than LR_CAP products take the products of the row's long B rows
    straight from B (long_dense reads their chunk segments through the btab
    table) instead of through the scratch.

    The batches are planned on the host from ONE read-back of the rows'
    product and entry counts, and the loop has no device->host sync (buffers
    are sized from that plan); the product-count consistency checks
    accumulate on the device and are read once at the end.

    ``defer``: instead of placing the rows at ``Crp``, append each batch's
    ``(rows, rt_off, rt_nnz, scratch)`` (chunk results still in the scratch)
    so the caller places them at final offsets once those are known
    (``place_long``): the pipelined one-pass skips a staging round trip."""
    dev = A.device
    lib = _native.hip()
    P = _native.ptr
    lgw, epw, maxch = _long_params()
    nch = (B.n + (1 << lgw) - 1) >> lgw
    if nch > maxch:
        raise ValueError(f"long-row path supports at most {maxch << lgw} columns, got {B.n}")
    lidx, btab = _long_btab(B, nch) if CONFIG.spgemm_long_btab else (None, None)
    direct = bool(CONFIG.spgemm_long_direct) and btab is not None and B.nnz < (1 << 32)
    rows = rows.long()
    nrows = rows.numel()
    if nrows == 0:
        return
    na_all = (A.rowptr[rows + 1] - A.rowptr[rows])
    host = torch.stack([nprod_rows.long(), na_all]).cpu()   # the one planning read-back
    np_h, na_h = host[0].numpy(), host[1].numpy()
    csum_h = np.cumsum(np_h)
    cap = max(GLOBAL_WS_BYTES // 8, int(np_h.max()))
    nwg_h = np.maximum((na_h + epw - 1) // epw, 1)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)   # rows whose counts disagree (device-side)
    nil = None
    # Side stream: a batch's accumulation (long_dense / long_rank: LDS-bound) and what follows
    # it run on the side stream, so the next batch's routing passes (HBM-write-bound) run
    # beside them on the main one; the main stream waits for the side one before returning
    sA = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    side = (sA is not None and CONFIG.spgemm_long_side and int(stream or 0) == int(sA.cuda_stream))
    sB = _side_stream(dev) if side else None
    bad_b = torch.zeros(1, dtype=torch.int64, device=dev) if side else bad   # (written on the side stream)
    start, done = 0, 0
    while start < nrows:
        # batch = the longest run of rows from start whose products fit cap (at least one row)
        end = int(np.searchsorted(csum_h, done + cap, side="right"))
        end = min(max(end, start + 1), nrows)
        rb = rows[start:end]
        R = end - start
        nwg = int(nwg_h[start:end].sum())
        a0 = A.rowptr[rb]
        na = na_all[start:end]
        nwg_r = torch.clamp((na + epw - 1) // epw, min=1)
        row_of_wg = torch.repeat_interleave(torch.arange(R, device=dev), nwg_r, output_size=nwg)
        first_wg = torch.cumsum(nwg_r, 0) - nwg_r
        kk = torch.arange(nwg, device=dev) - first_wg[row_of_wg]
        wg_e0 = (a0[row_of_wg] + kk * epw).contiguous()
        wg_e1 = torch.minimum(wg_e0 + epw, (a0 + na)[row_of_wg]).contiguous()
        wg_hist = torch.empty(nwg * nch, dtype=torch.int32, device=dev)
        wg_dhist = torch.empty(nwg * nch, dtype=torch.int32, device=dev) if direct else None
        wg_nlong = torch.empty(nwg, dtype=torch.int32, device=dev) if direct else None
        _native.check(lib.spmm_spgemm_long_route(0, P(A.col), P(A.val), P(B.rowptr), P(B.col), P(B.val), P(wg_e0),
                                                 P(wg_e1), nwg, nch, P(wg_hist), nil, nil, nil,
                                                 P(lidx) if lidx is not None else nil,
                                                 P(btab) if btab is not None else nil,
                                                 P(wg_dhist) if direct else nil, P(wg_nlong) if direct else nil,
                                                 nil, nil, nil, stream), "long_route")
        # the [workgroups x chunks] histogram becomes per-workgroup offsets in
        # place (one kernel); only the [rows x chunks] region sizes go through
        # torch
        T = torch.empty((R, nch), dtype=torch.int64, device=dev)
        D = torch.empty((R, nch), dtype=torch.int64, device=dev) if direct else None
        mode = torch.empty(R * nch, dtype=torch.uint8, device=dev) if direct else None
        _native.check(lib.spmm_spgemm_long_wg_scan(P(wg_hist), P(first_wg), P(nwg_r), R, nch, P(T),
                                                   P(wg_dhist) if direct else nil, P(D) if direct else nil,
                                                   P(mode) if direct else nil, stream), "long_wg_scan")
        del wg_dhist
        # scratch regions: the routed products; a direct item also holds its
        # compacted result (<= min(W, all its products) entries)
        region = torch.maximum(T, torch.clamp(T + D, max=1 << lgw)) if direct else T
        chunk_off = torch.cumsum(region, 1) - region
        row_reg = region.sum(1)
        row_base = torch.cumsum(row_reg, 0) - row_reg
        # the scatter pass writes exactly the histogram's slots, while the
        # scratch below is sized from the host plan's product counts (no
        # read-back).  Both count the same (A entry, B row) pairs, so they agree
        # unless a kernel is broken; this comparison, read once after the loop,
        # only DETECTS such a failure -- it does not keep the scatter in bounds.
        bad += ((T + D).sum(1) if direct else T.sum(1)).ne(nprod_rows[start:end]).sum()
        rt_off = (row_base[:, None] + chunk_off).reshape(-1).contiguous()   # each (row, chunk) region's base
        # sizes from the host plan (no read-back): the regions never exceed the
        # batch's products, the long-entry list never its A entries
        if direct:
            nl_r = wg_nlong.long()
            dl_off = (torch.cumsum(nl_r, 0) - nl_r).contiguous()
            dl_rp = torch.cat([dl_off[first_wg], (dl_off[-1:] + nl_r[-1:])]).contiguous()
            dl = torch.empty((max(int(na_h[start:end].sum()), 1), 4), dtype=torch.int32, device=dev)
        ntot = int(csum_h[end - 1]) - done
        scratch = torch.empty(max(ntot, 1), dtype=torch.int64, device=dev)
        wg_row = row_of_wg.to(torch.int32)
        _native.check(lib.spmm_spgemm_long_route(1, P(A.col), P(A.val), P(B.rowptr), P(B.col), P(B.val), P(wg_e0),
                                                 P(wg_e1), nwg, nch, P(wg_hist), P(wg_row), P(rt_off), P(scratch),
                                                 P(lidx) if lidx is not None else nil,
                                                 P(btab) if btab is not None else nil, nil, nil,
                                                 P(mode) if direct else nil, P(dl) if direct else nil,
                                                 P(dl_off) if direct else nil, stream), "long_route")
        del wg_hist, wg_row
        rt_cnt = T.reshape(-1)
        if LONG_STATS is not None:
            _long_stats(rt_cnt + D.reshape(-1) if direct else rt_cnt)
        if side:   # this batch's routed scratch is complete on the main stream
            sB.wait_stream(sA)
            for t in (rb, rt_off, T, scratch, *((D, dl, dl_rp, dl_off, mode) if direct else ())):
                t.record_stream(sB)
        with torch.cuda.stream(sB) if side else _nullctx():
            st = sB.cuda_stream if side else stream
            rt_nnz = torch.empty(R * nch, dtype=torch.int64, device=dev)
            lists = torch.empty(2 * R * nch + 4, dtype=torch.int32, device=dev)   # the two kernels' item lists + counters
            _native.check(lib.spmm_spgemm_long_dense(values, P(rt_off), P(rt_cnt), R * nch, nch, P(scratch), P(rt_nnz),
                                                     P(lists), P(D) if direct else nil, P(dl) if direct else nil,
                                                     P(dl_rp) if direct else nil, P(btab) if direct else nil,
                                                     P(B.col) if direct else nil, P(B.val) if direct else nil,
                                                     LONG_SIDE_GRID_PCT if side else 100, st),
                          "long_dense")
            del lists
            nnz_rt = rt_nnz.view(R, nch)
            nnz_r = nnz_rt.sum(1)
            if expect_nnz is not None:
                bad_b += nnz_r.ne(expect_nnz[rb].long()).sum()
            if out_nnz is not None:
                out_nnz[rb] = nnz_r.to(out_nnz.dtype)
            if values and defer is not None:
                defer.append((rb, rt_off, rt_nnz, scratch))
            elif values:
                dst = (Crp[rb][:, None] + torch.cumsum(nnz_rt, 1) - nnz_rt).reshape(-1).contiguous()
                _native.check(lib.spmm_spgemm_long_place(P(rt_off), P(dst), P(rt_nnz), R * nch, P(scratch), P(Cci),
                                                         P(Cv), st), "long_place")
        if side and values and defer is not None:
            rt_nnz.record_stream(sA)   # (allocated on the side stream, read by the caller's placement)
        if direct:
            del dl, dl_rp, dl_off, mode
        del scratch
        done = int(csum_h[end - 1])
        start = end
    if side:
        sA.wait_stream(sB)
        bad += bad_b
    nbad = int(bad)
    if nbad:
        raise RuntimeError(f"spgemm long rows: routing histogram or numeric count disagrees with the product / "
                           f"symbolic counts ({nbad} rows)")


def place_long(defer: list, rowptr: torch.Tensor, Cci: torch.Tensor, Cv: torch.Tensor, stream) -> None:
    """Copy deferred long-row results (``_long_rows(..., defer=)``) from their
    scratch to the final CSR rows at ``rowptr`` (on ``stream``; the caller
    keeps the scratch alive until that stream passes this point)."""
    lib = _native.hip()
    P = _native.ptr
    for rb, rt_off, rt_nnz, scratch in defer:
        nnz_rt = rt_nnz.view(rb.numel(), -1)
        dst = (rowptr[rb][:, None] + torch.cumsum(nnz_rt, 1) - nnz_rt).reshape(-1).contiguous()
        _native.check(lib.spmm_spgemm_long_place(P(rt_off), P(dst), P(rt_nnz), rt_nnz.numel(), P(scratch), P(Cci),
                                                 P(Cv), stream), "long_place")


def spgemm(A: CSR, B: CSR, info: Optional[SpgemmInfo] = None, B_ready=None) -> CSR:
    """C = A . B.  ``B_ready``: B's columns / values are still in flight (a
    distributed gather); ``B`` then only needs a valid row pointer, and
    ``B_ready()`` is called for the complete operand right before the first
    kernel that reads them (product counts and row binning overlap it).

    Memory admission is a forecast (free-memory fractions); when a one-pass
    mode still runs out of device memory, the product is redone with the
    two-phase symbolic + numeric path, which allocates exactly nnz(C) and no
    staging buffer (``info.rows_per_bin_num["oom_fallback"]`` records it).
    The retry starts only after the device has drained: kernels of the
    failed attempt (on this and on the side stream) may still be writing
    buffers the caching allocator would hand to the retry."""
    info = info if info is not None else SpgemmInfo()
    if A.device.type != "cuda":
        return _spgemm(A, B, info, B_ready)
    try:
        return _spgemm(A, B, info, B_ready)
    except torch.OutOfMemoryError:
        if CONFIG.spgemm_onepass == "off" and CONFIG.spgemm_bitmap == "off":
            raise   # already the lowest-memory path
    torch.cuda.synchronize(A.device)
    torch.cuda.empty_cache()
    info.rows_per_bin_num = {}
    C_ = _spgemm(A, B, info, B_ready, two_phase=True)
    info.rows_per_bin_num["oom_fallback"] = 1
    return C_


def _true_nnz(B: CSR) -> int:
    """nnz of an operand whose payload may still be in flight (a distributed
    gather's row-pointer-only CSR carries the total; ``CSR.nnz`` is len(col))."""
    return max(B.nnz, getattr(B, "_nnz_total", 0))


_native.register_hip("spmm_prim_spin", C.c_double, c_vp)
_native.register_hip("spmm_prim_scan_ws", C_I64, restype=C.c_size_t)
_native.register_hip("spmm_prim_scan", c_vp, C_INT, C_I64, c_vp, C_INT, c_vp, c_vp)


def device_scan(x: torch.Tensor, out: torch.Tensor, inclusive: bool) -> torch.Tensor:
    """out[i] = sum x[0..i] (inclusive) or x[0..i-1] (exclusive), int64, with
    the in-tree scan kernels (csrc/kernels/prim.hip: tile reduce, recursive
    scan of the tile sums, tile scan + carry).  Launches only -- capturable
    into a HIP graph; replaces the host prefix of the reference
    (sparse_matrix_mult.cu:214-216) and keeps rocPRIM out of the bitmap
    product's kernel set."""
    n = x.numel()
    assert out.dtype == torch.int64 and out.numel() >= n and x.dtype in (torch.int32, torch.int64)
    if n == 0:
        return out
    lib = _native.hip()
    ws = torch.empty(int(lib.spmm_prim_scan_ws(n)), dtype=torch.uint8, device=x.device)
    x = x.contiguous()
    _native.check(lib.spmm_prim_scan(_native.ptr(x), x.element_size(), n, _native.ptr(out), int(inclusive),
                                     _native.ptr(ws), _native.stream_ptr(x.device)), "prim_scan")
    return out


def _spgemm(A: CSR, B: CSR, info: SpgemmInfo, B_ready=None, two_phase: bool = False) -> CSR:
    """``two_phase``: symbolic + numeric only (no one-pass / bitmap modes),
    the exact-memory path the OOM fallback uses."""
    if A.n != B.m:
        raise ValueError(f"inner dimensions differ: {A.n} vs {B.m}")
    if A.device != B.device:
        raise ValueError("operands on different devices")
    if A.device.type != "cuda":
        return _spgemm_cpu(A, B_ready() if B_ready is not None else B, info)
    A = A if A.val.dtype == torch.float32 else A.with_values(A.val.float())
    B = B if B.val.dtype == torch.float32 else B.with_values(B.val.float())
    # every host decision below (limits, mode, ordered-unit split) from ONE
    # device->host read of the row plan (two kernels): each sync drains the
    # stream and exposes Python launch latency, which matters for the small
    # configs and for 8-way row panels (~20 ms steps)
    nprod, nsl, st = row_plan(A, B)
    tot, mx, nz, light, h1, h2, h4, h8, amax = st.tolist()[:9]
    pre = dict(max=mx, nonempty=nz, light=light, hist=[A.m - nz, h1, h2, 0, h4, 0, 0, 0, h8], nsl=nsl, amax=amax)
    if mx >= 1 << 31:   # per-row capacities and counts are int32 in the kernels
        raise ValueError(f"a row of A.B has {mx} intermediate products (limit 2^31 - 1)")
    info.flops = 2 * tot
    info.mean_seg = info.flops / 2 / max(A.nnz, 1)
    if B_ready is not None:
        cached = []
        fetch = B_ready

        def B_ready():   # noqa: F811  (resolve the gathered operand once)
            if not cached:
                cached.append(fetch())
            return cached[0]
        # the columns-only stage of a two-stage gather (see models.spgemm.OperandReady)
        B_ready.cols = getattr(fetch, "cols", B_ready)
        B_ready.local = getattr(fetch, "local", False)
    if not two_phase:
        if _bitmap_ok(A, B, info.flops // 2, pre):
            C_ = onepass_bitmap(A, B, info, B_ready, pre)
            if C_ is not None:
                return C_
            info.rows_per_bin_num = {}
        if CONFIG.spgemm_deterministic >= 2:   # strict: no unordered GPU path
            info.rows_per_bin_num["det_cpu_fallback"] = 1
            return _det_cpu(A, B_ready() if B_ready is not None else B, info)
        if CONFIG.spgemm_onepass == "auto" or CONFIG.spgemm_ordered == "auto":
            pre["free"] = _FreeMem(A.device)
        mode = _onepass_mode(info.flops // 2, A.device, pre_free=pre.get("free"))
        if mode is not None and _ordered_ok(nprod, info.flops // 2, A.device, pre):
            C_ = onepass_ordered(A, B, nprod, info, B_ready, pre)
            if C_ is not None:
                return C_
            info.rows_per_bin_num = {}
        if mode == "pipelined":
            C_ = onepass_pipelined(A, B, nprod, info, B_ready)
            if C_ is not None:
                return C_
            info.rows_per_bin_num = {}
            if _onepass_mode(info.flops // 2, A.device, allow_pipeline=False) == "plain":   # long / spilled rows
                mode = "plain"
        if mode == "plain":
            return onepass(A, B, nprod, info, B_ready)
    if B_ready is not None:
        B = B_ready()
    row_nnz = symbolic(A, B, nprod, info)
    return numeric(A, B, row_nnz, info, nprod)


def onepass(A: CSR, B: CSR, nprod: torch.Tensor, info: SpgemmInfo, B_ready=None) -> CSR:
    """Numeric without a symbolic phase: rows are binned by their product count
    and written at product-count offsets (an upper bound of their nnz), then
    compacted into the final CSR by one copy kernel.  Trades one extra pass
    over C for the whole symbolic phase.

    Hub rows (the HBM long-row path) skip the staging buffer: their chunk
    results stay in the long-row scratch and ``place_long`` copies them
    straight to their final rows once the row pointer exists, so the
    compaction only moves the LDS-bin rows (R-MAT: most of C is hub rows,
    which were otherwise written three times)."""
    dev = A.device
    m = A.m
    staged = torch.where(_bins(nprod, 1) == NUM_GLOBAL, torch.zeros_like(nprod), nprod)
    ub = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(staged, 0, out=ub[1:])
    tot = int(ub[-1])
    Uci = torch.empty(tot, dtype=torch.int32, device=dev)
    Uv = torch.empty(tot, dtype=torch.float32, device=dev)
    out_nnz = torch.zeros(m, dtype=torch.int32, device=dev)
    flags = torch.zeros(m, dtype=torch.int32, device=dev)
    cap = nprod.to(torch.int32)
    deferred = []
    _run_bins(1, A, B, nprod, cap, ub, Uci, Uv, flags, info.rows_per_bin_num, info.mean_seg, out_nnz=out_nnz,
              B_ready=B_ready, defer=deferred)
    for rb, *_ in deferred:   # placed by place_long, not copied by the compaction
        ub[rb] = -1
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(out_nnz, 0, out=rowptr[1:])
    nnz = int(rowptr[-1])
    info.nnz = nnz
    Cci = torch.empty(nnz, dtype=torch.int32, device=dev)
    Cv = torch.empty(nnz, dtype=torch.float32, device=dev)
    P = _native.ptr
    # (deferred_placement: the two copies below -- compaction of the LDS-bin rows, placement
    # of the hub rows -- run on the side stream and the product returns at once; R-MAT's
    # streamed panels: ~12 ms of copies a panel beside the next panel's planning)
    defer = getattr(_DEFER, "on", False) and dev.type == "cuda"
    sA = torch.cuda.current_stream(dev) if defer else None
    sB = _side_stream(dev) if defer else None
    if defer:
        sB.wait_stream(sA)
    with torch.cuda.stream(sB) if defer else _nullctx():
        stream = _native.stream_ptr(dev)
        _native.check(_native.hip().spmm_spgemm_compact(P(ub), P(rowptr), m, P(Uci), P(Uv), P(Cci), P(Cv), stream),
                      "spgemm_compact")
        place_long(deferred, rowptr, Cci, Cv, stream)
    C_ = CSR(m, B.n, rowptr, Cci, Cv)
    if defer:
        for t in (ub, rowptr, Uci, Uv, Cci, Cv, *[x for d in deferred for x in d]):
            t.record_stream(sB)
        ready = torch.cuda.Event()
        ready.record(sB)
        if bool(((flags & 1) != 0).any()):   # rows to re-sort (_finish, on this stream): C complete first
            sA.wait_event(ready)
        else:
            C_.ready = ready
    del Uci, Uv, deferred
    return _finish(C_, flags, info)


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


ORDERED_MAX_LIGHT = 0.05           # ordered mode: at most this share of non-empty rows below the ESC bins


def _ordered_slices(nprod: torch.Tensor) -> torch.Tensor:
    """Units per row of the ordered one-pass: 1 / 2 / 4 / 8 column ranges by
    product count (0 for empty rows)."""
    caps = torch.tensor([int(plan_params()[2] * CONFIG.spgemm_ordered_pcap) * k for k in (1, 2, 4)], device=nprod.device,
                        dtype=nprod.dtype)
    nsl = torch.pow(2, torch.bucketize(nprod, caps)).to(torch.int64)
    return torch.where(nprod > 0, nsl, torch.zeros_like(nsl))


def _ordered_ok(nprod: torch.Tensor, total_products: int, dev: torch.device, pre: Optional[dict] = None) -> bool:
    """Ordered one-pass: every non-empty row fits the bucketed-ESC kernel
    (no HBM long rows), few rows would be better served by the small LDS
    tables, and C fits at its product-count bound.  ``pre``: the row
    statistics already read back by ``spgemm`` (max / nonempty / light)."""
    mode = CONFIG.spgemm_ordered
    if mode == "off" or total_products == 0:
        return False
    mx = pre["max"] if pre is not None else int(nprod.max())
    if mx > int(plan_params()[2] * CONFIG.spgemm_ordered_pcap) * 8:
        return False
    if mode != "on":
        if pre is not None:
            nz, light = pre["nonempty"], pre["light"]
        else:
            nz = int((nprod > 0).sum())
            light = int(((nprod > 0) & (nprod <= ESC_MIN)).sum())
        if light > ORDERED_MAX_LIGHT * nz:
            return False
        free = pre["free"] if pre is not None and pre.get("free") is not None else _FreeMem(dev)
        if not free.fits(total_products * 8):
            return False
    return True


def onepass_ordered(A: CSR, B: CSR, nprod: torch.Tensor, info: SpgemmInfo, B_ready=None,
                    pre: Optional[dict] = None) -> Optional[CSR]:
    """One-pass numeric that writes every row at its FINAL offset: rows are
    split into units (row, column-eighth range) of the bucketed-ESC kernel
    (1 / 2 / 4 / 8 per row by product count), walked in row order, and each
    unit's position comes from a decoupled look-back over the counts of the
    units before it (csr_spgemm.hip ``EscOrd``).  No staging buffer and no
    compaction copy: C is written once.  Returns None if a unit overflowed its
    LDS slice (skewed columns); the caller then runs the binned path."""
    dev = A.device
    m = A.m
    tot = info.flops // 2
    pcap = CONFIG.spgemm_ordered_pcap
    if pre is not None:
        nsl, hist = pre["nsl"], pre["hist"]
    else:
        nsl = _ordered_slices(nprod)
        hist = torch.bincount(nsl, minlength=9).tolist()
    nunits = sum(k * hist[k] for k in (1, 2, 4, 8))
    unit_row = torch.empty(nunits, dtype=torch.int32, device=dev)
    unit_q = torch.empty(nunits, dtype=torch.uint8, device=dev)
    incl = torch.cumsum(nsl, 0)
    _native.check(_native.hip().spmm_spgemm_ordered_units(_native.ptr(nsl), _native.ptr(incl), m, _native.ptr(unit_row),
                                                          _native.ptr(unit_q), _native.stream_ptr(dev)),
                  "spgemm_ordered_units")
    del incl
    for sl, b in ((1, 7), (2, 8), (4, 9), (8, 10)):
        if hist[sl]:
            info.rows_per_bin_num[b] = hist[sl]
    info.rows_per_bin_num["ordered_units"] = nunits
    if B_ready is not None:
        B = B_ready()
    splits = _splits(B) if nunits > int(hist[1]) else None
    # lane groups from the typical segment length of a unit
    seg = info.mean_seg if info.mean_seg > 0 else B.nnz / max(B.m, 1)
    lg = _group_log2(seg / max(1.0, nunits / max(m - hist[0], 1)))   # B-segment length per unit
    z = torch.zeros(2 + 2 * m, dtype=torch.int32, device=dev)   # one fill for the four int32 zero arrays
    ticket, err, out_nnz, flags = z[0:1], z[1:2], z[2:2 + m], z[2 + m:]
    status = torch.zeros(nunits, dtype=torch.int64, device=dev)
    Cci = torch.empty(tot, dtype=torch.int32, device=dev)
    Cv = torch.empty(tot, dtype=torch.float32, device=dev)
    P = _native.ptr
    _native.check(_native.hip().spmm_spgemm_esc_ordered(
        P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col), P(B.val), P(splits) if splits is not None else None,
        P(unit_row), P(unit_q), nunits, B.n, lg, P(ticket), P(status), tot, P(err), P(out_nnz), P(Cci), P(Cv),
        P(flags), pcap, _native.stream_ptr(dev)), "spgemm_esc_ordered")
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(out_nnz, 0, out=rowptr[1:])
    # one read-back: error bits, nnz, and the flag summaries _finish needs
    e, nnz, f4, f1 = torch.stack([err[0].long(), rowptr[-1], ((flags & 4) != 0).sum(),
                                  ((flags & 1) != 0).sum()]).tolist()
    if e & 2:
        raise RuntimeError("spgemm ordered: output beyond the product-count bound (kernel invariant violated)")
    if e & 1:
        info.rows_per_bin_num["ordered_fallback"] = 1
        return None
    info.nnz = nnz
    return _finish(CSR(m, B.n, rowptr, Cci[:nnz], Cv[:nnz]), flags, info, (f4, f1))


class _BmOpts(C.Structure):   # csrc/kernels/bitmap_plan.hpp SpmmBmOpts
    _fields_ = [(n, C.c_int32) for n in ("mode", "cfg", "rows_mode", "det", "pad", "cv", "pipe",
                                         "use_ws8")]


class _BmPlan(C.Structure):   # csrc/kernels/bitmap_plan.hpp SpmmBmPlan
    _fields_ = ([(n, C.c_int32) for n in ("cfg", "lgw", "nwin", "nsub", "lg_count", "lg_c", "nsub_c", "lg_num",
                                          "count_rows", "rows", "det", "pipe", "ws8", "pad_num", "pad_cnt")]
                + [(n, C.c_int64) for n in ("m", "annz", "mb", "nnzb", "tot", "nunits", "ngc", "cap_bcv", "cap_colp",
                                            "ovf_cap", "o_split", "o_ucnt", "o_ws8", "o_plen", "o_plenc", "o_pbase",
                                            "o_cbase", "o_colp", "o_bcv", "o_ovf", "o_scan", "ws_bytes")])


_native.register_hip("spmm_spgemm_bm_choose", c_vp, C_I64, C_I64, C_I64, C_I64, C_I64, C_I64, C_I64, C_I64)
_native.register_hip("spmm_spgemm_bm_make_plan", c_vp, C_I64, C_I64, C_I64, C_I64, C_I64, C_I64, C_I64, C_I64,
                     C.c_double, c_vp)
_native.register_hip("spmm_spgemm_bm_front", c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_bm_back", c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_INT, c_vp, c_vp, c_vp, C_I64,
                     c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_bm_gathered_ok", c_vp)


class BmGathered(C.Structure):   # csrc/kernels/bitmap_plan.hpp SpmmBmGathered
    """B read in place from its all-gathered panels by the layout kernels
    (models.spgemm.RowblockGraph): panel r's columns at gc + r * cstride
    (packed to ``bits`` < 32, or raw), its value bits at gv + r * vstride;
    ebase / rbase: device int64 [W + 1] entry / row bounds of the panels."""
    _fields_ = [("gc", c_vp), ("gv", c_vp), ("ebase", c_vp), ("rbase", c_vp), ("cstride", C.c_int64),
                ("vstride", C.c_int64), ("W", C.c_int32), ("bits", C.c_int32)]


def _bm_opts(use_ws8: bool = True) -> _BmOpts:
    """CONFIG -> the native plan's options (csr_bitmap_plan.hip owns the decisions)."""
    tri = {"off": 0, "auto": 1, "on": 2}
    return _BmOpts(mode=tri.get(CONFIG.spgemm_bitmap, 1), cfg=CONFIG.spgemm_bitmap_cfg,
                   rows_mode=tri.get(CONFIG.spgemm_bitmap_rows, 1),
                   det=int(CONFIG.spgemm_deterministic > 0),
                   pad=int(CONFIG.spgemm_bitmap_pad > 0), cv=int(bool(CONFIG.spgemm_bitmap_cv)),
                   pipe=int(CONFIG.spgemm_bitmap_pipe > 0), use_ws8=int(use_ws8))


def _bitmap_ok(A: CSR, B: CSR, total_products: int, pre: dict) -> bool:
    """Bitmap-rank path (the native gate spmm_spgemm_bm_choose: uint32 B
    indices, every A row stageable by the reload kernel, row products not far
    above the mean -- a skewed matrix, e.g. R-MAT, takes the binned path) and
    the product-count bound of C in free device memory."""
    if CONFIG.spgemm_bitmap == "off" or total_products == 0:
        return False
    o = _bm_opts()
    cfg = _native.hip().spmm_spgemm_bm_choose(C.byref(o), A.m, A.nnz, B.n, _true_nnz(B), total_products,
                                              pre["nonempty"], pre["max"], pre.get("amax", 1 << 30))
    if cfg < 0:
        return False
    if CONFIG.spgemm_bitmap == "on":
        return True
    return _FreeMem(A.device).fits(total_products * 8 + A.m * 64)


@dataclass
class BitmapPlan:
    """Host decisions of one bitmap-rank product, made by the native planner
    (csr_bitmap_plan.hip spmm_spgemm_bm_make_plan, shared with the native
    engine): window configuration, lane groups, which kernels run, padded
    layout capacities, one workspace layout, and C's capacity in the lazy flow.
    Everything the kernels need besides the operands, so a plan made once can
    drive a captured HIP graph (``SpgemmGraph``)."""
    raw: _BmPlan
    opts: _BmOpts

    def __getattr__(self, name):
        if name in ("raw", "opts"):
            raise AttributeError(name)
        v = getattr(self.raw, name)
        return bool(v) if name in ("count_rows", "rows", "det", "ws8", "pad_num", "pad_cnt") else v


def _bitmap_plan(A: CSR, B: CSR, info: SpgemmInfo, pre: Optional[dict], use_ws8: bool = True) -> Optional[BitmapPlan]:
    o = _bm_opts(use_ws8)
    p = _BmPlan()
    nz = pre["nonempty"] if pre is not None else A.m
    amax = pre.get("amax", -1) if pre is not None else -1
    if _native.hip().spmm_spgemm_bm_make_plan(C.byref(o), A.m, A.nnz, B.m, B.n, _true_nnz(B), info.flops // 2, nz,
                                               amax, float(info.mean_seg), C.byref(p)):
        return None
    return BitmapPlan(raw=p, opts=o)


def bitmap_buffers(plan: BitmapPlan, dev: torch.device, cap: Optional[int] = None) -> dict:
    """Device buffers of one bitmap-rank product: the plan's workspace, the
    {error bits, deferred units} word pair, the unit offsets and (``cap``
    given) C's arrays.  Allocated outside any capture, so the launches that
    use them are graph-capturable as they are."""
    raw = plan.raw
    out = dict(ws=torch.empty(max(raw.ws_bytes, 1), dtype=torch.uint8, device=dev),
               # err, deferred count, numeric row ticket, spare (zeroed by the front)
               z=torch.empty(4, dtype=torch.int32, device=dev),
               uoff=torch.empty(raw.nunits + 1, dtype=torch.int64, device=dev), nunits=raw.nunits, ws8=bool(raw.ws8))
    if cap is not None:
        out.update(Cci=torch.empty(cap, dtype=torch.int32, device=dev),
                   Cv=torch.empty(cap, dtype=torch.float32, device=dev), cap=cap)
    return out


def bitmap_gathered_ok(plan: BitmapPlan) -> bool:
    """Whether the plan's kernels read B only through its padded layouts, so
    the layout passes may read B in place from gathered panels (BmGathered)."""
    return bool(_native.hip().spmm_spgemm_bm_gathered_ok(C.byref(plan.raw)))


def bitmap_front(A: CSR, B: CSR, plan: BitmapPlan, bufs: dict, values: bool, gathered=None) -> int:
    """B layouts + count kernel + unit-offset scan (csr_bitmap_plan.hip front)
    on the current stream; ``values``: B's values are readable (else only its
    columns: the padded pairs are then built by :func:`bitmap_back`).
    ``gathered``: a :class:`BmGathered` view B's layouts are read from (B's own
    column / value arrays are then not read).  Returns whether the padded
    pairs were built."""
    P = _native.ptr
    built = C.c_int(0)
    use_vals = values and gathered is None
    _native.check(_native.hip().spmm_spgemm_bm_front(
        C.byref(plan.raw), P(A.rowptr), P(A.col), P(B.rowptr), None if gathered is not None else P(B.col),
        P(B.val) if use_vals else None, P(bufs["ws"]), P(bufs["uoff"]), P(bufs["z"]), C.byref(built),
        C.byref(gathered) if gathered is not None else None, _native.stream_ptr(A.device)),
        "spgemm_bm_front")
    return built.value


def bitmap_back(A: CSR, B: CSR, plan: BitmapPlan, bufs: dict, built: int, gathered=None) -> None:
    """Padded pairs (unless built by the front) + numeric and reload kernels
    into ``bufs["Cci"] / ["Cv"]`` (csr_bitmap_plan.hip back); ``gathered``: as
    :func:`bitmap_front`."""
    P = _native.ptr
    g = gathered is not None
    _native.check(_native.hip().spmm_spgemm_bm_back(
        C.byref(plan.raw), P(A.rowptr), P(A.col), P(A.val), None if g else P(B.col), None if g else P(B.val), built,
        P(bufs["ws"]), P(bufs["uoff"]), P(bufs["z"]), bufs["cap"], P(bufs["Cci"]), P(bufs["Cv"]),
        C.byref(gathered) if g else None, _native.stream_ptr(A.device)),
        "spgemm_bm_back")


def _bitmap_launch(A: CSR, B: CSR, plan: BitmapPlan, lazy: bool, B_ready=None, info: Optional[SpgemmInfo] = None) -> dict:
    """The kernels of one bitmap-rank product, launched by the native front /
    back (csr_bitmap_plan.hip) into one workspace.  ``lazy``: C at the product
    bound, no host synchronisation at all (capturable into a HIP graph; the
    nnz and error bits stay on the device in ``out["z"]`` / ``out["uoff"]``).
    Eager: one read-back between count and numeric sizes C exactly."""
    dev = A.device
    if B_ready is not None:   # columns only: the values may still be in flight (two-stage gather)
        B = getattr(B_ready, "cols", B_ready)()
    raw = plan.raw
    out = bitmap_buffers(plan, dev)
    values_here = B_ready is None or getattr(B_ready, "local", False)
    built = bitmap_front(A, B, plan, out, values_here)
    z, uoff = out["z"], out["uoff"]
    if not lazy:
        nnz, e0 = torch.stack([uoff[-1], z[0].long()]).tolist()   # one read-back
        if e0 & 32:
            raise RuntimeError("spgemm bitmap: padded B layout overflow (kernel invariant violated)")
        out.update(nnz=nnz)
        # a window segment does not fit 16 bits (bit 3), or a count unit has more chunks
        # than the pipelined count kernel's descriptors (bit 6): the per-unit kernels
        if e0 & (8 | 64):
            out.update(truncated=True)
            return out
        if e0:
            raise RuntimeError(f"spgemm bitmap: count kernels flagged error bits {e0} (kernel invariant violated)")
        z[0].zero_()
    cap = max(raw.tot, 1) if lazy else out["nnz"]
    if B_ready is not None:   # the numeric kernels read the values
        B = B_ready()
    out.update(Cci=torch.empty(cap, dtype=torch.int32, device=dev), Cv=torch.empty(cap, dtype=torch.float32, device=dev),
               cap=cap, n=B.n)
    bitmap_back(A, B, plan, out, built)
    if info is not None and raw.ws8 and raw.rows:
        info.rows_per_bin_num["bitmap_rows"] = 1
    return out


def _bitmap_finish(A: CSR, B: CSR, plan: BitmapPlan, out: dict, info: SpgemmInfo, lazy: bool):
    """Read back (once) the nnz and error bits of a launched product and
    return its CSR, ``None`` (binned fallback), or ``"eager"`` (ws8 lengths
    truncated in the lazy flow: rerun eagerly on the per-unit kernels)."""
    z, uoff = out["z"], out["uoff"]
    if lazy:
        nnz, e, deferred = torch.stack([uoff[-1], z[0].long(), z[1].long()]).tolist()   # the one read-back
        if e & (8 | 64):   # ws8 lengths truncated / a count unit past the descriptors: rerun eagerly
            return "eager"
    else:
        nnz = out["nnz"]
        e, deferred = z[:2].tolist()
    info.nnz = nnz
    info.rows_per_bin_num["bitmap_units"] = out["nunits"]
    info.rows_per_bin_num["bitmap_cfg"] = plan.cfg
    info.rows_per_bin_num["bitmap_deferred"] = deferred
    if e & 2:
        raise RuntimeError("spgemm bitmap: numeric and count kernels disagree (kernel invariant violated)")
    if e & 32:
        raise RuntimeError("spgemm bitmap: padded B layout overflow (kernel invariant violated)")
    if plan.det and e & 21:
        # a unit beyond every deterministic kernel's budget (adversarial column
        # collisions): the CPU engine sums in the same (Gustavson) order
        info.rows_per_bin_num["det_cpu_fallback"] = 1
        return _det_cpu(A, B, info)
    if e & 5:
        info.rows_per_bin_num["bitmap_fallback"] = 1
        return None
    info.deterministic = bool(plan.det)
    nwin = plan.nwin
    rowptr = uoff[::nwin].contiguous() if nwin > 1 else uoff
    Cci, Cv = out["Cci"], out["Cv"]
    return CSR(A.m, out["n"], rowptr, Cci[:nnz] if lazy else Cci, Cv[:nnz] if lazy else Cv)


def onepass_bitmap(A: CSR, B: CSR, info: SpgemmInfo, B_ready=None, pre: Optional[dict] = None,
                   lazy: bool = False) -> Optional[CSR]:
    """Bitmap-rank SpGEMM (csr_spgemm_bitmap.hip): a count kernel gives the
    exact nnz of every (row, column window) unit, one scan gives every unit's
    final offset, and the numeric kernel writes each unit there once (no
    look-back, no staging buffer, no compaction).  Returns None when a unit
    does not fit even the reload kernel; the caller then runs the binned
    path.  ``lazy`` (the flow the captured graphs replay, ``SpgemmGraph``):
    C at the product-count bound (what ``_bitmap_ok`` admitted), no host sync
    between the kernels, one read-back after the product; eager (default):
    one read-back between count and numeric sizes C exactly (the two measure
    the same, PERF_LOG round 3)."""
    plan = _bitmap_plan(A, B, info, pre)
    if plan is None:
        return None
    lazy = lazy and not plan.det
    out = _bitmap_launch(A, B, plan, lazy, B_ready, info)
    if out.get("truncated"):   # eager: per-unit count and numeric kernels
        plan = _bitmap_plan(A, B, info, pre, use_ws8=False)
        out = _bitmap_launch(A, B, plan, False, B_ready, info)
    if B_ready is not None:
        B = B_ready()
    C_ = _bitmap_finish(A, B, plan, out, info, lazy)
    if isinstance(C_, str):
        del out
        return onepass_bitmap(A, B, info, None, pre)
    return C_


class SpgemmGraph:
    """C = A . B (bitmap-rank path) replayed from a captured HIP graph: the
    window splits, ws8 pack, count kernel, unit-offset scan, B interleave and
    numeric + reload kernels of one product, with NO host synchronisation
    inside (lazy flow: C allocated once at the product-count bound; the nnz
    and error bits are read only by :meth:`result`).  The host plan (row
    statistics -> window configuration, lane groups, capacities) is made once
    at construction from the operands' row plan, as a library's SpGEMM
    inspector does; every replay recomputes the whole product.  A replay on
    operands whose structure changed beyond the plan cannot write out of
    bounds (the kernels clamp to C's capacity and raise error bits), and
    :meth:`result` reports it.  Replaces the three read-backs of the eager
    flow (row plan, count total, error words) that leave the GPU idle on
    small products (BASELINE config 2)."""

    def __init__(self, A: CSR, B: CSR):
        if A.device.type != "cuda":
            raise ValueError("SpgemmGraph needs GPU operands")
        self.A, self.B = A, B
        info = SpgemmInfo()
        nprod, nsl, st = row_plan(A, B)
        tot, mx, nz, light, h1, h2, h4, h8, amax = st.tolist()[:9]
        pre = dict(max=mx, nonempty=nz, light=light, amax=amax)
        info.flops = 2 * tot
        info.mean_seg = tot / max(A.nnz, 1)
        if not _bitmap_ok(A, B, tot, pre):
            raise ValueError("SpgemmGraph: the product does not take the bitmap-rank path")
        self.plan = _bitmap_plan(A, B, info, pre)
        if self.plan is None or self.plan.det:
            raise ValueError("SpgemmGraph: no lazy bitmap plan for this product")
        self.flops = info.flops
        dev = A.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):   # warm-up outside the capture (allocator, lazy library state)
            for _ in range(2):
                warm = _bitmap_launch(A, B, self.plan, True)
                del warm
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = _bitmap_launch(A, B, self.plan, True)

    def run(self) -> dict:
        self.graph.replay()
        return self.out

    def result(self, info: Optional[SpgemmInfo] = None) -> Optional[CSR]:
        """The last replay's C (one read-back of nnz and error bits)."""
        info = info if info is not None else SpgemmInfo()
        C_ = _bitmap_finish(self.A, self.B, self.plan, self.out, info, True)
        if isinstance(C_, str):
            raise RuntimeError("SpgemmGraph: the operands no longer fit the row kernels (16-bit window lengths "
                               "or count descriptors)")
        return C_


def _det_cpu(A: CSR, B: CSR, info: SpgemmInfo) -> CSR:
    """Deterministic product on the CPU engine (sequential Gustavson order,
    the order the deterministic GPU kernels reproduce), back on A's device."""
    dev = A.device
    C_ = _spgemm_cpu(A.to("cpu"), B.to("cpu"), info)
    info.deterministic = True
    return C_.to(dev)


PIPE_MIN_PRODUCTS = 1 << 26        # smaller products: one compaction after all rows is cheaper
PIPE_CHUNK_PRODUCTS = 1 << 29      # staging per chunk (x 8 B = 4 GiB), two chunks in flight
_SIDE = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    """One side stream per (device, thread): loopback ranks are threads that
    share a device, and must not interleave their pipelines on one stream.
    High priority: HIP maps streams onto its GPU_MAX_HW_QUEUES hardware queues
    round-robin, and a side stream that lands on the main stream's queue runs
    strictly after it (an R-MAT kernel trace showed every kernel of both on one
    queue); a different priority is a different queue."""
    key = (dev.index, threading.get_ident())
    s = _SIDE.get(key)
    if s is None:
        s = _SIDE[key] = torch.cuda.Stream(dev, priority=-1)
    return s


_DEFER = threading.local()


class deferred_placement:
    """Inside this context the pipelined one-pass returns a product before its
    side-stream work -- the compaction and the long-row placement of its last
    chunk -- has finished: the row pointer and nnz are final, the column /
    value arrays are complete once the CSR's ``ready`` event has passed
    (:func:`wait_ready`).  Every kernel still runs; the caller's next work on
    the main stream (the next streamed panel's planning and kernels) overlaps
    the copy instead of waiting for it (``models.spgemm.streamed_spgemm``,
    ``overlap=True``)."""

    def __enter__(self):
        self._prev = getattr(_DEFER, "on", False)
        _DEFER.on = True
        return self

    def __exit__(self, *exc):
        _DEFER.on = self._prev
        return False


def wait_ready(C_: CSR, stream=None) -> CSR:
    """Make ``stream`` (default: the current one) wait until ``C_``'s arrays are
    complete (a product formed under :class:`deferred_placement`)."""
    ev = getattr(C_, "ready", None)
    if ev is not None:
        (stream if stream is not None else torch.cuda.current_stream(C_.rowptr.device)).wait_event(ev)
    return C_


def onepass_pipelined(A: CSR, B: CSR, nprod: torch.Tensor, info: SpgemmInfo, B_ready=None) -> Optional[CSR]:
    """One-pass numeric over contiguous row chunks with the compaction of chunk
    i (a copy kernel, HBM-bandwidth bound) on a side stream while the numeric
    kernels of chunk i+1 (LDS / latency bound, ~1.7 TB/s) run on the main one.

    Each chunk stages its rows at chunk-relative product-count offsets in one
    of two staging buffers (so staging is 2 x PIPE_CHUNK_PRODUCTS instead of
    every product of the matrix); its row pointer segment is a device-side
    cumsum carried from the previous chunk, so no host synchronisation sits
    between chunks.  C is allocated at the product-count bound and returned as
    a view of its first nnz entries.  Hub rows (HBM long-row path) and rows
    that overflowed an LDS bin are staged inside their chunk too (one host
    synchronisation per chunk for the overflow check)."""
    dev = A.device
    m = A.m
    tot = info.flops // 2
    bins = _bins(nprod, 1)
    ub = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nprod, 0, out=ub[1:])
    nch = max(2, -(-tot // PIPE_CHUNK_PRODUCTS))
    cuts = torch.searchsorted(ub[1:], torch.arange(1, nch, device=dev, dtype=torch.int64) * (tot // nch))
    bounds = [0] + sorted(set(min(max(int(c), 1), m - 1) for c in cuts.tolist())) + [m]
    nch = len(bounds) - 1
    bt = torch.tensor(bounds, dtype=torch.int64, device=dev)
    chunk_of = torch.bucketize(torch.arange(m, device=dev), bt[1:-1], right=True)
    key = chunk_of * 16 + (bins + 1)
    order = torch.argsort(key, stable=True).to(torch.int32)
    hist = torch.bincount(key, minlength=nch * 16).tolist()
    ub_at = ub[bt].tolist()
    for c in range(nch):
        for b in range(NUM_GLOBAL + 1):
            if hist[c * 16 + b + 1]:
                info.rows_per_bin_num[b] = info.rows_per_bin_num.get(b, 0) + hist[c * 16 + b + 1]
    ub_rel = ub[:-1] - ub[bt[:-1]][chunk_of]          # staging offset of each row inside its chunk
    cap = max(ub_at[i + 1] - ub_at[i] for i in range(nch))
    stage = [(torch.empty(cap, dtype=torch.int32, device=dev), torch.empty(cap, dtype=torch.float32, device=dev))
             for _ in range(2)]
    Cci = torch.empty(tot, dtype=torch.int32, device=dev)
    Cv = torch.empty(tot, dtype=torch.float32, device=dev)
    out_nnz = torch.zeros(m, dtype=torch.int32, device=dev)
    flags = torch.zeros(m, dtype=torch.int32, device=dev)
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    rcap = nprod.to(torch.int32)
    if B_ready is not None:
        B = B_ready()
    lib = _native.hip()
    P = _native.ptr
    splits = _splits(B) if any(hist[c * 16 + b + 1] for c in range(nch) for b in NUM_SLICED) else None
    seg = info.mean_seg if info.mean_seg > 0 else B.nnz / max(B.m, 1)
    sA = torch.cuda.current_stream(dev)
    sB = _side_stream(dev)
    sB.wait_stream(sA)
    free = [None, None]
    off = hist[0]
    defer = getattr(_DEFER, "on", False)
    rp_done, ok = None, False
    try:   # the side stream may still read this call's buffers: drain it even on an error
        for c in range(nch):
            lo, hi = bounds[c], bounds[c + 1]
            sci, sv = stage[c % 2]
            if free[c % 2] is not None:
                sA.wait_event(free[c % 2])              # chunk c-2's compaction has read this buffer
            long_rows = []
            for b in range(NUM_GLOBAL + 1):
                cnt = hist[c * 16 + b + 1]
                if cnt and b == NUM_GLOBAL:
                    long_rows.append(order[off:off + cnt])
                elif cnt:
                    _native.check(lib.spmm_spgemm_lds(b, 1, P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col),
                                                      P(B.val), P(splits) if splits is not None else None,
                                                      P(order) + 4 * off, cnt, B.n, _group_log2(seg / _slices(b, 1)),
                                                      P(rcap), P(out_nnz), P(ub_rel), P(sci), P(sv), P(flags),
                                                      sA.cuda_stream), "spgemm_lds(numeric, pipelined)")
                off += cnt
            off += hist[(c + 1) * 16] if c + 1 < nch else 0   # empty rows of the next chunk (bin -1)
            spill = ((flags[lo:hi] & 2) != 0).nonzero().flatten()
            if spill.numel():
                info.rows_per_bin_num["lds_overflow"] = info.rows_per_bin_num.get("lds_overflow", 0) + int(spill.numel())
                long_rows.append((spill + lo).to(torch.int32))
            deferred = []
            if long_rows:
                # hub rows stay in their chunk scratch and go straight to C once
                # the chunk's row pointer exists (the compaction skips them)
                rows = torch.cat(long_rows)
                _long_rows(1, A, B, rows, nprod[rows.long()], sA.cuda_stream, out_nnz=out_nnz, defer=deferred)
                ub_rel[rows.long()] = -1
            done = torch.cuda.Event()
            done.record(sA)
            with torch.cuda.stream(sB):
                sB.wait_event(done)
                torch.cumsum(out_nnz[lo:hi], 0, dtype=torch.int64, out=rowptr[lo + 1:hi + 1])
                rowptr[lo + 1:hi + 1] += rowptr[lo]
                if defer and c == nch - 1:   # the row pointer is final here, before the copies
                    rp_done = torch.cuda.Event()
                    rp_done.record(sB)
                _native.check(lib.spmm_spgemm_compact(P(ub_rel) + 8 * lo, P(rowptr) + 8 * lo, hi - lo, P(sci), P(sv),
                                                      P(Cci), P(Cv), sB.cuda_stream), "spgemm_compact(pipelined)")
                for d in deferred:   # allocated on sA, last read on sB
                    for t in d:
                        t.record_stream(sB)
                place_long(deferred, rowptr, Cci, Cv, sB.cuda_stream)
                del deferred
                free[c % 2] = torch.cuda.Event()
                free[c % 2].record(sB)
        ok = True
    finally:
        if not (ok and defer):
            sA.wait_stream(sB)
    ready = None
    if ok and defer:
        # return before the last chunk's compaction / placement has finished: the main stream
        # waits for the row pointer only, and every buffer the side stream still touches
        # stays out of the allocator's reach until it has passed
        sA.wait_event(rp_done)
        ready = torch.cuda.Event()
        ready.record(sB)
        for t in (out_nnz, rowptr, ub_rel, Cci, Cv, *[x for st in stage for x in st]):
            t.record_stream(sB)
    nnz = int(rowptr[-1])
    info.nnz = nnz
    C_ = CSR(m, B.n, rowptr, Cci[:nnz], Cv[:nnz])
    if ready is not None:
        if bool(((flags & 1) != 0).any()):   # rows to re-sort (_finish, on this stream): C complete first
            sA.wait_event(ready)
        else:
            C_.ready = ready
    return _finish(C_, flags, info)


def _finish(C_: CSR, flags: torch.Tensor, info: SpgemmInfo, counts=None) -> CSR:
    """``counts``: (rows flagged 4, rows flagged 1) when already read back."""
    f4, f1 = counts if counts is not None else (None, None)
    if f4 if f4 is not None else bool(((flags & 4) != 0).any()):
        raise RuntimeError("spgemm numeric: output position out of range (kernel invariant violated)")
    if f1 == 0:
        return C_
    bad = ((flags & 1) != 0).nonzero().flatten()
    if bad.numel():
        info.resorted_rows = int(bad.numel())
        C_ = sort_rows(C_, bad, inplace=True)
    return C_


def _dummies(dev):
    return (torch.zeros(1, dtype=torch.int64, device=dev), torch.zeros(1, dtype=torch.int32, device=dev),
            torch.zeros(1, dtype=torch.float32, device=dev))


def _slices(b: int, numeric: int) -> int:
    """Column slices of LDS bin b."""
    if numeric:
        return {8: 2, 9: 4, 10: 8}.get(b, 1)
    return {8: 2, 9: 4, 10: 8}.get(b, 1)


def _group_log2(seg_len: float) -> int:
    """log2 of the lanes per A-entry group in the LDS kernels: 64 lanes walk a
    long B-row segment, 32 / 16 share a wave for short ones."""
    if seg_len >= 40:
        return 6
    if seg_len >= 16:
        return 5
    return 4


def _splits(B: CSR) -> torch.Tensor:
    """Column-eighth split points of every row of B (csr_spgemm.hip row_splits).
    Memoised on the operand: a streamed product multiplies many row panels of
    A by the same B (R-MAT: 34 panels per rank, 1.8 ms each before)."""
    key = (B.rowptr.data_ptr(), B.col.data_ptr(), B.m, B.n, B.nnz)
    hit = getattr(B, "_splits_memo", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    sp = torch.empty(B.m * 7, dtype=torch.int64, device=B.device)
    _native.check(_native.hip().spmm_spgemm_row_splits(_native.ptr(B.rowptr), _native.ptr(B.col), B.m, B.n,
                                                        _native.ptr(sp), _native.stream_ptr(B.device)),
                  "spgemm_row_splits")
    B._splits_memo = (key, sp)
    return sp


def _run_bins(numeric: int, A: CSR, B: CSR, counts: torch.Tensor, row_nnz, Crp, Cci, Cv, flags, info_bins,
              mean_seg: float = 0.0, out_nnz: Optional[torch.Tensor] = None,
              nprod: Optional[torch.Tensor] = None, B_ready=None, defer: Optional[list] = None):
    """Run the LDS bins, then the HBM path for the rest.  Numeric: ``row_nnz`` is
    each row's capacity in the output (exact nnz, or the product count in
    one-pass mode where ``out_nnz`` receives the real counts).  ``defer``
    (one-pass): the long rows' results stay in their scratch for
    :func:`place_long` instead of being written at ``Crp``."""
    dev = A.device
    lib = _native.hip()
    P = _native.ptr
    stream = _native.stream_ptr(dev)
    sliced, glob = (NUM_SLICED, NUM_GLOBAL) if numeric else (SYM_SLICED, SYM_GLOBAL)
    order, groups = _group(_bins(counts, numeric), glob + 1)
    if B_ready is not None:   # operand payload in flight until here (distributed gather)
        B = B_ready()
    splits = None
    global_rows = []
    seg = mean_seg if mean_seg > 0 else B.nnz / max(B.m, 1)
    for b, off, cnt in groups:
        info_bins[b] = cnt
        rows = order[off:off + cnt]
        if b == glob:
            global_rows.append(rows)
            continue
        multi_slice = b in NUM_SLICED if numeric else b in SYM_SLICED[1:]
        if multi_slice and splits is None:
            splits = _splits(B)
        _native.check(lib.spmm_spgemm_lds(b, numeric, P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col),
                                          P(B.val), P(splits) if splits is not None else None, P(rows), cnt, B.n,
                                          _group_log2(seg / _slices(b, numeric)), P(row_nnz),
                                          P(out_nnz) if out_nnz is not None else None, P(Crp), P(Cci), P(Cv),
                                          P(flags), stream),
                      "spgemm_lds(numeric)" if numeric else "spgemm_lds(symbolic)")
    # rows whose column slice could overflow an LDS table were skipped by the kernel
    spill = ((flags & 2) != 0).nonzero().flatten().to(torch.int32)
    if spill.numel():
        info_bins["lds_overflow"] = int(spill.numel())
        global_rows.append(spill)
    if global_rows:
        rows = torch.cat(global_rows)
        nprod_rows = nprod[rows.long()] if nprod is not None else counts[rows.long()]
        if not numeric:            # symbolic: exact counts
            _long_rows(0, A, B, rows, nprod_rows, stream, out_nnz=row_nnz)
        elif out_nnz is not None:  # one-pass: values at product-count offsets, real counts out
            _long_rows(1, A, B, rows, nprod_rows, stream, out_nnz=out_nnz, Crp=Crp, Cci=Cci, Cv=Cv, defer=defer)
        else:                      # two-phase numeric: into the layout fixed by symbolic
            _long_rows(1, A, B, rows, nprod_rows, stream, Crp=Crp, Cci=Cci, Cv=Cv, expect_nnz=row_nnz)


def symbolic(A: CSR, B: CSR, nprod: torch.Tensor, info: SpgemmInfo) -> torch.Tensor:
    """Exact nnz per output row (int32, device)."""
    dev = A.device
    row_nnz = torch.zeros(A.m, dtype=torch.int32, device=dev)
    flags = torch.zeros(A.m, dtype=torch.int32, device=dev)
    d64, d32, df = _dummies(dev)
    _run_bins(0, A, B, nprod, row_nnz, d64, d32, df, flags, info.rows_per_bin_sym, info.mean_seg)
    return row_nnz


def numeric(A: CSR, B: CSR, row_nnz: torch.Tensor, info: SpgemmInfo,
            nprod: Optional[torch.Tensor] = None) -> CSR:
    """Values of C (column-sorted rows) into the layout fixed by ``row_nnz``."""
    if nprod is None:
        nprod = row_nprod(A, B)
    dev = A.device
    m = A.m
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(row_nnz, 0, out=rowptr[1:])
    nnz = int(rowptr[-1])
    info.nnz = nnz
    Cci = torch.empty(nnz, dtype=torch.int32, device=dev)
    Cv = torch.empty(nnz, dtype=torch.float32, device=dev)
    flags = torch.zeros(m, dtype=torch.int32, device=dev)
    _run_bins(1, A, B, nprod, row_nnz, rowptr, Cci, Cv, flags, info.rows_per_bin_num, info.mean_seg)
    return _finish(CSR(m, B.n, rowptr, Cci, Cv), flags, info)


def _spgemm_cpu(A: CSR, B: CSR, info: SpgemmInfo) -> CSR:
    lib = _native.host()
    P = _native.ptr
    A = A if A.val.dtype == torch.float32 else A.with_values(A.val.float())
    B = B if B.val.dtype == torch.float32 else B.with_values(B.val.float())
    A = CSR(A.m, A.n, A.rowptr.contiguous(), A.col.contiguous(), A.val.contiguous())
    nprod = torch.empty(A.m, dtype=torch.int64)
    info.flops = 2 * int(lib.spmm_cpu_csr_nprod(A.m, P(A.rowptr), P(A.col), P(B.rowptr), P(nprod), 0))
    rowptr = torch.empty(A.m + 1, dtype=torch.int64)
    nnz = int(lib.spmm_cpu_csr_spgemm_symbolic(A.m, B.n, P(A.rowptr), P(A.col), P(B.rowptr), P(B.col), P(rowptr), 0))
    col = torch.empty(nnz, dtype=torch.int32)
    val = torch.empty(nnz, dtype=torch.float32)
    lib.spmm_cpu_csr_spgemm_numeric(A.m, B.n, P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col), P(B.val),
                                    P(rowptr), P(col), P(val), 0)
    info.nnz = nnz
    return CSR(A.m, B.n, rowptr, col, val)


def csr_sum(parts, info: Optional[SpgemmInfo] = None) -> CSR:
    """Sum of same-shape CSR matrices, on the SpGEMM kernels: the sum of
    P_0 .. P_{s-1} (each m x n) is S . V with V = [P_0; ..; P_{s-1}] stacked
    by rows (s*m x n) and S = [I I .. I] (m x s*m), so row i of the result
    merges row i of every part.  The number of intermediate products is the
    total nnz of the parts; every product is one exact fp32 ``1 * v``, so the
    result equals a fp32 sum of the parts (up to summation order).  The ESC /
    hash accumulators sort and fold duplicates, which is exactly the sparse
    merge that a reduce-scatter of sparse partials needs (there is no sparse
    ``ncclSum``)."""
    parts = list(parts)
    if not parts:
        raise ValueError("csr_sum needs at least one part")
    m, n, dev = parts[0].m, parts[0].n, parts[0].device
    for p in parts:
        if (p.m, p.n) != (m, n):
            raise ValueError(f"csr_sum: shape {(p.m, p.n)} != {(m, n)}")
    s = len(parts)
    if s == 1:
        return parts[0]
    counts = torch.cat([p.rowptr[1:] - p.rowptr[:-1] for p in parts])
    vrp = torch.zeros(s * m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=vrp[1:])
    V = CSR(s * m, n, vrp, torch.cat([p.col for p in parts]),
            torch.cat([p.val.float() for p in parts]))
    srp = torch.arange(m + 1, dtype=torch.int64, device=dev) * s
    scol = (torch.arange(s, dtype=torch.int32, device=dev).view(1, s) * m
            + torch.arange(m, dtype=torch.int32, device=dev).view(m, 1)).reshape(-1)
    S = CSR(m, s * m, srp, scol.contiguous(), torch.ones(m * s, dtype=torch.float32, device=dev))
    return spgemm(S, V, info)
