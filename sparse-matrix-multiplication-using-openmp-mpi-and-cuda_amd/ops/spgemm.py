"""CSR x CSR SpGEMM (fp32): C = A . B.

GPU path (gfx950, ``csrc/kernels/csr_spgemm.hip``):
  1. ``nprod``: intermediate products per row (one wave per row).
  2. Symbolic: rows binned by nprod into LDS hash kernels with table sizes
     128 .. 32768 keys (load factor <= 0.75, 0.85 in the top bin); longer rows
     go to the HBM-workspace kernel.  Output: exact nnz per row.
  3. Row pointer by a device scan; C allocated once.
  4. Numeric: rows re-binned by their exact nnz (tables 128 .. 16384 key/value
     slots, 128 KiB of LDS at the top), monotone hashing + per-cluster sort, so
     rows come out column-sorted without a sort pass.
CPU path: OpenMP Gustavson (``libspmm_host.so``), identical output layout.

FLOPs are counted as 2 * sum(nprod) (one multiply + one add per intermediate
product), the convention of BASELINE.md.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from .. import _native
from .._native import c_vp
from .csr import CSR, sort_rows
import ctypes as C

C_I64 = C.c_int64
C_INT = C.c_int

_native.register_hip("spmm_spgemm_row_nprod", c_vp, c_vp, c_vp, C_I64, c_vp, c_vp)
_native.register_hip("spmm_spgemm_lds", C_INT, C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, C_INT,
                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spgemm_global", C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C_I64, c_vp, c_vp,
                     c_vp, c_vp, C_INT, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp)

SYM_MAX_BIN = 8      # table range 128 << 8 = 32768 keys (128 KiB)
NUM_MAX_BIN = 7      # 16384 key/value slots (128 KiB)
LOAD = 0.75
TOP_LOAD = 0.85
GLOBAL_WS_BYTES = 8 << 30   # HBM budget for one batch of global-table rows


@dataclass
class SpgemmInfo:
    flops: int = 0
    nnz: int = 0
    rows_per_bin_sym: Dict[int, int] = field(default_factory=dict)
    rows_per_bin_num: Dict[int, int] = field(default_factory=dict)
    resorted_rows: int = 0


def _bins(counts: torch.Tensor, max_bin: int) -> torch.Tensor:
    caps = [LOAD * (128 << b) for b in range(max_bin + 1)]
    caps[-1] = TOP_LOAD * (128 << max_bin)
    b = torch.bucketize(counts, torch.tensor([int(c) for c in caps], device=counts.device, dtype=counts.dtype))
    return torch.where(counts == 0, torch.full_like(b, -1), b)


def _group(bins: torch.Tensor, max_bin: int):
    """rows ordered by bin + host list of (bin, offset, count); bin max_bin+1 = global."""
    order = torch.argsort(bins, stable=True).to(torch.int32)
    hist = torch.bincount(bins + 1, minlength=max_bin + 3).tolist()
    groups, off = [], hist[0]
    for b in range(max_bin + 2):
        cnt = hist[b + 1]
        if cnt:
            groups.append((b, off, cnt))
        off += cnt
    return order, groups


def row_nprod(A: CSR, B: CSR) -> torch.Tensor:
    nprod = torch.empty(A.m, dtype=torch.int64, device=A.device)
    P = _native.ptr
    if A.device.type == "cuda":
        _native.check(_native.hip().spmm_spgemm_row_nprod(P(A.rowptr), P(A.col), P(B.rowptr), A.m, P(nprod),
                                                           _native.stream_ptr(A.device)), "spgemm_row_nprod")
    else:
        _native.host().spmm_cpu_csr_nprod(A.m, P(A.rowptr), P(A.col), P(B.rowptr), P(nprod), 0)
    return nprod


def _global_rows(numeric: int, A: CSR, B: CSR, rows: torch.Tensor, counts: torch.Tensor, row_nnz, Crp, Cci, Cv,
                 unsorted, stream) -> None:
    """Rows whose table exceeds LDS: HBM hash tables, processed in batches."""
    dev = A.device
    lib = _native.hip()
    P = _native.ptr
    cap = 1 << max(15, (max(B.n, 1) - 1).bit_length())
    cnt = counts.tolist()
    sizes = []
    for c in cnt:
        s = 1 << max(15, (int(c / 0.5) - 1).bit_length())
        sizes.append(min(s, cap * 2) + 1024)
    i = 0
    empty_f = torch.empty(0, dtype=torch.float32, device=dev)
    while i < len(sizes):
        j, tot = i, 0
        while j < len(sizes) and (j == i or (tot + sizes[j]) * 8 <= GLOBAL_WS_BYTES):
            tot += sizes[j]
            j += 1
        sz = torch.tensor(sizes[i:j], dtype=torch.int64, device=dev)
        off = torch.cumsum(sz, 0) - sz
        keys = torch.full((tot,), -1, dtype=torch.int32, device=dev)
        vals = torch.zeros(tot, dtype=torch.float32, device=dev) if numeric else empty_f
        r = rows[i:j].contiguous()
        _native.check(lib.spmm_spgemm_global(numeric, P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col),
                                             P(B.val), P(r), j - i, P(off), P(sz), P(keys), P(vals), B.n,
                                             P(row_nnz), P(Crp), P(Cci), P(Cv), P(unsorted), stream),
                      "spgemm_global")
        i = j


def spgemm(A: CSR, B: CSR, info: Optional[SpgemmInfo] = None) -> CSR:
    if A.n != B.m:
        raise ValueError(f"inner dimensions differ: {A.n} vs {B.m}")
    if A.device != B.device:
        raise ValueError("operands on different devices")
    info = info if info is not None else SpgemmInfo()
    if A.device.type != "cuda":
        return _spgemm_cpu(A, B, info)
    A = A if A.val.dtype == torch.float32 else A.with_values(A.val.float())
    B = B if B.val.dtype == torch.float32 else B.with_values(B.val.float())
    dev = A.device
    lib = _native.hip()
    P = _native.ptr
    stream = _native.stream_ptr(dev)
    m = A.m

    nprod = row_nprod(A, B)
    info.flops = 2 * int(nprod.sum())

    # symbolic
    row_nnz = torch.zeros(m, dtype=torch.int32, device=dev)
    sbins = _bins(nprod, SYM_MAX_BIN)
    order, groups = _group(sbins, SYM_MAX_BIN)
    dummy_i64 = torch.zeros(1, dtype=torch.int64, device=dev)
    dummy_i32 = torch.zeros(1, dtype=torch.int32, device=dev)
    dummy_f = torch.zeros(1, dtype=torch.float32, device=dev)
    for b, off, cnt in groups:
        info.rows_per_bin_sym[b] = cnt
        rows = order[off:off + cnt]
        if b <= SYM_MAX_BIN:
            _native.check(lib.spmm_spgemm_lds(b, 0, P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col),
                                              P(B.val), P(rows), cnt, B.n, P(row_nnz), P(dummy_i64), P(dummy_i32),
                                              P(dummy_f), P(dummy_i32), stream), "spgemm_lds(symbolic)")
        else:
            _global_rows(0, A, B, rows, nprod[rows.long()], row_nnz, dummy_i64, dummy_i32, dummy_f, dummy_i32,
                         stream)

    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(row_nnz, 0, out=rowptr[1:])
    nnz = int(rowptr[-1])
    info.nnz = nnz
    Cci = torch.empty(nnz, dtype=torch.int32, device=dev)
    Cv = torch.empty(nnz, dtype=torch.float32, device=dev)
    unsorted = torch.zeros(m, dtype=torch.int32, device=dev)

    # numeric
    nbins = _bins(row_nnz, NUM_MAX_BIN)
    order, groups = _group(nbins, NUM_MAX_BIN)
    for b, off, cnt in groups:
        info.rows_per_bin_num[b] = cnt
        rows = order[off:off + cnt]
        if b <= NUM_MAX_BIN:
            _native.check(lib.spmm_spgemm_lds(b, 1, P(A.rowptr), P(A.col), P(A.val), P(B.rowptr), P(B.col),
                                              P(B.val), P(rows), cnt, B.n, P(row_nnz), P(rowptr), P(Cci), P(Cv),
                                              P(unsorted), stream), "spgemm_lds(numeric)")
        else:
            _global_rows(1, A, B, rows, row_nnz[rows.long()], row_nnz, rowptr, Cci, Cv, unsorted, stream)
    C_ = CSR(m, B.n, rowptr, Cci, Cv)
    bad = unsorted.nonzero().flatten()
    if bad.numel():
        info.resorted_rows = int(bad.numel())
        C_ = sort_rows(C_, bad)
    return C_


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
