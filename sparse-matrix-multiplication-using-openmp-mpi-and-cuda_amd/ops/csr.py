"""CSR sparse matrices (north-star format; the reference has only block tiles).

Row pointers are int64 (SpGEMM outputs pass 2^31 non-zeros: 1M x 1M at 0.01 %
gives ~1e10), column indices int32, values fp32 (SpGEMM) or bf16 (SpMM).
Conversions are device-side torch ops; they are setup paths, not hot loops.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import ctypes as C

import torch

from .. import _native
from .._native import c_vp


@dataclass
class CSR:
    m: int
    n: int
    rowptr: torch.Tensor   # int64 [m+1]
    col: torch.Tensor      # int32 [nnz]
    val: torch.Tensor      # float32 / bfloat16 [nnz]

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    @property
    def device(self) -> torch.device:
        return self.col.device

    def to(self, device, non_blocking: bool = False) -> "CSR":
        return CSR(self.m, self.n, self.rowptr.to(device, non_blocking=non_blocking),
                   self.col.to(device, non_blocking=non_blocking), self.val.to(device, non_blocking=non_blocking))

    def with_values(self, val: torch.Tensor) -> "CSR":
        return CSR(self.m, self.n, self.rowptr, self.col, val)

    def nbytes(self) -> int:
        return self.rowptr.numel() * 8 + self.col.numel() * 4 + self.val.numel() * self.val.element_size()

    def row_ids(self) -> torch.Tensor:
        """int64 row index of every stored entry."""
        counts = self.rowptr[1:] - self.rowptr[:-1]
        return torch.repeat_interleave(torch.arange(self.m, device=self.device), counts, output_size=self.nnz)

    def to_dense(self, dtype=torch.float32) -> torch.Tensor:
        d = torch.zeros((self.m, self.n), dtype=dtype, device=self.device)
        if self.nnz:
            d.index_put_((self.row_ids(), self.col.long()), self.val.to(dtype), accumulate=True)
        return d

    def to_torch(self) -> torch.Tensor:
        return torch.sparse_csr_tensor(self.rowptr, self.col.long(), self.val, (self.m, self.n))

    def is_sorted(self) -> bool:
        """Columns strictly increasing inside every row (canonical form)."""
        if self.nnz < 2:
            return True
        code = self.row_ids() * self.n + self.col.long()
        return bool((code[1:] > code[:-1]).all())

    def transpose(self) -> "CSR":
        """A^T in canonical CSR: the gfx950 kernels of csr_transpose.hip on
        a GPU (``transpose_gpu``), a device sort otherwise."""
        if self.device.type == "cuda":
            return transpose_gpu(self)
        rows = self.row_ids()
        return from_coo(self.col.long(), rows, self.val, self.n, self.m)

    def col_slice(self, lo: int, hi: int) -> "CSR":
        """Columns [lo, hi), re-indexed from 0; all rows kept (the column panel
        of an inner-dimension split).  Column order inside a row is kept."""
        sel = (self.col >= lo) & (self.col < hi)
        cnt = torch.zeros(self.m + 1, dtype=torch.int64, device=self.device)
        if self.nnz:
            cnt[1:] = _row_sum(sel, self)
        return CSR(self.m, hi - lo, torch.cumsum(cnt, 0), (self.col[sel] - lo).to(torch.int32), self.val[sel])

    def row_slice(self, lo: int, hi: int) -> "CSR":
        s, e = int(self.rowptr[lo]), int(self.rowptr[hi])
        return CSR(hi - lo, self.n, (self.rowptr[lo:hi + 1] - s).contiguous(), self.col[s:e].contiguous(),
                   self.val[s:e].contiguous())


_native.register_hip("spmm_csr_col_count", c_vp, C.c_int64, c_vp, c_vp)
_native.register_hip("spmm_csr_t_scatter", c_vp, c_vp, C.c_int64, c_vp, c_vp, c_vp)
_native.register_hip("spmm_csr_t_sort", C.c_int, c_vp, c_vp, C.c_int64, c_vp, c_vp)
T_SORT_LDS = 2048   # csr_transpose.hip kSortLds


def transpose_gpu(A: "CSR") -> "CSR":
    """Column histogram -> scan -> atomic-cursor scatter of source indices ->
    per-segment sort (wave bitonic <= 64, LDS bitonic <= 2048, device radix
    sort for the few longer hub segments) -> gathers.  Requires A's columns
    sorted inside rows only for the output to be canonical (ascending source
    index is ascending row)."""
    lib = _native.hip()
    P, dev = _native.ptr, A.device
    st = _native.stream_ptr(dev)
    cnt = torch.zeros(A.n, dtype=torch.int64, device=dev)
    _native.check(lib.spmm_csr_col_count(P(A.col), A.nnz, P(cnt), st), "csr_col_count")
    trp = torch.zeros(A.n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt, 0, out=trp[1:])
    cursor = trp[:-1].clone()
    src = torch.empty(A.nnz, dtype=torch.int64, device=dev)
    _native.check(lib.spmm_csr_t_scatter(P(A.rowptr), P(A.col), A.m, P(cursor), P(src), st), "csr_t_scatter")
    short = torch.nonzero((cnt > 1) & (cnt <= 64)).view(-1)
    mid = torch.nonzero((cnt > 64) & (cnt <= T_SORT_LDS)).view(-1)
    long_ = torch.nonzero(cnt > T_SORT_LDS).view(-1)
    _native.check(lib.spmm_csr_t_sort(0, P(trp), P(short), short.numel(), P(src), st), "csr_t_sort")
    _native.check(lib.spmm_csr_t_sort(1, P(trp), P(mid), mid.numel(), P(src), st), "csr_t_sort")
    if long_.numel():
        lens = cnt[long_]
        seg = torch.repeat_interleave(torch.arange(long_.numel(), device=dev), lens)
        starts = torch.repeat_interleave(trp[long_], lens)
        idx = starts + (torch.arange(seg.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens))
        keyed = torch.sort(seg * (A.nnz + 1) + src[idx]).values
        src[idx] = keyed - seg * (A.nnz + 1)
    return CSR(A.n, A.m, trp, A.row_ids()[src].to(torch.int32), A.val[src])


def _row_sum(mask: torch.Tensor, A: "CSR") -> torch.Tensor:
    out = torch.zeros(A.m, dtype=torch.int64, device=A.device)
    out.index_add_(0, A.row_ids(), mask.to(torch.int64))
    return out


def rowptr_from_rows(rows_sorted: torch.Tensor, m: int) -> torch.Tensor:
    rp = torch.zeros(m + 1, dtype=torch.int64, device=rows_sorted.device)
    if rows_sorted.numel():
        torch.cumsum(torch.bincount(rows_sorted, minlength=m), 0, out=rp[1:])
    return rp


def from_coo(rows: torch.Tensor, cols: torch.Tensor, vals: Optional[torch.Tensor], m: int, n: int,
             sum_duplicates: bool = True, dtype=torch.float32) -> CSR:
    """COO -> canonical CSR (sorted columns, duplicates summed)."""
    dev = rows.device
    if vals is None:
        vals = torch.ones(rows.shape[0], dtype=dtype, device=dev)
    code = rows.to(torch.int64) * n + cols.to(torch.int64)
    code, perm = torch.sort(code)
    vals = vals[perm].to(dtype)
    if sum_duplicates and code.numel() > 1:
        uniq, inv = torch.unique_consecutive(code, return_inverse=True)
        if uniq.numel() != code.numel():
            acc = torch.zeros(uniq.numel(), dtype=torch.float32, device=dev)
            acc.index_add_(0, inv, vals.float())
            code, vals = uniq, acc.to(dtype)
    r = torch.div(code, n, rounding_mode="floor")
    c = (code - r * n).to(torch.int32)
    return CSR(m, n, rowptr_from_rows(r, m), c, vals.contiguous())


def from_dense(d: torch.Tensor) -> CSR:
    r, c = d.nonzero(as_tuple=True)
    return from_coo(r, c, d[r, c], d.shape[0], d.shape[1], sum_duplicates=False, dtype=d.dtype)


def from_torch(t: torch.Tensor) -> CSR:
    t = t.to_sparse_csr()
    return CSR(t.shape[0], t.shape[1], t.crow_indices().to(torch.int64), t.col_indices().to(torch.int32),
               t.values())


_native.register_hip("spmm_csr_sort_rows_ws", C.c_int64, C.c_int64, C.c_int64, restype=C.c_size_t)
_native.register_hip("spmm_csr_sort_rows", c_vp, c_vp, C.c_int64, C.c_int64, C.c_int64, c_vp, c_vp, c_vp, c_vp)


def sort_rows(C: CSR, rows: Optional[torch.Tensor] = None, inplace: bool = False) -> CSR:
    """Re-sort columns inside rows (all rows, or only ``rows``).  On the GPU
    the listed rows are sorted by csr_rowsort.hip (bitonic per wave / LDS
    workgroup, the in-tree radix sort for rows beyond 16384 entries): one
    read-back of their total and longest length, no per-row host work.
    ``inplace``: sort C's own arrays (the SpGEMM's fresh output)."""
    if (rows is not None and rows.numel() and C.col.is_cuda and C.col.dtype == torch.int32
            and C.val.dtype == torch.float32 and rows.numel() < C.m):
        r = rows.long().contiguous()
        lens = C.rowptr[r + 1] - C.rowptr[r]
        total, maxlen = torch.stack([lens.sum(), lens.max()]).tolist()
        col, val = (C.col, C.val) if inplace else (C.col.clone(), C.val.clone())
        lib = _native.hip()
        ws = torch.empty(max(int(lib.spmm_csr_sort_rows_ws(r.numel(), total, maxlen)), 1), dtype=torch.uint8,
                         device=C.col.device)
        _native.check(lib.spmm_csr_sort_rows(_native.ptr(C.rowptr), _native.ptr(r), r.numel(), total, maxlen,
                                             _native.ptr(col), _native.ptr(val), _native.ptr(ws),
                                             _native.stream_ptr(C.col.device)), "csr_sort_rows")
        return CSR(C.m, C.n, C.rowptr, col, val)
    if rows is None or rows.numel() == C.m:
        r = C.row_ids()
        code = r * C.n + C.col.long()
        code, perm = torch.sort(code)
        return CSR(C.m, C.n, C.rowptr, (code - torch.div(code, C.n, rounding_mode="floor") * C.n).to(torch.int32),
                   C.val[perm])
    col, val = C.col.clone(), C.val.clone()
    for i in rows.tolist():
        s, e = int(C.rowptr[i]), int(C.rowptr[i + 1])
        cs, p = torch.sort(col[s:e])
        col[s:e] = cs
        val[s:e] = val[s:e][p]
    return CSR(C.m, C.n, C.rowptr, col, val)
