"""CSR sparse matrices (north-star format; the reference has only block tiles).

Row pointers are int64 (SpGEMM outputs pass 2^31 non-zeros: 1M x 1M at 0.01 %
gives ~1e10), column indices int32, values fp32 (SpGEMM) or bf16 (SpMM).
Conversions are device-side torch ops; they are setup paths, not hot loops.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


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


def sort_rows(C: CSR, rows: Optional[torch.Tensor] = None) -> CSR:
    """Re-sort columns inside rows (all rows, or only ``rows``)."""
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
