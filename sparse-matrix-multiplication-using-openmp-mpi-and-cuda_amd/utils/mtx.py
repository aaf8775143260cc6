"""Matrix Market (coordinate) I/O for CSR matrices (north-star requirement;
the reference only has its own folder format).

Parsing and formatting are done by ``libspmm_host.so`` (mmap + all-thread
tokenizer, shortest round-trip float text); symmetric / skew-symmetric /
hermitian (real) files are expanded to general, duplicates are summed.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, List, Optional

import torch

from .. import _native
from ..ops.csr import CSR, from_coo


class MtxError(RuntimeError):
    pass


def _open(path: str):
    lib = _native.host()
    err = C.create_string_buffer(512)
    m, n, nnz = C.c_int64(), C.c_int64(), C.c_int64()
    field, sym = C.c_int32(), C.c_int32()
    h = lib.spmm_mtx_open(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(field), C.byref(sym),
                          err, 512)
    if not h:
        raise MtxError(f"{path}: {err.value.decode()}")
    return h, m.value, n.value, nnz.value, field.value, sym.value


def read_mtx_coo(path: str, part: int = 0, nparts: int = 1, nthreads: int = 0,
                 gather_counts: Optional[Callable[[int], List[int]]] = None):
    """Entries of part ``part`` of ``nparts`` of the file (line-aligned byte
    ranges of the entry section: a distributed read parses 1/nparts of the
    text per rank), symmetric storage expanded.  Returns (m, n, rows, cols,
    values) as int64 / int64 / float64 host tensors, 0-based, any order.

    ``gather_counts`` (required for nparts > 1): all-gathers this part's
    entry count (-1: the part does not hold whole entries) and returns every
    part's, in part order.  With them every part applies the 1-part rules
    exactly: a file with fewer entries than the header's nnz is rejected (by
    every part), entries past the nnz-th are ignored, so the matrix does not
    depend on the number of parts."""
    lib = _native.host()
    h, m, n, nnz, field, sym = _open(path)
    try:
        if nparts == 1:
            ne = nnz
            ri = torch.empty(ne, dtype=torch.int64)
            ci = torch.empty(ne, dtype=torch.int64)
            v = torch.empty(ne, dtype=torch.float64)
            err = C.create_string_buffer(512)
            if ne and lib.spmm_mtx_fill(h, ri.data_ptr(), ci.data_ptr(), v.data_ptr(), nthreads, err, 512) != 0:
                raise MtxError(f"{path}: {err.value.decode()}")
        else:
            if gather_counts is None:
                raise ValueError("read_mtx_coo: a partial read needs gather_counts")
            b0, b1, ne_ = C.c_int64(), C.c_int64(), C.c_int64()
            whole = lib.spmm_mtx_part(h, part, nparts, C.byref(b0), C.byref(b1), C.byref(ne_), nthreads) == 0
            counts = gather_counts(ne_.value if whole else -1)   # every part takes part in this, even a bad one
            if min(counts) < 0:
                bad = [p for p, c in enumerate(counts) if c < 0]
                raise MtxError(f"{path}: part(s) {bad} of {nparts} do not hold whole entries")
            total = sum(counts)
            if total < nnz:
                raise MtxError(f"{path}: file has {total} entries, expected {nnz}")
            start = sum(counts[:part])
            ne = max(0, min(counts[part], nnz - start))   # entries past the nnz-th are ignored, as in a 1-part read
            ri = torch.empty(ne, dtype=torch.int64)
            ci = torch.empty(ne, dtype=torch.int64)
            v = torch.ones(ne, dtype=torch.float64)
            if ne:
                per = 2 if field == 2 else 3
                got = lib.spmm_mtx_fill_part(h, b0.value, b1.value, ne, ri.data_ptr(), ci.data_ptr(), v.data_ptr(),
                                             nthreads)
                if got != counts[part] * per:
                    raise MtxError(f"{path}: part {part}/{nparts} parsed {got} tokens, expected {counts[part] * per}")
    finally:
        lib.spmm_mtx_close(h)
    if ne and (int(ri.min()) < 0 or int(ri.max()) >= m or int(ci.min()) < 0 or int(ci.max()) >= n):
        raise MtxError(f"{path}: coordinates out of range")
    if sym in (1, 2, 3):
        off = ri != ci
        sign = -1.0 if sym == 2 else 1.0
        ri, ci, v = torch.cat([ri, ci[off]]), torch.cat([ci, ri[off]]), torch.cat([v, sign * v[off]])
    return m, n, ri, ci, v


def read_mtx(path: str, device="cpu", dtype=torch.float32, nthreads: int = 0) -> CSR:
    m, n, ri, ci, v = read_mtx_coo(path, nthreads=nthreads)
    return from_coo(ri.to(device), ci.to(device), v.to(device), m, n, sum_duplicates=True, dtype=dtype)


class MtxWriter:
    """Streaming coordinate-file writer: the header (total nnz known up
    front), then row panels appended in row order (``write_rows_p2p`` feeds
    it one received panel of C at a time), then ``close``.  The bytes are the
    same for any split of the matrix into panels."""

    def __init__(self, path: str, m: int, n: int, nnz: int, pattern: bool = False, nthreads: int = 0):
        self.path, self.pattern, self.nthreads = path, pattern, nthreads
        self.h = _native.host().spmm_mtx_write_begin(path.encode(), m, n, nnz, int(pattern))
        if not self.h:
            raise OSError(f"cannot open {path} for writing")

    def panel(self, row0: int, M: CSR) -> None:
        rp = M.rowptr.to("cpu", torch.int64).contiguous()
        ci = M.col.to("cpu", torch.int32).contiguous()
        vals = None if self.pattern else M.val.to("cpu", torch.float32).contiguous()
        rc = _native.host().spmm_mtx_write_panel(self.h, row0, M.m, rp.data_ptr(), ci.data_ptr(),
                                                  vals.data_ptr() if vals is not None else None, self.nthreads)
        if rc != 0:
            raise OSError(-rc, f"writing {self.path} failed")

    def close(self) -> None:
        if self.h:
            rc = _native.host().spmm_mtx_write_end(self.h)
            self.h = None
            if rc != 0:
                raise OSError(-rc, f"writing {self.path} failed")


def write_mtx(path: str, M: CSR, pattern: bool = False, nthreads: int = 0) -> None:
    w = MtxWriter(path, M.m, M.n, M.nnz, pattern, nthreads)
    try:
        w.panel(0, M)
    finally:
        w.close()
