"""Matrix Market (coordinate) I/O for CSR matrices (north-star requirement;
the reference only has its own folder format).

Parsing and formatting are done by ``libspmm_host.so`` (mmap + all-thread
tokenizer, shortest round-trip float text); symmetric / skew-symmetric /
hermitian (real) files are expanded to general, duplicates are summed.
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native
from ..ops.csr import CSR, from_coo


class MtxError(RuntimeError):
    pass


def read_mtx(path: str, device="cpu", dtype=torch.float32, nthreads: int = 0) -> CSR:
    lib = _native.host()
    err = C.create_string_buffer(512)
    m, n, nnz = C.c_int64(), C.c_int64(), C.c_int64()
    field, sym = C.c_int32(), C.c_int32()
    h = lib.spmm_mtx_open(path.encode(), C.byref(m), C.byref(n), C.byref(nnz), C.byref(field), C.byref(sym),
                          err, 512)
    if not h:
        raise MtxError(f"{path}: {err.value.decode()}")
    try:
        ri = torch.empty(nnz.value, dtype=torch.int64)
        ci = torch.empty(nnz.value, dtype=torch.int64)
        v = torch.empty(nnz.value, dtype=torch.float64)
        if nnz.value and lib.spmm_mtx_fill(h, ri.data_ptr(), ci.data_ptr(), v.data_ptr(), nthreads, err, 512) != 0:
            raise MtxError(f"{path}: {err.value.decode()}")
    finally:
        lib.spmm_mtx_close(h)
    if nnz.value and (int(ri.min()) < 0 or int(ri.max()) >= m.value or int(ci.min()) < 0 or int(ci.max()) >= n.value):
        raise MtxError(f"{path}: coordinates out of range")
    if sym.value in (1, 2, 3):
        off = ri != ci
        sign = -1.0 if sym.value == 2 else 1.0
        ri, ci, v = torch.cat([ri, ci[off]]), torch.cat([ci, ri[off]]), torch.cat([v, sign * v[off]])
    M = from_coo(ri.to(device), ci.to(device), v.to(device), m.value, n.value, sum_duplicates=True, dtype=dtype)
    return M


def write_mtx(path: str, M: CSR, pattern: bool = False, nthreads: int = 0) -> None:
    rp = M.rowptr.to("cpu", torch.int64).contiguous()
    ci = M.col.to("cpu", torch.int32).contiguous()
    vals = None if pattern else M.val.to("cpu", torch.float32).contiguous()
    rc = _native.host().spmm_mtx_write(path.encode(), M.m, M.n, rp.data_ptr(), ci.data_ptr(),
                                        vals.data_ptr() if vals is not None else None, nthreads)
    if rc != 0:
        raise OSError(-rc, f"writing {path} failed")
