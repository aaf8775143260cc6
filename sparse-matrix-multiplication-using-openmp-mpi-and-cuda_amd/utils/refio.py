"""Reference folder format I/O (``<folder>/size``, ``<folder>/matrix<i>``, ``./matrix``).

Parity: size file read at sparse_matrix_mult.cu:411-419, per-matrix parser
:342-391 (one OpenMP task per file, ``ifstream >>``), writer :595-608.
Parsing and formatting run in ``libspmm_host.so`` (mmap + all-thread
tokenizer, ``to_chars`` writer); tiles can be parsed straight into pinned
memory so the H2D copy is a single async DMA.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Tuple

import torch

from .. import _native
from ..ops.bsr import BSR, canonicalize


class FormatError(RuntimeError):
    pass


def read_size(folder: str) -> Tuple[int, int]:
    """``<folder>/size`` holds ``N k``: chain length and tile edge."""
    path = os.path.join(folder, "size")
    try:
        with open(path) as f:
            tok = f.read().split()
    except OSError as e:
        raise FormatError(f"Cannot open size file! ({path}: {e.strerror})") from e
    if len(tok) < 2:
        raise FormatError(f"size file {path} must contain 'N k'")
    return int(tok[0]), int(tok[1])


def matrix_path(folder: str, i: int) -> str:
    """1-based file index, as the reference (``"/matrix" + to_string(i)``, :342-345)."""
    return os.path.join(folder, f"matrix{i}")


def read_matrix(path: str, k: int, nthreads: int = 0, pin: bool = False) -> BSR:
    """Parse one reference-format matrix into a canonical (sorted, deduplicated)
    CPU BSR.  ``pin=True`` parses into page-locked memory."""
    lib = _native.host()
    err = C.create_string_buffer(512)
    rows, cols, nb = C.c_int64(), C.c_int64(), C.c_int64()
    h = lib.spmm_ref_open(path.encode(), k, C.byref(rows), C.byref(cols), C.byref(nb), err, 512)
    if not h:
        raise FormatError(err.value.decode())
    try:
        pin = pin and torch.cuda.is_available()
        keys = torch.empty((nb.value, 2), dtype=torch.int32, pin_memory=pin)
        vals = torch.empty((nb.value, k, k), dtype=torch.int64, pin_memory=pin)
        if nb.value:
            rc = lib.spmm_ref_fill(h, keys.data_ptr(), vals.data_ptr(), nthreads, err, 512)
            if rc != 0:
                raise FormatError(f"{path}: {err.value.decode()}")
    finally:
        lib.spmm_ref_close(h)
    keys, vals = canonicalize(keys, vals)
    return BSR(rows.value, cols.value, k, keys, vals)


def write_matrix(path: str, M: BSR, nthreads: int = 0) -> None:
    """Write M in the reference output layout.  M must be canonical and pruned
    (the caller decides about zero tiles, as the reference does at :577-592)."""
    keys = M.keys.to("cpu").contiguous()
    vals = M.vals.to("cpu").contiguous()
    rc = _native.host().spmm_ref_write(path.encode(), M.rows, M.cols, M.nb, keys.data_ptr(), vals.data_ptr(),
                                        M.k, nthreads)
    if rc != 0:
        raise OSError(-rc, f"writing {path} failed")


def write_folder(folder: str, mats, k: int) -> None:
    """Write a whole chain as a reference input folder (generator output)."""
    os.makedirs(folder, exist_ok=True)
    with open(os.path.join(folder, "size"), "w") as f:
        f.write(f"{len(mats)} {k}\n")
    for i, M in enumerate(mats, start=1):
        write_matrix(matrix_path(folder, i), M)
