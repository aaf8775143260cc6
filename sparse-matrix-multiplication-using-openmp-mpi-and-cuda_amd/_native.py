"""ctypes bindings for the in-tree native libraries.

Two libraries, both C ABI (no torch headers, no hipify):

* ``libspmm_host.so`` (C++/OpenMP) — always required.
* ``libspmm_hip.so`` (HIP, gfx950) — required whenever a GPU is used.  It is
  loaded AFTER ``import torch`` so it binds to the HIP runtime torch already
  loaded (same SONAME ``libamdhip64.so.7``): one runtime, one device context,
  shared streams and allocations.

There is deliberately no silent fallback: on a GPU box a missing or broken
HIP library raises instead of quietly running PyTorch/CPU code.
"""
from __future__ import annotations

import ctypes as C
import fcntl
import os
import threading

from . import _build

_lock = threading.Lock()
_host = None
_hip = None

c_i32p = C.POINTER(C.c_int32)
c_i64p = C.POINTER(C.c_int64)
c_vp = C.c_void_p


def _build_locked(which: str) -> None:
    os.makedirs(_build.LIB_DIR, exist_ok=True)
    with open(os.path.join(_build.LIB_DIR, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if which == "host":
                _build.build_host()
            else:
                _build.build_hip()
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _sig(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)


def host():
    """The C++/OpenMP host library (builds it on first use if needed)."""
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                if not os.path.exists(_build.HOST_LIB) or os.environ.get("SPMM_REBUILD"):
                    _build_locked("host")
                lib = C.CDLL(_build.HOST_LIB)
                _sig(lib, "spmm_ref_open", c_vp, C.c_char_p, C.c_int, c_i64p, c_i64p, c_i64p, C.c_char_p, C.c_int)
                _sig(lib, "spmm_ref_fill", C.c_int, c_vp, c_vp, c_vp, C.c_int, C.c_char_p, C.c_int)
                _sig(lib, "spmm_ref_close", None, c_vp)
                _sig(lib, "spmm_ref_write", C.c_int, C.c_char_p, C.c_int64, C.c_int64, C.c_int64, c_vp, c_vp,
                     C.c_int, C.c_int)
                _sig(lib, "spmm_mtx_open", c_vp, C.c_char_p, c_i64p, c_i64p, c_i64p, c_i32p, c_i32p,
                     C.c_char_p, C.c_int)
                _sig(lib, "spmm_mtx_fill", C.c_int, c_vp, c_vp, c_vp, c_vp, C.c_int, C.c_char_p, C.c_int)
                _sig(lib, "spmm_mtx_close", None, c_vp)
                _sig(lib, "spmm_mtx_write", C.c_int, C.c_char_p, C.c_int64, C.c_int64, c_vp, c_vp, c_vp, C.c_int)
                _sig(lib, "spmm_mtx_part", C.c_int, c_vp, C.c_int, C.c_int, c_i64p, c_i64p, c_i64p, C.c_int)
                _sig(lib, "spmm_mtx_fill_part", C.c_int64, c_vp, C.c_int64, C.c_int64, C.c_int64, c_vp, c_vp, c_vp,
                     C.c_int)
                _sig(lib, "spmm_mtx_write_begin", c_vp, C.c_char_p, C.c_int64, C.c_int64, C.c_int64, C.c_int)
                _sig(lib, "spmm_mtx_write_panel", C.c_int, c_vp, C.c_int64, C.c_int64, c_vp, c_vp, c_vp, C.c_int)
                _sig(lib, "spmm_mtx_write_end", C.c_int, c_vp)
                _sig(lib, "spmm_cpu_bsr_u64_numeric", C.c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                     C.c_int, C.c_int64, C.c_int)
                _sig(lib, "spmm_cpu_bsr_u64_nonzero", C.c_int, c_vp, C.c_int, C.c_int64, c_vp, C.c_int)
                _sig(lib, "spmm_cpu_csr_nprod", C.c_int64, C.c_int64, c_vp, c_vp, c_vp, c_vp, C.c_int)
                _sig(lib, "spmm_cpu_csr_spgemm_symbolic", C.c_int64, C.c_int64, C.c_int64, c_vp, c_vp, c_vp,
                     c_vp, c_vp, C.c_int)
                _sig(lib, "spmm_cpu_csr_spgemm_numeric", C.c_int, C.c_int64, C.c_int64, c_vp, c_vp, c_vp,
                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C.c_int)
                _sig(lib, "spmm_cpu_csr_spmm", C.c_int, C.c_int64, C.c_int64, c_vp, c_vp, c_vp, c_vp, c_vp,
                     C.c_int)
                _host = lib
    return _host


def hip():
    """The gfx950 kernel library.  Raises if it cannot be built or loaded."""
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                import torch  # noqa: F401  (bind to torch's HIP runtime first)

                path = os.environ.get("SPMM_HIP_LIB")   # a diagnostic build (tools/bm_stamps.py)
                if not path:
                    if not os.path.exists(_build.HIP_LIB) or os.environ.get("SPMM_REBUILD"):
                        _build_locked("hip")
                    path = _build.HIP_LIB
                lib = C.CDLL(path)
                _sig(lib, "spmm_bsr_u64_numeric", C.c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C.c_int,
                     C.c_int64, c_vp)
                _sig(lib, "spmm_bsr_u64_nonzero", C.c_int, c_vp, C.c_int, C.c_int64, c_vp, c_vp)
                for name, (res, args) in _HIP_EXTRA.items():
                    if hasattr(lib, name):
                        _sig(lib, name, res, *args)
                _hip = lib
    return _hip


# Signatures of launchers added by other kernel files (registered lazily so a
# partially built library still exposes what it has).
_HIP_EXTRA: dict = {}


def register_hip(name: str, *argtypes, restype=C.c_int) -> None:
    _HIP_EXTRA[name] = (restype, argtypes)
    if _hip is not None and hasattr(_hip, name):
        _sig(_hip, name, restype, *argtypes)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error {rc}")


def ptr(t) -> int:
    """Raw data pointer of a torch tensor / numpy array (0 for empty; None,
    i.e. a null pointer, for None)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
