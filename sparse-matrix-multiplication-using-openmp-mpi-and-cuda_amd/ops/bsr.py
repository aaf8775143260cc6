"""Block-sparse (BSR) uint64 matrices and their pairwise product.

Capability parity with ``helper()`` (sparse_matrix_mult.cu:97-286) and the
data model ``one_matrix`` (:26-32):

* The reference keeps each matrix as ``std::map<(r,c), vector<vector<u64>>>``
  on the host and rebuilds flat buffers + hash indexes for every product
  (:102-138), joins tiles on the host (:140-156), packs every contributing tile
  pair into an 8 GB staging buffer (:189-218) and round-trips it over PCIe in
  rounds of 500 output tiles (:227-253).
* Here a matrix is two device tensors — ``keys`` int32 [nb, 2] sorted
  lexicographically (the std::map order) and ``vals`` int64 [nb, k, k]
  (uint64 bit patterns) — resident in HBM for its whole life.  The tile join
  (symbolic phase) runs on the device, and the numeric phase is the gfx950
  kernel ``spmm_bsr_u64_numeric`` that gathers A/B tiles by index: no staging
  copy, no rounds, no PCIe traffic.
* All-zero tiles are dropped after every product.  With the reference
  arithmetic a zero tile only ever contributes the identity term, so this is
  output-preserving and shrinks later products and messages.

The same code runs on CPU tensors, where the numeric phase is the OpenMP
kernel of ``libspmm_host.so`` with identical arithmetic.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import ctypes as C

import torch

from .. import _native
from .._native import c_vp

# the shared symbolic phase (csrc/kernels/prim.hip), also used by the native a4 engine
_native.register_hip("spmm_bsr_sym_plan_ws", C.c_int64, restype=C.c_size_t)
_native.register_hip("spmm_bsr_sym_plan", c_vp, C.c_int64, c_vp, C.c_int64, c_vp, c_vp, c_vp, c_vp, c_vp)
_native.register_hip("spmm_bsr_sym_build_ws", C.c_int64, restype=C.c_size_t)
_native.register_hip("spmm_bsr_sym_build", c_vp, c_vp, C.c_int64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                     c_vp)
_native.register_hip("spmm_prim_scan_ws", C.c_int64, restype=C.c_size_t)
_native.register_hip("spmm_prim_scan", c_vp, C.c_int, C.c_int64, c_vp, C.c_int, c_vp, c_vp)
_native.register_hip("spmm_prim_sort_ws", C.c_int64, restype=C.c_size_t)
_native.register_hip("spmm_prim_sort_pairs_u64", c_vp, c_vp, C.c_int64, C.c_int, c_vp, c_vp)

U64_MAX = (1 << 64) - 1
_OFF = 1 << 31


def encode_keys(r: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """Order-preserving int64 code of signed int32 pairs (lexicographic (r, c))."""
    return (r.to(torch.int64) << 32) + (c.to(torch.int64) + _OFF)


def decode_keys(code: torch.Tensor) -> torch.Tensor:
    r = torch.div(code, 1 << 32, rounding_mode="floor")
    c = code - (r << 32) - _OFF
    return torch.stack([r, c], dim=1).to(torch.int32)


@dataclass
class BSR:
    """A block-sparse matrix of k x k uint64 tiles.

    ``keys[t] = (r, c)`` are the reference's opaque tile coordinates, sorted
    and unique; ``vals[t]`` is the row-major k x k tile (int64 storage of
    uint64 bit patterns).  ``rows``/``cols`` are the header dimensions.
    """

    rows: int
    cols: int
    k: int
    keys: torch.Tensor
    vals: torch.Tensor

    @property
    def nb(self) -> int:
        return int(self.keys.shape[0])

    @property
    def device(self) -> torch.device:
        return self.vals.device

    def to(self, device, non_blocking: bool = False) -> "BSR":
        return BSR(self.rows, self.cols, self.k, self.keys.to(device, non_blocking=non_blocking),
                   self.vals.to(device, non_blocking=non_blocking))

    def nbytes(self) -> int:
        return self.keys.numel() * 4 + self.vals.numel() * 8

    @staticmethod
    def empty(rows: int, cols: int, k: int, device="cpu") -> "BSR":
        return BSR(rows, cols, k, torch.empty((0, 2), dtype=torch.int32, device=device),
                   torch.empty((0, k, k), dtype=torch.int64, device=device))

    def to_dict(self) -> dict:
        """{(r, c): numpy uint64 [k, k]} — debugging / tests (the reference's map view)."""
        keys = self.keys.cpu().numpy()
        vals = self.vals.cpu().numpy().view("uint64")
        return {(int(r), int(c)): vals[i] for i, (r, c) in enumerate(keys)}


def canonicalize(keys: torch.Tensor, vals: torch.Tensor):
    """Sort tiles by (r, c); for duplicate keys keep the LAST occurrence.

    Mirrors the reference loader's ``m[{row1,col1}] = v`` into a std::map
    (sparse_matrix_mult.cu:383): later tiles overwrite earlier ones and
    iteration is in key order.
    """
    n = keys.shape[0]
    if n <= 1:
        return keys.contiguous(), vals.contiguous()
    code = encode_keys(keys[:, 0], keys[:, 1])
    if bool((code[1:] > code[:-1]).all()):
        return keys.contiguous(), vals.contiguous()
    sc, perm = torch.sort(code, stable=True)
    last = torch.ones(n, dtype=torch.bool, device=keys.device)
    last[:-1] = sc[1:] != sc[:-1]
    sel = perm[last]
    return keys[sel].contiguous(), vals[sel].contiguous()


@dataclass
class BsrPairs:
    """Output of the symbolic phase: for output tile t, the (A tile, B tile)
    pairs ``pa/pb[tile_ptr[t]:tile_ptr[t+1]]`` in ascending middle index."""

    keys: torch.Tensor      # int32 [ntiles, 2]
    tile_ptr: torch.Tensor  # int64 [ntiles + 1]
    pa: torch.Tensor        # int32 [npairs]
    pb: torch.Tensor        # int32 [npairs]

    @property
    def ntiles(self) -> int:
        return int(self.keys.shape[0])

    @property
    def npairs(self) -> int:
        return int(self.pa.shape[0])


def bsr_symbolic(a_keys: torch.Tensor, b_keys: torch.Tensor) -> BsrPairs:
    """Tile-level join C(i,k) <- {(A(i,j), B(j,k))}, on the tensors' device.

    Replaces the host hash join of sparse_matrix_mult.cu:140-156.  A's tiles
    are in (i, j) order and each B block-row in k order, so the expanded pairs
    are already in ascending j for every (i, k); a stable sort by (i, k) groups
    them without disturbing that order — which is the per-element summation
    order the reference's kernel uses (:54-56), needed for bit-exactness.

    On the GPU this is the in-tree symbolic phase of csrc/kernels/prim.hip
    (pair counts, scan, fill with compact keys, stable LSD radix sort,
    run-length encode) — the same code the native ``a4`` engine runs; the
    torch formulation below serves CPU tensors.
    """
    if a_keys.device.type == "cuda":
        return _bsr_symbolic_native(a_keys.contiguous(), b_keys.contiguous())
    dev = a_keys.device
    a_r = a_keys[:, 0].contiguous()
    a_c = a_keys[:, 1].contiguous()
    b_r = b_keys[:, 0].contiguous()
    b_c = b_keys[:, 1].contiguous()
    lo = torch.searchsorted(b_r, a_c)
    hi = torch.searchsorted(b_r, a_c, right=True)
    cnt = hi - lo
    total = int(cnt.sum()) if cnt.numel() else 0
    if total == 0:
        z = torch.zeros(1, dtype=torch.int64, device=dev)
        e32 = torch.empty(0, dtype=torch.int32, device=dev)
        return BsrPairs(torch.empty((0, 2), dtype=torch.int32, device=dev), z, e32, e32)
    a_idx = torch.repeat_interleave(torch.arange(a_keys.shape[0], device=dev), cnt, output_size=total)
    starts = torch.cumsum(cnt, 0) - cnt
    b_idx = lo[a_idx] + (torch.arange(total, device=dev) - starts[a_idx])
    code = encode_keys(a_r[a_idx], b_c[b_idx])
    code, perm = torch.sort(code, stable=True)
    uniq, counts = torch.unique_consecutive(code, return_counts=True)
    tile_ptr = torch.zeros(uniq.shape[0] + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=tile_ptr[1:])
    return BsrPairs(decode_keys(uniq), tile_ptr, a_idx[perm].to(torch.int32), b_idx[perm].to(torch.int32))


def _bsr_symbolic_native(a_keys: torch.Tensor, b_keys: torch.Tensor) -> BsrPairs:
    dev = a_keys.device
    lib = _native.hip()
    P = _native.ptr
    st = _native.stream_ptr(dev)
    na, nb = a_keys.shape[0], b_keys.shape[0]
    z = torch.zeros(1, dtype=torch.int64, device=dev)
    e32 = torch.empty(0, dtype=torch.int32, device=dev)
    empty = BsrPairs(torch.empty((0, 2), dtype=torch.int32, device=dev), z, e32, e32)
    if na == 0 or nb == 0:
        return empty
    start = torch.empty(na + 1, dtype=torch.int64, device=dev)
    lo = torch.empty(na, dtype=torch.int64, device=dev)
    ws = torch.empty(int(lib.spmm_bsr_sym_plan_ws(na)), dtype=torch.uint8, device=dev)
    plan = (C.c_int64 * 5)()
    _native.check(lib.spmm_bsr_sym_plan(P(a_keys), na, P(b_keys), nb, P(start), P(lo), P(ws), plan, st),
                  "spmm_bsr_sym_plan")
    np_ = plan[0]
    if np_ == 0:
        return empty
    del ws
    ws = torch.empty(int(lib.spmm_bsr_sym_build_ws(np_)), dtype=torch.uint8, device=dev)
    okeys = torch.empty((np_, 2), dtype=torch.int32, device=dev)
    tile_ptr = torch.empty(np_ + 1, dtype=torch.int64, device=dev)
    pa = torch.empty(np_, dtype=torch.int32, device=dev)
    pb = torch.empty(np_, dtype=torch.int32, device=dev)
    nt = C.c_int64()
    _native.check(lib.spmm_bsr_sym_build(P(a_keys), P(b_keys), na, P(start), P(lo), plan, P(ws), P(okeys),
                                         P(tile_ptr), P(pa), P(pb), C.byref(nt), st), "spmm_bsr_sym_build")
    n = nt.value
    return BsrPairs(okeys[:n].clone(), tile_ptr[:n + 1].clone(), pa, pb)   # (release the np-sized buffers)


def bsr_numeric(A: BSR, B: BSR, sym: BsrPairs):
    """Numeric phase: returns (vals [ntiles,k,k] int64, nonzero flags int32)."""
    k = A.k
    dev = A.device
    n = sym.ntiles
    vals = torch.empty((n, k, k), dtype=torch.int64, device=dev)
    nz = torch.zeros(n, dtype=torch.int32, device=dev)
    if n == 0:
        return vals, nz
    Av, Bv = A.vals.contiguous(), B.vals.contiguous()
    P = _native.ptr
    if dev.type == "cuda":
        rc = _native.hip().spmm_bsr_u64_numeric(P(Av), P(Bv), P(sym.pa), P(sym.pb), P(sym.tile_ptr), P(vals),
                                                 P(nz), k, n, _native.stream_ptr(dev))
        _native.check(rc, "spmm_bsr_u64_numeric")
    else:
        rc = _native.host().spmm_cpu_bsr_u64_numeric(P(Av), P(Bv), P(sym.pa), P(sym.pb), P(sym.tile_ptr),
                                                      P(vals), P(nz), k, n, 0)
        _native.check(rc, "spmm_cpu_bsr_u64_numeric")
    return vals, nz


def nonzero_tiles(M: BSR) -> torch.Tensor:
    """int32 flag per tile: 1 if any element is non-zero."""
    n = M.nb
    nz = torch.empty(n, dtype=torch.int32, device=M.device)
    if n == 0:
        return nz
    v = M.vals.contiguous()
    if M.device.type == "cuda":
        _native.check(_native.hip().spmm_bsr_u64_nonzero(_native.ptr(v), M.k, n, _native.ptr(nz),
                                                          _native.stream_ptr(M.device)), "spmm_bsr_u64_nonzero")
    else:
        _native.check(_native.host().spmm_cpu_bsr_u64_nonzero(_native.ptr(v), M.k, n, _native.ptr(nz), 0),
                      "spmm_cpu_bsr_u64_nonzero")
    return nz


def prune_zero_tiles(M: BSR, nz: Optional[torch.Tensor] = None) -> BSR:
    """Drop all-zero tiles (the reference's final erase loop, :577-592, without
    its erase-during-iteration UB)."""
    if nz is None:
        nz = nonzero_tiles(M)
    keep = nz.bool()
    if M.nb and bool(keep.all()):
        return M
    return BSR(M.rows, M.cols, M.k, M.keys[keep].contiguous(), M.vals[keep].contiguous())


def bsr_matmul(A: BSR, B: BSR, prune: bool = True) -> BSR:
    """C = A . B (reference arithmetic).  C.rows = A.rows, C.cols = B.cols,
    as in the reference (:280-283) — tile keys, not dimensions, drive the join."""
    if A.k != B.k:
        raise ValueError(f"tile size mismatch: {A.k} vs {B.k}")
    if A.device != B.device:
        raise ValueError("operands on different devices")
    sym = bsr_symbolic(A.keys, B.keys)
    vals, nz = bsr_numeric(A, B, sym)
    C = BSR(A.rows, B.cols, A.k, sym.keys, vals)
    return prune_zero_tiles(C, nz) if prune else C


def tile_pair_count(A: BSR, B: BSR) -> int:
    """Number of tile-pair products of A.B (each is 2*k^3 integer ops)."""
    b_r = B.keys[:, 0].contiguous()
    a_c = A.keys[:, 1].contiguous()
    return int((torch.searchsorted(b_r, a_c, right=True) - torch.searchsorted(b_r, a_c)).sum())
