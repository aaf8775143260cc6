"""CSR x dense SpMM: Y = A . X  (A bf16 CSR, X bf16 [n, D], fp32 accumulate).

gfx950 kernels (``csrc/kernels/csr_spmm.hip``):

* ``mfma``    — row-group MFMA kernel (D = 128; other multiples of 128 take
  ``panel``): a wave owns 16 consecutive rows, takes their entries in chunks
  of 32 with the sweep's 16-byte gathers (16 in flight a wave), transposes
  the gathered X rows through LDS and multiplies with
  v_mfma_f32_16x16x32_bf16 (K = the chunk's entries).  No inspector.
* ``panel``   — panel MFMA kernel: an inspector (:func:`plan_panels`, run once
  per matrix) lists each 64-row panel's sorted union of columns in chunks of
  64; the kernel gathers each chunk's X rows into LDS once, scatters the
  chunk's entries into a dense 64x64 A tile and runs the same MFMA.  X rows
  shared by several rows of a panel are fetched once.
* ``rowwise`` — VALU row-gather kernel, no inspector; one wave per row.
* ``sweep``   — VALU row-owning sweep (D = 128): a resident grid of waves,
  each owning up to 16 rows staged in LDS, walks A's columns slice by slice
  with 16 independent 16-byte gathers in flight per wave (:func:`sweep_ok`
  checks once per operand that the rows fit).

Both MFMA kernels multiply zero A slots into X rows of other rows of the
group: a non-finite X value reaches every output row of its 16-row group
(panel: 64-row panel) as NaN, where the VALU kernels keep it to the rows
that use it.

``auto`` picks ``panel`` when the panel column reuse (nnz / union columns) is
at least ``MFMA_MIN_REUSE`` — i.e. when the panel path moves fewer bytes —
and ``rowwise`` otherwise (``models.spmm.bench_setup`` times every
candidate instead).  CPU tensors use the OpenMP kernel.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import torch

from .. import _native
from .._native import c_vp
from ..utils.config import CONFIG
from .csr import CSR

_native.register_hip("spmm_spmm_panel_mfma", c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, C.c_int64, C.c_int64, C.c_int64,
                     c_vp, C.c_int64, C.c_int, c_vp)
_native.register_hip("spmm_spmm_rows_mfma", c_vp, c_vp, c_vp, c_vp, C.c_int64, C.c_int64, C.c_int64, c_vp,
                     C.c_int64, C.c_int, c_vp)
_native.register_hip("spmm_spmm_rowwise", c_vp, c_vp, c_vp, c_vp, C.c_int64, C.c_int64, C.c_int64, c_vp,
                     C.c_int64, C.c_int, c_vp)
_native.register_hip("spmm_spmm_sweep", c_vp, c_vp, c_vp, c_vp, C.c_int64, C.c_int64, C.c_int64, C.c_int64, c_vp,
                     C.c_int64, C.c_int, c_vp, c_vp)
_native.register_hip("spmm_spmm_sweep_geometry", C.c_int64, C.c_int64, c_vp, c_vp, c_vp)
_native.register_hip("spmm_spmm_plan_count", c_vp, c_vp, C.c_int64, C.c_int64, c_vp, c_vp)
_native.register_hip("spmm_spmm_plan_fill", c_vp, c_vp, c_vp, C.c_int, C.c_int64, C.c_int64, c_vp, c_vp, c_vp, c_vp,
                     c_vp, c_vp, c_vp)

PANEL = 64
CHUNK = 64
MFMA_MIN_REUSE = CONFIG.spmm_mfma_min_reuse


@dataclass
class PanelPlan:
    m: int
    n: int
    panel_chunk_ptr: torch.Tensor   # int64 [npanels + 1]
    chunk_cols: torch.Tensor        # int32 [nchunks * 64], -1 = padding
    chunk_ent_ptr: torch.Tensor     # int64 [nchunks + 1]
    ent_rc: torch.Tensor            # int32 [nnz]: row_in_panel * 64 + slot
    ent_val: torch.Tensor           # bf16 [nnz]
    union_cols: int                 # X rows gathered per pass (sum over panels)
    nnz: int

    @property
    def reuse(self) -> float:
        return self.nnz / max(self.union_cols, 1)


def plan_panels(A: CSR, device_kernel: bool = True) -> PanelPlan:
    """Inspector for the MFMA kernel, done once per sparse operand.  On a GPU
    it is two hand-written kernels (``csr_spmm.hip`` spmm_plan: per panel an
    LDS column bitmap, union ranks, chunk counts and scan) with one read-back
    of the chunk total; panels whose union exceeds 65536 columns, and CPU
    tensors, use the torch formulation below (same plan up to the order of
    entries inside a chunk)."""
    if device_kernel and A.device.type == "cuda" and A.m > 0:
        plan = _plan_panels_hip(A)
        if plan is not None:
            return plan
    return _plan_panels_torch(A)


def _plan_panels_hip(A: CSR) -> Optional[PanelPlan]:
    dev = A.device
    P = _native.ptr
    lib = _native.hip()
    st = _native.stream_ptr(dev)
    npan = (A.m + PANEL - 1) // PANEL
    col = A.col if A.col.dtype == torch.int32 else A.col.to(torch.int32)
    val_f32 = A.val.dtype == torch.float32
    av = A.val if val_f32 or A.val.dtype == torch.bfloat16 else A.val.float()
    val_f32 = av.dtype == torch.float32
    nunion = torch.empty(npan, dtype=torch.int64, device=dev)
    _native.check(lib.spmm_spmm_plan_count(P(A.rowptr), P(col), A.m, A.n, P(nunion), st), "spmm_plan_count")
    pcp = torch.zeros(npan + 1, dtype=torch.int64, device=dev)
    torch.cumsum(torch.div(nunion + CHUNK - 1, CHUNK, rounding_mode="floor"), 0, out=pcp[1:])
    total_ch, union_cols, widest = torch.stack([pcp[-1], nunion.sum(), nunion.max()]).tolist()   # one read-back
    if widest > 1024 * CHUNK:
        return None
    chunk_cols = torch.empty(total_ch * CHUNK, dtype=torch.int32, device=dev)
    chunk_ent_ptr = torch.zeros(total_ch + 1, dtype=torch.int64, device=dev)
    ent_rc = torch.empty(A.nnz, dtype=torch.int32, device=dev)
    ent_val = torch.empty(A.nnz, dtype=torch.bfloat16, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _native.check(lib.spmm_spmm_plan_fill(P(A.rowptr), P(col), P(av), int(val_f32), A.m, A.n, P(pcp), P(chunk_cols),
                                          P(chunk_ent_ptr), P(ent_rc), P(ent_val), P(err), st), "spmm_plan_fill")
    return PanelPlan(A.m, A.n, pcp, chunk_cols, chunk_ent_ptr, ent_rc, ent_val, int(union_cols), A.nnz)


def _plan_panels_torch(A: CSR) -> PanelPlan:
    """The inspector as device-side torch ops (reference formulation)."""
    dev = A.device
    n = A.n
    npan = (A.m + PANEL - 1) // PANEL
    r = A.row_ids()
    p = torch.div(r, PANEL, rounding_mode="floor")
    key, perm = torch.sort(p * n + A.col.long(), stable=True)
    r, p = r[perm], p[perm]
    vals = A.val[perm].to(torch.bfloat16)
    uniq, inv = torch.unique_consecutive(key, return_inverse=True)
    up = torch.div(uniq, n, rounding_mode="floor")
    ucol = uniq - up * n
    ucount = torch.bincount(up, minlength=npan)
    ustart = torch.cumsum(ucount, 0) - ucount
    uidx = torch.arange(uniq.numel(), device=dev) - ustart[up]
    nch = torch.div(ucount + CHUNK - 1, CHUNK, rounding_mode="floor")
    chend = torch.cumsum(nch, 0)
    chstart = chend - nch
    total_ch = int(chend[-1]) if npan else 0
    panel_chunk_ptr = torch.zeros(npan + 1, dtype=torch.int64, device=dev)
    panel_chunk_ptr[1:] = chend
    chunk_cols = torch.full((total_ch * CHUNK,), -1, dtype=torch.int32, device=dev)
    chunk_cols[chstart[up] * CHUNK + uidx] = ucol.to(torch.int32)
    e_upos = uidx[inv]
    e_chunk = chstart[p] + torch.div(e_upos, CHUNK, rounding_mode="floor")
    ent_rc = ((r - p * PANEL) * CHUNK + e_upos % CHUNK).to(torch.int32)
    chunk_ent_ptr = torch.zeros(total_ch + 1, dtype=torch.int64, device=dev)
    if total_ch:
        torch.cumsum(torch.bincount(e_chunk, minlength=total_ch), 0, out=chunk_ent_ptr[1:])
    return PanelPlan(A.m, n, panel_chunk_ptr, chunk_cols, chunk_ent_ptr, ent_rc.contiguous(), vals.contiguous(),
                     int(uniq.numel()), A.nnz)


def sweep_ok(A: CSR) -> bool:
    """Whether the row-owning sweep kernel (``method="sweep"``,
    csr_spmm.hip spmm_sweep) can take A on this GPU: every row's columns are
    non-decreasing (the kernel splits a row into column slices by counting
    its entries below each slice boundary, which assumes sorted columns; CSR
    does not guarantee that), its resident grid holds every row (<= 16 rows
    per wave) and no wave's rows hold more entries than its LDS stage.  One
    read-back; done once per operand (an inspector step, like
    :func:`plan_panels`)."""
    if A.device.type != "cuda" or A.m == 0:
        return False
    cached = getattr(A, "_sweep_ok", None)
    if cached is not None:
        return cached
    A._sweep_ok = _cols_nondecreasing(A) and _sweep_fits(A)
    return A._sweep_ok


def _cols_nondecreasing(A: CSR) -> bool:
    if A.nnz < 2:
        return True
    code = A.row_ids() * A.n + A.col.long()
    return bool((code[1:] >= code[:-1]).all())


def _sweep_fits(A: CSR) -> bool:
    waves, rpw, cap = C.c_int64(), C.c_int(), C.c_int()
    _native.check(_native.hip().spmm_spmm_sweep_geometry(A.m, A.n, C.byref(waves), C.byref(rpw), C.byref(cap)),
                  "spmm_sweep_geometry")
    G = waves.value
    if G == 0:
        return False
    lens = (A.rowptr[1:] - A.rowptr[:-1]).to(torch.int64)
    padded = torch.zeros(rpw.value * G, dtype=torch.int64, device=A.device)
    padded[:A.m] = lens
    return int(padded.view(rpw.value, G).sum(0).max()) <= cap.value   # row k of wave w = w + k G


def spmm(A: CSR, X: torch.Tensor, out_dtype=torch.float32, method: str = "auto",
         plan: Optional[PanelPlan] = None) -> torch.Tensor:
    if X.dim() != 2 or X.shape[0] != A.n:
        raise ValueError(f"X must be [{A.n}, D], got {tuple(X.shape)}")
    D = X.shape[1]
    dev = A.device
    if dev.type != "cuda":
        Af = A.val.float().contiguous()
        Xf = X.float().contiguous()
        Y = torch.empty((A.m, D), dtype=torch.float32)
        _native.host().spmm_cpu_csr_spmm(A.m, D, _native.ptr(A.rowptr), _native.ptr(A.col), _native.ptr(Af),
                                         _native.ptr(Xf), _native.ptr(Y), 0)
        return Y.to(out_dtype)
    X = X.to(torch.bfloat16).contiguous()
    Y = torch.empty((A.m, D), dtype=out_dtype, device=dev)
    out_bf16 = 1 if out_dtype == torch.bfloat16 else 0
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("out_dtype must be float32 or bfloat16")
    P = _native.ptr
    lib = _native.hip()
    stream = _native.stream_ptr(dev)
    if method == "auto":
        if D % 128 == 0 and (plan is not None and plan.reuse >= MFMA_MIN_REUSE):
            method = "panel"
        else:
            method = "rowwise"
    if method == "mfma" and D != 128:
        method = "panel"   # (the row-group kernel covers one 128-column block)
    if method == "mfma":
        av = A.val.to(torch.bfloat16).contiguous()
        _native.check(lib.spmm_spmm_rows_mfma(P(A.rowptr), P(A.col), P(av), P(X), D, A.m, D, P(Y), D, out_bf16,
                                              stream), "spmm_rows_mfma")
    elif method == "panel":
        if D % 128 != 0:
            raise ValueError("MFMA SpMM needs D % 128 == 0")
        plan = plan if plan is not None else plan_panels(A)
        _native.check(lib.spmm_spmm_panel_mfma(P(plan.panel_chunk_ptr), P(plan.chunk_cols), P(plan.chunk_ent_ptr),
                                               P(plan.ent_rc), P(plan.ent_val), P(X), D, A.m, D, P(Y), D, out_bf16,
                                               stream), "spmm_panel_mfma")
    elif method == "sweep":
        if D != 128:
            raise ValueError("the sweep SpMM kernel needs D == 128")
        if getattr(A, "_sweep_ok", None) is None and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("spmm(method='sweep') inside a graph capture: call sweep_ok(A) before capturing")
        if not sweep_ok(A):   # (cached per operand after the first call)
            raise ValueError("the sweep SpMM kernel cannot stage this operand (sweep_ok(A) is False)")
        # (the kernel's err word flags the same condition device-side: a wave over its LDS stage
        # writes zero rows; the plan check above rules it out, so no word is passed or read back)
        av = A.val.to(torch.bfloat16).contiguous()
        _native.check(lib.spmm_spmm_sweep(P(A.rowptr), P(A.col), P(av), P(X), D, A.m, A.n, D, P(Y), D, out_bf16,
                                          None, stream), "spmm_sweep")
    elif method == "rowwise":
        av = A.val.to(torch.bfloat16).contiguous()
        _native.check(lib.spmm_spmm_rowwise(P(A.rowptr), P(A.col), P(av), P(X), D, A.m, D, P(Y), D, out_bf16,
                                            stream), "spmm_rowwise")
    else:
        raise ValueError(f"unknown method {method!r}")
    return Y


class SpmmGraph:
    """Y = A . X replayed from a captured HIP graph.

    The inspected SpMM has no host synchronisation, so its launches (input
    cast, output allocation, MFMA or row kernel) are captured once into a
    graph and replayed: a launch-bound 65536^2 x 128 step (~0.15 ms of GPU
    work) stops paying per-kernel launch and Python dispatch costs.  ``X`` is
    a static input buffer: copy new operands into ``graph.X`` before
    ``run()``; ``run()`` returns the static output tensor.
    """

    def __init__(self, A: CSR, X: torch.Tensor, out_dtype=torch.float32, method: str = "auto",
                 plan: Optional[PanelPlan] = None):
        if A.device.type != "cuda":
            raise ValueError("SpmmGraph needs a GPU operand")
        self.X = X.to(torch.bfloat16).contiguous().clone()
        side = torch.cuda.Stream(A.device)
        side.wait_stream(torch.cuda.current_stream(A.device))
        with torch.cuda.stream(side):
            for _ in range(2):   # warm-up outside the capture (allocator, lazy library state)
                spmm(A, self.X, out_dtype, method, plan)
        torch.cuda.current_stream(A.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.Y = spmm(A, self.X, out_dtype, method, plan)

    def run(self) -> torch.Tensor:
        self.graph.replay()
        return self.Y
