"""Distributed SpMM over RCCL / xGMI: Y = A . X, A sparse (bf16), X dense [n, D].

Two decompositions (north-star: "all-gather of B row panels plus
reduce-scatter of C"):

* ``rowblock_spmm`` — rank r holds A's row panel r and X's row panel r;
  X is all-gathered (ring over xGMI), Y's row panel is computed locally.
  Communication: (P-1)/P * n * D * 2 B per rank.
* ``innerdim_spmm`` — rank r holds A's COLUMN panel r (all rows) and X's
  row panel r; each rank computes a full-height fp32 partial Y_r = A[:, r] .
  X_r, and a reduce-scatter sums the partials into row panels.
  Communication: (P-1)/P * m * D * 4 B per rank, no X replication — the
  right choice when X (n x D) is much larger than Y, or X cannot be
  replicated.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops.csr import CSR
from ..ops.spmm import PanelPlan, SpmmGraph, plan_panels, spmm, sweep_ok
from ..parallel.comm import Comm
from ..parallel.partition import row_panels
from ..utils.config import CONFIG
from ..utils.gen_csr import uniform_csr


def allgather_rows(Xp: torch.Tensor, comm: Comm, counts) -> torch.Tensor:
    """Concatenate row panels of a dense matrix (uneven panels padded)."""
    if not comm.is_dist:
        return Xp
    mx = max(counts)
    buf = torch.zeros((mx, Xp.shape[1]), dtype=Xp.dtype, device=Xp.device)
    buf[:Xp.shape[0]] = Xp
    parts = comm.all_gather(buf).view(comm.world, mx, -1)
    if all(c == mx for c in counts):
        return parts.reshape(comm.world * mx, -1)
    return torch.cat([parts[r, :counts[r]] for r in range(comm.world)])


def rowblock_spmm(A_panel: CSR, X_panel: torch.Tensor, comm: Comm, counts, plan: Optional[PanelPlan] = None,
                  method: str = "auto", out_dtype=torch.float32) -> torch.Tensor:
    X = allgather_rows(X_panel, comm, counts)
    return spmm(A_panel, X, out_dtype=out_dtype, method=method, plan=plan)


def innerdim_spmm(A_colpanel: CSR, X_panel: torch.Tensor, comm: Comm, row_counts, method: str = "auto",
                  plan: Optional[PanelPlan] = None) -> torch.Tensor:
    """A_colpanel: all m rows, columns of this rank's panel (re-indexed from 0).
    Returns this rank's fp32 row panel of Y."""
    Yp = spmm(A_colpanel, X_panel, out_dtype=torch.float32, method=method, plan=plan)
    if not comm.is_dist:
        return Yp
    mx = max(row_counts)
    D = Yp.shape[1]
    full = torch.zeros((comm.world * mx, D), dtype=torch.float32, device=Yp.device)
    off = 0
    for r, c in enumerate(row_counts):
        full[r * mx:r * mx + c] = Yp[off:off + c]
        off += c
    return comm.reduce_scatter(full)[:row_counts[comm.rank]]


def column_panel(A: CSR, lo: int, hi: int) -> CSR:
    """Columns [lo, hi) of A, re-indexed to start at 0 (all rows kept)."""
    return A.col_slice(lo, hi)


def bench_setup(comm: Comm, n: int = 65536, density: float = 1e-3, cols: int = 128, seed: int = 1,
                method: str = "auto"):
    """BASELINE config 3: 65536^2 CSR (bf16) x dense [65536, 128] (bf16).
    One step = all-gather of X row panels (P > 1) + SpMM of this rank's rows.
    The kernel is what ``auto`` picks from the inspected plan.  The inspector
    (``plan_panels``: A's panel / chunk layout) runs once per sparse operand,
    as a library's SpMM preprocessing does; its time is reported separately
    (``inspector_ms``) rather than hidden."""
    panels = row_panels(n, comm.world)
    lo, hi = panels[comm.rank]
    A = uniform_csr(n, n, density, seed=seed, device=comm.device, rows=(lo, hi), dtype=torch.bfloat16)
    g = torch.Generator(device=comm.device)
    g.manual_seed(seed * 31 + comm.rank)
    Xp = (torch.rand((hi - lo, cols), generator=g, device=comm.device) * 2 - 1).to(torch.bfloat16)
    counts = [b - a for a, b in panels]
    plan, inspector_ms, inspector_first_ms = None, None, None
    import time

    if method not in ("auto", "mfma", "panel", "sweep", "rowwise"):
        raise ValueError(f"unknown SpMM method {method!r}")
    if comm.device.type == "cuda" and method in ("auto", "panel"):
        times = []
        for _ in range(2):   # first call: includes loading the kernels; second: the steady state
            torch.cuda.synchronize(comm.device)
            t0 = time.perf_counter()
            plan = plan_panels(A)
            torch.cuda.synchronize(comm.device)
            times.append((time.perf_counter() - t0) * 1e3)
        inspector_ms = times[1]
        inspector_first_ms = times[0]
    kernel_ms = {}
    if method == "auto":
        method = "panel" if plan is not None and cols % 128 == 0 and plan.reuse >= CONFIG.spmm_mfma_min_reuse else "rowwise"
        if comm.device.type == "cuda":
            # executor choice at inspection time: time every kernel that can
            # take this operand (one local SpMM each, warm, 10 calls) and keep
            # the fastest; all times are reported.  Panel reuse decides the
            # order (tools/probes/spmm_reuse.py: MFMA from reuse ~1.6 up, the
            # sweep / row kernels near 1), but the measured time decides.
            # Timed on the real X (the step's all-gathered operand): an
            # all-zero X would flatter kernels whose cost depends on the data.
            Xfull = allgather_rows(Xp, comm, counts)
            cands = (("panel",) if plan is not None and cols % 128 == 0 else ()) + ("rowwise",) + (
                ("sweep",) if cols == 128 and sweep_ok(A) else ()) + (("mfma",) if cols == 128 else ())
            for meth in cands:
                spmm(A, Xfull, method=meth, plan=plan)
                torch.cuda.synchronize(comm.device)
                t0 = time.perf_counter()
                for _ in range(10):
                    spmm(A, Xfull, method=meth, plan=plan)
                torch.cuda.synchronize(comm.device)
                kernel_ms[meth] = (time.perf_counter() - t0) * 1e3 / 10
            del Xfull
            # the slowest rank's view decides, so every rank runs the same kernel
            # (a kernel not available on some rank counts as infinitely slow there)
            worst = {k: comm.allreduce_max(kernel_ms.get(k, float("inf"))) for k in ("mfma", "panel", "rowwise", "sweep")}
            method = min(worst, key=worst.get)
    step = lambda: rowblock_spmm(A, Xp, comm, counts, plan=plan, method=method)  # noqa: E731
    if not comm.is_dist and comm.device.type == "cuda":
        # one GPU: the step is a single launch-bound SpMM -> replay it from a HIP graph
        graph = SpmmGraph(A, Xp, method=method, plan=plan)
        step = graph.run
    nnz_a = A.nnz
    if comm.is_dist:
        nnz_a = sum(comm.gather_ints(nnz_a))
    flops = 2 * nnz_a * cols
    kernel = {"mfma": "MFMA row-group kernel (v_mfma_f32_16x16x32_bf16)",
              "panel": "MFMA panel kernel (v_mfma_f32_16x16x32_bf16)", "sweep": "VALU row-owning sweep kernel",
              "rowwise": "VALU row-gather kernel"}[method]
    extra = dict(nnz_A=nnz_a, spmm_method=method, spmm_kernel=kernel,
                 panel_reuse=(plan.reuse if plan is not None else None),
                 inspector_ms=inspector_ms, inspector_first_ms=inspector_first_ms,
                 autotune_ms=kernel_ms or None, hip_graph=not comm.is_dist and comm.device.type == "cuda")
    cfg = dict(model=f"{n}x{n} CSR SpMM (sparse x dense {cols}-col) at {density * 100:g}% density, bf16, {kernel}",
               n=n, density=density, cols=cols, global_batch=1, seq_len=n, parallelism=f"rowblock{comm.world}")
    return step, flops, extra, cfg
