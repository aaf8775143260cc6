"""Distributed CSR SpGEMM: 1D row-block decomposition over RCCL / xGMI.

North-star config "1M x 1M CSR SpGEMM at 0.01 % density, 1D row-block over
8 x MI355X" (BASELINE.json).  The reference distributes a *chain* over MPI
ranks (sparse_matrix_mult.cu:437-456) and funnels partials to rank 0
(:466-571); it has no decomposition of a single product.  Here:

* rank r owns row panel r of A and of B (contiguous rows, chunk-aligned so the
  synthetic matrices do not depend on P);
* B's row panels are all-gathered (one ``all_gather_into_tensor`` per array,
  ring over the xGMI links — B is ~0.8 GB for the 1M config, small against
  288 GB of HBM, so replicating it is the right trade);
* each rank computes its C row panel = A_panel . B with the local gfx950
  SpGEMM; C stays distributed (no reduce needed: rows are disjoint).

``gather_rows`` reassembles a distributed CSR on one rank (tests, output).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops.csr import CSR
from ..ops.spgemm import SpgemmInfo, spgemm
from ..parallel.comm import Comm
from ..parallel.partition import row_panels
from ..utils.gen_csr import uniform_csr


def _allgather_equal(comm: Comm, t: torch.Tensor) -> torch.Tensor:
    """[world * t.numel()] gather of equally sized 1-D tensors, rank order."""
    if comm.backend == "nccl":
        out = torch.empty(comm.world * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous())
        return out
    parts = [torch.empty_like(t) for _ in range(comm.world)]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts)


def allgather_csr_rows(panel: CSR, comm: Comm) -> CSR:
    """Concatenate every rank's row panel (same column space) in rank order."""
    if not comm.is_dist:
        return panel
    wd = panel.device if comm.backend == "nccl" else torch.device("cpu")
    meta = _allgather_equal(comm, torch.tensor([panel.m, panel.nnz], dtype=torch.int64, device=wd)).view(-1, 2)
    ms, nnzs = meta[:, 0].tolist(), meta[:, 1].tolist()
    mmax, emax = max(ms), max(nnzs)
    cnt = torch.zeros(mmax, dtype=torch.int64, device=wd)
    cnt[:panel.m] = (panel.rowptr[1:] - panel.rowptr[:-1]).to(wd)
    col = torch.zeros(emax, dtype=panel.col.dtype, device=wd)
    col[:panel.nnz] = panel.col.to(wd)
    val = torch.zeros(emax, dtype=panel.val.dtype, device=wd)
    val[:panel.nnz] = panel.val.to(wd)
    g_cnt = _allgather_equal(comm, cnt).view(comm.world, mmax)
    g_col = _allgather_equal(comm, col).view(comm.world, emax)
    g_val = _allgather_equal(comm, val).view(comm.world, emax)
    if all(x == mmax for x in ms) and all(x == emax for x in nnzs):
        cnts, cols, vals = g_cnt.reshape(-1), g_col.reshape(-1), g_val.reshape(-1)
    else:
        cnts = torch.cat([g_cnt[r, :ms[r]] for r in range(comm.world)])
        cols = torch.cat([g_col[r, :nnzs[r]] for r in range(comm.world)])
        vals = torch.cat([g_val[r, :nnzs[r]] for r in range(comm.world)])
    m = sum(ms)
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=wd)
    torch.cumsum(cnts, 0, out=rowptr[1:])
    out = CSR(m, panel.n, rowptr, cols.contiguous(), vals.contiguous())
    return out.to(panel.device)


def gather_rows(panel: CSR, comm: Comm, dst: int = 0) -> Optional[CSR]:
    full = allgather_csr_rows(panel, comm)
    return full if comm.rank == dst else None


def allgather_operand(panel: CSR, comm: Comm) -> CSR:
    """Right operand of the row-block SpGEMM: every rank's B row panel, with ONE
    collective of the payload (instead of one per array).

    Each rank packs [row counts (int64 as 2 x int32) | columns | value bits]
    into one int32 buffer of a common size S; a single ``all_gather_into_tensor``
    (ring over the xGMI links) replicates it, then the panels' columns and
    values are packed back-to-back (two device copies, ~0.4 ms for the 1M
    config's 0.9 GB against a multi-ms collective) so row r ends where row r+1
    starts, as every CSR consumer expects.
    """
    if not comm.is_dist:
        return panel
    wd = panel.device if comm.backend == "nccl" else torch.device("cpu")
    meta = _allgather_equal(comm, torch.tensor([panel.m, panel.nnz], dtype=torch.int64, device=wd)).view(-1, 2)
    ms, nnzs = meta[:, 0].tolist(), meta[:, 1].tolist()
    mmax, emax = max(ms), max(nnzs)
    S = 2 * mmax + 2 * emax
    buf = torch.zeros(S, dtype=torch.int32, device=wd)
    buf[:2 * mmax].view(torch.int64)[:panel.m] = (panel.rowptr[1:] - panel.rowptr[:-1]).to(wd)
    buf[2 * mmax:2 * mmax + panel.nnz] = panel.col.to(wd)
    buf[2 * mmax + emax:2 * mmax + emax + panel.nnz] = panel.val.float().to(wd).view(torch.int32)
    G = _allgather_equal(comm, buf).to(panel.device)
    Gv = G.view(comm.world, S)
    cnt = Gv[:, :2 * mmax].contiguous().view(torch.int64)          # [world, mmax]
    W = range(comm.world)
    counts = cnt.reshape(-1) if all(x == mmax for x in ms) else torch.cat([cnt[r, :ms[r]] for r in W])
    col = torch.cat([Gv[r, 2 * mmax:2 * mmax + nnzs[r]] for r in W])
    val = torch.cat([Gv[r, 2 * mmax + emax:2 * mmax + emax + nnzs[r]] for r in W]).view(torch.float32)
    m = sum(ms)
    rowptr = torch.zeros(m + 1, dtype=torch.int64, device=G.device)
    torch.cumsum(counts, 0, out=rowptr[1:])
    return CSR(m, panel.n, rowptr, col, val)


def rowblock_spgemm(A_panel: CSR, B_panel: CSR, comm: Comm, info: Optional[SpgemmInfo] = None) -> CSR:
    """C_panel = A_panel . B, where B = rows of every rank's B_panel."""
    B = allgather_operand(B_panel, comm)
    return spgemm(A_panel, B, info)


@dataclass
class UniformProblem:
    """A, B uniform random n x n at ``density``; this rank's row panels."""

    n: int
    density: float
    seed: int
    rows: Tuple[int, int]
    A: CSR
    B: CSR

    @staticmethod
    def build(n: int, density: float, comm: Comm, seed: int = 1) -> "UniformProblem":
        # any split yields the same global matrices (the generator is chunk-seeded)
        panels = row_panels(n, comm.world)
        lo, hi = panels[comm.rank]
        A = uniform_csr(n, n, density, seed=seed, device=comm.device, rows=(lo, hi))
        B = uniform_csr(n, n, density, seed=seed + 1, device=comm.device, rows=(lo, hi))
        return UniformProblem(n, density, seed, (lo, hi), A, B)


def smoke(dev: torch.device) -> None:
    """Tiny SpGEMM on the GPU vs a dense fp32 PyTorch reference."""
    A = uniform_csr(300, 257, 0.05, seed=3, device=dev)
    B = uniform_csr(257, 311, 0.05, seed=4, device=dev)
    C = spgemm(A, B)
    ref = A.to_dense() @ B.to_dense()
    got = C.to_dense()
    assert C.is_sorted(), "SpGEMM output not column-sorted"
    err = (got - ref).abs().max().item()
    assert err < 1e-4, f"SpGEMM mismatch {err}"
    # structural: every reference non-zero present
    assert int(((ref != 0) & (got == 0)).sum()) == 0
