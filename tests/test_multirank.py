"""Multi-rank (gloo, CPU) coverage of every 1D decomposition at world sizes
4, 7 and 8 with uneven and EMPTY panels: row-block SpGEMM
(B all-gathered), inner-dimension SpGEMM (sparse reduce-scatter of C),
row-block SpMM (X all-gathered), inner-dimension SpMM (reduce-scatter of Y).
Each world is one spawned job running all four; the parent checks the
gathered pieces against single-process products."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import spmm_amd  # noqa: F401
from spmm_amd.ops import csr as CS
from spmm_amd.ops import spgemm as SG
from spmm_amd.utils import gen_csr

M, K, N, D = 230, 190, 260, 8


def _cuts(total: int, world: int, seed: int):
    """Uneven panel boundaries with empty panels at rank 1 and the last rank."""
    g = torch.Generator().manual_seed(seed)
    w = torch.rand(world, generator=g) + 0.2
    w[1] = 0.0
    w[world - 1] = 0.0
    sizes = (w / w.sum() * total).floor().long()
    sizes[0] += total - int(sizes.sum())
    cuts = [0]
    for s in sizes.tolist():
        cuts.append(cuts[-1] + s)
    return cuts


def _operands():
    A = gen_csr.uniform_csr(M, K, 0.05, seed=11)
    B = gen_csr.uniform_csr(K, N, 0.05, seed=12)
    X = (torch.arange(K * D, dtype=torch.float32).view(K, D) % 5 - 2).to(torch.bfloat16)
    Ab = A.with_values((torch.round(A.val * 4) / 4).to(torch.bfloat16))
    return A, B, X, Ab


def _worker(rank, world, port, tmp):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from spmm_amd.models import spgemm as MS
    from spmm_amd.models import spmm as MM
    from spmm_amd.parallel import comm as CM

    comm = CM.init(backend="gloo", device="cpu", timeout_s=180)
    try:
        A, B, X, Ab = _operands()
        rc, kc = _cuts(M, world, 1), _cuts(K, world, 2)
        lo, hi = rc[rank], rc[rank + 1]
        klo, khi = kc[rank], kc[rank + 1]
        row_counts = [rc[r + 1] - rc[r] for r in range(world)]
        k_counts = [kc[r + 1] - kc[r] for r in range(world)]
        out = {}
        # row-block SpGEMM: A rows [lo, hi), B rows [klo, khi) all-gathered
        C1 = MS.rowblock_spgemm(A.row_slice(lo, hi), B.row_slice(klo, khi), comm)
        out["rb_spgemm"] = (C1.rowptr, C1.col, C1.val)
        # inner-dimension SpGEMM: A[:, klo:khi] x B[klo:khi, :], C reduce-scattered to row panels rc
        C2 = MS.innerdim_spgemm(A.col_slice(klo, khi), B.row_slice(klo, khi), comm, row_counts)
        out["in_spgemm"] = (C2.rowptr, C2.col, C2.val)
        # row-block SpMM: Ab rows [lo, hi), X rows [klo, khi) all-gathered
        out["rb_spmm"] = MM.rowblock_spmm(Ab.row_slice(lo, hi), X[klo:khi], comm, k_counts)
        # inner-dimension SpMM: Ab[:, klo:khi] x X[klo:khi], Y reduce-scattered to row panels rc
        out["in_spmm"] = MM.innerdim_spmm(MM.column_panel(Ab, klo, khi), X[klo:khi], comm, row_counts)
        torch.save(out, os.path.join(tmp, f"r{rank}.pt"))
    finally:
        comm.close()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stack_csr(parts, n):
    rps, cols, vals, base = [torch.zeros(1, dtype=torch.int64)], [], [], 0
    for rp, col, val in parts:
        rps.append(rp[1:] + base)
        base += int(rp[-1])
        cols.append(col)
        vals.append(val)
    rp = torch.cat(rps)
    return CS.CSR(rp.numel() - 1, n, rp, torch.cat(cols), torch.cat(vals))


@pytest.mark.parametrize("world", [4, 7, 8])
def test_all_decompositions_uneven_and_empty_panels(tmp_path, world):
    mp.start_processes(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    got = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    A, B, X, Ab = _operands()
    rc = _cuts(M, world, 1)
    assert rc[2] - rc[1] == 0 and rc[world] - rc[world - 1] == 0   # empty panels really exercised
    C = SG.spgemm(A, B)
    Cd = C.to_dense().double()
    for key in ("rb_spgemm", "in_spgemm"):
        parts = [g[key] for g in got]
        for r in range(world):
            assert parts[r][0].numel() - 1 == rc[r + 1] - rc[r], (key, r)
        S = _stack_csr(parts, N)
        assert S.is_sorted(), key
        assert torch.allclose(S.to_dense().double(), Cd, atol=1e-5), key
        if key == "rb_spgemm":   # same kernels, same order: identical structure
            assert torch.equal(S.rowptr, C.rowptr) and torch.equal(S.col, C.col)
    Y = Ab.to_dense(torch.float32) @ X.float()
    for key in ("rb_spmm", "in_spmm"):
        Yg = torch.cat([g[key] for g in got])
        assert Yg.shape == Y.shape and torch.allclose(Yg, Y, atol=1e-3), key
