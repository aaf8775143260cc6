"""SpMM: CPU / GPU (rowwise VALU and MFMA panel kernels) against a plain
PyTorch fp32 reference on the same bf16-rounded inputs; inspector invariants;
row-block (all-gather) and inner-dimension (reduce-scatter) decompositions."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import spmm_amd  # noqa: F401
from spmm_amd.ops import csr as CS
from spmm_amd.ops import spmm as SM
from spmm_amd.utils import gen_csr


def ref(A, X):
    return A.to_dense(torch.float32) @ X.float()


def test_spmm_cpu():
    A = gen_csr.uniform_csr(300, 200, 0.05, seed=1, dtype=torch.bfloat16)
    X = torch.randn(200, 64).to(torch.bfloat16)
    Y = SM.spmm(A, X)
    assert torch.allclose(Y, ref(A, X), atol=1e-4, rtol=1e-4)


def test_plan_panels_invariants():
    A = gen_csr.uniform_csr(200, 500, 0.05, seed=2, dtype=torch.bfloat16)
    P = SM.plan_panels(A)
    assert P.nnz == A.nnz
    assert int(P.chunk_ent_ptr[-1]) == A.nnz
    # reconstruct A from the plan
    dense = torch.zeros(A.m, A.n)
    cc = P.chunk_cols
    npan = P.panel_chunk_ptr.numel() - 1
    for p in range(npan):
        for ch in range(int(P.panel_chunk_ptr[p]), int(P.panel_chunk_ptr[p + 1])):
            for e in range(int(P.chunk_ent_ptr[ch]), int(P.chunk_ent_ptr[ch + 1])):
                rc = int(P.ent_rc[e])
                row = p * 64 + rc // 64
                col = int(cc[ch * 64 + rc % 64])
                dense[row, col] += float(P.ent_val[e])
    assert torch.equal(dense, A.to_dense())
    assert P.union_cols <= A.nnz


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from spmm_amd.models import spmm as MM
    from spmm_amd.parallel import comm as CM
    from spmm_amd.parallel.partition import row_panels

    comm = CM.init(backend="gloo", device="cpu", timeout_s=120)
    try:
        m, n, D = 150, 130, 16
        A = gen_csr.uniform_csr(m, n, 0.08, seed=5, dtype=torch.bfloat16)
        X = (torch.arange(n * D, dtype=torch.float32).view(n, D) % 7 - 3).to(torch.bfloat16)
        rp = row_panels(m, world)
        xp = row_panels(n, world)
        lo, hi = rp[rank]
        xlo, xhi = xp[rank]
        Y1 = MM.rowblock_spmm(A.row_slice(lo, hi), X[xlo:xhi], comm, [b - a for a, b in xp])
        Acol = MM.column_panel(A, xlo, xhi)
        Y2 = MM.innerdim_spmm(Acol, X[xlo:xhi], comm, [b - a for a, b in rp])
        torch.save({"y1": Y1, "y2": Y2}, os.path.join(tmp, f"y{rank}.pt"))
    finally:
        comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_spmm_gloo(tmp_path, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    m, n, D = 150, 130, 16
    A = gen_csr.uniform_csr(m, n, 0.08, seed=5, dtype=torch.bfloat16)
    X = (torch.arange(n * D, dtype=torch.float32).view(n, D) % 7 - 3).to(torch.bfloat16)
    want = ref(A, X)
    parts = [torch.load(os.path.join(tmp_path, f"y{r}.pt"), weights_only=True) for r in range(world)]
    assert torch.allclose(torch.cat([p["y1"] for p in parts]), want, atol=1e-4)
    assert torch.allclose(torch.cat([p["y2"] for p in parts]), want, atol=1e-4)


# ----------------------------------------------------------------- GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("method", ["rowwise", "mfma", "panel"])
@pytest.mark.parametrize("m,n,D,d", [(1000, 800, 128, 0.02), (333, 4096, 256, 0.01), (64, 64, 128, 0.5),
                                     (4097, 300, 128, 0.05)])
def test_spmm_gpu(method, m, n, D, d):
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, n, d, seed=3, device=dev, dtype=torch.bfloat16)
    X = torch.randn(n, D, device=dev).to(torch.bfloat16)
    Y = SM.spmm(A, X, method=method)
    R = ref(A, X)
    assert torch.allclose(Y, R, atol=2e-3, rtol=2e-3), (Y - R).abs().max()
    Yb = SM.spmm(A, X, method=method, out_dtype=torch.bfloat16)
    assert torch.allclose(Yb.float(), R, atol=3e-2, rtol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["mfma", "panel"])
@pytest.mark.parametrize("m,n,d", [(130, 200, 0.1), (4099, 3000, 0.02), (40, 100, 0.0), (17, 64, 1.0),
                                   (48, 4096, 0.025)])
def test_spmm_mfma_exact_small_integers(method, m, n, d):
    """Exact integer data catches any fragment-layout / transpose mistake:
    row groups past m, empty rows / matrix, rows longer than a chunk, chunks
    straddling rows (row-group kernel; 48 x 4096 @ 2.5 %: ~1600 entries per
    16 rows), fp32 and bf16 outputs."""
    dev = torch.device("cuda")
    D = 128
    A = gen_csr.uniform_csr(m, n, d, seed=9, device=dev, values="small_int", dtype=torch.bfloat16)
    X = (torch.arange(n * D, device=dev).view(n, D) % 11 - 5).to(torch.bfloat16)
    R = ref(A, X)
    assert torch.equal(SM.spmm(A, X, method=method), R)
    assert torch.equal(SM.spmm(A, X, method=method, out_dtype=torch.bfloat16).float(), R.to(torch.bfloat16).float())


@pytest.mark.gpu
def test_spmm_mfma_row_kernel_segments():
    """The row-group kernel on rows whose entries all sit in one half of the
    columns, empty rows between them, rows crossing the middle, and the same
    matrix with its columns NOT sorted inside the rows (CSR allows it): exact
    on integers."""
    dev = torch.device("cuda")
    m, n, D = 37, 1000, 128
    g = torch.Generator().manual_seed(11)
    rows, cols = [], []
    for r in range(m):
        kind = r % 4
        if kind == 3:
            continue   # empty row
        lo, hi = {0: (0, 512), 1: (512, 1000), 2: (400, 700)}[kind]
        c = torch.randperm(hi - lo, generator=g)[:min(40, hi - lo)] + lo
        rows.append(torch.full((c.numel(),), r))
        cols.append(c)
    rows, cols = torch.cat(rows), torch.cat(cols)
    vals = torch.randint(-3, 4, (rows.numel(),), generator=g).float()
    A = CS.from_coo(rows, cols, vals, m, n).to(dev)
    A = CS.CSR(A.m, A.n, A.rowptr, A.col, A.val.to(torch.bfloat16))
    X = (torch.arange(n * D, device=dev).view(n, D) % 11 - 5).to(torch.bfloat16)
    assert torch.equal(SM.spmm(A, X, method="mfma"), ref(A, X))
    # columns NOT sorted inside the rows
    perm = torch.cat([torch.randperm(int(b - a), generator=g) + int(a)
                      for a, b in zip(A.rowptr[:-1].tolist(), A.rowptr[1:].tolist())]).to(dev)
    U = CS.CSR(A.m, A.n, A.rowptr, A.col[perm].contiguous(), A.val[perm].contiguous())
    assert torch.equal(SM.spmm(U, X, method="mfma"), ref(A, X))


@pytest.mark.gpu
@pytest.mark.parametrize("D", [128, 256, 72, 130])
def test_spmm_rowwise_exact_small_integers(D):
    """Row kernels (16-byte gathers when D % 8 == 0, incl. a partial 128-column
    block at D = 72; 4-byte gathers at D = 130) on exact integer data: rows of
    0 .. ~150 entries (several 64-entry rounds), a row count that leaves the
    last wave partly empty, both output types."""
    dev = torch.device("cuda")
    m, n = 301, 2000
    A = gen_csr.uniform_csr(m, n, 0.05, seed=19, values="small_int")
    keep = (A.row_ids() % 7) != 3                       # every 7th row empty
    A = CS.from_coo(A.row_ids()[keep], A.col[keep].long(), A.val[keep].float(), m, n)
    A = A.with_values(A.val.to(torch.bfloat16)).to(dev)
    X = (torch.arange(n * D, device=dev).view(n, D) % 13 - 6).to(torch.bfloat16)
    R = ref(A, X)
    assert torch.equal(SM.spmm(A, X, method="rowwise"), R)
    assert torch.equal(SM.spmm(A, X, method="rowwise", out_dtype=torch.bfloat16).float(), R.to(torch.bfloat16).float())


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,d", [(301, 2000, 0.05), (65536, 65536, 1e-3), (7, 100000, 0.01), (20000, 1000, 0.02)])
def test_spmm_sweep_exact_small_integers(m, n, d):
    """Row-owning sweep kernel on exact integer data: empty rows, a row
    count that leaves waves with fewer rows than their 16, the bench operand
    (16 rows per wave), a ragged last column slice (n = 100000), few columns;
    both output types equal the fp32 reference bit for bit."""
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, n, d, seed=23, values="small_int")
    keep = (A.row_ids() % 7) != 3                       # every 7th row empty
    A = CS.from_coo(A.row_ids()[keep], A.col[keep].long(), A.val[keep].float(), m, n)
    A = A.with_values(A.val.to(torch.bfloat16)).to(dev)
    assert SM.sweep_ok(A)
    X = (torch.arange(n * 128, device=dev).view(n, 128) % 13 - 6).to(torch.bfloat16)
    R = ref(A, X)
    assert torch.equal(SM.spmm(A, X, method="sweep"), R)
    assert torch.equal(SM.spmm(A, X, method="sweep", out_dtype=torch.bfloat16).float(), R.to(torch.bfloat16).float())


@pytest.mark.gpu
def test_spmm_sweep_refuses_what_it_cannot_stage():
    """sweep_ok: rows whose entries overflow a wave's LDS stage (here every
    row has 2000 entries) or more rows than the resident grid holds at 16 per
    wave are refused, so the autotuner never offers the kernel for them."""
    dev = torch.device("cuda")
    dense_rows = gen_csr.uniform_csr(64, 4000, 0.5, seed=1, device=dev, dtype=torch.bfloat16)
    assert not SM.sweep_ok(dense_rows)
    tall = gen_csr.uniform_csr(1 << 21, 64, 0.01, seed=2, device=dev, dtype=torch.bfloat16)
    assert not SM.sweep_ok(tall)
    with pytest.raises(ValueError):
        SM.spmm(dense_rows, torch.zeros(4000, 128, device=dev, dtype=torch.bfloat16), method="sweep")


@pytest.mark.gpu
def test_spmm_graph_replay_matches_eager():
    """The HIP-graph replay of the SpMM step gives the eager result, also after
    new operands are copied into the static input."""
    from spmm_amd.ops.spmm import SpmmGraph, plan_panels, spmm

    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(3000, 2500, 0.01, seed=41, device=dev, dtype=torch.bfloat16)
    X = (torch.rand((2500, 128), device=dev) * 2 - 1).to(torch.bfloat16)
    plan = plan_panels(A)
    for method in ("panel", "mfma"):
        g = SpmmGraph(A, X, method=method, plan=plan)
        assert torch.equal(g.run(), spmm(A, X, method=method, plan=plan))
        X2 = (torch.rand((2500, 128), device=dev) * 2 - 1).to(torch.bfloat16)
        g.X.copy_(X2)
        assert torch.equal(g.run(), spmm(A, X2, method=method, plan=plan))


def _plan_chunks(P):
    """(panel_chunk_ptr, chunk_cols, chunk_ent_ptr, per-chunk sorted (rc, val) lists) on the host."""
    cep = P.chunk_ent_ptr.cpu()
    rc, val = P.ent_rc.cpu(), P.ent_val.cpu().float()
    per = []
    for ch in range(cep.numel() - 1):
        s, e = int(cep[ch]), int(cep[ch + 1])
        k, o = torch.sort(rc[s:e])
        per.append((k, val[s:e][o]))
    return P.panel_chunk_ptr.cpu(), P.chunk_cols.cpu(), cep, per


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,d,dt", [(65536, 65536, 1e-3, torch.bfloat16), (1000, 300000, 2e-4, torch.float32),
                                      (777, 5000, 0.02, torch.bfloat16), (64, 70000, 0.01, torch.bfloat16)])
def test_plan_panels_device_kernel_matches_torch(m, n, d, dt):
    """The HIP inspector (count + fill kernels, column windows of 2^16, empty
    panels, fp32 or bf16 values) builds the torch inspector's plan: same
    chunk layout and columns, same entries per chunk (the order inside a
    chunk is free)."""
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, n, d, seed=7, device=dev, dtype=dt)
    Pk = SM.plan_panels(A)
    Pt = SM.plan_panels(A, device_kernel=False)
    a, b = _plan_chunks(Pk), _plan_chunks(Pt)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert all(torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) for x, y in zip(a[3], b[3]))
    assert Pk.union_cols == Pt.union_cols and Pk.nnz == Pt.nnz


@pytest.mark.gpu
@pytest.mark.parametrize("db", ["0", "1"])
def test_spmm_mfma_kernels_match_reference(monkeypatch, db):
    """Single-buffered and double-buffered MFMA panel kernels (SPMM_SPMM_MFMA_DB,
    read once per process: run in a subprocess) equal the fp32 reference, incl.
    a chunk with more than 512 entries (dense panel columns)."""
    import subprocess
    import sys

    code = """
import torch, spmm_amd
from spmm_amd.ops import spmm as SM
from spmm_amd.utils import gen_csr
dev = torch.device("cuda")
for (m, n, d) in [(4096, 3000, 0.01), (300, 200, 0.9), (70, 65, 1.0)]:
    A = gen_csr.uniform_csr(m, n, d, seed=3, device=dev, dtype=torch.bfloat16)
    X = (torch.randn(n, 256, device=dev) * 0.5).to(torch.bfloat16)
    Y = SM.spmm(A, X, method="panel")
    R = A.to_dense(torch.float32) @ X.float()
    err = float((Y - R).abs().max()) / max(1.0, float(R.abs().max()))
    assert err < 1e-3, (m, n, d, err)
print("ok")
"""
    env = dict(os.environ, SPMM_SPMM_MFMA_DB=db,
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]
