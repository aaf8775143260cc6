"""CSR SpGEMM: CPU (OpenMP) and GPU (gfx950 hash kernels) against a plain
PyTorch fp32 dense reference; generators; row-block distribution (gloo)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import spmm_amd  # noqa: F401
from spmm_amd.ops import csr as CS
from spmm_amd.ops import spgemm as SG
from spmm_amd.utils import gen_csr


def dense_ref(A, B):
    return A.to_dense().double() @ B.to_dense().double()


def check(C, A, B, tol=1e-4):
    ref = dense_ref(A, B)
    got = C.to_dense().double()
    assert C.is_sorted()
    assert torch.allclose(got, ref, atol=tol, rtol=1e-4), (got - ref).abs().max()
    # exact structure: C stores exactly the structural non-zeros of A.B
    pat = (A.to_dense() != 0).double() @ (B.to_dense() != 0).double()
    assert C.nnz == int((pat != 0).sum())


def test_coo_csr_roundtrip():
    r = torch.tensor([2, 0, 2, 1, 0])
    c = torch.tensor([1, 3, 1, 0, 0])
    v = torch.tensor([1.0, 2.0, 3.0, 4.0, 5.0])
    M = CS.from_coo(r, c, v, 3, 4)
    assert M.rowptr.tolist() == [0, 2, 3, 4]
    assert M.col.tolist() == [0, 3, 0, 1]
    assert M.val.tolist() == [5.0, 2.0, 4.0, 4.0]
    assert torch.equal(M.transpose().transpose().to_dense(), M.to_dense())


def test_uniform_generator_partition_independent():
    full = gen_csr.uniform_csr(1000, 500, 0.02, seed=5)
    top = gen_csr.uniform_csr(1000, 500, 0.02, seed=5, rows=(0, 400))
    bot = gen_csr.uniform_csr(1000, 500, 0.02, seed=5, rows=(400, 1000))
    assert torch.equal(full.to_dense()[:400], top.to_dense())
    assert torch.equal(full.to_dense()[400:], bot.to_dense())
    assert full.is_sorted()
    d = full.nnz / (1000 * 500)
    assert 0.015 < d < 0.025


def test_rmat_generator():
    M = gen_csr.rmat_csr(10, 8, seed=1)
    assert M.m == 1024 and M.is_sorted()
    deg = (M.rowptr[1:] - M.rowptr[:-1]).float()
    assert deg.max() > 4 * deg.mean()   # power-law: hubs exist


@pytest.mark.parametrize("m,k,n,d", [(1024, 1024, 1024, 0.01), (200, 300, 150, 0.05), (64, 64, 64, 0.3)])
def test_spgemm_cpu(m, k, n, d):
    A = gen_csr.uniform_csr(m, k, d, seed=1)
    B = gen_csr.uniform_csr(k, n, d, seed=2)
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, B, info)
    check(C, A, B)
    assert info.flops == 2 * int(SG.row_nprod(A, B).sum())


def test_spgemm_cpu_empty_rows():
    A = gen_csr.uniform_csr(50, 40, 0.0, seed=1)
    B = gen_csr.uniform_csr(40, 30, 0.2, seed=2)
    C = SG.spgemm(A, B)
    assert C.nnz == 0 and C.rowptr.shape[0] == 51


def _worker(rank, world, port, n, d, tmp):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from spmm_amd.models import spgemm as MS
    from spmm_amd.parallel import comm as CM

    comm = CM.init(backend="gloo", device="cpu", timeout_s=120)
    try:
        prob = MS.UniformProblem.build(n, d, comm, seed=7)
        Cp = MS.rowblock_spgemm(prob.A, prob.B, comm)
        C = MS.gather_rows(Cp, comm)
        if rank == 0:
            torch.save({"rp": C.rowptr, "col": C.col, "val": C.val}, os.path.join(tmp, "C.pt"))
    finally:
        comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_rowblock_spgemm_gloo(tmp_path, world):
    n, d = 600, 0.02
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_worker, args=(world, port, n, d, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(os.path.join(tmp_path, "C.pt"), weights_only=True)
    A = gen_csr.uniform_csr(n, n, d, seed=7)
    B = gen_csr.uniform_csr(n, n, d, seed=8)
    C = CS.CSR(n, n, got["rp"], got["col"], got["val"])
    check(C, A, B)


def test_col_slice_and_csr_sum():
    A = gen_csr.uniform_csr(90, 120, 0.08, seed=3)
    Ad = A.to_dense()
    for lo, hi in [(0, 40), (40, 120), (7, 8), (50, 50)]:
        P = A.col_slice(lo, hi)
        assert P.m == 90 and P.n == hi - lo and P.is_sorted()
        assert torch.equal(P.to_dense(), Ad[:, lo:hi])
    parts = [gen_csr.uniform_csr(90, 120, 0.05, seed=s) for s in range(5)] + [gen_csr.uniform_csr(90, 120, 0.0, seed=9)]
    C = SG.csr_sum(parts)
    ref = sum(p.to_dense() for p in parts)
    assert C.is_sorted() and torch.allclose(C.to_dense(), ref, atol=1e-6)
    assert C.nnz == int((ref != 0).sum())


def _inner_worker(rank, world, port, n, d, tmp):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from spmm_amd.models import spgemm as MS
    from spmm_amd.parallel import comm as CM
    from spmm_amd.parallel.partition import row_panels

    comm = CM.init(backend="gloo", device="cpu", timeout_s=120)
    try:
        prob = MS.UniformProblem.build(n, d, comm, seed=7)
        counts = [b - a for a, b in row_panels(n, world)]
        info = SG.SpgemmInfo()
        Cp = MS.innerdim_spgemm(prob.inner_operand(), prob.B, comm, counts, info)
        assert Cp.m == counts[rank] and Cp.is_sorted() and info.partial_nnz > 0
        C = MS.gather_rows(Cp, comm)
        if rank == 0:
            torch.save({"rp": C.rowptr, "col": C.col, "val": C.val}, os.path.join(tmp, "C.pt"))
    finally:
        comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_innerdim_spgemm_gloo(tmp_path, world):
    """Inner-dimension split (A column panel x B row panel per rank) + sparse
    reduce-scatter (all-to-all-v + SpGEMM-kernel merge) equals A . B."""
    n, d = 500, 0.03
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_inner_worker, args=(world, port, n, d, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(os.path.join(tmp_path, "C.pt"), weights_only=True)
    A = gen_csr.uniform_csr(n, n, d, seed=7)
    B = gen_csr.uniform_csr(n, n, d, seed=8)
    C = CS.CSR(n, n, got["rp"], got["col"], got["val"])
    check(C, A, B)


# ----------------------------------------------------------------- GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n,d", [(1024, 1024, 1024, 0.01), (3000, 2000, 2500, 0.004), (500, 400, 300, 0.1),
                                     (200, 3000, 5000, 0.03), (64, 64, 64, 0.5)])
def test_spgemm_gpu_vs_dense(m, k, n, d):
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, k, d, seed=11, device=dev)
    B = gen_csr.uniform_csr(k, n, d, seed=12, device=dev)
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, B, info)
    check(C, A, B)
    assert info.resorted_rows == 0


@pytest.mark.gpu
def test_spgemm_gpu_matches_cpu_structure_all_bins():
    """Row lengths spread over every LDS bin and the HBM (global) path."""
    dev = torch.device("cuda")
    # rows with very different product counts: dense-ish rows hit the global bins
    m, k, n = 700, 2000, 40000
    A = gen_csr.uniform_csr(m, k, 0.004, seed=1)
    # make a few heavy rows
    heavy = gen_csr.uniform_csr(6, k, 0.9, seed=2)
    rows = torch.cat([A.row_ids(), heavy.row_ids() + m])
    cols = torch.cat([A.col, heavy.col]).long()
    vals = torch.cat([A.val, heavy.val])
    A = CS.from_coo(rows, cols, vals, m + 6, k)
    B = gen_csr.uniform_csr(k, n, 0.01, seed=3)
    Cc = SG.spgemm(A, B)
    info = SG.SpgemmInfo()
    Cg = SG.spgemm(A.to(dev), B.to(dev), info)
    assert SG.SYM_GLOBAL in info.rows_per_bin_sym or SG.NUM_GLOBAL in info.rows_per_bin_num
    assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
    assert torch.equal(Cg.col.cpu(), Cc.col)
    assert torch.allclose(Cg.val.cpu(), Cc.val, atol=1e-3, rtol=1e-4)


@pytest.mark.gpu
def test_spgemm_gpu_rmat_aat():
    dev = torch.device("cuda")
    A = gen_csr.rmat_csr(12, 8, seed=2, device=dev)
    At = A.transpose()
    Cg = SG.spgemm(A, At)
    Cc = SG.spgemm(A.to("cpu"), At.to("cpu"))
    assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
    assert torch.equal(Cg.col.cpu(), Cc.col)
    assert torch.allclose(Cg.val.cpu(), Cc.val, atol=1e-3, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("brow,bcols", [(60, 200000), (100, 200000), (100, 40000)])
def test_spgemm_gpu_column_sliced_bins(monkeypatch, brow, bcols):
    """Rows long enough for the 2- and 4-slice LDS passes (and the overflow
    hand-off to the HBM path) must match the CPU result exactly in structure.
    (The bitmap path, which would take the uniform rows, is switched off.)"""
    from spmm_amd.utils.config import CONFIG

    monkeypatch.setattr(CONFIG, "spgemm_bitmap", "off")
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(300, 2000, 0.1, seed=5)
    B = gen_csr.uniform_csr(2000, bcols, brow / bcols, seed=6)
    Cc = SG.spgemm(A, B)
    info = SG.SpgemmInfo()
    Cg = SG.spgemm(A.to(dev), B.to(dev), info)
    assert any(b in info.rows_per_bin_sym for b in SG.SYM_SLICED) or any(b in info.rows_per_bin_num for b in SG.NUM_SLICED)
    assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
    assert torch.equal(Cg.col.cpu(), Cc.col)
    assert torch.allclose(Cg.val.cpu(), Cc.val, atol=1e-3, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n,d", [(3000, 2000, 2500, 0.004), (300, 2000, 40000, 0.05)])
def test_spgemm_gpu_onepass_matches_two_phase(monkeypatch, m, k, n, d):
    """One-pass (product-count staging + compaction) and symbolic+numeric give
    the same CSR."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, k, d, seed=21, device=dev)
    B = gen_csr.uniform_csr(k, n, d, seed=22, device=dev)
    monkeypatch.setattr(CONFIG, "spgemm_onepass", "on")
    C1 = SG.spgemm(A, B)
    monkeypatch.setattr(CONFIG, "spgemm_onepass", "off")
    C2 = SG.spgemm(A, B)
    assert torch.equal(C1.rowptr, C2.rowptr)
    assert torch.equal(C1.col, C2.col)
    assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    check(C1.to("cpu"), A.to("cpu"), B.to("cpu"))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform", "rmat"])
def test_spgemm_gpu_pipelined_onepass_matches_plain(monkeypatch, kind):
    """Row-chunked one-pass with the compaction overlapped on a side stream
    (forced to many small chunks) gives the same CSR as the plain one-pass;
    a matrix with hub rows (HBM long-row path) falls back to the plain path."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    if kind == "uniform":
        A = gen_csr.uniform_csr(40000, 40000, 2e-3, seed=31, device=dev)
        B = gen_csr.uniform_csr(40000, 40000, 2e-3, seed=32, device=dev)
    else:
        A = gen_csr.rmat_csr(13, 16, seed=33, device=dev)
        B = A.transpose()
    monkeypatch.setattr(CONFIG, "spgemm_onepass", "on")
    monkeypatch.setattr(SG, "PIPE_MIN_PRODUCTS", 1 << 20)
    monkeypatch.setattr(SG, "PIPE_CHUNK_PRODUCTS", 1 << 22)
    monkeypatch.setattr(CONFIG, "spgemm_pipeline", "on")
    C1 = SG.spgemm(A, B)
    monkeypatch.setattr(CONFIG, "spgemm_pipeline", "off")
    C2 = SG.spgemm(A, B)
    assert torch.equal(C1.rowptr, C2.rowptr)
    assert torch.equal(C1.col, C2.col)
    assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    if kind == "uniform":
        nz = C1.val.numel()
        assert nz == int(C1.rowptr[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", ["on", "off"])
def test_spgemm_gpu_long_rows_side_stream_equal(monkeypatch, onepass):
    """The long-row batches' accumulation on the side stream (beside the next
    batch's routing; several batches forced by a small scratch budget) gives
    the same CSR as the serialised flow, one-pass and two-phase."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    A = gen_csr.rmat_csr(13, 16, seed=35, device=dev)
    B = A.transpose()
    monkeypatch.setattr(CONFIG, "spgemm_onepass", onepass)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap", "off")
    monkeypatch.setattr(SG, "GLOBAL_WS_BYTES", 1 << 22)   # many small long-row batches
    out = []
    for side in (0, 1):
        monkeypatch.setattr(CONFIG, "spgemm_long_side", side)
        info = SG.SpgemmInfo()
        out.append((SG.spgemm(A, B, info), info))
    (C0, i0), (C1, i1) = out
    assert i0.rows_per_bin_num.get(SG.NUM_GLOBAL, 0) > 0   # hub rows took the long-row path
    assert torch.equal(C0.rowptr, C1.rowptr) and torch.equal(C0.col, C1.col)
    assert torch.allclose(C0.val, C1.val, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", ["on", "off"])
def test_streamed_spgemm_gpu_overlap_panels_equal(monkeypatch, pipeline):
    """Streamed panels with ``overlap=True`` (each panel's last compaction and
    long-row placement still running on the side stream when it is handed
    over; the consumer waits on its ``ready`` event) equal the panels of the
    serialised flow, hub rows included."""
    from spmm_amd.models import spgemm as MS
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    A = gen_csr.rmat_csr(13, 16, seed=33, device=dev)
    B = A.transpose()
    monkeypatch.setattr(CONFIG, "spgemm_onepass", "on")
    monkeypatch.setattr(CONFIG, "spgemm_pipeline", pipeline)   # (off: the plain one-pass, R-MAT 24's panels)
    monkeypatch.setattr(SG, "PIPE_MIN_PRODUCTS", 1 << 20)
    monkeypatch.setattr(SG, "PIPE_CHUNK_PRODUCTS", 1 << 22)
    budget = max(int(SG.row_nprod(A, B).sum()) // 4, 1 << 21)
    out = {}
    for overlap in (False, True):
        got = []

        def consume(lo, hi, C, got=got):
            got.append((lo, hi, getattr(C, "ready", None) is not None))
            SG.wait_ready(C)
            got.append((C.rowptr.clone(), C.col.clone(), C.val.clone()))

        MS.streamed_spgemm(A, B, consume, budget=budget, overlap=overlap)
        torch.cuda.synchronize()
        out[overlap] = got
    assert len(out[True]) == len(out[False]) >= 4
    assert any(g[2] for g in out[True][0::2]) and not any(g[2] for g in out[False][0::2])
    for (p1, c1), (p2, c2) in zip(zip(out[False][0::2], out[False][1::2]), zip(out[True][0::2], out[True][1::2])):
        assert p1[:2] == p2[:2]
        assert torch.equal(c1[0], c2[0]) and torch.equal(c1[1], c2[1])
        assert torch.allclose(c1[2], c2[2], atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", ["on", "off"])
def test_spgemm_gpu_long_rows_keep_cancelled_and_signed_zero_entries(monkeypatch, onepass):
    """Hub rows (HBM long-row path) whose products cancel exactly or are -0.0
    still store every structural entry: the long-row accumulator marks
    occupancy with a -0.0 sentinel, so a -0 product or an exact cancellation
    must not read as an empty slot."""
    from spmm_amd.utils.config import CONFIG

    k, n = 2000, 40000
    B0 = gen_csr.uniform_csr(k // 2, n, 0.01, seed=41)
    # B rows 2i and 2i+1 identical: A entries +1 / -1 on them cancel to exactly
    # 0 in any summation order (values are multiples of 1/8: every partial sum is exact)
    v0 = torch.round(B0.val * 8) / 8 + 0.125
    v0[::7] = -0.0
    rows = torch.cat([B0.row_ids() * 2, B0.row_ids() * 2 + 1])
    cols = torch.cat([B0.col, B0.col]).long()
    vals = torch.cat([v0, v0])
    B = CS.from_coo(rows, cols, vals, k, n, sum_duplicates=False)
    ar, ac, av = [], [], []
    for r in range(4):   # 4 hub rows over all of B: ~800k products each
        ar.append(torch.full((k,), r))
        ac.append(torch.arange(k))
        av.append(torch.where(torch.arange(k) % 2 == 0, 1.0, -1.0) if r % 2 == 0 else torch.rand(k) - 0.5)
    A = CS.from_coo(torch.cat(ar), torch.cat(ac), torch.cat(av), 4, k)
    Cc = SG.spgemm(A, B)
    monkeypatch.setattr(CONFIG, "spgemm_onepass", onepass)
    info = SG.SpgemmInfo()
    dev = torch.device("cuda")
    Cg = SG.spgemm(A.to(dev), B.to(dev), info)
    assert SG.NUM_GLOBAL in info.rows_per_bin_num
    pat = (A.to_dense() != 0).double() @ torch.sparse_coo_tensor(
        torch.stack([B.row_ids(), B.col.long()]), torch.ones(B.nnz, dtype=torch.float64), (k, n)).to_dense()
    assert Cg.nnz == int((pat != 0).sum()) == Cc.nnz
    assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
    assert torch.equal(Cg.col.cpu(), Cc.col)
    assert torch.allclose(Cg.val.cpu(), Cc.val, atol=1e-3, rtol=1e-4)
    assert int((Cg.val[:int(Cg.rowptr[1])] == 0).sum()) == int(Cg.rowptr[1])   # row 0 cancels exactly


@pytest.mark.gpu
def test_rowblock_spgemm_rccl_one_rank(monkeypatch):
    """The distributed SpGEMM path (count gather, async packed payload gather
    over RCCL, deferred operand) in a one-rank RCCL group equals the local
    product."""
    from spmm_amd.models import spgemm as MS
    from spmm_amd.parallel import comm as CM

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    for k, v in dict(SPMM_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                     WORLD_SIZE="1", LOCAL_RANK="0").items():
        monkeypatch.setenv(k, v)
    comm = CM.init(backend="nccl", device="cuda")
    try:
        assert comm.is_dist and comm.backend == "nccl"
        for n, d in ((50000, 4e-4), (65536, 1e-3)):
            prob = MS.UniformProblem.build(n, d, comm, seed=5)
            info = SG.SpgemmInfo()
            C1 = MS.rowblock_spgemm(prob.A, prob.B, comm, info)
            C2 = SG.spgemm(prob.A, prob.B)
            assert torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
            assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
        # the second one ran the bitmap kernels on the two-stage gather (columns
        # unpacked first for the count kernel, values + pairs before the numeric)
        assert "bitmap_units" in info.rows_per_bin_num
        # the host-sync-free step: RCCL gathers between two captured graphs,
        # replayed after in-place value changes of both operands; cfg 1 and cfg 0 on
        # the row kernel with more rows than its static schedule (row tickets: the
        # first graph's reset of the ticket / deferred words must hold on replay)
        for n, d in ((65536, 1e-3), (262144, 1e-4)):
            prob = MS.UniformProblem.build(n, d, comm, seed=7)
            g = MS.RowblockGraph(prob.A, prob.B, comm)
            assert g.gview is not None and g.plan.raw.rows
            va, vb = prob.A.val.clone(), prob.B.val.clone()
            for s in (1.0, -0.5, 2.0):
                prob.A.val.copy_(va * s)
                prob.B.val.copy_(vb * (s + 1.0))
                g.run()
                C1 = g.result()
                C2 = SG.spgemm(prob.A, prob.B)
                assert torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
                assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5), (n, s)
            torch.cuda.synchronize()
            del g
    finally:
        comm.close()


def test_streamed_spgemm_panels_concatenate_to_full_product():
    """C produced in product-bounded row panels (C never resident) equals the
    one-shot product, panel by panel, and every panel respects the budget
    unless it is a single row."""
    from spmm_amd.models import spgemm as MS

    A = gen_csr.rmat_csr(10, 8, seed=3)
    At = A.transpose()
    full = SG.spgemm(A, At)
    nprod = SG.row_nprod(A, At)
    budget = int(nprod.sum()) // 7
    panels = MS.stream_panels(nprod, budget)
    assert panels[0][0] == 0 and panels[-1][1] == A.m and len(panels) >= 7
    assert all(a[1] == b[0] for a, b in zip(panels, panels[1:]))
    assert all(int(nprod[lo:hi].sum()) <= budget or hi - lo == 1 for lo, hi in panels)
    got = []
    info = MS.streamed_spgemm(A, At, lambda lo, hi, C: got.append((lo, hi, C)), budget=budget)
    assert [(lo, hi) for lo, hi, _ in got] == panels
    assert info.nnz == full.nnz and info.flops == 2 * int(nprod.sum())
    for lo, hi, C in got:
        ref = full.row_slice(lo, hi)
        assert torch.equal(C.rowptr, ref.rowptr) and torch.equal(C.col, ref.col)
        assert torch.allclose(C.val, ref.val)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uniform1", "uniform2", "uniform4", "wide8", "skewed_fallback"])
def test_spgemm_gpu_ordered_onepass_matches_binned(monkeypatch, case):
    """Ordered one-pass (units in row order, final offsets from a decoupled
    look-back, no compaction) equals the binned path bit for bit in structure;
    rows of 1 / 2 / 4 / 8 ESC slices; a row whose products crowd one column
    eighth overflows its unit and falls back to the binned path."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    if case == "skewed_fallback":
        k, n = 3000, 80000
        A = gen_csr.uniform_csr(200, k, 0.05, seed=51, device=dev)
        B = gen_csr.uniform_csr(k, n // 8, 0.03, seed=52, device=dev)   # every column in the first eighth
        B = CS.CSR(k, n, B.rowptr, B.col, B.val)
    else:
        m, k, n, d = dict(uniform1=(3000, 8000, 8000, 0.012), uniform2=(2000, 10000, 20000, 0.011),
                          uniform4=(1500, 10000, 20000, 0.0095), wide8=(300, 20000, 20000, 0.01))[case]
        A = gen_csr.uniform_csr(m, k, d, seed=53, device=dev)
        B = gen_csr.uniform_csr(k, n, d, seed=54, device=dev)
    monkeypatch.setattr(CONFIG, "spgemm_onepass", "on")
    monkeypatch.setattr(CONFIG, "spgemm_ordered", "on")
    i1 = SG.SpgemmInfo()
    C1 = SG.spgemm(A, B, i1)
    monkeypatch.setattr(CONFIG, "spgemm_ordered", "off")
    C2 = SG.spgemm(A, B)
    if case == "skewed_fallback":
        assert i1.rows_per_bin_num.get("ordered_fallback") is None   # info reset by the fallback
    else:
        assert "ordered_units" in i1.rows_per_bin_num
    assert torch.equal(C1.rowptr, C2.rowptr)
    assert torch.equal(C1.col, C2.col)
    assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    assert C1.is_sorted()


@pytest.mark.gpu
def test_csr_sum_gpu_vs_dense():
    """Sparse sum of partials on the gfx950 SpGEMM kernels (selector-matrix
    product) vs a dense fp32 sum."""
    dev = torch.device("cuda", 0)
    parts = [gen_csr.uniform_csr(3000, 5000, 0.004 * (s + 1), seed=s, device=dev) for s in range(6)]
    C = SG.csr_sum(parts)
    ref = sum(p.to_dense() for p in parts)
    assert C.is_sorted()
    assert torch.allclose(C.to_dense(), ref, atol=1e-5)
    assert C.nnz == int((sum((p.to_dense() != 0).float() for p in parts) != 0).sum())


@pytest.mark.gpu
def test_innerdim_spgemm_rccl_one_rank(monkeypatch):
    """Inner-dimension SpGEMM through the RCCL all-to-all-v path (one-rank
    group) equals the local product."""
    from spmm_amd.models import spgemm as MS
    from spmm_amd.parallel import comm as CM

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    for k, v in dict(SPMM_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                     WORLD_SIZE="1", LOCAL_RANK="0").items():
        monkeypatch.setenv(k, v)
    comm = CM.init(backend="nccl", device="cuda")
    try:
        prob = MS.UniformProblem.build(40000, 5e-4, comm, seed=5)
        info = SG.SpgemmInfo()
        C1 = MS.innerdim_spgemm(prob.inner_operand(), prob.B, comm, [40000], info)
        C2 = SG.spgemm(prob.A, prob.B)
        assert info.flops > 0
        assert torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
        assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    finally:
        comm.close()


@pytest.mark.gpu
def test_csr_transpose_gpu_all_segment_classes():
    """gfx950 transpose (histogram, atomic scatter, wave / LDS bitonic and
    radix sorted segments) equals the CPU sort-based transpose, incl. a hub
    column longer than the LDS sort and R-MAT power-law columns."""
    dev = torch.device("cuda", 0)
    rows = torch.cat([torch.arange(6000), torch.arange(0, 6000, 37), torch.arange(100, 1900, 3), torch.arange(50)])
    cols = torch.cat([torch.full((6000,), 7), torch.full((163,), 11), torch.full((600,), 900), torch.arange(50) * 19])
    vals = torch.randn(rows.numel())
    hub = CS.from_coo(rows, cols, vals, 6000, 1000)
    for A in (hub, gen_csr.uniform_csr(3000, 2500, 0.01, seed=3), gen_csr.rmat_csr(14, 16, seed=2)):
        Tc = A.transpose()
        Tg = A.to(dev).transpose()
        assert Tg.m == A.n and Tg.n == A.m
        assert torch.equal(Tg.rowptr.cpu(), Tc.rowptr) and torch.equal(Tg.col.cpu(), Tc.col)
        assert torch.equal(Tg.val.cpu(), Tc.val)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,n,d", [(0, 10, 10, 0.1), (1, 50, 50, 0.2), (5000, 3000, 4000, 0.004),
                                     (700, 20000, 20000, 0.012)])
def test_spgemm_row_plan_matches_torch(m, k, n, d):
    """spgemm_row_plan + spgemm_plan_finish (one launch pair, one read-back)
    against the PyTorch computation it replaces: per-row product counts, the
    ordered unit counts, and the folded statistics; spgemm_ordered_units
    against repeat_interleave."""
    from spmm_amd import _native

    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, k, d, seed=61, device=dev)
    B = gen_csr.uniform_csr(k, n, d, seed=62, device=dev)
    nprod, nsl, st = SG.row_plan(A, B)
    ref = SG.row_nprod(A, B)
    assert torch.equal(nprod, ref)
    assert torch.equal(nsl, SG._ordered_slices(ref))
    tot, mx, nz, light, h1, h2, h4, h8, amax = st.tolist()[:9]
    assert tot == int(ref.sum()) and mx == (int(ref.max()) if m else 0)
    assert amax == (int((A.rowptr[1:] - A.rowptr[:-1]).max()) if m else 0)
    assert nz == int((ref > 0).sum()) and light == int(((ref > 0) & (ref <= SG.ESC_MIN)).sum())
    hist = torch.bincount(nsl.cpu(), minlength=9).tolist()
    assert [h1, h2, h4, h8] == [hist[1], hist[2], hist[4], hist[8]]
    if m == 0:
        return
    nunits = int(nsl.sum())
    unit_row = torch.empty(nunits, dtype=torch.int32, device=dev)
    unit_q = torch.empty(nunits, dtype=torch.uint8, device=dev)
    incl = torch.cumsum(nsl, 0)
    P = _native.ptr
    _native.check(_native.hip().spmm_spgemm_ordered_units(P(nsl), P(incl), m, P(unit_row), P(unit_q),
                                                          _native.stream_ptr(dev)), "spgemm_ordered_units")
    rows = torch.repeat_interleave(torch.arange(m, device=dev, dtype=torch.int32), nsl)
    assert torch.equal(unit_row, rows)
    kk = torch.arange(nunits, device=dev) - (incl - nsl)[rows.long()]
    s = nsl[rows.long()]
    assert torch.equal(unit_q, ((kk * 8 // s) | (((kk + 1) * 8 // s) << 4)).to(torch.uint8))


def test_free_mem_asks_allocator_only_when_needed(monkeypatch):
    """The dispatcher's free-memory check reads the caching allocator's
    statistics (slow) only when the driver's free figure alone is too small."""
    calls = []
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (1000, 4000))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda dev=None: calls.append("r") or 3000)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda dev=None: calls.append("a") or 1000)
    f = SG._FreeMem(torch.device("cpu"))
    assert f.fits(800) and not calls             # 800 <= 0.8 * 1000
    assert f.fits(2000) and calls == ["r", "a"]  # 2000 <= 0.8 * (1000 + 2000)
    assert not f.fits(2500) and calls == ["r", "a"]   # spare cached


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,d,empty", [(3000, 3000, 0.02, False), (70000, 70000, 0.0015, False),
                                         (2999, 1237, 0.01, True), (5001, 77777, 0.0004, True)])
def test_spgemm_row_splits_match_searchsorted(m, n, d, empty):
    """Eighth split points of every B row (8 lanes per row, one binary search
    per lane) against torch.searchsorted on each row; rectangular B whose
    column count is not a multiple of 8 (the floor in q * n / 8 matters) and
    with empty rows."""
    dev = torch.device("cuda")
    B = gen_csr.uniform_csr(m, n, d, seed=81)
    if empty:   # every 5th row empty, and the last one
        keep = (B.row_ids() % 5 != 0) & (B.row_ids() != m - 1)
        B = CS.from_coo(B.row_ids()[keep], B.col[keep].long(), B.val[keep], m, n)
        assert int((B.rowptr[1:] == B.rowptr[:-1]).sum()) >= m // 5
    B = B.to(dev)
    B = CS.CSR(B.m, B.n, B.rowptr, B.col, B.val)
    sp = SG._splits(B).view(B.m, 7).cpu()
    rp, col = B.rowptr.cpu(), B.col.cpu()
    bounds = torch.tensor([(q * B.n) >> 3 for q in range(1, 8)], dtype=torch.int32)
    for j in list(range(min(B.m, 300))) + [B.m - 1]:
        lo, hi = int(rp[j]), int(rp[j + 1])
        ref = lo + torch.searchsorted(col[lo:hi].contiguous(), bounds)
        assert torch.equal(sp[j], ref.to(torch.int64)), j


def _bitmap_vs_binned(monkeypatch, A, B, cfg):
    from spmm_amd.utils.config import CONFIG

    monkeypatch.setattr(CONFIG, "spgemm_bitmap", "on")
    monkeypatch.setattr(CONFIG, "spgemm_bitmap_cfg", cfg)
    i1 = SG.SpgemmInfo()
    C1 = SG.spgemm(A, B, i1)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap", "off")
    C2 = SG.spgemm(A, B)
    assert torch.equal(C1.rowptr, C2.rowptr)
    assert torch.equal(C1.col, C2.col)
    assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    assert C1.is_sorted()
    return i1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,m,k,n,da,db", [(0, 2000, 20000, 300000, 0.002, 2.7e-4),
                                             (1, 3000, 10000, 65536, 0.006, 0.001),
                                             (2, 2500, 9000, 200001, 0.006, 5e-4), (1, 700, 3000, 1000, 0.01, 0.01),
                                             (0, 500, 400, 50, 0.2, 0.2)])
def test_spgemm_gpu_bitmap_matches_binned(monkeypatch, cfg, m, k, n, da, db):
    """Bitmap-rank path (count kernel -> unit offsets -> numeric kernel) equals
    the binned path bit for bit in structure, for every window configuration,
    ragged last windows (n not a multiple of the window) and n below one
    window."""
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(m, k, da, seed=91, device=dev)
    B = gen_csr.uniform_csr(k, n, db, seed=92, device=dev)
    info = _bitmap_vs_binned(monkeypatch, A, B, cfg)
    assert info.rows_per_bin_num["bitmap_cfg"] == cfg and "bitmap_fallback" not in info.rows_per_bin_num


@pytest.mark.gpu
@pytest.mark.parametrize("n", [700000, 1 << 20, 300000])
def test_spgemm_gpu_bitmap_count_units(monkeypatch, n):
    """Row count kernel (units of 2 windows) over the padded column groups
    (16-byte column loads), the 1M config's window (cfg 0: 2^17): ragged last
    window (n = 700000: 6 windows, the last count unit partly past the end),
    exactly 8 windows, and 3 windows (an odd count: the last unit is one
    window)."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(3000, 20000, 0.004, seed=61, device=dev)
    B = gen_csr.uniform_csr(20000, n, 100.0 / n, seed=62, device=dev)
    info = _bitmap_vs_binned(monkeypatch, A, B, 0)
    assert info.rows_per_bin_num.get("bitmap_cfg") == 0 and info.rows_per_bin_num.get("bitmap_rows") == 1, \
        info.rows_per_bin_num


@pytest.mark.gpu
@pytest.mark.parametrize("rows,pad,pipe,cv", [("on", 1, 1, 1), ("on", 0, 1, 1), ("on", 1, 0, 1), ("off", 1, 1, 1),
                                          ("on", 1, 1, 0)])
def test_spgemm_gpu_bitmap_row_kernels(monkeypatch, rows, pad, pipe, cv):
    """The two numeric paths of the widest-window configuration on a product
    with 5 windows per row (ragged last window): the pipelined row kernels
    (B's pairs with every window segment padded to a 128-byte line) and the
    per-unit kernels, which take every product the row kernels cannot (no
    padded layout, SPMM_SPGEMM_BITMAP_PIPE=0, no (column, value) pairs, rows
    off); all equal the binned path."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(1500, 20000, 0.002, seed=95, device=dev)
    B = gen_csr.uniform_csr(20000, 600000, 1.4e-4, seed=96, device=dev)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap_rows", rows)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap_pad", pad)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap_pipe", pipe)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap_cv", cv)
    info = _bitmap_vs_binned(monkeypatch, A, B, 0)
    assert info.rows_per_bin_num.get("bitmap_rows", 0) == (1 if (rows, pad, pipe, cv) == ("on", 1, 1, 1) else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uniform", "empty_rows", "deferred", "tiny"])
def test_spgemm_gpu_bitmap_row_kernel_cases(monkeypatch, case):
    """Row count + row-major numeric kernels equal the binned path: 20000
    rows (many rows per workgroup), runs of empty rows (rows that never reach
    pass 1), units deferred to the reload kernel, and a 5-row product."""
    dev = torch.device("cuda")
    k, n = 20000, 600000
    if case == "deferred":
        k, n = 6000, 300000
        base = gen_csr.uniform_csr(1500, k, 0.01, seed=93)
        big = torch.arange(0, 1500, 97)   # rows of 250 entries: ~6.5k products per window > 2048 (fast capacity)
        r0, c0 = base.row_ids(), base.col.long()
        keep = torch.isin(r0, big, invert=True)
        rows = torch.cat([r0[keep], big.repeat_interleave(250)])
        cols = torch.cat([c0[keep], torch.cat([torch.randperm(k)[:250] for _ in range(big.numel())])])
        A = CS.from_coo(rows, cols, torch.rand(rows.numel()) - 0.5, 1500, k).to(dev)
        B = gen_csr.uniform_csr(k, n, 2e-4, seed=94, device=dev)
    elif case == "empty_rows":
        base = gen_csr.uniform_csr(6000, k, 0.002, seed=97)
        r0 = base.row_ids()
        keep = ((r0 // 300) % 3 != 1) & (r0 != 0) & (r0 != 5999)   # blocks of 300 empty rows, first/last empty
        A = CS.from_coo(r0[keep], base.col.long()[keep], base.val[keep], 6000, k).to(dev)
        B = gen_csr.uniform_csr(k, n, 1.4e-4, seed=98, device=dev)
    else:
        A = gen_csr.uniform_csr(5 if case == "tiny" else 20000, k, 0.002, seed=97, device=dev)
        B = gen_csr.uniform_csr(k, n, 1.4e-4, seed=98, device=dev)
    info = _bitmap_vs_binned(monkeypatch, A, B, 0)
    assert info.rows_per_bin_num.get("bitmap_rows", 0) == 1
    if case == "deferred":
        assert info.rows_per_bin_num["bitmap_deferred"] >= 16


@pytest.mark.gpu
@pytest.mark.parametrize("lazy", [1, 0])
def test_spgemm_gpu_bitmap_truncated_window_lengths(monkeypatch, lazy):
    """A B row with >= 65536 entries inside one window does not fit the row
    kernels' 16-bit window lengths (ws8, err bit 3).  Eager flow: the row
    count stands down and the per-unit kernels count; lazy flow (C at the
    product bound, one read-back): the numeric kernels stand down too and the
    product reruns eagerly.  Either way C equals the binned path (the long B
    row is never referenced by A, so no unit exceeds the reload budget)."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    k, n = 4000, 300000
    base = gen_csr.uniform_csr(k, n, 2e-4, seed=31)
    r0, c0 = base.row_ids(), base.col.long()
    keep = r0 != 17
    long_cols = torch.randperm(1 << 17)[:70000]
    rows = torch.cat([r0[keep], torch.full((70000,), 17)])
    cols = torch.cat([c0[keep], long_cols])
    B = CS.from_coo(rows, cols, torch.rand(rows.numel()) - 0.5, k, n).to(dev)
    A = gen_csr.uniform_csr(600, k, 0.01, seed=32)
    ka = A.col.long() != 17
    A = CS.from_coo(A.row_ids()[ka], A.col.long()[ka], A.val[ka], 600, k).to(dev)
    if lazy:   # the flow the captured graphs replay: numeric stands down too, the product reruns eagerly
        monkeypatch.setattr(CONFIG, "spgemm_bitmap", "on")
        monkeypatch.setattr(CONFIG, "spgemm_bitmap_cfg", 0)
        info = SG.SpgemmInfo()
        nprod, _, st = SG.row_plan(A, B)
        tot, mx, nz, light, h1, h2, h4, h8, amax = st.tolist()[:9]
        info.flops, info.mean_seg = 2 * tot, tot / max(A.nnz, 1)
        C1 = SG.onepass_bitmap(A, B, info, pre=dict(max=mx, nonempty=nz, light=light, amax=amax), lazy=True)
        monkeypatch.setattr(CONFIG, "spgemm_bitmap", "off")
        C2 = SG.spgemm(A, B)
        assert torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
        assert torch.allclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    else:
        info = _bitmap_vs_binned(monkeypatch, A, B, 0)
    assert "bitmap_units" in info.rows_per_bin_num


@pytest.mark.gpu
def test_spgemm_gpu_bitmap_deferred_units_and_fallback(monkeypatch):
    """Rows too long for the fast kernel (A rows > 256 entries, windows above
    its product capacity) are deferred to the reload kernel; a unit beyond the
    reload budget (> 12288 products in one window) sends the whole product to
    the binned path; empty rows give empty units."""
    dev = torch.device("cuda")
    k, n = 6000, 300000
    base = gen_csr.uniform_csr(1500, k, 0.01, seed=93)
    rows = [base.row_ids(), torch.full((400,), 3), torch.full((300,), 1000)]
    cols = [base.col.long(), torch.randperm(k)[:400], torch.randperm(k)[:300]]
    keep = (rows[0] != 3) & (rows[0] != 1000) & (rows[0] != 7)   # row 7 empty
    A = CS.from_coo(torch.cat([rows[0][keep]] + rows[1:]), torch.cat([cols[0][keep]] + cols[1:]),
                    torch.rand(int(keep.sum()) + 700) - 0.5, 1500, k).to(dev)
    B = gen_csr.uniform_csr(k, n, 2e-4, seed=94, device=dev)
    info = _bitmap_vs_binned(monkeypatch, A, B, 0)
    assert info.rows_per_bin_num["bitmap_deferred"] >= 6   # rows 3 and 1000 (> 256 entries) in their 3 windows
    # one window crowded beyond the reload capacity -> binned fallback
    Bc = gen_csr.uniform_csr(k, 1 << 17, 0.03, seed=95)
    Bc = CS.CSR(k, n, Bc.rowptr, Bc.col, Bc.val).to(dev)   # every column in window 0 of cfg 0
    Ac = CS.from_coo(torch.full((900,), 5), torch.randperm(k)[:900], torch.rand(900), 64, k).to(dev)
    info = _bitmap_vs_binned(monkeypatch, Ac, Bc, 0)
    assert info.rows_per_bin_num.get("bitmap_fallback") is None   # info reset by the fallback
    assert "bitmap_units" not in info.rows_per_bin_num


@pytest.mark.gpu
def test_spgemm_gpu_bitmap_count_descriptor_batches(monkeypatch):
    """A two-window count unit of more chunks than the pipelined count
    kernel's 768 descriptors: 256-entry A rows over B rows of exactly 65 or
    97 entries inside the first two windows (cfg 0, 8 windows; the mean
    segment gives 32-column chunks: 3 or 4 chunks per entry, ~800 per unit)
    while every window stays inside the reload kernel's 12288 products.
    The pipelined count kernel flags such a unit (err bit 6) and the product
    is recounted on the per-unit kernels, which take descriptors in batches;
    before, the chunks past the buffer were dropped and the numeric kernel
    raised on the short count."""
    dev = torch.device("cuda")
    k, n = 2000, 1 << 20
    g = torch.Generator().manual_seed(7)
    rows, cols = [], []
    for j in range(k):
        w0, w1 = (49, 48) if j % 8 == 0 else (33, 32)   # 97 or 65 columns in [0, 2^18)
        c = torch.cat([torch.randperm(1 << 17, generator=g)[:w0], (1 << 17) + torch.randperm(1 << 17, generator=g)[:w1]])
        rows.append(torch.full((c.numel(),), j))
        cols.append(c)
    rows, cols = torch.cat(rows), torch.cat(cols)
    B = CS.from_coo(rows, cols, torch.rand(rows.numel(), generator=g) - 0.5, k, n).to(dev)
    m = 48
    ar = torch.arange(m).repeat_interleave(256)
    ac = torch.cat([torch.randperm(k, generator=g)[:256] for _ in range(m)])
    A = CS.from_coo(ar, ac, torch.rand(ar.numel(), generator=g) - 0.5, m, k).to(dev)
    info = _bitmap_vs_binned(monkeypatch, A, B, 0)
    assert info.rows_per_bin_num.get("bitmap_cfg") == 0 and "bitmap_units" in info.rows_per_bin_num, \
        info.rows_per_bin_num
    assert info.rows_per_bin_num["bitmap_deferred"] >= m   # every row's first windows: the reload kernel


def sampled_rows_check(A, B, C, nrows: int, seed: int = 0) -> float:
    """Gustavson in fp64 on the CPU for ``nrows`` random rows of C = A.B:
    asserts the exact column structure of each row, returns the max value error
    relative to the sum of |products| of the entry (values in [-1, 1) cancel, so
    |ref| itself can be arbitrarily small: fp32 accumulation error is bounded by
    a few ulps of sum |a_ik b_kj|)."""
    g = torch.Generator().manual_seed(seed)
    rows = torch.randint(0, A.m, (nrows,), generator=g).unique()
    Arp, Aci, Av = A.rowptr.cpu(), A.col.cpu().long(), A.val.cpu().double()
    Brp, Bci, Bv = B.rowptr.cpu(), B.col.cpu().long(), B.val.cpu().double()
    Crp = C.rowptr.cpu()
    worst = 0.0
    for i in rows.tolist():
        s, e = int(Arp[i]), int(Arp[i + 1])
        js, avs = Aci[s:e], Av[s:e]
        lens = Brp[js + 1] - Brp[js]
        idx = torch.repeat_interleave(Brp[js], lens) + (torch.arange(int(lens.sum())) -
                                                         torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens))
        cols, prods = Bci[idx], Bv[idx] * torch.repeat_interleave(avs, lens)
        uc, inv = torch.unique(cols, return_inverse=True)
        ref = torch.zeros(uc.numel(), dtype=torch.float64).index_add_(0, inv, prods)
        mag = torch.zeros(uc.numel(), dtype=torch.float64).index_add_(0, inv, prods.abs())
        cs, ce = int(Crp[i]), int(Crp[i + 1])
        got_c = C.col[cs:ce].cpu().long()
        got_v = C.val[cs:ce].cpu().double()
        assert torch.equal(got_c, uc), f"row {i}: column structure differs"
        if uc.numel():
            worst = max(worst, float(((got_v - ref).abs() / (mag + 1e-30)).max()))
    return worst


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,ordered", [(65536, 1e-3, False), (65536, 1e-3, True), (1 << 20, 1e-4, False)])
def test_spgemm_bench_scale_sampled_rows(monkeypatch, n, d, ordered):
    """BASELINE configs 2 and 4 at full size, on the path the bench takes
    (bitmap-rank; ordered one-pass with ``ordered``): 4096 random rows against
    fp64 Gustavson on the CPU (structure exact, values to fp32 accumulation
    error), and the total nnz against the two-phase symbolic count."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(n, n, d, seed=1, device=dev)
    B = gen_csr.uniform_csr(n, n, d, seed=2, device=dev)
    if ordered:
        monkeypatch.setattr(CONFIG, "spgemm_bitmap", "off")
        monkeypatch.setattr(CONFIG, "spgemm_ordered", "on")
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, B, info)
    assert ("ordered_units" if ordered else "bitmap_units") in info.rows_per_bin_num
    assert C.rowptr[-1] == C.nnz == info.nnz
    err = sampled_rows_check(A, B, C, 4096)
    assert err < 1e-6, err
    row_nnz = SG.symbolic(A, B, SG.row_nprod(A, B), SG.SpgemmInfo())
    assert torch.equal((C.rowptr[1:] - C.rowptr[:-1]).to(torch.int32), row_nnz)


def _rmat_worker(rank, world, port, scale, ef, chunk, stream, tmp):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from spmm_amd.models import spgemm as MS
    from spmm_amd.parallel import comm as CM

    comm = CM.init(backend="gloo", device="cpu", timeout_s=120)
    try:
        prob = MS.RmatProblem.build(scale, ef, comm, seed=5, chunk=chunk)
        info = SG.SpgemmInfo()
        if stream:
            got = []
            MS.streamed_spgemm(prob.A, prob.right_operand(comm), lambda lo, hi, C: got.append(C), budget=3000,
                               info=info)
            Cp = got[0] if len(got) == 1 else CS.CSR(prob.A.m, prob.A.n, *_cat_panels(got))
        else:
            Cp = prob.step(comm, info)
        Ag = MS.gather_rows(prob.A, comm)
        Atg = MS.gather_rows(prob.At, comm)
        Cg = MS.gather_rows(Cp, comm)
        flops = torch.tensor([info.flops], dtype=torch.int64)
        if comm.is_dist:
            torch.distributed.all_reduce(flops)
        if rank == 0:
            torch.save({"A": (Ag.rowptr, Ag.col), "At": (Atg.rowptr, Atg.col), "C": (Cg.rowptr, Cg.col, Cg.val),
                        "flops": int(flops), "cuts": prob.cuts}, os.path.join(tmp, "rmat.pt"))
    finally:
        comm.close()


def _cat_panels(panels):
    rp = [torch.zeros(1, dtype=torch.int64)]
    base = 0
    for C in panels:
        rp.append(C.rowptr[1:] + base)
        base += C.nnz
    return torch.cat(rp), torch.cat([C.col for C in panels]), torch.cat([C.val for C in panels])


@pytest.mark.parametrize("world,stream", [(1, False), (4, False), (7, True), (8, False)])
def test_rmat_distributed_gloo(tmp_path, world, stream):
    """BASELINE config 5 the distributed way (chunked generation per rank,
    product-balanced panels, all-to-all-v row shuffle, all-to-all-v
    transpose, all-gathered A^T): at world 1, 4, 7 and 8 (7: streamed C
    panels, uneven panels) the gathered A, A^T and C = A.A^T equal the
    single-process product of the same graph, and the FLOPs summed over ranks
    are the same."""
    scale, ef, chunk = 9, 8, 256   # 16 edge chunks over the ranks
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_rmat_worker, args=(world, port, scale, ef, chunk, stream, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = torch.load(os.path.join(tmp_path, "rmat.pt"), weights_only=True)
    n = 1 << scale
    A = gen_csr.rmat_csr(scale, ef, seed=5, chunk=chunk)
    assert torch.equal(got["A"][0], A.rowptr) and torch.equal(got["A"][1], A.col)
    At = A.transpose()
    assert torch.equal(got["At"][0], At.rowptr) and torch.equal(got["At"][1], At.col)
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, At, info)
    assert got["flops"] == info.flops
    assert torch.equal(got["C"][0], C.rowptr) and torch.equal(got["C"][1], C.col)
    assert torch.allclose(got["C"][2], C.val)
    cuts = got["cuts"]
    assert len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == n and cuts == sorted(cuts)


@pytest.mark.gpu
def test_spgemm_gpu_rmat18_streamed_panels_match_resident():
    """R-MAT scale-18 A.A^T streamed in row panels (a budget that forces
    several panels, hub rows included) vs the resident product: every panel
    equals the same rows of C (structure exact, values to fp32 rounding:
    unit weights, so entries are exact integer counts)."""
    from spmm_amd.models import spgemm as MS

    dev = torch.device("cuda")
    A = gen_csr.rmat_csr(18, 16, seed=4, device=dev)
    At = A.transpose()
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, At, info)
    budget = info.flops // 2 // 6 + 1
    seen = []

    def consume(lo, hi, Cp):
        ref = C.row_slice(lo, hi)
        assert Cp.m == hi - lo and torch.equal(Cp.rowptr, ref.rowptr) and torch.equal(Cp.col, ref.col), (lo, hi)
        assert torch.equal(Cp.val, ref.val), (lo, hi)
        seen.append((lo, hi))

    sinfo = MS.streamed_spgemm(A, At, consume, budget=budget)
    assert len(seen) >= 4 and seen[0][0] == 0 and seen[-1][1] == A.m
    assert all(a[1] == b[0] for a, b in zip(seen, seen[1:]))
    assert sinfo.flops == info.flops and sinfo.nnz == info.nnz == C.nnz


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", ["on", "off"])
def test_spgemm_gpu_long_rows_wave_items(monkeypatch, onepass):
    """Hub rows spread over 256 column chunks: items of a few hundred
    products go to the wave-per-item kernel (long_rank), the heavy rows'
    items (> 1024 products) to long_dense, in the same product; duplicates
    within an item are summed and exact cancellations keep their entry."""
    from spmm_amd.utils.config import CONFIG

    k, n = 20000, 1 << 22
    B = gen_csr.uniform_csr(k, n, 16 / n, seed=51, values="small_int")
    rows, cols, vals = [], [], []
    g = torch.Generator().manual_seed(5)
    for r, na in enumerate([8000, 8000, 12000, 19000, 0, 9000]):   # ~128k .. ~300k products per hub row
        if na:
            rows.append(torch.full((na,), r))
            cols.append(torch.randperm(k, generator=g)[:na])
            vals.append(torch.randint(-2, 3, (na,), generator=g).float())
    light = gen_csr.uniform_csr(40, k, 0.002, seed=52)   # ordinary rows around them
    rows.append(light.row_ids() + 6)
    cols.append(light.col.long())
    vals.append(light.val)
    A = CS.from_coo(torch.cat(rows), torch.cat(cols), torch.cat(vals), 46, k)
    # one hub row made of two identical halves with opposite signs: exact 0 everywhere
    cancel = torch.randperm(k // 2, generator=g)[:5000]
    A2 = CS.from_coo(torch.cat([torch.cat(rows), torch.full((10000,), 46)]),
                     torch.cat([torch.cat(cols), cancel, cancel + k // 2]),
                     torch.cat([torch.cat(vals), torch.ones(5000), -torch.ones(5000)]), 47, k)
    Bc = CS.from_coo(torch.cat([B.row_ids(), (B.row_ids() + k // 2) % k]), torch.cat([B.col, B.col]).long(),
                     torch.cat([B.val, B.val]), k, n, sum_duplicates=True)
    for Am, Bm in ((A, B), (A2, Bc)):
        Cc = SG.spgemm(Am, Bm)
        monkeypatch.setattr(CONFIG, "spgemm_onepass", onepass)
        info = SG.SpgemmInfo()
        dev = torch.device("cuda")
        Cg = SG.spgemm(Am.to(dev), Bm.to(dev), info)
        assert SG.NUM_GLOBAL in info.rows_per_bin_num
        assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
        assert torch.equal(Cg.col.cpu(), Cc.col)
        assert torch.equal(Cg.val.cpu(), Cc.val)   # small integers: every order sums exactly


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", ["on", "off"])
def test_spgemm_gpu_long_rows_btab_histogram(monkeypatch, onepass):
    """B with hub rows (>= LONG_BTAB_MIN entries per column chunk) next to
    short rows: the routing histogram takes the hub rows' chunk counts from
    the chunk-offset table (long_btab) and the short rows from their
    columns; C is identical with the table on and off and matches the CPU
    product (small integers: exact in every summation order)."""
    from spmm_amd.ops import spgemm as OS
    from spmm_amd.utils.config import CONFIG

    k, n = 6000, (1 << 20) + 77                   # nch = 33 column chunks, a partial last one
    g = torch.Generator().manual_seed(11)
    rows, cols = [], []
    for r in range(k):
        ln = 3000 if r % 97 == 0 else (140 if r % 13 == 0 else 9)   # hub / near-threshold / short
        rows.append(torch.full((ln,), r))
        cols.append(torch.randperm(n, generator=g)[:ln])
    rr, cc = torch.cat(rows), torch.cat(cols)
    B = CS.from_coo(rr, cc, torch.randint(-3, 4, (rr.numel(),), generator=g).float(), k, n)
    ra, ca = [], []
    for r, na in enumerate([2500, 0, 4000, 1800, 3000]):
        ra.append(torch.full((na,), r))
        ca.append(torch.randperm(k, generator=g)[:na])
    ra, ca = torch.cat(ra), torch.cat(ca)
    A = CS.from_coo(ra, ca, torch.randint(-2, 3, (ra.numel(),), generator=g).float(), 5, k)
    Cc = SG.spgemm(A, B)
    dev = torch.device("cuda")
    Ad, Bd = A.to(dev), B.to(dev)
    lidx, btab = OS._long_btab(Bd, (n + (1 << OS._long_params()[0]) - 1) >> OS._long_params()[0])
    assert lidx is not None and int((lidx >= 0).sum()) == int(((B.rowptr[1:] - B.rowptr[:-1]) >= 4 * 33).sum())
    monkeypatch.setattr(CONFIG, "spgemm_onepass", onepass)
    for tab, direct in ((1, 1), (1, 0), (0, 0)):
        monkeypatch.setattr(CONFIG, "spgemm_long_btab", tab)
        monkeypatch.setattr(CONFIG, "spgemm_long_direct", direct)
        info = SG.SpgemmInfo()
        Cg = SG.spgemm(Ad, Bd, info)
        assert SG.NUM_GLOBAL in info.rows_per_bin_num
        assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
        assert torch.equal(Cg.col.cpu(), Cc.col)
        assert torch.equal(Cg.val.cpu(), Cc.val)


@pytest.mark.gpu
@pytest.mark.parametrize("onepass", ["on", "off"])
def test_spgemm_gpu_long_rows_direct_products(monkeypatch, onepass):
    """Direct long-row products: items of > 1024 products read their long B
    rows' chunk segments straight from B (long_dense), items of <= 1024
    products route them through the scratch with the short rows (long_rank,
    mode 0), rows without long B rows stay routed; hub rows with 0, 1 and many
    64-entry blocks of long entries.  C equals the CPU product exactly (small
    integers) and the run with the direct mode off."""
    from spmm_amd.utils.config import CONFIG

    k, n = 9000, (1 << 22) + 5                     # 129 column chunks, a partial last one
    g = torch.Generator().manual_seed(17)
    r_ = torch.arange(k)
    lens = torch.where(r_ % 50 == 0, 6000, torch.where(r_ % 7 == 0, 600, 12))   # hub / long (>= 4 * 129) / short
    rr = torch.repeat_interleave(r_, lens)
    cc = torch.randint(0, n, (rr.numel(),), generator=g)   # (rare repeats are summed)
    B = CS.from_coo(rr, cc, torch.randint(-3, 4, (rr.numel(),), generator=g).float(), k, n)
    ra, ca = [], []
    short = torch.tensor([r for r in range(k) if r % 7 and r % 50])
    for r, na in enumerate([4000, 500, 1500, 0, 800]):
        ra.append(torch.full((na,), r))
        ca.append(torch.randperm(k, generator=g)[:na])
    ra.append(torch.full((6000,), 5))                  # a hub row over short B rows only: no long entries
    ca.append(short[torch.randperm(short.numel(), generator=g)[:6000]])
    light = gen_csr.uniform_csr(30, k, 0.001, seed=18)
    ra.append(light.row_ids() + 6)
    ca.append(light.col.long())
    ra, ca = torch.cat(ra), torch.cat(ca)
    A = CS.from_coo(ra, ca, torch.randint(-2, 3, (ra.numel(),), generator=g).float(), 36, k)
    Cc = SG.spgemm(A, B)
    dev = torch.device("cuda")
    Ad, Bd = A.to(dev), B.to(dev)
    monkeypatch.setattr(CONFIG, "spgemm_onepass", onepass)
    outs = []
    for direct in (1, 0):
        monkeypatch.setattr(CONFIG, "spgemm_long_direct", direct)
        info = SG.SpgemmInfo()
        Cg = SG.spgemm(Ad, Bd, info)
        assert SG.NUM_GLOBAL in info.rows_per_bin_num
        assert torch.equal(Cg.rowptr.cpu(), Cc.rowptr)
        assert torch.equal(Cg.col.cpu(), Cc.col)
        assert torch.equal(Cg.val.cpu(), Cc.val)
        outs.append(Cg)
    # both modes' item sizes: long rows with items above and below 1024 products
    nprod = SG.row_nprod(Ad, Bd).cpu()
    assert int((nprod[:6] > 1024 * 129).sum()) >= 2 and int(((nprod[:6] > 60000) & (nprod[:6] < 1024 * 129)).sum()) >= 1


def test_streamed_spgemm_splits_panels_on_oom(monkeypatch):
    """A streamed panel that runs out of device memory is split in half and
    retried: consumers still get contiguous panels in row order and the
    product is unchanged."""
    from spmm_amd.models import spgemm as MS

    A = gen_csr.uniform_csr(300, 200, 0.05, seed=61)
    B = gen_csr.uniform_csr(200, 250, 0.05, seed=62)
    real = MS.spgemm

    def flaky(Ap, Bm, info=None, B_ready=None):
        if Ap.m > 37:
            raise torch.OutOfMemoryError("simulated")
        return real(Ap, Bm, info)

    monkeypatch.setattr(MS, "spgemm", flaky)
    got = []
    info = MS.streamed_spgemm(A, B, lambda lo, hi, C: got.append((lo, hi, C)), budget=10 ** 9)
    assert info.rows_per_bin_num["oom_splits"] >= 3
    assert got[0][0] == 0 and got[-1][1] == A.m and all(a[1] == b[0] for a, b in zip(got, got[1:]))
    assert all(hi - lo <= 37 for lo, hi, _ in got)
    ref = real(A, B)
    dense = torch.cat([C.to_dense() for _, _, C in got])
    assert torch.allclose(dense, ref.to_dense(), atol=1e-6)
    assert info.nnz == ref.nnz


@pytest.mark.gpu
def test_spgemm_gpu_oom_falls_back_to_two_phase(monkeypatch):
    """A one-pass mode that runs out of memory is redone by the two-phase
    symbolic + numeric path (exact allocation), with the same result."""
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(4000, 3000, 0.004, seed=63, device=dev)
    B = gen_csr.uniform_csr(3000, 200000, 0.0004, seed=64, device=dev)
    ref = SG.spgemm(A, B)

    def oom(*a, **k):
        raise torch.OutOfMemoryError("simulated")

    monkeypatch.setattr(SG, "onepass_bitmap", oom)
    monkeypatch.setattr(SG, "onepass_ordered", oom)
    monkeypatch.setattr(SG, "onepass", oom)
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, B, info)
    assert info.rows_per_bin_num.get("oom_fallback") == 1
    assert torch.equal(C.rowptr, ref.rowptr) and torch.equal(C.col, ref.col)
    assert torch.allclose(C.val, ref.val, atol=1e-5, rtol=1e-5)


def _rows_subset(A, rows):
    """CSR of the given rows of A (host)."""
    Arp, Aci, Av = A.rowptr.cpu(), A.col.cpu(), A.val.cpu()
    lens = Arp[rows + 1] - Arp[rows]
    idx = torch.repeat_interleave(Arp[rows], lens) + (torch.arange(int(lens.sum())) -
                                                       torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens))
    rp = torch.zeros(rows.numel() + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=rp[1:])
    return CS.CSR(rows.numel(), A.n, rp, Aci[idx], Av[idx])


def _digest(t: torch.Tensor) -> int:
    """Order-sensitive digest of a tensor's bits, chunked (C of the 1M product
    is 46 GB of values)."""
    bits = t.view(torch.int32)
    acc = 0
    step = 1 << 27
    for s in range(0, bits.numel(), step):
        x = bits[s:s + step].long()
        w = (torch.arange(s, s + x.numel(), device=x.device) % 1000003) + 1
        acc = (acc + int((x * w).sum())) & ((1 << 64) - 1)
    return acc


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["rows_cfg0", "rows_cfg1", "generic", "collide_fast", "collide_reload",
                                  "collide_cpu"])
def test_spgemm_gpu_deterministic_equals_cpu_order(monkeypatch, case):
    """Deterministic mode (SPMM_SPGEMM_DETERMINISTIC=1): the bitmap kernels sum
    every output in Gustavson order, so C equals the CPU engine's result value
    for value, and two runs are bitwise equal.  Cases: the row-major kernel
    (two window configurations), the per-unit kernel, heavy column collisions
    (the >= 3-product fix-up in the fast kernel, in the reload kernel, and its
    CPU fallback when even the reload list overflows)."""
    from spmm_amd.utils.config import CONFIG

    dev = torch.device("cuda")
    monkeypatch.setattr(CONFIG, "spgemm_deterministic", 1)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap", "on")
    cfg = {"rows_cfg1": 1}.get(case, 0)
    monkeypatch.setattr(CONFIG, "spgemm_bitmap_cfg", cfg)
    if case == "generic":
        monkeypatch.setattr(CONFIG, "spgemm_bitmap_rows", "off")
    if case in ("rows_cfg0", "generic"):
        A = gen_csr.uniform_csr(2000, 20000, 0.002, seed=191, device=dev)
        B = gen_csr.uniform_csr(20000, 300000, 2.7e-4, seed=192, device=dev)
    elif case == "rows_cfg1":
        A = gen_csr.uniform_csr(3000, 10000, 0.006, seed=193, device=dev)
        B = gen_csr.uniform_csr(10000, 65536, 0.001, seed=194, device=dev)
    elif case == "collide_fast":    # ~1500 products per row into 20000 columns: pairs and a few triples
        A = gen_csr.uniform_csr(1500, 4000, 0.01, seed=195, device=dev)
        B = gen_csr.uniform_csr(4000, 20000, 0.00075, seed=196, device=dev)
    elif case == "collide_reload":  # ~3000 products per row (> fast capacity) into 20000 columns
        A = gen_csr.uniform_csr(800, 4000, 0.05, seed=197, device=dev)
        B = gen_csr.uniform_csr(4000, 20000, 0.00075, seed=198, device=dev)
    else:                           # ~1500 products into 300 columns: beyond every fix-up list
        A = gen_csr.uniform_csr(300, 4000, 0.05, seed=199, device=dev)
        B = gen_csr.uniform_csr(4000, 300, 0.025, seed=200, device=dev)
    i1 = SG.SpgemmInfo()
    C1 = SG.spgemm(A, B, i1)
    C2 = SG.spgemm(A, B)
    assert i1.deterministic
    assert torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
    assert torch.equal(C1.val.view(torch.int32), C2.val.view(torch.int32))
    R = SG.spgemm(A.to("cpu"), B.to("cpu"))
    assert torch.equal(C1.rowptr.cpu(), R.rowptr) and torch.equal(C1.col.cpu(), R.col)
    assert torch.equal(C1.val.cpu(), R.val)   # (value equality: +0.0 == -0.0)
    bins = i1.rows_per_bin_num
    if case == "collide_cpu":
        assert bins.get("det_cpu_fallback") == 1
    else:
        assert "det_cpu_fallback" not in bins and bins.get("bitmap_cfg") == cfg
    if case == "collide_reload":
        assert bins.get("bitmap_deferred", 0) > 0


@pytest.mark.gpu
def test_spgemm_bench_scale_deterministic_bitwise(monkeypatch):
    """BASELINE config 4 (1M^2 @ 0.01 %, the headline product) in
    deterministic mode: two runs give bitwise-equal C, and 2048 sampled rows
    equal the CPU engine's sequential Gustavson sums value for value."""
    from spmm_amd.utils.config import CONFIG

    monkeypatch.setattr(CONFIG, "spgemm_deterministic", 1)
    dev = torch.device("cuda")
    n, d = 1 << 20, 1e-4
    A = gen_csr.uniform_csr(n, n, d, seed=1, device=dev)
    B = gen_csr.uniform_csr(n, n, d, seed=2, device=dev)
    info = SG.SpgemmInfo()
    C = SG.spgemm(A, B, info)
    assert info.deterministic and "bitmap_units" in info.rows_per_bin_num
    d1, dc1, rp1 = _digest(C.val), _digest(C.col), C.rowptr.clone()
    g = torch.Generator().manual_seed(3)
    rows = torch.randint(0, n, (2048,), generator=g).unique()
    R = SG.spgemm(_rows_subset(A, rows), B.to("cpu"))
    Crp = C.rowptr.cpu()
    for t, i in enumerate(rows.tolist()):
        cs, ce = int(Crp[i]), int(Crp[i + 1])
        rs, re = int(R.rowptr[t]), int(R.rowptr[t + 1])
        assert torch.equal(C.col[cs:ce].cpu(), R.col[rs:re]) and torch.equal(C.val[cs:ce].cpu(), R.val[rs:re]), i
    del C
    torch.cuda.empty_cache()
    C = SG.spgemm(A, B)
    assert torch.equal(C.rowptr, rp1) and _digest(C.col) == dc1 and _digest(C.val) == d1


@pytest.mark.gpu
@pytest.mark.parametrize("n,d", [(65536, 1e-3), (300000, 3e-4)])
def test_spgemm_graph_replay_matches_eager(n, d):
    """SpgemmGraph (the bitmap product captured into one HIP graph, no host
    sync inside, C at the product bound) gives the eager product on every
    replay, and reports the same nnz."""
    dev = torch.device("cuda")
    A = gen_csr.uniform_csr(n, n, d, seed=3, device=dev)
    B = gen_csr.uniform_csr(n, n, d, seed=4, device=dev)
    C1 = SG.spgemm(A, B)
    g = SG.SpgemmGraph(A, B)
    for _ in range(2):
        g.run()
        info = SG.SpgemmInfo()
        C2 = g.result(info)
        assert info.nnz == C1.nnz
        assert torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
        assert torch.allclose(C1.val, C2.val, atol=1e-6, rtol=1e-5)


@pytest.mark.gpu
def test_spgemm_graph_replay_after_value_change():
    """Values of B changed IN PLACE between replays: the next replay of the
    captured graph computes the product of the new values (the graph holds
    pointers, not a cached C), matching a fresh eager product."""
    dev = torch.device("cuda")
    n, d = 65536, 1e-3
    A = gen_csr.uniform_csr(n, n, d, seed=13, device=dev)
    B = gen_csr.uniform_csr(n, n, d, seed=14, device=dev)
    g = SG.SpgemmGraph(A, B)
    g.run()
    v0 = g.result().val.clone()   # (result() views the graph's own C buffers)
    gen = torch.Generator(device=dev).manual_seed(5)
    B.val.copy_(torch.rand(B.val.shape, generator=gen, device=dev) * 2 - 1)   # new values, same structure
    A.val.mul_(-0.5)
    g.run()
    C1 = g.result()
    ref = SG.spgemm(A, B)
    assert torch.equal(ref.rowptr, C1.rowptr) and torch.equal(ref.col, C1.col)
    assert torch.allclose(ref.val, C1.val, atol=1e-6, rtol=1e-5)
    assert not torch.allclose(v0, C1.val)   # the replay did recompute


@pytest.mark.gpu
def test_spgemm_graph_replay_structure_change():
    """B's column structure changed in place (same row lengths): every
    kernel of the product is in the graph, so the replay gives the new
    product.  A's rows changed so that the product exceeds the plan's C
    capacity: result() reports it (no C is returned) and nothing outside C
    is written -- a canary allocated next to the operands is intact and a
    later eager product is still exact."""
    dev = torch.device("cuda")
    n, d = 65536, 1e-3
    A = gen_csr.uniform_csr(n, n, d, seed=23, device=dev)
    B = gen_csr.uniform_csr(n, n, d, seed=24, device=dev)
    g = SG.SpgemmGraph(A, B)
    # (1) new B columns: shift every column by a row-dependent offset, re-sorted per row
    rows = torch.repeat_interleave(torch.arange(n, device=dev), B.rowptr[1:] - B.rowptr[:-1])
    newc = (B.col.long() + 7 * rows + 1) % n
    key = rows * n + newc
    order = torch.argsort(key)
    B.col.copy_(newc[order].to(B.col.dtype))
    B.val.copy_(B.val[order])
    g.run()
    C1 = g.result()
    ref = SG.spgemm(A, B)
    assert torch.equal(ref.rowptr, C1.rowptr) and torch.equal(ref.col, C1.col)
    assert torch.allclose(ref.val, C1.val, atol=1e-6, rtol=1e-5)
    # (2) B's entries moved into the first half of its rows (each about twice
    # as long) and A's columns folded onto those rows: about twice the
    # products the graph's C capacity was planned for
    canary = torch.full((1 << 20,), 7, dtype=torch.int32, device=dev)
    nnz_b, half = B.nnz, n // 2
    lens = torch.full((half,), nnz_b // half, dtype=torch.int64, device=dev)
    lens[: nnz_b - int(lens.sum())] += 1
    rp = torch.zeros(n + 1, dtype=B.rowptr.dtype, device=dev)
    rp[1:half + 1] = torch.cumsum(lens, 0).to(rp.dtype)
    rp[half + 1:] = nnz_b
    B.rowptr.copy_(rp)
    brow = torch.repeat_interleave(torch.arange(half, device=dev), lens)
    k = torch.arange(nnz_b, device=dev) - (rp[:-1].long())[brow]
    bcol = (k * 499 + brow * 7) % n   # distinct within a row (499 * k < n)
    order = torch.argsort(brow * n + bcol)
    B.col.copy_(bcol[order].to(B.col.dtype))
    A.col.copy_((A.col.long() % half).to(A.col.dtype))
    arows = torch.repeat_interleave(torch.arange(n, device=dev), A.rowptr[1:] - A.rowptr[:-1])
    order = torch.argsort(arows * n + A.col.long())
    A.col.copy_(A.col[order])
    A.val.copy_(A.val[order])
    assert int(SG.row_nprod(A, B).sum()) > g.plan.tot
    g.run()
    with pytest.raises(RuntimeError):
        g.result()
    torch.cuda.synchronize()
    assert int((canary != 7).sum()) == 0
    C3 = SG.spgemm(A, B)   # the device is still sound: a fresh eager product is exact
    assert C3.is_sorted()
    for r in torch.randint(0, n, (8,)).tolist():
        want = torch.zeros(n, dtype=torch.float64, device=dev)
        for e in range(int(A.rowptr[r]), int(A.rowptr[r + 1])):
            j, a = int(A.col[e]), float(A.val[e])
            lo, hi = int(B.rowptr[j]), int(B.rowptr[j + 1])
            want.index_add_(0, B.col[lo:hi].long(), a * B.val[lo:hi].double())
        got = torch.zeros(n, dtype=torch.float64, device=dev)
        lo, hi = int(C3.rowptr[r]), int(C3.rowptr[r + 1])
        got[C3.col[lo:hi].long()] = C3.val[lo:hi].double()
        assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), r


def test_bitmap_plan_defaults_match_native():
    """The bitmap planner is native (csr_bitmap_plan.hip, shared with the a4 engine); the
    Python knobs (utils/config.py) and the native engine's environment defaults agree, and
    the native plan of a 1M-like product picks the wide-window row kernels."""
    import ctypes as C

    from spmm_amd import _native
    from spmm_amd.ops import spgemm as SG

    env = SG._BmOpts()
    _native.hip().spmm_spgemm_bm_env_opts(C.byref(env))
    py = SG._bm_opts()
    for f, _ in SG._BmOpts._fields_:
        assert getattr(env, f) == getattr(py, f), f
    p = SG._BmPlan()
    m, n, annz = 1 << 20, 1 << 20, 104857600
    tot = 10_995_116_277
    assert _native.hip().spmm_spgemm_bm_make_plan(C.byref(py), m, annz, n, n, annz, tot, m, 140,
                                                   float(tot / annz), C.byref(p)) == 0
    assert p.cfg == 0 and p.nwin == 8 and p.rows and p.count_rows and p.pad_num and p.pad_cnt
    assert p.ws_bytes >= p.cap_bcv * 8 + p.cap_colp * 4
