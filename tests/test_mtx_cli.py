"""Matrix Market I/O and the spgemm CLI (north-star plumbing config:
1024 x 1024 CSR x CSR at 1 % density on CPU/OpenMP, single process)."""
import json
import os
import subprocess
import sys

import pytest
import torch

import spmm_amd  # noqa: F401
from spmm_amd.ops import csr as CS
from spmm_amd.utils import gen_csr, mtx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mtx_roundtrip(tmp_path):
    A = gen_csr.uniform_csr(120, 90, 0.05, seed=1)
    p = str(tmp_path / "a.mtx")
    mtx.write_mtx(p, A)
    B = mtx.read_mtx(p)
    assert torch.equal(A.rowptr, B.rowptr) and torch.equal(A.col, B.col)
    assert torch.equal(A.val, B.val)   # shortest round-trip float text is exact


def test_mtx_symmetric_pattern_and_duplicates(tmp_path):
    p = tmp_path / "s.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real symmetric\n% c\n3 3 4\n1 1 2.0\n2 1 -1.5\n3 2 4\n3 2 1\n")
    M = mtx.read_mtx(str(p))
    d = M.to_dense()
    want = torch.tensor([[2.0, -1.5, 0], [-1.5, 0, 5.0], [0, 5.0, 0]])
    assert torch.equal(d, want)
    q = tmp_path / "p.mtx"
    q.write_text("%%MatrixMarket matrix coordinate pattern general\n2 3 2\n1 3\n2 1\n")
    P = mtx.read_mtx(str(q))
    assert P.to_dense().tolist() == [[0, 0, 1], [1, 0, 0]]
    with pytest.raises(mtx.MtxError):
        bad = tmp_path / "b.mtx"
        bad.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
        mtx.read_mtx(str(bad))


def test_spgemm_cli_plumbing_config(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    a = str(tmp_path / "A.mtx")
    b = str(tmp_path / "B.mtx")
    c = str(tmp_path / "C.mtx")
    for path, seed in ((a, 1), (b, 2)):
        r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.spgemm", "gen", "uniform", "--n", "1024",
                            "--density", "0.01", "--seed", str(seed), "--device", "cpu", "-o", path],
                           env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
    r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.spgemm", "mult", a, b, "-o", c, "--device", "cpu"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    A, B, C = mtx.read_mtx(a), mtx.read_mtx(b), mtx.read_mtx(c)
    ref = A.to_dense().double() @ B.to_dense().double()
    assert torch.allclose(C.to_dense().double(), ref, atol=1e-5)
    assert rec["flops"] > 0 and rec["nnz_C"] == C.nnz


def _shuffled_mtx(path, M, seed, symmetric=False):
    """Write M as a coordinate file with its entries in random line order
    (symmetric: the lower triangle of M + M^T with symmetric storage)."""
    r, c, v = M.row_ids(), M.col.long(), M.val.double()
    if symmetric:
        keep = r >= c
        r, c, v = r[keep], c[keep], v[keep]
    p = torch.randperm(r.numel(), generator=torch.Generator().manual_seed(seed))
    kind = "symmetric" if symmetric else "general"
    lines = [f"%%MatrixMarket matrix coordinate real {kind}", f"{M.m} {M.n} {r.numel()}"]
    lines += [f"{int(r[i]) + 1} {int(c[i]) + 1} {float(v[i])!r}" for i in p.tolist()]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


@pytest.mark.parametrize("mode", ["ab", "aat", "sym"])
def test_spgemm_cli_four_ranks_byte_identical(tmp_path, mode):
    """``apps.spgemm mult -o`` on 4 gloo ranks (each rank parses a quarter of
    every input file, entries shuffled to their row owners, C streamed to rank
    0 point-to-point) writes the same bytes as the 1-rank run; inputs with
    random line order, duplicate-free general and symmetric storage."""
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    A = gen_csr.uniform_csr(700, 500, 0.02, seed=3)
    B = gen_csr.uniform_csr(500, 900, 0.02, seed=4)
    a, b = str(tmp_path / "A.mtx"), str(tmp_path / "B.mtx")
    if mode == "sym":
        S = gen_csr.uniform_csr(600, 600, 0.02, seed=5)
        _shuffled_mtx(a, S, 1, symmetric=True)
        _shuffled_mtx(b, S, 2, symmetric=True)
    else:
        _shuffled_mtx(a, A, 1)
        _shuffled_mtx(b, B, 2)
    out = {}
    for world in (1, 4):
        c = str(tmp_path / f"C{world}.mtx")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={29650 + world + 10 * ['ab', 'aat', 'sym'].index(mode)}",
               "-m", "spmm_amd.apps.spgemm", "mult", a] + (["--aat"] if mode == "aat" else [b]) + \
              ["-o", c, "--device", "cpu", "--comm", "gloo"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
        assert r.returncode == 0, r.stderr[-3000:]
        out[world] = (json.loads(r.stdout.strip().splitlines()[-1]), open(c, "rb").read())
    assert out[1][1] == out[4][1]
    assert out[4][0]["ranks"] == 4 and out[1][0]["flops"] == out[4][0]["flops"]
    Am = mtx.read_mtx(a)
    Bm = Am.transpose() if mode == "aat" else mtx.read_mtx(b)
    C = mtx.read_mtx(str(tmp_path / "C4.mtx"))
    assert torch.allclose(C.to_dense().double(), Am.to_dense().double() @ Bm.to_dense().double(), atol=1e-5)


@pytest.mark.parametrize("world", [1, 3])
def test_a4_format_mtx_chain(tmp_path, world):
    """One command line for both workloads: ``a4 --format mtx`` multiplies a
    chain of Matrix Market files on the CSR engine (1 and 3 gloo ranks, a
    folder of naturally ordered files), prints the reference's stdout lines
    and writes the product."""
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    d = tmp_path / "chain"
    d.mkdir()
    dims = [300, 250, 280, 260, 310]
    mats = [gen_csr.uniform_csr(dims[i], dims[i + 1], 0.03, seed=10 + i) for i in range(4)]
    for i, M in enumerate(mats):
        mtx.write_mtx(str(d / f"m{i + 1}.mtx"), M)
    out = str(tmp_path / f"P{world}.mtx")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={29690 + world}", "-m", "spmm_amd.apps.a4", "--format", "mtx",
           str(d), "--out", out, "--device", "cpu", "--comm", "gloo"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert [x for x in lines if x.startswith("multiplying")] == ["multiplying 1 2", "multiplying 2 3", "multiplying 3 4"]
    assert sum(x.startswith("time taken ") for x in lines) == world
    ref = mats[0].to_dense().double()
    for M in mats[1:]:
        ref = ref @ M.to_dense().double()
    got = mtx.read_mtx(out).to_dense().double()
    assert got.shape == ref.shape and torch.allclose(got, ref, atol=1e-4)
