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
