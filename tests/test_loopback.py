"""In-process loopback backend: P ranks as threads run the
distributed chain (reference split, binomial tree with row-panel splits, fast
split) byte-identical to the golden model at the same P — no processes."""
import os
import subprocess
import sys

import pytest

import spmm_amd  # noqa: F401
from spmm_amd.models import chain as CH
from spmm_amd.parallel.loopback import run_loopback
from spmm_amd.utils import gen, golden, refio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,p,split", [(7, 2, True), (6, 3, True), (9, 4, False), (16, 8, True), (3, 5, True),
                                       (1, 1, True), (12, 7, True)])
def test_loopback_chain_matches_golden(tmp_path, n, p, split):
    mats = gen.random_chain(n, 4, 2, 0.55, "adversarial", seed=7 * n + p)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, 2)
    out = str(tmp_path / "matrix")
    logs = []
    run_loopback(p, lambda comm: CH.run_chain(folder, comm, out_path=out, log=logs.append, nthreads=1, split=split))
    with open(out) as f:
        assert f.read() == golden.to_text(golden.chain([golden.from_bsr(m) for m in mats], p=p))
    assert len(logs) == n - 1   # every product logged once across the ranks


def test_loopback_rank_failure_is_raised():
    def body(comm):
        if comm.rank == 1:
            raise RuntimeError("rank 1 failed")
        comm.barrier()   # released by the abort, not left hanging

    with pytest.raises(RuntimeError, match="rank 1 failed"):
        run_loopback(3, body, timeout_s=30)


def test_a4_cli_loopback(tmp_path):
    mats = gen.random_chain(9, 4, 2, 0.55, "adversarial", seed=3)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, 2)
    out = str(tmp_path / "matrix")
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.a4", folder, "--comm", "loopback", "--ranks", "4",
                        "--device", "cpu", "--out", out], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("multiplying") == 8 and r.stdout.count("time taken") == 4
    with open(out) as f:
        assert f.read() == golden.to_text(golden.chain([golden.from_bsr(m) for m in mats], p=4))


def test_loopback_collectives_let_the_caller_reuse_its_buffer():
    """A rank may overwrite its input as soon as a collective returns (as
    under RCCL's stream order): peers still receive the posted values."""
    import torch

    def body(comm):
        x = torch.full((4,), float(comm.rank))
        fin = comm.all_gather_async(x)
        x.fill_(-1.0)   # reuse right after posting
        g = fin()
        y = torch.arange(2 * comm.world, dtype=torch.float32) + 10 * comm.rank
        out = comm.all_to_all_v(y, [2] * comm.world, [2] * comm.world)
        y.fill_(-1.0)
        comm.barrier()
        return g, out

    res = run_loopback(3, body, timeout_s=30)
    for r, (g, out) in enumerate(res):
        assert torch.equal(g, torch.tensor([0.0] * 4 + [1.0] * 4 + [2.0] * 4))
        assert torch.equal(out, torch.tensor([10.0 * s + 2 * r + i for s in range(3) for i in range(2)]))
