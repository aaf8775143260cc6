"""Multi-process chain product over gloo (CPU): byte-identical output vs the
golden model at the same P, for every partition case of the reference
(N > P with remainder, N == P, N < P fallback)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import spmm_amd  # noqa: F401
from spmm_amd.utils import gen, golden, refio


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, folder, out, logdir, fast=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from spmm_amd.models import chain as CH
    from spmm_amd.parallel import comm as CM

    comm = CM.init(backend="gloo", device="cpu", timeout_s=120)
    lines = []
    try:
        CH.run_chain(folder, comm, out_path=out, log=lines.append, nthreads=2, fast=fast)
    finally:
        comm.close()
    with open(os.path.join(logdir, f"log{rank}"), "w") as f:
        f.write("\n".join(lines))


@pytest.mark.parametrize("n,p", [(7, 2), (6, 3), (9, 4), (4, 4), (2, 3), (5, 5)])
def test_distributed_chain_matches_golden(tmp_path, n, p):
    k = 2
    mats = gen.random_chain(n, 4, k, 0.55, "adversarial", seed=10 * n + p)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, k)
    out = str(tmp_path / "matrix")
    mp.start_processes(_worker, args=(p, _free_port(), folder, out, str(tmp_path)), nprocs=p, join=True,
                       start_method="spawn")
    want = golden.chain([golden.from_bsr(m) for m in mats], p=p)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
    # every product is logged exactly once across ranks
    total = sum(len([l for l in (tmp_path / f"log{r}").read_text().splitlines() if l]) for r in range(p))
    assert total == n - 1


# unequal tile grids (heavy first half): the balanced split differs from the count split
FAST_SHAPES = [12, 14, 12, 13, 3, 2, 3, 2, 3]


@pytest.mark.parametrize("p", [2, 3])
def test_distributed_chain_fast_split(tmp_path, p):
    """``--fast``: chain ranges balanced on file sizes re-associate the chain;
    with uniform 64-bit values no partial sum hits the 2^64-1 collapse, so the
    output equals the exact (reference-split) golden product at the same P."""
    from spmm_amd.parallel.partition import chain_ranges, chain_ranges_balanced

    k = 4
    mats = gen.random_chain(len(FAST_SHAPES) - 1, 0, k, 0.6, "full", seed=40 + p, shapes=FAST_SHAPES)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, k)
    costs = [os.path.getsize(refio.matrix_path(folder, i + 1)) for i in range(len(mats))]
    assert chain_ranges_balanced(costs, p) != chain_ranges(len(mats), p)   # the split really changes
    out = str(tmp_path / "matrix")
    mp.start_processes(_worker, args=(p, _free_port(), folder, out, str(tmp_path), True), nprocs=p, join=True,
                       start_method="spawn")
    want = golden.chain([golden.from_bsr(m) for m in mats], p=p)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
