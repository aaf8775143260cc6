"""Native ``a4`` executable (csrc/runtime): mpiexec-launched, byte-identical
``./matrix`` vs the golden model at the same P, reference stdout lines,
checkpoint/resume, fail-fast fault injection.  CPU engine + MPI here; the GPU
engine (and RCCL at P=1) on the GPU box."""
import json
import os
import re
import shutil
import subprocess

import pytest

import spmm_amd  # noqa: F401
from spmm_amd import _build
from spmm_amd.utils import gen, golden, refio

MPIEXEC = os.path.join(_build.mpi_home(), "bin", "mpiexec")


@pytest.fixture(scope="module")
def a4_bin():
    if not os.path.exists(MPIEXEC):
        pytest.skip("no MPICH")
    path = _build.build_a4()
    if path is None:
        pytest.skip("native a4 not built (no mpi.h)")
    return path


def _run(a4_bin, p, folder, *args, check=True, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("SPMM_FAULT_INJECT", None)
    cmd = [MPIEXEC, "-n", str(p), a4_bin, folder] + list(args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    if check and r.returncode != 0:
        raise AssertionError(f"a4 failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    return r


def _chain(tmp_path, n, blocks=4, k=2, seed=0):
    mats = gen.random_chain(n, blocks, k, 0.55, "adversarial", seed=seed)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, k)
    return mats, folder


@pytest.mark.parametrize("n,p", [(7, 2), (6, 3), (9, 4), (4, 4), (2, 3), (1, 1), (5, 1)])
def test_a4_cpu_matches_golden(tmp_path, a4_bin, n, p):
    mats, folder = _chain(tmp_path, n, seed=10 * n + p)
    out = str(tmp_path / "matrix")
    r = _run(a4_bin, p, folder, "--device", "cpu", "--out", out, "--threads", "2")
    want = golden.chain([golden.from_bsr(m) for m in mats], p=p)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
    # ranks' lines can interleave in mpiexec's merged stdout: count tokens, not lines
    assert len(re.findall(r"multiplying \d+ \d+", r.stdout)) == n - 1
    assert len(re.findall(r"time taken [0-9.e+-]+ seconds", r.stdout)) == p


@pytest.mark.parametrize("n,p", [(9, 4), (12, 3), (16, 8)])
def test_a4_cpu_row_panel_split_matches_unsplit(tmp_path, a4_bin, n, p):
    """Cross-rank products split by row panels over the idle ranks of each tree
    group give the same bytes as one rank per product (and the golden model)."""
    mats, folder = _chain(tmp_path, n, blocks=7, seed=100 + n)
    outs = []
    for flag in ([], ["--no-split"]):
        out = str(tmp_path / f"matrix{len(outs)}")
        met = str(tmp_path / f"m{len(outs)}.json")
        r = _run(a4_bin, p, folder, "--device", "cpu", "--out", out, "--threads", "1", "--metrics-json", met, *flag)
        assert len(re.findall(r"multiplying \d+ \d+", r.stdout)) == n - 1
        outs.append(open(out).read())
        assert json.load(open(met))["split"] == (not flag)
    assert outs[0] == outs[1] == golden.to_text(golden.chain([golden.from_bsr(m) for m in mats], p=p))


@pytest.mark.parametrize("p", [2, 3])
def test_a4_cpu_fast_split(tmp_path, a4_bin, p):
    """Native ``--fast`` (chain ranges balanced on file sizes) on unequal tile
    grids: same output as the exact golden product (uniform 64-bit values
    never hit the 2^64-1 collapse), every product logged once."""
    shapes = [12, 14, 12, 13, 3, 2, 3, 2, 3]
    mats = gen.random_chain(len(shapes) - 1, 0, 4, 0.6, "full", seed=40 + p, shapes=shapes)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, 4)
    out = str(tmp_path / "matrix")
    r = _run(a4_bin, p, folder, "--device", "cpu", "--out", out, "--threads", "2", "--fast")
    want = golden.chain([golden.from_bsr(m) for m in mats], p=p)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
    assert len(re.findall(r"multiplying \d+ \d+", r.stdout)) == len(mats) - 1


def test_a4_missing_size_file(tmp_path, a4_bin):
    r = _run(a4_bin, 1, str(tmp_path / "nowhere"), "--device", "cpu", check=False)
    assert r.returncode != 0
    assert "Cannot open size file!" in r.stderr


@pytest.mark.parametrize("p", [1, 3])
def test_a4_empty_chain_writes_empty_matrix(tmp_path, a4_bin, p):
    """A size file with N = 0: rank 0 writes an empty product instead of
    dereferencing a partial that was never built."""
    folder = tmp_path / "in"
    folder.mkdir()
    (folder / "size").write_text("0 2\n")
    out = str(tmp_path / "matrix")
    r = _run(a4_bin, p, str(folder), "--device", "cpu", "--out", out)
    assert open(out).read() == "0 0\n0\n"
    assert len(re.findall(r"time taken [0-9.e+-]+ seconds", r.stdout)) == p


def test_a4_checkpoint_resume_and_metrics(tmp_path, a4_bin):
    mats, folder = _chain(tmp_path, 8, seed=3)
    ck = str(tmp_path / "ck")
    out1, out2 = str(tmp_path / "m1"), str(tmp_path / "m2")
    _run(a4_bin, 2, folder, "--device", "cpu", "--out", out1, "--save-partials", ck, "--quiet")
    assert sorted(os.listdir(ck)) == ["partial_0", "partial_1"]
    met = str(tmp_path / "met.json")
    r = _run(a4_bin, 2, folder, "--device", "cpu", "--out", out2, "--load-partials", ck, "--metrics-json", met)
    assert open(out1).read() == open(out2).read()
    # resumed run skips the local trees: only the cross-rank product is printed
    assert sum(1 for l in r.stdout.splitlines() if l.startswith("multiplying ")) == 1
    m = json.load(open(met))
    assert m["engine"] == "native" and m["ranks"] == 2 and m["products"] == 1


def test_a4_fault_injection_fails_fast(tmp_path, a4_bin):
    _, folder = _chain(tmp_path, 6, seed=4)
    env = dict(os.environ, OMP_NUM_THREADS="2", SPMM_FAULT_INJECT="send:1")
    r = subprocess.run([MPIEXEC, "-n", "2", a4_bin, folder, "--device", "cpu", "--out", str(tmp_path / "m")],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "injected fault" in r.stderr


def test_a4_dump(tmp_path, a4_bin):
    _, folder = _chain(tmp_path, 2, seed=5)
    r = _run(a4_bin, 1, folder, "--device", "cpu", "--out", str(tmp_path / "m"), "--dump")
    assert r.stdout.count("[dump] ") == 3   # two inputs + the result


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,comm", [(9, 1, "auto"), (5, 1, "rccl"), (7, 2, "mpi"), (8, 4, "mpi"), (6, 2, "rccl"),
                                      (9, 4, "rccl")])
def test_a4_gpu_matches_golden(tmp_path, a4_bin, n, p, comm):
    """P ranks over MPI (host-staged; ranks may share a GPU) or RCCL (one GPU
    per rank: the split tree steps' grouped fan-out / fan-in; RCCL refuses two
    ranks on one device, so those cases need a node with >= P GPUs)."""
    import torch

    if comm == "rccl" and p > torch.cuda.device_count():
        pytest.skip(f"RCCL needs one GPU per rank ({p} ranks, {torch.cuda.device_count()} GPU(s))")
    mats, folder = _chain(tmp_path, n, blocks=6, k=4, seed=n + p)
    out = str(tmp_path / "matrix")
    _run(a4_bin, p, folder, "--device", "hip", "--comm", comm, "--out", out, "--streams", "3")
    want = golden.chain([golden.from_bsr(m) for m in mats], p=p)
    with open(out) as f:
        assert f.read() == golden.to_text(want)


@pytest.mark.gpu
def test_a4_gpu_concurrent_levels_match_python_engine(tmp_path, a4_bin):
    """Dense-filling chain: four concurrent level-0 products on the stream pool,
    loader uploads in flight, stream-ordered buffers freed across streams;
    output must equal the in-process GPU engine (same P=1 association)."""
    import torch

    from spmm_amd.models.chain import chain_product

    mats = gen.random_chain(8, 40, 32, 0.2, "full", seed=21)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, 32)
    _run(a4_bin, 1, folder, "--device", "hip", "--out", str(tmp_path / "g"), "--quiet", "--streams", "4")
    want = chain_product([m.to(torch.device("cuda", 0)) for m in mats])
    refio.write_matrix(str(tmp_path / "p"), want)
    assert open(tmp_path / "g").read() == open(tmp_path / "p").read()


@pytest.mark.gpu
def test_a4_gpu_k32_matches_cpu_engine(tmp_path, a4_bin):
    mats = gen.random_chain(6, 8, 32, 0.4, "full", seed=9)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, 32)
    _run(a4_bin, 1, folder, "--device", "hip", "--out", str(tmp_path / "g"), "--quiet")
    _run(a4_bin, 1, folder, "--device", "cpu", "--out", str(tmp_path / "c"), "--quiet")
    assert open(tmp_path / "g").read() == open(tmp_path / "c").read()
