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


# ---- a4 --format mtx (csr_chain.cpp) ----------------------------------------

def _mtx_chain(d, dims, density=0.03, seed=10):
    from spmm_amd.utils import gen_csr, mtx

    d.mkdir(exist_ok=True)
    mats = [gen_csr.uniform_csr(dims[i], dims[i + 1], density, seed=seed + i) for i in range(len(dims) - 1)]
    for i, M in enumerate(mats):
        mtx.write_mtx(str(d / f"m{i + 1}.mtx"), M)
    return mats


def _python_mtx(tmp_path, inputs, out):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.a4", "--format", "mtx", *inputs, "--out", out,
                        "--device", "cpu", "--comm", "gloo", "--quiet"], env=env, capture_output=True, text=True,
                       timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("p", [1, 2, 3, 8])
def test_a4_mtx_native_matches_python_cli(tmp_path, a4_bin, p):
    """Native ``a4 --format mtx`` at P MPI ranks (each rank parses 1/P of every
    file, entries shuffled to their row owners, B all-gathered, C written
    through rank 0) writes the same bytes as the Python front-end's one-rank
    run (both on the OpenMP Gustavson engine), with the reference's stdout."""
    import torch

    from spmm_amd.utils import mtx

    mats = _mtx_chain(tmp_path / "chain", [300, 250, 280, 260, 310])
    want = str(tmp_path / "py.mtx")
    _python_mtx(tmp_path, [str(tmp_path / "chain")], want)
    out, met = str(tmp_path / "n.mtx"), str(tmp_path / "met.json")
    r = _run(a4_bin, p, str(tmp_path / "chain"), "--format", "mtx", "--device", "cpu", "--out", out, "--threads", "2",
             "--metrics-json", met)
    assert open(out, "rb").read() == open(want, "rb").read()
    assert re.findall(r"multiplying \d+ \d+", r.stdout) == ["multiplying 1 2", "multiplying 2 3", "multiplying 3 4"]
    assert len(re.findall(r"time taken [0-9.e+-]+ seconds", r.stdout)) == p
    m = json.load(open(met))
    assert m["format"] == "mtx" and m["ranks"] == p and m["n_files"] == 4
    ref = mats[0].to_dense().double()
    for M in mats[1:]:
        ref = ref @ M.to_dense().double()
    assert torch.allclose(mtx.read_mtx(out).to_dense().double(), ref, atol=1e-4)


@pytest.mark.parametrize("p", [1, 4])
def test_a4_mtx_symmetric_shuffled_natural_order(tmp_path, a4_bin, p):
    """Symmetric storage expanded, entries in random line order, a folder of
    11 files taken in natural order (m2 before m10: lexicographic order breaks
    the chain's shapes), an explicit file list giving the same bytes."""
    import torch

    from spmm_amd.utils import gen_csr, mtx

    d = tmp_path / "chain"
    d.mkdir()
    dims = [40 + 3 * i for i in range(12)]
    mats = [gen_csr.uniform_csr(dims[i], dims[i + 1], 0.08, seed=30 + i) for i in range(11)]
    for i, M in enumerate(mats):
        mtx.write_mtx(str(d / f"m{i + 1}.mtx"), M)
    S = gen_csr.uniform_csr(dims[-1], dims[-1], 0.05, seed=99)
    S = _symmetrize(S)
    lines = ["%%MatrixMarket matrix coordinate real symmetric", f"{S.m} {S.n} 0"]
    r_, c_, v_ = S.row_ids().tolist(), S.col.tolist(), S.val.tolist()
    ent = [(r_[i], c_[i], v_[i]) for i in range(len(r_)) if r_[i] >= c_[i]]
    import random

    random.Random(5).shuffle(ent)
    lines[1] = f"{S.m} {S.n} {len(ent)}"
    lines += [f"{a + 1} {b + 1} {v!r}" for a, b, v in ent]
    (tmp_path / "sym.mtx").write_text("\n".join(lines) + "\n")
    d2 = tmp_path / "chain2"
    d2.mkdir()
    for i in range(11):
        shutil.copy(d / f"m{i + 1}.mtx", d2 / f"m{i + 1}.mtx")
    shutil.copy(tmp_path / "sym.mtx", d2 / "m12.mtx")
    out1, out2 = str(tmp_path / "a.mtx"), str(tmp_path / "b.mtx")
    _run(a4_bin, p, str(d2), "--format", "mtx", "--device", "cpu", "--out", out1, "--quiet")
    files = [str(d2 / f"m{i + 1}.mtx") for i in range(12)]
    _run(a4_bin, p, *files[:1], *files[1:], "--format", "mtx", "--device", "cpu", "--out", out2, "--quiet")
    assert open(out1, "rb").read() == open(out2, "rb").read()
    ref = mats[0].to_dense().double()
    for M in mats[1:]:
        ref = ref @ M.to_dense().double()
    ref = ref @ S.to_dense().double()
    assert torch.allclose(mtx.read_mtx(out1).to_dense().double(), ref, rtol=1e-4, atol=1e-4)


def _symmetrize(S):
    """S + S^T."""
    import torch

    from spmm_amd.ops import csr as CS

    St = S.transpose()
    return CS.from_coo(torch.cat([S.row_ids(), St.row_ids()]), torch.cat([S.col.long(), St.col.long()]),
                       torch.cat([S.val, St.val]), S.m, S.n)


@pytest.mark.parametrize("p", [1, 3])
def test_a4_mtx_truncated_and_overlong_files(tmp_path, a4_bin, p):
    """The 1-rank rules at any P: a file short of its header's nnz is rejected
    (every rank exits non-zero with the count), entries past it are ignored."""
    d = tmp_path / "c"
    _mtx_chain(d, [60, 50, 70], density=0.1)
    good = str(tmp_path / "good.mtx")
    _run(a4_bin, 1, str(d), "--format", "mtx", "--device", "cpu", "--out", good, "--quiet")
    text = (d / "m2.mtx").read_text().splitlines()
    hdr = next(i for i, l in enumerate(text) if not l.startswith("%"))
    nnz = int(text[hdr].split()[2])
    (d / "m2.mtx").write_text("\n".join(text + ["1 1 7.0", "2 2 3.0"]) + "\n")   # 2 entries past nnz
    out = str(tmp_path / "long.mtx")
    _run(a4_bin, p, str(d), "--format", "mtx", "--device", "cpu", "--out", out, "--quiet")
    assert open(out, "rb").read() == open(good, "rb").read()
    (d / "m2.mtx").write_text("\n".join(text[:-5]) + "\n")
    r = _run(a4_bin, p, str(d), "--format", "mtx", "--device", "cpu", "--out", out, "--quiet", check=False)
    assert r.returncode != 0
    assert f"file has {nnz - 5} entries, expected {nnz}" in r.stderr


def test_a4_mtx_bad_format_flag(tmp_path, a4_bin):
    r = _run(a4_bin, 1, str(tmp_path), "--format", "coo", check=False)
    assert r.returncode != 0 and "--format must be ref or mtx" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("p", [1, 2])
def test_a4_mtx_gpu_bitmap_matches_cpu(tmp_path, a4_bin, p):
    """The products run on the GPU's bitmap-rank kernels through their C ABI:
    same structure as the CPU engine, values to fp32 summation order."""
    import numpy as np

    from spmm_amd.utils import mtx

    _mtx_chain(tmp_path / "c", [3000, 2500, 2800, 2600], density=0.004, seed=3)
    g, c, met = str(tmp_path / "g.mtx"), str(tmp_path / "c.mtx"), str(tmp_path / "met.json")
    _run(a4_bin, p, str(tmp_path / "c"), "--format", "mtx", "--device", "hip", "--out", g, "--quiet",
         "--metrics-json", met)
    _run(a4_bin, p, str(tmp_path / "c"), "--format", "mtx", "--device", "cpu", "--out", c, "--quiet")
    assert json.load(open(met))["gpu_products"] == 2
    G, C = mtx.read_mtx(g), mtx.read_mtx(c)
    assert G.nnz == C.nnz and bool((G.rowptr == C.rowptr).all()) and bool((G.col == C.col).all())
    np.testing.assert_allclose(G.val.numpy(), C.val.numpy(), rtol=1e-5, atol=1e-6)


def _skewed(m, n, base, hubs, hub_len, seed):
    """m x n CSR with ~base entries per row and a few hub rows of hub_len."""
    import torch

    from spmm_amd.ops import csr as CS

    g = torch.Generator().manual_seed(seed)
    rows, cols = [], []
    for i in range(m):
        k = hub_len if i in hubs else int(torch.randint(max(base // 2, 1), base * 2, (1,), generator=g))
        c = torch.randperm(n, generator=g)[:k]
        rows.append(torch.full((k,), i))
        cols.append(c)
    r, c = torch.cat(rows), torch.cat(cols)
    return CS.from_coo(r, c, torch.rand(r.numel(), generator=g) - 0.5, m, n)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [1, 2])
def test_a4_mtx_gpu_skewed_chain_has_no_cpu_fallback(tmp_path, a4_bin, p):
    """A skewed (hub-row) chain stays on the GPU: the products that fail the
    bitmap gate take the binned LDS path, and output rows of > 55296
    intermediate products go through the long-row pipeline (long_route /
    long_dense / long_place) -- recorded in --metrics-json, no CPU product.
    Same structure as the CPU engine, values to fp32 summation order."""
    import numpy as np

    from spmm_amd.utils import mtx

    d = tmp_path / "c"
    d.mkdir()
    mats = [_skewed(1200, 3000, 6, {0, 7}, 2500, 1), _skewed(3000, 2600, 30, set(range(0, 3000, 150)), 1800, 2),
            _skewed(2600, 2200, 8, {3, 4}, 1500, 3)]
    for i, M in enumerate(mats):
        mtx.write_mtx(str(d / f"m{i + 1}.mtx"), M)
    g, c, met = str(tmp_path / "g.mtx"), str(tmp_path / "c.mtx"), str(tmp_path / "met.json")
    _run(a4_bin, p, str(d), "--format", "mtx", "--device", "hip", "--out", g, "--quiet", "--metrics-json", met)
    _run(a4_bin, p, str(d), "--format", "mtx", "--device", "cpu", "--out", c, "--quiet")
    m = json.load(open(met))
    assert m["device_resident"] and m["cpu_products"] == 0 and m["gpu_products"] == 2, m
    assert m["gpu_binned_products"] >= 1 and m["gpu_long_rows"] >= 1, m
    assert m["host_resorted_rows"] == 0, m   # flagged rows are re-sorted on the device (csr_rowsort.hip)
    G, C = mtx.read_mtx(g), mtx.read_mtx(c)
    assert G.nnz == C.nnz and bool((G.rowptr == C.rowptr).all()) and bool((G.col == C.col).all())
    np.testing.assert_allclose(G.val.numpy(), C.val.numpy(), rtol=1e-4, atol=1e-5)


def test_counter_order_tree_is_the_reference_tree():
    """a4_main.cpp gpu_reduce_local submits the products in binary-counter order
    (a level-k product as soon as its two halves exist, the stack folded from
    the right at the end).  That is the same association as the reference's
    level-by-level pairwise tree with the odd node carried up
    (sparse_matrix_mult.cu:290-326) for every chain length -- the arithmetic is
    not associative in its edge cases, so the tree must match exactly."""
    def ref(n):
        arr = [(i, i + 1) for i in range(0, n - 1, 2)] + ([n - 1] if n % 2 else [])
        while len(arr) > 1:
            nxt = [(arr[i], arr[i + 1]) for i in range(0, len(arr) - 1, 2)]
            if len(arr) % 2:
                nxt.append(arr[-1])
            arr = nxt
        return arr[0]

    def counter(n):
        st = []
        for i in range(0, n - 1, 2):
            lv, x = 0, (i, i + 1)
            while st and st[-1][0] == lv:
                x = (st.pop()[1], x)
                lv += 1
            st.append((lv, x))
        if n % 2:
            st.append((0, n - 1))
        x = st.pop()[1]
        while st:
            x = (st.pop()[1], x)
        return x

    for n in range(1, 300):
        assert ref(n) == counter(n), n
