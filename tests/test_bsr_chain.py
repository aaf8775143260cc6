"""Block-sparse uint64 chain product: arithmetic, join, numeric, I/O, CLI.

Reference behaviour pinned by an independent golden model
(spmm_amd.utils.golden) — the reference ships no tests or fixtures
(SURVEY.md §4), so parity is against its documented semantics.
"""
import os
import random
import subprocess
import sys

import numpy as np
import pytest
import torch

import spmm_amd  # noqa: F401
from spmm_amd.ops import bsr as B
from spmm_amd.models import chain as CH
from spmm_amd.parallel import comm as CM
from spmm_amd.parallel.partition import chain_ranges, binomial_tree_schedule
from spmm_amd.utils import gen, golden, refio

MAX = (1 << 64) - 1
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ref_step_mod(acc, a, b):
    """Literal reference form: wrap, then % MAX (sparse_matrix_mult.cu:59-61)."""
    t = ((a * b) % (1 << 64)) % MAX
    return ((acc + t) % (1 << 64)) % MAX


def test_division_free_step_matches_modulo_form():
    rnd = random.Random(1)
    edge = [0, 1, 2, MAX, MAX - 1, 1 << 63, (1 << 63) - 1, (1 << 32) - 1, 1 << 32]
    for _ in range(20000):
        acc = rnd.choice(edge + [rnd.getrandbits(64)])
        a = rnd.choice(edge + [rnd.getrandbits(64)])
        b = rnd.choice(edge + [rnd.getrandbits(64)])
        if acc == MAX:
            acc = 0
        want = ref_step_mod(acc, a, b)
        got = golden.step(np.array([acc], np.uint64), np.array([a], np.uint64), np.array([b], np.uint64))[0]
        assert int(got) == want
    # the collapse really fires: a*b == 2^64-1
    a = 3
    b = (-pow(3, -1, 1 << 64)) % (1 << 64)
    assert (a * b) % (1 << 64) == MAX
    assert ref_step_mod(5, a, b) == 5


def test_keys_roundtrip_order():
    r = torch.tensor([-5, -5, 0, 3, 2 ** 31 - 1, -2 ** 31], dtype=torch.int32)
    c = torch.tensor([7, -9, 0, -1, 2 ** 31 - 1, -2 ** 31], dtype=torch.int32)
    code = B.encode_keys(r, c)
    back = B.decode_keys(code)
    assert torch.equal(back[:, 0], r) and torch.equal(back[:, 1], c)
    pairs = sorted(zip(r.tolist(), c.tolist()))
    assert [tuple(x) for x in B.decode_keys(torch.sort(code).values).tolist()] == pairs


def test_canonicalize_last_duplicate_wins():
    keys = torch.tensor([[2, 0], [0, 1], [2, 0], [0, 0]], dtype=torch.int32)
    vals = torch.arange(4, dtype=torch.int64).view(4, 1, 1)
    k2, v2 = B.canonicalize(keys, vals)
    assert k2.tolist() == [[0, 0], [0, 1], [2, 0]]
    assert v2.view(-1).tolist() == [3, 1, 2]


@pytest.mark.parametrize("k", [1, 2, 3, 5])
@pytest.mark.parametrize("mode", ["small", "full", "adversarial"])
def test_bsr_matmul_cpu_matches_golden(k, mode):
    rng = np.random.default_rng(k * 7 + len(mode))
    A = gen.random_bsr(5, 6, k, 0.5, mode, rng)
    Bm = gen.random_bsr(6, 4, k, 0.5, mode, rng)
    C = B.bsr_matmul(A, Bm, prune=False)
    G = golden.multiply(golden.from_bsr(A), golden.from_bsr(Bm))
    got = C.to_dict()
    assert set(got) == set(G.tiles)
    for key, v in G.tiles.items():
        np.testing.assert_array_equal(got[key], v)
    # pruning drops exactly the all-zero tiles
    Cp = B.bsr_matmul(A, Bm, prune=True)
    assert set(Cp.to_dict()) == {kk for kk, v in G.tiles.items() if v.any()}


def test_symbolic_pair_order_ascending_middle():
    k = 1
    A = B.BSR(3, 3, k, torch.tensor([[0, 0], [0, 1], [0, 2]], dtype=torch.int32), torch.ones(3, 1, 1, dtype=torch.int64))
    Bm = B.BSR(3, 3, k, torch.tensor([[0, 5], [1, 5], [2, 5]], dtype=torch.int32), torch.ones(3, 1, 1, dtype=torch.int64))
    sym = B.bsr_symbolic(A.keys, Bm.keys)
    assert sym.keys.tolist() == [[0, 5]]
    assert sym.pa.tolist() == [0, 1, 2] and sym.pb.tolist() == [0, 1, 2]


def test_order_sensitivity_is_reproduced():
    """(-2) + 1 + 1 = 1 but 1 + 1 + (-2) = 0 under the collapse rule: the
    engine must sum pairs in ascending middle key."""
    k = 1
    m2 = MAX - 1  # == -2
    vals_a = torch.tensor([m2, 1, 1], dtype=torch.uint64).view(torch.int64).view(3, 1, 1)
    A = B.BSR(1, 3, k, torch.tensor([[0, 0], [0, 1], [0, 2]], dtype=torch.int32), vals_a)
    Bm = B.BSR(3, 1, k, torch.tensor([[0, 0], [1, 0], [2, 0]], dtype=torch.int32), torch.ones(3, 1, 1, dtype=torch.int64))
    C = B.bsr_matmul(A, Bm, prune=False)
    assert int(C.vals.view(-1)[0]) == 1
    vals_a2 = torch.tensor([1, 1, m2], dtype=torch.uint64).view(torch.int64).view(3, 1, 1)
    C2 = B.bsr_matmul(B.BSR(1, 3, k, A.keys, vals_a2), Bm, prune=False)
    assert int(C2.vals.view(-1)[0]) == 0


def test_partition_rule():
    assert chain_ranges(10, 3) == [(0, 2), (3, 5), (6, 9)]
    assert chain_ranges(2, 4) == [(0, 1), None, None, None]
    assert chain_ranges(4, 4) == [(0, 0), (1, 1), (2, 2), (3, 3)]
    assert list(binomial_tree_schedule(5)) == [(1, 0, 1), (1, 2, 3), (2, 0, 2), (4, 0, 4)]


def _write_chain(tmp_path, mats, k):
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, k)
    return folder


def test_refio_roundtrip(tmp_path):
    k = 3
    M = gen.random_bsr(7, 5, k, 0.4, "full", np.random.default_rng(3))
    p = str(tmp_path / "m")
    refio.write_matrix(p, M)
    R = refio.read_matrix(p, k)
    assert (R.rows, R.cols) == (M.rows, M.cols)
    assert torch.equal(R.keys, M.keys) and torch.equal(R.vals, M.vals)
    # writer bytes == golden text bytes
    with open(p) as f:
        assert f.read() == golden.to_text(golden.from_bsr(M))


def test_refio_parser_tolerates_whitespace_and_order(tmp_path):
    p = tmp_path / "m"
    p.write_text("4 4\n2\n2 2\r\n 5 6\n7\t8\n0 0\n1 2 3\n18446744073709551615\n")
    R = refio.read_matrix(str(p), 2)
    assert R.keys.tolist() == [[0, 0], [2, 2]]
    v = R.to_dict()
    assert v[(2, 2)].tolist() == [[5, 6], [7, 8]]
    assert v[(0, 0)].tolist() == [[1, 2], [3, MAX]]


def test_refio_large_file_parallel_parse(tmp_path):
    # > 1 MiB so the multi-threaded tokenizer path is used
    k = 8
    M = gen.random_bsr(40, 40, k, 0.5, "full", np.random.default_rng(9))
    p = str(tmp_path / "big")
    refio.write_matrix(p, M)
    assert os.path.getsize(p) > (1 << 20)
    R = refio.read_matrix(p, k, nthreads=7)
    assert torch.equal(R.keys, M.keys) and torch.equal(R.vals, M.vals)


def test_refio_writer_digit_boundaries_and_swar_parser(tmp_path):
    """Every decimal length 1..20 (incl. 0, 10^n - 1, 10^n, 2^64 - 1) through the
    multi-threaded writer (sizing pass, exact offsets) and the 8-digit SWAR parser."""
    k = 6
    edge = [0, 2 ** 64 - 1, 2 ** 63, 2 ** 63 - 1]
    for n in range(1, 20):
        edge += [10 ** n - 1, 10 ** n, 10 ** n + 1]
    edge += [10 ** 19, 10 ** 19 - 1, 18446744073709551614]
    rng = np.random.default_rng(4)
    nb = 300
    vals = rng.choice(np.array(edge, dtype=np.uint64), size=(nb, k, k))
    keys = np.stack(np.divmod(np.arange(nb), 20), 1).astype(np.int32) * k
    keys[::7, 1] *= -1                       # negative tile coordinates print with '-'
    M = B.BSR(120 * k, 20 * k, k, *B.canonicalize(torch.from_numpy(keys), torch.from_numpy(vals.view(np.int64))))
    p = str(tmp_path / "m")
    refio.write_matrix(p, M, nthreads=5)
    with open(p) as f:
        assert f.read() == golden.to_text(golden.from_bsr(M))
    R = refio.read_matrix(p, k, nthreads=3)
    assert torch.equal(R.keys, M.keys) and torch.equal(R.vals, M.vals)


def test_refio_short_file_errors(tmp_path):
    p = tmp_path / "m"
    p.write_text("2 2\n1\n0 0\n1 2 3\n")
    with pytest.raises(refio.FormatError):
        refio.read_matrix(str(p), 2)
    with pytest.raises(refio.FormatError):
        refio.read_size(str(tmp_path / "nope"))


@pytest.mark.parametrize("n", [1, 2, 5, 8])
def test_run_chain_single_process_cpu(tmp_path, n):
    k = 2
    mats = gen.random_chain(n, 4, k, 0.5, "adversarial", seed=n)
    folder = _write_chain(tmp_path, mats, k)
    comm = CM.Comm(0, 1, 0, torch.device("cpu"), None)
    out = str(tmp_path / "matrix")
    lines = []
    CH.run_chain(folder, comm, out_path=out, log=lines.append)
    want = golden.chain([golden.from_bsr(m) for m in mats], p=1)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
    assert len(lines) == n - 1
    if n == 5:
        assert lines == ["multiplying 0 1", "multiplying 2 3", "multiplying 0 1", "multiplying 0 1"]


def test_a4_cli_single_process(tmp_path):
    k = 3
    mats = gen.random_chain(3, 3, k, 0.6, "full", seed=11)
    folder = _write_chain(tmp_path, mats, k)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.a4", folder, "--device", "cpu"], cwd=str(tmp_path),
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    assert out[:2] == ["multiplying 0 1", "multiplying 0 1"]
    assert out[-1].startswith("time taken ") and out[-1].endswith(" seconds")
    want = golden.chain([golden.from_bsr(m) for m in mats], p=1)
    assert (tmp_path / "matrix").read_text() == golden.to_text(want)


def test_a4_cli_missing_size(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.a4", str(tmp_path / "none"), "--device", "cpu"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 1
    assert "Cannot open size file!" in r.stderr


# ----------------------------------------------------------------- GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 3, 4, 8, 16, 17, 24, 31, 32, 33, 48, 64])
def test_bsr_numeric_gpu_matches_cpu(k):
    rng = np.random.default_rng(100 + k)
    A = gen.random_bsr(9, 7, k, 0.45, "full" if k % 2 else "adversarial", rng)
    Bm = gen.random_bsr(7, 8, k, 0.45, "adversarial" if k % 2 else "full", rng)
    Cc = B.bsr_matmul(A, Bm, prune=False)
    Cg = B.bsr_matmul(A.to("cuda"), Bm.to("cuda"), prune=False)
    assert torch.equal(Cg.keys.cpu(), Cc.keys)
    assert torch.equal(Cg.vals.cpu(), Cc.vals)
    nz_cpu = B.nonzero_tiles(Cc)
    assert torch.equal(B.nonzero_tiles(Cg).cpu(), nz_cpu)


@pytest.mark.gpu
def test_bsr_numeric_gpu_matches_golden_k32():
    k = 32
    rng = np.random.default_rng(5)
    A = gen.random_bsr(4, 5, k, 0.5, "adversarial", rng)
    Bm = gen.random_bsr(5, 3, k, 0.5, "adversarial", rng)
    Cg = B.bsr_matmul(A.to("cuda"), Bm.to("cuda"), prune=False)
    G = golden.multiply(golden.from_bsr(A), golden.from_bsr(Bm))
    got = Cg.to_dict()
    assert set(got) == set(G.tiles)
    for key, v in G.tiles.items():
        np.testing.assert_array_equal(got[key], v)


@pytest.mark.gpu
@pytest.mark.parametrize("streams", [1, 4])
def test_run_chain_gpu_k32(tmp_path, streams):
    """Also with the products of each tree level on a pool of 4 HIP streams
    (``a4 --streams 4``): same bytes as the golden model."""
    k = 32
    mats = gen.random_chain(11, 5, k, 0.4, "adversarial", seed=21)
    folder = _write_chain(tmp_path, mats, k)
    comm = CM.Comm(0, 1, 0, torch.device("cuda", 0), None)
    out = str(tmp_path / "matrix")
    lines = []
    CH.run_chain(folder, comm, out_path=out, log=lines.append, streams=streams)
    want = golden.chain([golden.from_bsr(m) for m in mats], p=1)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
    assert len(lines) == 10


def test_a4_cli_streams_flag_cpu(tmp_path):
    """``--streams`` is accepted by the Python front-end as by the native one
    (a no-op on the CPU engine)."""
    k = 2
    mats = gen.random_chain(5, 3, k, 0.6, "full", seed=12)
    folder = _write_chain(tmp_path, mats, k)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "spmm_amd.apps.a4", folder, "--device", "cpu", "--streams", "3"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    want = golden.chain([golden.from_bsr(m) for m in mats], p=1)
    assert (tmp_path / "matrix").read_text() == golden.to_text(want)


def test_weighted_row_panels_balance():
    from spmm_amd.parallel.partition import weighted_row_panels

    w = [1] * 100 + [50] * 4 + [1] * 96          # a hub block in the middle
    pre = list(np.cumsum(w))
    panels = weighted_row_panels(pre, 4)
    assert panels[0][0] == 0 and panels[-1][1] == len(w)
    assert all(a[1] == b[0] for a, b in zip(panels, panels[1:]))
    loads = [sum(w[lo:hi]) for lo, hi in panels]
    assert max(loads) <= sum(w) / 4 + 50          # within one heavy row of perfect
    import torch
    for p in (1, 2, 3, 4, 7):                     # device-tensor prefix: same cuts as the list
        assert weighted_row_panels(torch.tensor(pre), p) == weighted_row_panels(pre, p)
