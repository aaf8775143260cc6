"""In-tree device primitives (csrc/kernels/prim.hip) against torch: scan,
stable LSD radix sort of (key, payload) pairs, and the block-sparse symbolic
phase shared by the native a4 engine and ops/bsr.py."""
import ctypes as C

import pytest
import torch

import spmm_amd  # noqa: F401
from spmm_amd import _native
from spmm_amd.ops import bsr as BS


def _lib():
    return _native.hip()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 5, 2047, 2048, 2049, 300_001, 5_000_000])
@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
def test_prim_scan(n, dtype):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(n)
    x = torch.randint(-50, 1000, (n,), generator=g, device=dev, dtype=dtype)
    ws = torch.empty(int(_lib().spmm_prim_scan_ws(n)), dtype=torch.uint8, device=dev)
    ref = torch.cumsum(x.long(), 0)
    for inclusive in (1, 0):
        out = torch.empty(n, dtype=torch.int64, device=dev)
        _native.check(_lib().spmm_prim_scan(_native.ptr(x), x.element_size(), n, _native.ptr(out), inclusive,
                                            _native.ptr(ws), _native.stream_ptr(dev)), "scan")
        want = ref if inclusive else ref - x.long()
        assert torch.equal(out, want)


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits", [(1, 8), (100, 3), (2048, 12), (70_001, 20), (1_000_003, 33), (262_144, 64)])
def test_prim_sort_pairs_stable(n, bits):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(bits * 7 + n)
    hi = (1 << min(bits, 62))
    k = torch.randint(0, hi, (n,), generator=g, device=dev, dtype=torch.int64)
    if bits == 64:
        k = k * 4 - (1 << 62)   # negative int64 = high-bit-set uint64 patterns
    k[: n // 3] = k[0]          # many equal keys: stability matters
    v = torch.arange(n, device=dev, dtype=torch.int64)
    ws = torch.empty(int(_lib().spmm_prim_sort_ws(n)), dtype=torch.uint8, device=dev)
    ks, vs = k.clone(), v.clone()
    _native.check(_lib().spmm_prim_sort_pairs_u64(_native.ptr(ks), _native.ptr(vs), n, bits, _native.ptr(ws),
                                                  _native.stream_ptr(dev)), "sort")
    # reference: stable sort on the unsigned value of the low `bits` bits
    mask = -1 if bits == 64 else (1 << bits) - 1
    key = k & mask if bits < 64 else k
    if bits == 64:   # unsigned order of int64 patterns: flip the sign bit
        key = k ^ (-(1 << 63))
    order = torch.sort(key, stable=True).indices
    assert torch.equal(vs, v[order]) and torch.equal(ks, k[order])


def _random_bsr_keys(nr, nc, density, seed, dev):
    g = torch.Generator().manual_seed(seed)
    m = torch.rand(nr, nc, generator=g) < density
    r, c = m.nonzero(as_tuple=True)
    return torch.stack([r, c], 1).to(torch.int32).to(dev)   # row-major = sorted (r, c)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(40, 50, 60, 0.1), (200, 300, 150, 0.03), (7, 1, 9, 1.0), (64, 64, 64, 0.0)])
def test_bsr_symbolic_native_matches_torch(shape):
    nr, nk, nc, d = shape
    dev = torch.device("cuda")
    ak = _random_bsr_keys(nr, nk, d, 1, dev)
    bk = _random_bsr_keys(nk, nc, d, 2, dev)
    if ak.shape[0]:
        ak[:, 0] += 1000   # offset tile coordinates: the compact key must subtract them again
    if bk.shape[0]:
        bk[:, 1] -= 500
    got = BS.bsr_symbolic(ak, bk)
    ref = BS.bsr_symbolic(ak.cpu(), bk.cpu())
    assert torch.equal(got.keys.cpu(), ref.keys)
    assert torch.equal(got.tile_ptr.cpu(), ref.tile_ptr)
    assert torch.equal(got.pa.cpu(), ref.pa) and torch.equal(got.pb.cpu(), ref.pb)


@pytest.mark.gpu
@pytest.mark.parametrize("long_rows", [False, True])
def test_csr_sort_rows_device(long_rows):
    """ops.csr.sort_rows on listed rows (csr_rowsort.hip: wave / LDS bitonic, radix beyond
    16384 entries) equals a per-row torch sort; unlisted rows stay as they were."""
    from spmm_amd.ops.csr import CSR, sort_rows

    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5 + long_rows)
    lens = [0, 1, 2, 63, 64, 65, 100, 2047, 2048, 2049, 16384, 5, 700]
    if long_rows:
        lens += [16385, 40000]
    m, n = len(lens), 1 << 20
    cols, vals = [], []
    for ln in lens:
        cols.append(torch.randperm(n, generator=g)[:ln].to(torch.int32))   # distinct, unsorted
        vals.append(torch.randn(ln, generator=g))
    rowptr = torch.zeros(m + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.tensor(lens), 0)
    Cm = CSR(m, n, rowptr.to(dev), torch.cat(cols).to(dev), torch.cat(vals).to(dev))
    rows = torch.tensor([i for i in range(m) if i % 4 != 3], dtype=torch.int64, device=dev)
    out = sort_rows(Cm, rows)
    for i in range(m):
        s, e = int(rowptr[i]), int(rowptr[i + 1])
        if i % 4 == 3:
            assert torch.equal(out.col[s:e], Cm.col[s:e])
            continue
        c, p = torch.sort(Cm.col[s:e])
        assert torch.equal(out.col[s:e], c), i
        assert torch.equal(out.val[s:e], Cm.val[s:e][p]), i
