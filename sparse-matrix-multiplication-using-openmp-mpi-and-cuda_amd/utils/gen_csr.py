"""Synthetic CSR generators (north-star configs: uniform random sparse matrices
at fixed density, and R-MAT power-law graphs).

Both are generated on the device with torch RNG, and the uniform generator is
chunked by row blocks with a per-chunk seed so that the same global matrix
comes out whatever the row partition (a P-GPU run and a 1-GPU run of the same
config multiply the same matrices: strong scaling is well defined).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..ops.csr import CSR, rowptr_from_rows

CHUNK_ROWS = 65536


def _gen(device, seed: int) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    return g


def _uniform_chunk(rows: int, n: int, density: float, seed: int, device, values: str, dtype):
    g = _gen(device, seed)
    lam = torch.full((rows,), n * density, dtype=torch.float32, device=device)
    cnt = torch.poisson(lam, generator=g).to(torch.int64).clamp_(max=n)
    total = int(cnt.sum())
    rid = torch.repeat_interleave(torch.arange(rows, device=device), cnt, output_size=total)
    col = torch.randint(0, n, (total,), generator=g, device=device, dtype=torch.int64)
    code = torch.sort(rid * n + col).values
    if total > 1:
        keep = torch.ones(total, dtype=torch.bool, device=device)
        keep[1:] = code[1:] != code[:-1]
        code = code[keep]
    r = torch.div(code, n, rounding_mode="floor")
    c = (code - r * n).to(torch.int32)
    nnz = c.shape[0]
    if values == "ones":
        v = torch.ones(nnz, dtype=dtype, device=device)
    elif values == "small_int":
        v = torch.randint(-3, 4, (nnz,), generator=g, device=device).to(dtype)
    else:
        v = (torch.rand(nnz, generator=g, device=device) * 2 - 1).to(dtype)
    return r, c, v


def uniform_csr(m: int, n: int, density: float, seed: int = 0, device="cpu", rows: Optional[Tuple[int, int]] = None,
                values: str = "uniform", dtype=torch.float32) -> CSR:
    """Rows ``rows=(lo, hi)`` (default all) of an m x n matrix whose entries are
    present independently with probability ``density`` (row counts Poisson,
    columns uniform, duplicates merged), values uniform in [-1, 1)."""
    lo, hi = rows if rows is not None else (0, m)
    rs, cs, vs = [], [], []
    c0 = lo // CHUNK_ROWS
    c1 = (hi + CHUNK_ROWS - 1) // CHUNK_ROWS
    for ch in range(c0, c1):
        clo = ch * CHUNK_ROWS
        chi = min(m, clo + CHUNK_ROWS)
        r, c, v = _uniform_chunk(chi - clo, n, density, seed * 1000003 + ch, device, values, dtype)
        r = r + clo
        if clo < lo or chi > hi:
            sel = (r >= lo) & (r < hi)
            r, c, v = r[sel], c[sel], v[sel]
        rs.append(r - lo)
        cs.append(c)
        vs.append(v)
    r = torch.cat(rs) if rs else torch.empty(0, dtype=torch.int64, device=device)
    c = torch.cat(cs) if cs else torch.empty(0, dtype=torch.int32, device=device)
    v = torch.cat(vs) if vs else torch.empty(0, dtype=dtype, device=device)
    return CSR(hi - lo, n, rowptr_from_rows(r, hi - lo), c, v)


RMAT_CHUNK_EDGES = 1 << 22


def rmat_nchunks(scale: int, edge_factor: int = 16, chunk: int = RMAT_CHUNK_EDGES) -> int:
    return (edge_factor * (1 << scale) + chunk - 1) // chunk


def rmat_perm(scale: int, seed: int = 0, device="cpu") -> torch.Tensor:
    """The vertex relabelling of the R-MAT graph (same on every rank: one
    fixed-seed generator)."""
    return torch.randperm(1 << scale, generator=_gen(device, seed * 7919 + scale), device=device)


def rmat_edges(scale: int, edge_factor: int = 16, a: float = 0.57, b: float = 0.19, c: float = 0.19,
               seed: int = 0, device="cpu", permute: bool = True, chunk: int = RMAT_CHUNK_EDGES,
               chunks: Optional[Tuple[int, int]] = None, perm: Optional[torch.Tensor] = None):
    """Graph500-style R-MAT edge list (src, dst) int64, 2^scale vertices.

    The edges come in chunks of ``chunk`` with a generator seeded per chunk,
    so ``chunks=(k0, k1)`` yields exactly those chunks of the global list:
    P ranks that each generate a share of the chunks hold, together, the same
    graph as one rank that generates all of them (any P, strong scaling)."""
    n = 1 << scale
    ne = edge_factor * n
    nck = (ne + chunk - 1) // chunk
    k0, k1 = chunks if chunks is not None else (0, nck)
    srcs, dsts = [], []
    ab, abc = a + b, a + b + c
    for k in range(max(k0, 0), min(k1, nck)):
        g = _gen(device, (seed * 7919 + scale) * 1000003 + k + 1)
        e = min(chunk, ne - k * chunk)
        s = torch.zeros(e, dtype=torch.int64, device=device)
        d = torch.zeros(e, dtype=torch.int64, device=device)
        for lvl in range(scale):
            u = torch.rand(e, generator=g, device=device)
            sb = (u >= ab)
            db = ((u >= a) & (u < ab)) | (u >= abc)
            s |= sb.to(torch.int64) << lvl
            d |= db.to(torch.int64) << lvl
        srcs.append(s)
        dsts.append(d)
    s = torch.cat(srcs) if srcs else torch.empty(0, dtype=torch.int64, device=device)
    d = torch.cat(dsts) if dsts else torch.empty(0, dtype=torch.int64, device=device)
    if permute:
        perm = perm if perm is not None else rmat_perm(scale, seed, device)
        s, d = perm[s], perm[d]
    return s, d, n


def pattern_csr(s: torch.Tensor, d: torch.Tensor, m: int, n: int, row0: int = 0, dtype=torch.float32) -> CSR:
    """Rows row0 .. row0 + m of the 0/1 pattern of the edges (s, d) (every s
    in that range), duplicates merged, unit values."""
    code = torch.unique((s - row0) * n + d)   # sorted, unique
    r = torch.div(code, n, rounding_mode="floor")
    col = (code - r * n).to(torch.int32)
    return CSR(m, n, rowptr_from_rows(r, m), col, torch.ones(col.numel(), dtype=dtype, device=s.device))


def rmat_csr(scale: int, edge_factor: int = 16, seed: int = 0, device="cpu", dtype=torch.float32,
             chunk: int = RMAT_CHUNK_EDGES) -> CSR:
    """R-MAT adjacency matrix (duplicates merged, unit weights)."""
    s, d, n = rmat_edges(scale, edge_factor, seed=seed, device=device, chunk=chunk)
    return pattern_csr(s, d, n, n, dtype=dtype)
