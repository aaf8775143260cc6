"""Independent golden model of the reference semantics (tests only).

Deliberately simple and separate from the engine: tiles live in a Python
dict (the reference's std::map view), the join is done with plain loops, and
the arithmetic is numpy uint64 (which wraps mod 2^64 like the reference's
C++), vectorised only across the k x k output elements of one tile.  The
order is exactly the reference's: for each output tile, pairs in ascending
middle key, then inner index 0..k-1 (sparse_matrix_mult.cu:54-62); chain
association = per-rank helper2 tree over the C12 range split, then helper2
over the P partials (:287-327, :437-571).  Intermediate zero tiles are KEPT,
as in the reference, so the engine's intermediate pruning is checked too.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Tuple

import numpy as np

from ..parallel.partition import chain_ranges

MAXU = np.uint64(0xFFFFFFFFFFFFFFFF)
Tiles = Dict[Tuple[int, int], np.ndarray]


class GoldenMatrix:
    def __init__(self, rows: int, cols: int, k: int, tiles: Tiles):
        self.rows, self.cols, self.k, self.tiles = rows, cols, k, tiles


def step(acc: np.ndarray, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """One reference step over arrays: t=(a*b)%MAX; acc=(acc+t)%MAX, wrapping first."""
    with np.errstate(over="ignore"):
        t = a * b
        t[t == MAXU] = 0
        s = acc + t
    s[s == MAXU] = 0
    return s


def multiply(A: GoldenMatrix, B: GoldenMatrix) -> GoldenMatrix:
    k = A.k
    brow = defaultdict(list)
    for (j, c) in sorted(B.tiles):
        brow[j].append(c)
    d = defaultdict(list)
    for (i, j) in sorted(A.tiles):
        for c in brow.get(j, ()):
            d[(i, c)].append(j)
    out: Tiles = {}
    for key in sorted(d):
        acc = np.zeros((k, k), dtype=np.uint64)
        for j in d[key]:
            a = A.tiles[(key[0], j)]
            b = B.tiles[(j, key[1])]
            for jj in range(k):
                acc = step(acc, np.repeat(a[:, jj:jj + 1], k, axis=1), np.repeat(b[jj:jj + 1, :], k, axis=0))
        out[key] = acc
    return GoldenMatrix(A.rows, B.cols, k, out)


def helper2(arr: List[GoldenMatrix]) -> GoldenMatrix:
    arr = list(arr)
    while len(arr) > 1:
        nxt = [multiply(arr[i], arr[i + 1]) for i in range(0, len(arr) - 1, 2)]
        if len(arr) % 2:
            nxt.append(arr[-1])
        arr = nxt
    return arr[0]


def chain(mats: List[GoldenMatrix], p: int = 1) -> GoldenMatrix:
    """Reference result for P MPI ranks, final zero tiles pruned."""
    ranges = chain_ranges(len(mats), p)
    if len(mats) // p == 0:
        res = helper2(mats)
    else:
        partials = [helper2(mats[lo:hi + 1]) for (lo, hi) in ranges]
        res = helper2(partials)
    tiles = {key: v for key, v in res.tiles.items() if v.any()}
    return GoldenMatrix(res.rows, res.cols, res.k, tiles)


def to_text(M: GoldenMatrix) -> str:
    """The reference writer's exact bytes (sparse_matrix_mult.cu:595-608)."""
    out = [f"{M.rows} {M.cols}\n{len(M.tiles)}\n"]
    for (r, c) in sorted(M.tiles):
        out.append(f"{r} {c}\n")
        for row in M.tiles[(r, c)]:
            out.append(" ".join(str(int(x)) for x in row) + "\n")
    return "".join(out)


def from_bsr(M) -> GoldenMatrix:
    return GoldenMatrix(M.rows, M.cols, M.k, {key: v.copy() for key, v in M.to_dict().items()})
