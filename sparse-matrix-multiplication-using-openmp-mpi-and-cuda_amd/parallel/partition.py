"""Work decomposition rules.

``chain_ranges`` is the reference's chain split (sparse_matrix_mult.cu:437-456,
612-615): ``op = N // P``; rank r < P-1 owns ``[r*op, (r+1)*op - 1]``, the last
rank owns ``[(P-1)*op, N-1]`` (the remainder); when ``op == 0`` (N < P) rank 0
owns the whole chain and the other ranks idle.  Exact mode must keep this
split: together with the per-range tree and the cross-rank tree it fixes the
association order, which the reference arithmetic is sensitive to.

``chain_ranges_balanced`` is the fast-mode alternative: contiguous ranges
balanced by an estimated per-matrix cost (not bit-compatible with the
reference for adversarial data; identical for inputs whose partial sums never
hit 2^64-1).

``row_panels`` splits rows for the 1D row-block SpGEMM / SpMM decomposition;
``weighted_row_panels`` splits them at equal cumulative work (e.g. the
per-row product counts of a SpGEMM), which is what power-law matrices (R-MAT
hub rows at low indices) need for balance.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

Range = Optional[Tuple[int, int]]


def chain_ranges(n: int, p: int) -> List[Range]:
    op = n // p
    if op == 0:
        return [(0, n - 1) if r == 0 and n > 0 else None for r in range(p)]
    out: List[Range] = []
    for r in range(p):
        lo = r * op
        hi = (r + 1) * op - 1 if r != p - 1 else n - 1
        out.append((lo, hi))
    return out


def chain_ranges_balanced(costs: Sequence[float], p: int) -> List[Range]:
    """Contiguous split of a chain minimising the max per-rank cost (greedy on
    prefix sums; every rank gets >= 1 matrix when len(costs) >= p)."""
    n = len(costs)
    if n < p:
        return chain_ranges(n, p)
    total = float(sum(costs))
    out: List[Range] = []
    lo = 0
    acc = 0.0
    for r in range(p):
        if r == p - 1:
            out.append((lo, n - 1))
            break
        target = total * (r + 1) / p
        hi = lo
        acc += costs[hi]
        # keep at least one matrix for each remaining rank
        while hi + 1 < n - (p - r - 1) and acc + costs[hi + 1] / 2 <= target:
            hi += 1
            acc += costs[hi]
        out.append((lo, hi))
        lo = hi + 1
    return out


def row_panels(m: int, p: int, align: int = 1) -> List[Tuple[int, int]]:
    """[lo, hi) row ranges of near-equal size, boundaries multiples of align."""
    out = []
    for r in range(p):
        lo = (m * r // p) // align * align
        hi = m if r == p - 1 else (m * (r + 1) // p) // align * align
        out.append((lo, hi))
    return out


def weighted_row_panels(prefix: Sequence[int], p: int) -> List[Tuple[int, int]]:
    """[lo, hi) row ranges with near-equal work: ``prefix`` is the inclusive
    cumulative work per row (length m, non-decreasing).  Cut r is the first row
    whose prefix reaches r/p of the total; panels may be empty.  ``prefix``
    may be an integer tensor (searched where it lives: no host copy of a
    16M-row prefix)."""
    import bisect

    m = len(prefix)
    total = int(prefix[-1]) if m else 0
    import torch

    if m and isinstance(prefix, torch.Tensor):
        targets = torch.tensor([-(-total * r // p) for r in range(1, p)], dtype=prefix.dtype, device=prefix.device)
        found = torch.searchsorted(prefix, targets).tolist() if p > 1 else []
    else:
        found = [bisect.bisect_left(prefix, total * r / p) for r in range(1, p)]
    cuts = [0]
    for r in range(1, p):
        c = found[r - 1] + 1 if total else m * r // p
        cuts.append(min(max(c, cuts[-1]), m))
    cuts.append(m)
    return [(cuts[r], cuts[r + 1]) for r in range(p)]


def binomial_tree_schedule(p: int):
    """The cross-rank reduction the reference performs on rank 0 with
    helper2 (:569-571), expressed as a distributed binomial tree: at step s
    (1, 2, 4, ...) rank r with r % 2s == 0 receives from r + s (if it exists)
    and computes (own . received).  Yields (step, receiver, sender); the pair
    is the reference's helper2 pair (r/s, r/s + 1) at level log2(s)."""
    s = 1
    while s < p:
        for r in range(0, p, 2 * s):
            if r + s < p:
                yield s, r, r + s
        s *= 2
