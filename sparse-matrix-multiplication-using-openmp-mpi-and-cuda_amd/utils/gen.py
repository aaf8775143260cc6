"""Synthetic block-sparse chains (the reference ships no inputs or generator;
``<random>`` is included at sparse_matrix_mult.cu:6 but never used).

Tile keys are element offsets of the tile's top-left corner (multiples of k),
the convention the reference's commented clipping code assumes (:636-637);
consecutive matrices share the inner dimension so the chain is conformant.

Value modes:
  small        0..9                        (exact-integer regime)
  full         uniform 64-bit              (wrap regime)
  adversarial  values near 2^64-1, odd a with b = -a^{-1} (a*b == 2^64-1), 0/1,
               so both collapse branches of the reference step fire.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ..ops.bsr import BSR, canonicalize

U64 = np.uint64


def _inv_mod_2_64(a: int) -> int:
    return pow(a, -1, 1 << 64)


def random_values(n: int, k: int, mode: str, rng: np.random.Generator) -> np.ndarray:
    shape = (n, k, k)
    if mode == "small":
        v = rng.integers(0, 10, size=shape, dtype=np.uint64)
    elif mode == "full":
        v = rng.integers(0, 1 << 63, size=shape, dtype=np.uint64) * U64(2) + rng.integers(0, 2, size=shape,
                                                                                            dtype=np.uint64)
    elif mode == "adversarial":
        pool = [0, 1, 2, 3, (1 << 64) - 1, (1 << 64) - 2, 1 << 63, (1 << 63) - 1]
        for _ in range(8):
            a = int(rng.integers(0, 1 << 62)) * 2 + 1
            pool += [a, (-_inv_mod_2_64(a)) % (1 << 64)]
        pool_arr = np.array(pool, dtype=np.uint64)
        v = pool_arr[rng.integers(0, len(pool), size=shape)]
    else:
        raise ValueError(f"unknown value mode {mode!r}")
    return v.astype(np.uint64)


def random_bsr(rb: int, cb: int, k: int, density: float, mode: str = "small",
               rng: Optional[np.random.Generator] = None, min_tiles: int = 1) -> BSR:
    """rb x cb grid of k x k tiles, each present with probability ``density``."""
    rng = rng or np.random.default_rng(0)
    mask = rng.random((rb, cb)) < density
    if mask.sum() < min_tiles:
        flat = rng.choice(rb * cb, size=min(min_tiles, rb * cb), replace=False)
        mask.flat[flat] = True
    r, c = np.nonzero(mask)
    keys = np.stack([r * k, c * k], axis=1).astype(np.int32)
    vals = random_values(len(r), k, mode, rng)
    kt, vt = canonicalize(torch.from_numpy(keys), torch.from_numpy(vals.view(np.int64)))
    return BSR(rb * k, cb * k, k, kt, vt)


def random_chain(n: int, blocks: int, k: int, density: float, mode: str = "small", seed: int = 0,
                 shapes: Optional[List[int]] = None) -> List[BSR]:
    """n conformant square-ish matrices of ``blocks`` x ``blocks`` tiles
    (or block dims ``shapes[i] x shapes[i+1]``)."""
    rng = np.random.default_rng(seed)
    dims = shapes if shapes is not None else [blocks] * (n + 1)
    return [random_bsr(dims[i], dims[i + 1], k, density, mode, rng) for i in range(n)]
