"""Benchmark the block-sparse uint64 chain product (the reference's workload).

In-memory mode (default): a synthetic chain is generated on the device and
the exact-mode tree reduction is timed; reports tile pairs, integer GOP/s
(2*k^3 ops per tile pair, the report's op count) and ms per chain.

Folder mode (--folder): end-to-end like the reference's Table 1 (parse +
upload + reduce + prune + write), via the a4 pipeline on one process.

Report presets (report.pdf p.3 Table 1 gives tile counts only; shapes here are
ours, chosen so the whole chain holds the stated number of input tiles):
  small   N=8, 128x128 tile grid, density 0.076  (~10k tiles)
  medium  N=8, 256x256 tile grid, density 0.19   (~100k tiles)
  large   N=16, 512x512 tile grid, density 0.24  (~1M tiles)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.ops.bsr import BSR, canonicalize, tile_pair_count  # noqa: E402
from spmm_amd.models.chain import chain_product, ChainStats, reduce_tree  # noqa: E402

PRESETS = {
    "small": dict(n=8, blocks=128, density=0.076),
    "medium": dict(n=8, blocks=256, density=0.19),
    "large": dict(n=16, blocks=512, density=0.24),
}


def device_random_bsr(b: int, k: int, density: float, gen: torch.Generator, device) -> BSR:
    mask = torch.rand((b, b), generator=gen, device=device) < density
    rc = mask.nonzero().to(torch.int32)
    keys = rc * k
    vals = torch.randint(-(2 ** 63), 2 ** 63 - 1, (rc.shape[0], k, k), generator=gen, device=device,
                         dtype=torch.int64)
    keys, vals = canonicalize(keys, vals)
    return BSR(b * k, b * k, k, keys, vals)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(PRESETS), default="medium")
    ap.add_argument("--n", type=int)
    ap.add_argument("--blocks", type=int)
    ap.add_argument("--density", type=float)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    cfg = dict(PRESETS[a.preset])
    for key in ("n", "blocks", "density"):
        if getattr(a, key) is not None:
            cfg[key] = getattr(a, key)
    dev = torch.device(a.device)
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed)
    mats = [device_random_bsr(cfg["blocks"], a.k, cfg["density"], g, dev) for _ in range(cfg["n"])]
    tiles = sum(m.nb for m in mats)
    stats = ChainStats()
    reduce_tree(mats, 0, None, stats)   # warm + count pairs
    pairs = stats.tile_pairs
    for _ in range(a.warmup - 1):
        chain_product(mats)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        C = chain_product(mats)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    ops = pairs * 2 * a.k ** 3
    rec = dict(metric="bsr_chain_int_GOPs", preset=a.preset, **cfg, k=a.k, input_tiles=tiles, tile_pairs=pairs,
               out_tiles=C.nb, ms_per_chain=dt * 1e3, gops=ops / dt / 1e9, device=str(dev),
               ref_kernel_gops_p100=500.0)
    print(json.dumps(rec))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
