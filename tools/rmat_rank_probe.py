"""What one rank of an N-GPU R-MAT A.A^T step computes, timed on one GPU.

Generates the full R-MAT matrix (BASELINE config 5: scale 24, edge factor 16)
on the device, splits rows at equal intermediate-product counts exactly as
``bench.py --workload rmat`` does for world size N, and times rank r's local
product (C streamed in row panels when its product bound does not fit, as in
the bench).  Predicts the per-rank step time of the 8-GPU run without an
8-GPU node.

    python tools/rmat_rank_probe.py [--scale 24] [--world 8] [--ranks 0,7] [--steps 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _native  # noqa: E402
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.ops.spgemm import SpgemmInfo, row_nprod, spgemm  # noqa: E402
from spmm_amd.parallel.partition import weighted_row_panels  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--stream", default="auto", choices=["auto", "on", "off"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    _native.hip()
    t0 = time.perf_counter()
    A = gen_csr.rmat_csr(a.scale, a.edge_factor, seed=a.seed, device=dev)
    At = A.transpose()
    nprod = row_nprod(A, At)
    panels = weighted_row_panels(torch.cumsum(nprod, 0), a.world)
    total = int(nprod.sum())
    torch.cuda.synchronize()
    print(json.dumps(dict(scale=a.scale, nnz_A=A.nnz, products=total, max_row_products=int(nprod.max()),
                          gen_s=round(time.perf_counter() - t0, 2))), flush=True)
    for r in [int(x) for x in a.ranks.split(",")]:
        lo, hi = panels[r]
        Ap = A.row_slice(lo, hi)
        local = int(nprod[lo:hi].sum())
        stream = a.stream == "on" or (a.stream == "auto" and local > MS.stream_budget(dev))
        info = SpgemmInfo()
        if stream:
            run = lambda i=None: MS.streamed_spgemm(Ap, At, lambda *_: None, info=i)  # noqa: E731
        else:
            def run(i=None):
                C = spgemm(Ap, At, i)
                del C
        run(info)   # warm-up, counts
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps(dict(world=a.world, rank=r, rows=hi - lo, products=local, flops=info.flops, nnz_C=info.nnz,
                              streamed=stream, ms=round(dt * 1e3, 1), gflops=round(info.flops / dt / 1e9, 1),
                              bins={str(k): v for k, v in info.rows_per_bin_num.items()})), flush=True)
        del Ap
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
