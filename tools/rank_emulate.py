"""Per-rank cost of the row-block SpGEMM step at world size N, on one GPU.

Builds exactly what rank r of an N-GPU run holds (A's row panel r; B already
all-gathered, i.e. the full B) and times the local part of the step
(``spgemm(A_panel, B)``), plus a device copy of the B bytes a rank would
receive as a stand-in for the all-gather.  Used to predict strong scaling of
``bench.py`` without an 8-GPU node.

    python tools/rank_emulate.py --world 8 [--rank 0] [--n 1048576] [--density 1e-4]
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
from spmm_amd.ops.spgemm import SpgemmGraph, SpgemmInfo, spgemm  # noqa: E402
from spmm_amd.parallel.partition import row_panels  # noqa: E402
from spmm_amd.utils.gen_csr import uniform_csr  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--density", type=float, default=1e-4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--graph", action="store_true", help="time the local product as a SpgemmGraph replay")
    ap.add_argument("--per-step", action="store_true", help="print every timed step's ms and the path taken")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    _native.hip()
    lo, hi = row_panels(a.n, a.world)[a.rank]
    A = uniform_csr(a.n, a.n, a.density, seed=a.seed, device=dev, rows=(lo, hi))
    B = uniform_csr(a.n, a.n, a.density, seed=a.seed + 1, device=dev)
    info = SpgemmInfo()
    C = spgemm(A, B, info)
    del C
    recv = (a.world - 1) / a.world * (B.nnz * 8 + B.m * 8)
    src = torch.empty(int(recv) // 4 + 1, dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    run = lambda: spgemm(A, B)  # noqa: E731
    if a.graph:
        g = SpgemmGraph(A, B)
        run = g.run
    if a.per_step:
        print(json.dumps(dict(first_run=info.rows_per_bin_num)), file=sys.stderr, flush=True)
        for k in range(a.steps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            si = SpgemmInfo()
            C = spgemm(A, B, si) if not a.graph else run()
            del C
            torch.cuda.synchronize()
            print(json.dumps(dict(step=k, ms=round((time.perf_counter() - t1) * 1e3, 3), path=si.rows_per_bin_num)),
                  file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        C = run()
        del C
    torch.cuda.synchronize()
    t_local = (time.perf_counter() - t0) / a.steps
    t0 = time.perf_counter()
    for _ in range(a.steps):
        dst.copy_(src)
    torch.cuda.synchronize()
    t_copy = (time.perf_counter() - t0) / a.steps
    print(json.dumps(dict(world=a.world, rank=a.rank, graph=a.graph, rows=hi - lo, flops=info.flops, nnz_C=info.nnz,
                          local_ms=round(t_local * 1e3, 3), gflops_local=round(info.flops / t_local / 1e9, 1),
                          allgather_recv_bytes=int(recv), device_copy_ms=round(t_copy * 1e3, 3))), flush=True)


if __name__ == "__main__":
    main()
