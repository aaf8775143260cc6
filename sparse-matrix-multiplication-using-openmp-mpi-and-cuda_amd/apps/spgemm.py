"""CSR SpGEMM / SpMM command line (north-star configs).

    # C = A . B from Matrix Market files (one process, or torchrun/mpirun P ranks:
    # 1D row-block, B all-gathered over RCCL, C gathered to rank 0 for output)
    python -m spmm_amd.apps.spgemm mult A.mtx B.mtx -o C.mtx

    # C = A . A^T  (e.g. R-MAT graphs)
    python -m spmm_amd.apps.spgemm mult A.mtx --aat -o C.mtx

    # synthetic inputs (uniform at fixed density, or R-MAT)
    python -m spmm_amd.apps.spgemm gen uniform --n 65536 --density 1e-3 -o A.mtx
    python -m spmm_amd.apps.spgemm gen rmat --scale 16 --edge-factor 16 -o G.mtx

Prints one JSON line with wall-clock, FLOPs (2 x intermediate products) and
GFLOP/s of the multiply (load / write timed separately).
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def _sync(comm):
    import torch

    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)


def cmd_mult(args) -> int:
    import torch

    from ..models.spgemm import allgather_csr_rows, gather_rows
    from ..ops.spgemm import SpgemmInfo, spgemm
    from ..parallel import comm as CM
    from ..parallel.partition import row_panels
    from ..utils.mtx import read_mtx, write_mtx

    comm = CM.init(backend=args.comm, device=args.device)
    t0 = time.perf_counter()
    A = read_mtx(args.a, device=comm.device)
    B = A.transpose() if args.aat else read_mtx(args.b, device=comm.device)
    lo, hi = row_panels(A.m, comm.world)[comm.rank]
    Ap = A.row_slice(lo, hi)
    blo, bhi = row_panels(B.m, comm.world)[comm.rank]
    Bp = B.row_slice(blo, bhi)
    del A, B
    _sync(comm)
    t_load = time.perf_counter() - t0
    comm.barrier()
    t1 = time.perf_counter()
    info = SpgemmInfo()
    Bfull = allgather_csr_rows(Bp, comm)
    Cp = spgemm(Ap, Bfull, info)
    _sync(comm)
    t_mult = comm.allreduce_max(time.perf_counter() - t1)
    flops = info.flops
    if comm.is_dist:
        import torch.distributed as dist

        t = torch.tensor([float(flops)], dtype=torch.float64,
                         device=comm.device if comm.backend == "nccl" else "cpu")
        dist.all_reduce(t)
        flops = int(t.item())
    C = gather_rows(Cp, comm) if args.output else None
    t2 = time.perf_counter()
    if comm.rank == 0 and args.output:
        write_mtx(args.output, C)
    t_write = time.perf_counter() - t2
    if comm.rank == 0:
        print(json.dumps(dict(op="spgemm", ranks=comm.world, device=str(comm.device), m=Ap.m if comm.world == 1 else None,
                              nnz_C=(C.nnz if C is not None else None), flops=flops, t_load_s=t_load,
                              t_mult_s=t_mult, t_write_s=t_write, gflops=flops / t_mult / 1e9 if t_mult > 0 else None)))
    comm.close()
    return 0


def cmd_gen(args) -> int:
    import torch

    from ..utils import gen_csr
    from ..utils.mtx import write_mtx

    dev = torch.device(args.device if args.device != "auto" else ("cuda" if torch.cuda.is_available() else "cpu"))
    if args.kind == "uniform":
        M = gen_csr.uniform_csr(args.n, args.n if args.cols is None else args.cols, args.density, seed=args.seed,
                                device=dev)
    else:
        M = gen_csr.rmat_csr(args.scale, args.edge_factor, seed=args.seed, device=dev)
    write_mtx(args.output, M)
    print(json.dumps(dict(kind=args.kind, m=M.m, n=M.n, nnz=M.nnz, path=args.output)))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="spgemm", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    m = sub.add_parser("mult")
    m.add_argument("a")
    m.add_argument("b", nargs="?")
    m.add_argument("--aat", action="store_true")
    m.add_argument("-o", "--output")
    m.add_argument("--device", default="auto")
    m.add_argument("--comm", default="auto")
    g = sub.add_parser("gen")
    g.add_argument("kind", choices=["uniform", "rmat"])
    g.add_argument("--n", type=int, default=1024)
    g.add_argument("--cols", type=int)
    g.add_argument("--density", type=float, default=0.01)
    g.add_argument("--scale", type=int, default=10)
    g.add_argument("--edge-factor", type=int, default=16)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--device", default="auto")
    g.add_argument("-o", "--output", required=True)
    args = ap.parse_args(argv)
    if args.cmd == "mult":
        if not args.aat and not args.b:
            ap.error("mult needs B (or --aat)")
        return cmd_mult(args)
    return cmd_gen(args)


if __name__ == "__main__":
    sys.exit(main())
