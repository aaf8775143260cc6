"""CSR SpGEMM / SpMM command line (north-star configs).

    # C = A . B from Matrix Market files (one process, or torchrun P ranks: each
    # rank parses 1/P of the files, 1D row-block, B all-gathered over RCCL, C
    # streamed to rank 0 point-to-point and written as it arrives)
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
    """Every rank parses 1/P of each input file and gets its row panel by an
    all-to-all-v shuffle (``read_mtx_rowblock``); B (or A^T, by a distributed
    transpose) is all-gathered inside the multiply; C's panels are streamed
    to rank 0 point-to-point and appended to the output file as they arrive."""
    import torch

    from ..models import spgemm as MS
    from ..ops.spgemm import SpgemmInfo
    from ..parallel import comm as CM

    comm = CM.init(backend=args.comm, device=args.device)
    t0 = time.perf_counter()
    Ap, row0, cuts = MS.read_mtx_rowblock(args.a, comm)
    if args.aat:
        Bp, _ = MS.transpose_rowblock(Ap, row0, cuts[-1], comm)
    else:
        Bp, _, bcuts = MS.read_mtx_rowblock(args.b, comm)
        if bcuts[-1] != Ap.n:
            raise SystemExit(f"inner dimensions differ: A has {Ap.n} columns, B has {bcuts[-1]} rows")
    _sync(comm)
    t_load = comm.allreduce_max(time.perf_counter() - t0)
    comm.barrier()
    t1 = time.perf_counter()
    info = SpgemmInfo()
    Cp = MS.rowblock_spgemm(Ap, Bp, comm, info)
    _sync(comm)
    t_mult = comm.allreduce_max(time.perf_counter() - t1)
    flops, nnz_c = info.flops, Cp.nnz
    if comm.is_dist:
        flops, nnz_c = sum(comm.gather_ints(flops)), sum(comm.gather_ints(nnz_c))
    t2 = time.perf_counter()
    if args.output:
        MS.write_rows_p2p(args.output, Cp, row0, comm)
    t_write = comm.allreduce_max(time.perf_counter() - t2)
    if comm.rank == 0:
        print(json.dumps(dict(op="spgemm", ranks=comm.world, device=str(comm.device), m=cuts[-1], n=Cp.n,
                              nnz_C=nnz_c, flops=flops, t_load_s=t_load, t_mult_s=t_mult, t_write_s=t_write,
                              gflops=flops / t_mult / 1e9 if t_mult > 0 else None)))
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
