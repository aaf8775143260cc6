"""Drop-in replacement for the reference binary ``a4`` (sparse_matrix_mult.cu:402-681).

    mpirun -np P python -m spmm_amd.apps.a4 <folder>            # MPI launcher
    torchrun --nproc-per-node P -m spmm_amd.apps.a4 <folder>    # torch launcher
    python -m spmm_amd.apps.a4 <folder>                         # one process

Same inputs (``<folder>/size``, ``<folder>/matrix1..N``), same output
(``./matrix`` in the current directory, byte-identical to the reference for
the same P), same stdout lines (``multiplying <i> <i+1>`` per product and
``time taken <s> seconds`` on every rank, clock started before process-group
init and stopped after teardown as in :403/:677-679).

Matrix Market chains (CSR engine, fp32, same launchers and stdout lines):

    python -m spmm_amd.apps.a4 --format mtx M1.mtx M2.mtx [M3.mtx ...]
    python -m spmm_amd.apps.a4 --format mtx <folder of *.mtx, natural order>

Extra options (all optional; env equivalents SPMM_*):
  --format ref|mtx    input format (default ref: the reference folder format)
  --out PATH          output file (default ./matrix, ./matrix.mtx for mtx)
  --device cuda|cpu   compute device (default: cuda when present)
  --comm nccl|gloo|loopback
                      process-group backend (default: nccl on GPU, gloo on CPU);
                      loopback runs --ranks P ranks as threads of this process
  --threads N         host parser/writer threads (default: all)
  --streams N         concurrent products per tree level on the GPU (default 4,
                      as the native a4)
  --quiet             suppress the "multiplying" lines
  --metrics-json PATH per-rank phase times, bytes moved and throughput
  --no-split          cross-rank tree products on one rank each (default: each
                      product is row-panel split over the ranks of its group)
  --exact / --fast    chain split: the reference's count split (default, bit-exact
                      by construction) or ranges balanced on the files' sizes
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None) -> int:
    t_start = time.perf_counter()
    ap = argparse.ArgumentParser(prog="a4", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("inputs", nargs="+", metavar="folder", help="reference folder (or, with --format mtx, the "
                    "chain's .mtx files / a folder of them)")
    ap.add_argument("--format", choices=["ref", "mtx"], default=os.environ.get("SPMM_FORMAT", "ref"))
    ap.add_argument("--out", default=os.environ.get("SPMM_OUT"))
    ap.add_argument("--device", default=os.environ.get("SPMM_DEVICE", "auto"))
    ap.add_argument("--comm", default=os.environ.get("SPMM_COMM", "auto"))
    ap.add_argument("--threads", type=int, default=int(os.environ.get("SPMM_THREADS", "0")))
    ap.add_argument("--streams", type=int, default=int(os.environ.get("SPMM_STREAMS", "4")))
    ap.add_argument("--ranks", type=int, default=int(os.environ.get("SPMM_RANKS", "1")),
                    help="--comm loopback: in-process ranks")
    ap.add_argument("--quiet", action="store_true", default=bool(os.environ.get("SPMM_QUIET")))
    ap.add_argument("--metrics-json", default=os.environ.get("SPMM_METRICS_JSON"))
    ap.add_argument("--no-split", action="store_true", default=bool(os.environ.get("SPMM_NO_SPLIT")))
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--fast", action="store_true", default=bool(os.environ.get("SPMM_FAST")))
    g.add_argument("--exact", dest="fast", action="store_false")
    args = ap.parse_args(argv)
    if args.format == "ref" and len(args.inputs) != 1:
        ap.error("the reference format takes one folder")
    args.folder = args.inputs[0]
    if args.out is None:
        args.out = "matrix.mtx" if args.format == "mtx" else "matrix"

    import torch  # noqa: F401  (after argparse so --help is instant)

    if args.format == "mtx":
        return _main_mtx(args, t_start)
    if args.comm == "loopback":
        return _main_loopback(args, t_start)

    from ..models.chain import ChainStats, run_chain
    from ..parallel import comm as commmod
    from ..utils import refio

    comm = commmod.init(backend=args.comm, device=args.device)
    stats = ChainStats()
    rc = 0
    try:
        log = None if args.quiet else (lambda s: print(s, flush=True))
        run_chain(args.folder, comm, out_path=args.out, log=log, nthreads=args.threads, stats=stats,
                  split=not args.no_split, fast=args.fast, streams=max(1, args.streams))
    except refio.FormatError as e:
        print(str(e), file=sys.stderr)
        rc = 1
    finally:
        comm.close()
    elapsed = time.perf_counter() - t_start
    print(f"time taken {elapsed} seconds", flush=True)
    if args.metrics_json and rc == 0:
        try:
            k = refio.read_size(args.folder)[1]
        except refio.FormatError:
            k = 0
        rec = dict(rank=comm.rank, world=comm.world, device=str(comm.device), split=not args.no_split, wall_s=elapsed,
                   **stats.as_dict(k))
        path = args.metrics_json if comm.world == 1 else f"{args.metrics_json}.rank{comm.rank}"
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
    return rc


def _main_loopback(args, t_start: float) -> int:
    """P ranks as threads of this process (parallel/loopback.py): the same
    chain split, cross-rank tree and output as P processes."""
    import torch

    from ..models.chain import ChainStats, run_chain
    from ..parallel.loopback import run_loopback
    from ..utils import refio

    dev = args.device if args.device != "auto" else ("cuda" if torch.cuda.is_available() else "cpu")
    log = None if args.quiet else (lambda s: print(s, flush=True))

    def rank_main(comm):
        st = ChainStats()
        run_chain(args.folder, comm, out_path=args.out, log=log, nthreads=args.threads, stats=st,
                  split=not args.no_split, fast=args.fast, streams=max(1, args.streams))
        return st

    try:
        run_loopback(max(1, args.ranks), rank_main, device=dev)
    except refio.FormatError as e:
        print(str(e), file=sys.stderr)
        return 1
    elapsed = time.perf_counter() - t_start
    for _ in range(max(1, args.ranks)):   # one line per rank, as P processes print
        print(f"time taken {elapsed} seconds", flush=True)
    return 0


def _mtx_paths(inputs):
    import re

    if len(inputs) == 1 and os.path.isdir(inputs[0]):
        names = [f for f in os.listdir(inputs[0]) if f.endswith(".mtx")]
        key = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]  # noqa: E731
        return [os.path.join(inputs[0], f) for f in sorted(names, key=key)]
    return list(inputs)


def _main_mtx(args, t_start: float) -> int:
    from ..models.spgemm import csr_chain
    from ..ops.spgemm import SpgemmInfo
    from ..parallel import comm as commmod
    from ..utils.mtx import MtxError

    comm = commmod.init(backend=args.comm, device=args.device)
    rc = 0
    info = SpgemmInfo()
    t_mult = 0.0
    try:
        paths = _mtx_paths(args.inputs)
        log = None if args.quiet else (lambda s: print(s, flush=True))
        t0 = time.perf_counter()
        csr_chain(paths, comm, out_path=args.out, log=log, info=info)
        t_mult = time.perf_counter() - t0
    except (MtxError, ValueError, OSError) as e:
        print(str(e), file=sys.stderr)
        rc = 1
    finally:
        comm.close()
    elapsed = time.perf_counter() - t_start
    print(f"time taken {elapsed} seconds", flush=True)
    if args.metrics_json and rc == 0:
        rec = dict(rank=comm.rank, world=comm.world, device=str(comm.device), format="mtx", wall_s=elapsed,
                   t_chain_s=t_mult, flops_local=info.flops)
        path = args.metrics_json if comm.world == 1 else f"{args.metrics_json}.rank{comm.rank}"
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
    return rc


if __name__ == "__main__":
    sys.exit(main())
