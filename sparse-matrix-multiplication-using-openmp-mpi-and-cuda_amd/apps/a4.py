"""Drop-in replacement for the reference binary ``a4`` (sparse_matrix_mult.cu:402-681).

    mpirun -np P python -m spmm_amd.apps.a4 <folder>            # MPI launcher
    torchrun --nproc-per-node P -m spmm_amd.apps.a4 <folder>    # torch launcher
    python -m spmm_amd.apps.a4 <folder>                         # one process

Same inputs (``<folder>/size``, ``<folder>/matrix1..N``), same output
(``./matrix`` in the current directory, byte-identical to the reference for
the same P), same stdout lines (``multiplying <i> <i+1>`` per product and
``time taken <s> seconds`` on every rank, clock started before process-group
init and stopped after teardown as in :403/:677-679).

Extra options (all optional; env equivalents SPMM_*):
  --out PATH          output file (default ./matrix)
  --device cuda|cpu   compute device (default: cuda when present)
  --comm nccl|gloo    process-group backend (default: nccl on GPU, gloo on CPU)
  --threads N         host parser/writer threads (default: all)
  --quiet             suppress the "multiplying" lines
  --metrics-json PATH per-rank phase times, bytes moved and throughput
  --no-split          cross-rank tree products on one rank each (default: each
                      product is row-panel split over the ranks of its group)
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
    ap.add_argument("folder")
    ap.add_argument("--out", default=os.environ.get("SPMM_OUT", "matrix"))
    ap.add_argument("--device", default=os.environ.get("SPMM_DEVICE", "auto"))
    ap.add_argument("--comm", default=os.environ.get("SPMM_COMM", "auto"))
    ap.add_argument("--threads", type=int, default=int(os.environ.get("SPMM_THREADS", "0")))
    ap.add_argument("--quiet", action="store_true", default=bool(os.environ.get("SPMM_QUIET")))
    ap.add_argument("--metrics-json", default=os.environ.get("SPMM_METRICS_JSON"))
    ap.add_argument("--no-split", action="store_true", default=bool(os.environ.get("SPMM_NO_SPLIT")))
    args = ap.parse_args(argv)

    import torch  # noqa: F401  (after argparse so --help is instant)

    from ..models.chain import ChainStats, run_chain
    from ..parallel import comm as commmod
    from ..utils import refio

    comm = commmod.init(backend=args.comm, device=args.device)
    stats = ChainStats()
    rc = 0
    try:
        log = None if args.quiet else (lambda s: print(s, flush=True))
        run_chain(args.folder, comm, out_path=args.out, log=log, nthreads=args.threads, stats=stats,
                  split=not args.no_split)
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


if __name__ == "__main__":
    sys.exit(main())
