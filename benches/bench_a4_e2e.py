"""End-to-end benchmark of the native ``a4`` executable on report-sized inputs.

This is the reference's own headline measurement: report.pdf p.3 Table 1 times
the whole program (``mpirun -np 8 ./a4 <folder>``: parse the text files,
multiply the chain, write ``./matrix``) on Small / Medium / Large inputs of
10k / 100k / 1M k=32 tiles, 3.4 s / 32.1 s / 320.5 s on a P100 (CPU-only:
15.2 s / 152 s / 1530 s).  The report gives tile counts only, so the chain
shapes are ours (benches/bench_chain.py PRESETS: N matrices of a square tile
grid at a density that totals the stated tile count) and values are uniform
64-bit (the wrap regime, the slowest to parse and print).

The input folder is generated (device RNG when a GPU is visible) and written
with the native formatter; generation is not timed.  Then

    mpiexec -n P a4 <folder> --quiet --out <tmp>/matrix --metrics-json <tmp>/m.json

is timed by this script's own clock around the subprocess, and the program's
``time taken`` line (max over ranks, the reference's clock) and its phase
metrics are reported.

    python benches/bench_a4_e2e.py --preset medium [--p 1] [--device hip|cpu]

Several runs over the same generated input (comma lists, cartesian product):
the CPU-only column of report Table 1 and the thread scaling of Table 3
(1 rank, 100k tiles, 4 / 8 / 16 / 32 threads) come from

    python benches/bench_a4_e2e.py --preset medium --device hip,cpu
    python benches/bench_a4_e2e.py --preset medium --device cpu --threads 4,8,16,32
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benches"))

REPORT = {  # report.pdf p.3 Table 1: (tiles, optimized s, CPU-only s), P = 8 ranks x 16 threads, P100
    "small": (10_000, 3.4, 15.2),
    "medium": (100_000, 32.1, 152.0),
    "large": (1_000_000, 320.5, 1530.0),
}


def generate(folder: str, preset: str, seed: int, k: int = 32) -> dict:
    import torch

    from bench_chain import PRESETS, device_random_bsr
    from spmm_amd.utils import refio

    cfg = PRESETS[preset]
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    os.makedirs(folder, exist_ok=True)
    with open(os.path.join(folder, "size"), "w") as f:
        f.write(f"{cfg['n']} {k}\n")
    tiles = 0
    for i in range(1, cfg["n"] + 1):   # one matrix at a time: host memory stays small
        M = device_random_bsr(cfg["blocks"], k, cfg["density"], g, dev)
        tiles += M.nb
        refio.write_matrix(refio.matrix_path(folder, i), M.to("cpu"))
        del M
        print(f"[generate] matrix {i}/{cfg['n']} written", file=sys.stderr, flush=True)
    nbytes = sum(os.path.getsize(os.path.join(folder, f)) for f in os.listdir(folder))
    return dict(cfg, k=k, input_tiles=tiles, input_bytes=nbytes)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(REPORT), default="medium")
    ap.add_argument("--p", default="1", help="MPI ranks (one GPU each when GPUs are visible); comma list")
    ap.add_argument("--device", default="auto", help="auto / hip / cpu; comma list")
    ap.add_argument("--threads", default="0", help="a4 --threads (host parser/writer/CPU-engine threads; 0 = all); "
                    "comma list")
    ap.add_argument("--comm", default="auto")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--workdir", default=None, help="where the input folder goes (default: a temp dir)")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--json", default=None)
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--streams", type=int, default=None, help="a4 --streams (concurrent products per level)")
    a = ap.parse_args()

    from spmm_amd import _build

    a4 = _build.build_a4()
    if a4 is None:
        raise SystemExit("native a4 not built (no MPI headers)")
    mpiexec = os.path.join(_build.mpi_home(), "bin", "mpiexec")
    work = tempfile.mkdtemp(prefix="a4e2e_", dir=a.workdir)
    try:
        folder = os.path.join(work, "in")
        t0 = time.perf_counter()
        info = generate(folder, a.preset, a.seed)
        t_gen = time.perf_counter() - t0
        runs = [(d, int(p), int(t)) for d in a.device.split(",") for p in a.p.split(",") for t in a.threads.split(",")]
        recs = []
        for dev, nranks, threads in runs:
            out = os.path.join(work, "matrix")
            met = os.path.join(work, "m.json")
            cmd = [mpiexec, "-n", str(nranks), a4, folder, "--quiet", "--out", out, "--metrics-json", met,
                   "--device", dev, "--comm", a.comm, "--threads", str(threads)]
            if a.streams is not None:
                cmd += ["--streams", str(a.streams)]
            t0 = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout)
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
                raise SystemExit(f"a4 failed with {r.returncode}")
            taken = max(float(x) for x in re.findall(r"time taken ([0-9.eE+-]+) seconds", r.stdout))
            m = json.load(open(met))
            tiles_ref, t_opt, t_cpu = REPORT[a.preset]
            rec = dict(metric="a4 end-to-end wall-clock (report.pdf Table 1)", preset=a.preset, ranks=nranks,
                       threads=m.get("threads", threads), streams=a.streams, device=m.get("device"), comm=m.get("comm"),
                       value=round(taken, 3), unit="s", higher_is_better=False, wall_s_outer=round(wall, 3),
                       report_tiles=tiles_ref, report_optimized_s=t_opt, report_cpu_only_s=t_cpu,
                       speedup_vs_report=round(t_opt / taken, 2),
                       speedup_vs_report_cpu_only=round(t_cpu / taken, 2), output_bytes=os.path.getsize(out),
                       gen_s=round(t_gen, 2), **info, metrics=m)
            print(json.dumps(rec), flush=True)
            recs.append(rec)
        if a.json:
            with open(a.json, "w") as f:
                json.dump(recs if len(recs) > 1 else recs[0], f, indent=1)
    finally:
        if not a.keep:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
