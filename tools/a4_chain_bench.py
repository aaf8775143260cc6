"""Native Matrix-Market chain (a4 --format mtx --device hip) against the Python front end on
the same products: per-product wall time of both (device products only: upload, gather,
file parse and output excluded on both sides).

    python tools/a4_chain_bench.py [--n 1048576] [--nnz-row 6] [--mats 3] [--dir /tmp/a4c] [--reps 2]

Prints one JSON line: the products' intermediate-product counts, the native and Python
seconds per product (best of --reps runs), and their ratio.  BASELINE-style config: a chain
of uniform n x n matrices, fp32 (the reference's CLI workload shape, sparse_matrix_mult.cu:402-681).
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _build  # noqa: E402
from spmm_amd.ops.spgemm import SpgemmInfo, spgemm  # noqa: E402
from spmm_amd.utils import mtx  # noqa: E402
from spmm_amd.utils.gen_csr import uniform_csr  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--nnz-row", type=float, default=6.0)
    ap.add_argument("--mats", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/a4c")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    os.makedirs(a.dir, exist_ok=True)
    dens = a.nnz_row / a.n
    mats = [uniform_csr(a.n, a.n, dens, seed=100 + i, device=dev) for i in range(a.mats)]
    for i, M in enumerate(mats):
        mtx.write_mtx(os.path.join(a.dir, f"m{i + 1}.mtx"), M.to("cpu"))
    print(f"wrote {a.mats} matrices of {mats[0].nnz} entries", file=sys.stderr, flush=True)
    a4 = os.path.join(_build.BIN_DIR, "a4")
    mpiexec = os.path.join(_build.mpi_home(), "bin", "mpiexec")
    native = None
    for _ in range(a.reps):
        met = os.path.join(a.dir, "met.json")
        subprocess.run([mpiexec, "-n", "1", a4, a.dir, "--format", "mtx", "--device", "hip", "--out", "/dev/null",
                        "--quiet", "--metrics-json", met], check=True, timeout=900)
        m = json.load(open(met))
        t = m["t_products_s"]
        native = t if native is None else [min(x, y) for x, y in zip(native, t)]
    info_n = m
    # Python front end on the same matrices (eager spgemm: row plan + product, as the a4 engine)
    py, prods = None, []
    for rep in range(a.reps):
        P, ts = mats[0], []
        for B in mats[1:]:
            info = SpgemmInfo()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            C = spgemm(P, B, info)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            if rep == 0:
                prods.append(info.flops // 2)
            P = C
        del P
        torch.cuda.empty_cache()
        py = ts if py is None else [min(x, y) for x, y in zip(py, ts)]
    out = dict(config=dict(n=a.n, nnz_row=a.nnz_row, mats=a.mats, dtype="fp32"), products=prods,
               native_s=[round(x, 5) for x in native], python_s=[round(x, 5) for x in py],
               native_over_python=[round(x / y, 3) for x, y in zip(native, py)],
               native_total_over_python=round(sum(native) / sum(py), 3),
               native_metrics={k: info_n[k] for k in ("gpu_bitmap_products", "gpu_binned_products", "host_resorted_rows",
                                                      "device_sorted_rows", "cpu_products")})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
