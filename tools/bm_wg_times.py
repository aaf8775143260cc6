"""Per-workgroup timeline of the pipelined bitmap numeric kernel (stamps build):
when every persistent workgroup starts and ends its row loop, on the 100 MHz
real-time counter, for rank r's A row panel of a W-rank 1M step against the
full B.  Answers "ramp, tail or rate?" for the row-block step's numeric
kernel.

    python tools/bm_wg_times.py [--world 8] [--rank 0] [--n 1048576] [--density 1e-4]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spmm_amd import _build  # noqa: E402

_lib = os.path.join(_build.LIB_DIR, "diag", "libspmm_hip_stamps.so")
if os.environ.get("SPMM_STAMPS_PREBUILT") and os.path.exists(_lib):
    os.environ["SPMM_HIP_LIB"] = _lib
else:
    os.environ["SPMM_HIP_LIB"] = _build.build_hip(out=_lib, extra=["-DSPMM_BM_STAMPS"])

import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _native  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.parallel.partition import row_panels  # noqa: E402
from spmm_amd.utils.gen_csr import uniform_csr  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--density", type=float, default=1e-4)
    a = ap.parse_args()
    dev = torch.device("cuda")
    lo, hi = row_panels(a.n, a.world)[a.rank]
    A = uniform_csr(a.n, a.n, a.density, seed=1, device=dev, rows=(lo, hi))
    B = uniform_csr(a.n, a.n, a.density, seed=2, device=dev)
    lib = _native.hip()
    SG.spgemm(A, B)
    torch.cuda.synchronize()
    lib.spmm_spgemm_bm_wg_times(1, None, 0)
    lib.spmm_spgemm_bm_stamps(1, None)
    SG.spgemm(A, B)
    torch.cuda.synchronize()
    nmax = 8192
    buf = (C.c_ulonglong * (3 * nmax))()
    lib.spmm_spgemm_bm_wg_times(0, buf, nmax)
    lib.spmm_spgemm_bm_stamps(0, None)
    rows = [(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(nmax) if buf[3 * i + 1]]
    t0 = min(r[0] for r in rows)
    us = lambda t: (t - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
    starts = [us(r[0]) for r in rows]
    ends = [us(r[1]) for r in rows]
    busy = [e - s for s, e in zip(starts, ends)]
    units = [r[2] & 0xFFFFFFFF for r in rows]
    xcd = {}
    for (s, e, x) in rows:
        xcd.setdefault(x >> 32, []).append(us(e))
    rec = dict(world=a.world, rank=a.rank, rows=hi - lo, workgroups=len(rows),
               start_us=dict(max=round(max(starts), 1), p50=round(pct(starts, 0.5), 1)),
               end_us=dict(min=round(min(ends), 1), p10=round(pct(ends, 0.1), 1), p50=round(pct(ends, 0.5), 1),
                           p90=round(pct(ends, 0.9), 1), max=round(max(ends), 1)),
               busy_us_mean=round(sum(busy) / len(busy), 1),
               units=dict(min=min(units), max=max(units), mean=round(sum(units) / len(units), 1)),
               tail_share=round(1 - (sum(busy) / len(busy)) / max(ends), 4),
               xcd_end_us={str(k): dict(n=len(v), mean=round(sum(v) / len(v), 1), max=round(max(v), 1))
                           for k, v in sorted(xcd.items())})
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
