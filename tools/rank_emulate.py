"""Per-rank cost of the row-block SpGEMM step at world size N, on one GPU.

Builds exactly what rank r of an N-GPU run holds (A's row panel r; every
rank's B row panel) and times:

* ``local_ms``: the local product against the full B (``spgemm(A_panel, B)``,
  eager, or ``--graph``: a SpgemmGraph replay) -- the step without the gather;
* ``step_ms[gbps]`` (``--gather-gbps 0,300,...``): the whole rank-r step of
  ``bench.py`` at N ranks, i.e. ``models.spgemm.RowblockGraph.run`` (pack
  of the own panel into the send buffers, column gather, graph 1 = unpack +
  B layouts + count kernel, value gather, graph 2 = unpack + padded pairs +
  numeric), through ``parallel.loopback.PanelComm``: every rank's payload is
  built from its panel on a "link" stream while a "wire" stream runs a
  stream-ordered delay of (bytes this rank receives) / gbps per payload, in
  RCCL's issue order (columns, then values); a payload is readable when
  both are done, i.e. when a link of that rate would deliver it, and the
  count kernel overlaps the value transfer as on the real node.  Not
  modelled: the CUs RCCL's own kernels take while they run.  0 = delay-free
  (the payload writes only).
* ``step_ms_link[gbps]``: the same step with the payloads written once
  (``PanelComm(prefill=True)``): the link delay alone, as on a node where
  the peers push the bytes and this GPU's CUs copy none of them (the
  ``step_ms`` model charges this GPU for writing all N payloads every step).

    python tools/rank_emulate.py --world 8 [--rank 0] [--gather-gbps 0,150,300]
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
from spmm_amd.ops.spgemm import SpgemmGraph, SpgemmInfo, spgemm  # noqa: E402
from spmm_amd.parallel.loopback import PanelComm  # noqa: E402
from spmm_amd.parallel.partition import row_panels  # noqa: E402
from spmm_amd.utils.gen_csr import uniform_csr  # noqa: E402

def timed(fn, steps: int) -> float:
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--density", type=float, default=1e-4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--graph", action="store_true", help="time the local product as a SpgemmGraph replay")
    ap.add_argument("--gather-gbps", default="", help="comma list: emulate the whole step at these link rates")
    ap.add_argument("--no-local", action="store_true", help="skip the local-product timings")
    ap.add_argument("--link-priority", type=int, default=0,
                    help="stream priority of the emulated link (-1: high, dispatched ahead of the compute grids)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    _native.hip()
    pan = row_panels(a.n, a.world)
    lo, hi = pan[a.rank]
    A = uniform_csr(a.n, a.n, a.density, seed=a.seed, device=dev, rows=(lo, hi))
    rec = dict(world=a.world, rank=a.rank, rows=hi - lo)
    if not a.no_local:
        B = uniform_csr(a.n, a.n, a.density, seed=a.seed + 1, device=dev)
        info = SpgemmInfo()
        C = spgemm(A, B, info)
        del C
        rec.update(flops=info.flops, nnz_C=info.nnz)
        run = (lambda: spgemm(A, B)) if not a.graph else SpgemmGraph(A, B).run
        rec.update(graph=a.graph, local_ms=round(timed(run, a.steps), 3))
        rec["gflops_local"] = round(info.flops / rec["local_ms"] / 1e6, 1)
        rec["allgather_recv_bytes"] = int((a.world - 1) / a.world * (B.nnz * 8))
        del B, run
        torch.cuda.empty_cache()
    if a.gather_gbps:
        panels = [uniform_csr(a.n, a.n, a.density, seed=a.seed + 1, device=dev, rows=p) for p in pan]
        steps = {}
        link = {}
        keep = []   # (graphs stay alive until the end: see tests/test_dist_device.py _graph_case_panels)
        for g in [float(x) for x in a.gather_gbps.split(",")]:
            for prefill, d in ((False, steps), (True, link)):
                comm = PanelComm(a.rank, a.world, dev, panels, g, link_priority=a.link_priority, prefill=prefill)
                rg = MS.RowblockGraph(A, panels[a.rank], comm)
                d[str(g)] = round(timed(rg.run, a.steps), 3)
                C = rg.result()
                rec.setdefault("step_nnz_C", C.nnz)
                if C.nnz != rec["step_nnz_C"]:
                    raise RuntimeError("emulated steps disagree on nnz(C)")
                keep.append(rg)
                del C
        rec["step_ms"] = steps
        rec["step_ms_link"] = link
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
