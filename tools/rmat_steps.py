"""R-MAT A.A^T: build the problem, run K streamed steps (consume = count nnz only, as the
timed bench step), print ms per step.  For kernel profiles of the step alone (no setup
checksum).  usage: python tools/rmat_steps.py [scale] [steps]"""
import sys
import time

import torch

import os  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import spmm_amd  # noqa: F401,E402
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.parallel import comm as CM  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
comm = CM.init(backend="auto", device="auto")
if comm.device.type == "cuda":   # the side stream first (see bench.py)
    from spmm_amd.ops import spgemm as SG  # noqa: E402

    SG._side_stream(comm.device)
sync = torch.cuda.synchronize if comm.device.type == "cuda" else (lambda: None)
t = time.time()
prob = MS.RmatProblem.build(scale, 16, comm, seed=1)
sync()
print(f"build {time.time() - t:.1f} s", flush=True)
for s in range(steps):
    nnz = [0]

    def consume(_lo, _hi, C):
        nnz[0] += C.nnz

    sync()
    t = time.time()
    prob.step(comm, None, consume, overlap=os.environ.get("RMAT_OVERLAP", "1") == "1")
    sync()
    print(f"step {s}: {(time.time() - t) * 1e3:.1f} ms nnz {nnz[0]}", flush=True)
