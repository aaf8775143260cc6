"""RowblockGraph at 65536^2 (one-rank RCCL group): replays after value changes vs eager;
prints the mismatching rows and the kernels' z words (diagnostic)."""
import os
import socket

import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd.models import spgemm as MS
from spmm_amd.ops import spgemm as SG
from spmm_amd.parallel import comm as CM

s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
os.environ.update(SPMM_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                  LOCAL_RANK="0")
comm = CM.init(backend="nccl", device="cuda")
prob = MS.UniformProblem.build(65536, 1e-3, comm, seed=5)
g = MS.RowblockGraph(prob.A, prob.B, comm)
print("plan rows", g.plan.raw.rows, "cfg", g.plan.raw.cfg, "gview", g.gview is not None, flush=True)
va, vb = prob.A.val.clone(), prob.B.val.clone()
for sc in (1.0, -0.5, 2.0):
    prob.A.val.copy_(va * sc)
    prob.B.val.copy_(vb * (sc + 1.0))
    for mode in ("replay", "eager"):
        if mode == "replay":
            g.run()
        else:
            g._step(None, None)
        C1 = g.result()
        C2 = SG.spgemm(prob.A, prob.B)
        z = g.bufs["z"].tolist()
        bad = ~torch.isclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
        rows = torch.searchsorted(C1.rowptr, bad.nonzero().flatten(), right=True) - 1
        ur = torch.unique(rows)
        print(f"s={sc} {mode}: z={z} bad entries {int(bad.sum())} rows {ur.numel()} "
              f"first {ur[:8].tolist()} last {ur[-4:].tolist()}", flush=True)
comm.close()
