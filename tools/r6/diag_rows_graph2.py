"""65536^2 cfg 1 on the row kernel: (a) SpgemmGraph replays after value changes, (b) RowblockGraph EAGER
steps (no replay) after value changes, each vs the eager product (diagnostic)."""
import os
import socket
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.parallel import comm as CM  # noqa: E402


def report(tag, C1, C2, z):
    torch.cuda.synchronize()
    same = torch.equal(C1.rowptr, C2.rowptr) and torch.equal(C1.col, C2.col)
    bad = ~torch.isclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    rows = torch.searchsorted(C1.rowptr, bad.nonzero().flatten(), right=True) - 1
    ur = torch.unique(rows)
    print(f"{tag}: struct {same} z={z} bad entries {int(bad.sum())} rows {ur.numel()} first {ur[:6].tolist()} "
          f"last {ur[-3:].tolist()}", flush=True)


s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
os.environ.update(SPMM_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                  LOCAL_RANK="0")
comm = CM.init(backend="nccl", device="cuda")
prob = MS.UniformProblem.build(65536, 1e-3, comm, seed=5)
va, vb = prob.A.val.clone(), prob.B.val.clone()
mode = sys.argv[1]
if mode == "a":
    g = SG.SpgemmGraph(prob.A, prob.B)
    print("plan rows", g.plan.raw.rows, "cfg", g.plan.raw.cfg, flush=True)
    for sc in (1.0, -0.5, 2.0):
        prob.A.val.copy_(va * sc)
        prob.B.val.copy_(vb * (sc + 1.0))
        g.run()
        report(f"a s={sc} replay", g.result(), SG.spgemm(prob.A, prob.B), g.out["z"].tolist())
else:
    g = MS.RowblockGraph(prob.A, prob.B, comm)
    print("plan rows", g.plan.raw.rows, "cfg", g.plan.raw.cfg, "gview", g.gview is not None, flush=True)
    for sc in (1.0, -0.5, 2.0):
        prob.A.val.copy_(va * sc)
        prob.B.val.copy_(vb * (sc + 1.0))
        g._step(None, None)
        report(f"b s={sc} eager step", g.result(), SG.spgemm(prob.A, prob.B), g.bufs["z"].tolist())
comm.close()
