"""RowblockGraph: does graph 1 (front) reset z on replay?  Replays graph 1 alone with sentinels in z
(no numeric kernel), then graph 2 only after z is zeroed by hand (diagnostic)."""
import os
import socket
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.parallel import comm as CM  # noqa: E402

s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
os.environ.update(SPMM_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                  LOCAL_RANK="0")
comm = CM.init(backend="nccl", device="cuda")
for n, d in ((int(sys.argv[1]), float(sys.argv[2])),):
    prob = MS.UniformProblem.build(n, d, comm, seed=5)
    g = MS.RowblockGraph(prob.A, prob.B, comm)
    z = g.bufs["z"]
    print(n, "plan rows", g.plan.raw.rows, "cfg", g.plan.raw.cfg, "gview", g.gview is not None,
          "z after eager", z.tolist(), "uoff[0]", int(g.bufs["uoff"][0]), flush=True)
    z.copy_(torch.tensor([0, 111, 222, 333], dtype=torch.int32, device=z.device))
    g.bufs["uoff"][0] = 444
    torch.cuda.synchronize()
    g.g1.replay()
    torch.cuda.synchronize()
    print(n, "z after graph-1 replay (sentinels 0,111,222,333; uoff[0] 444)", z.tolist(), int(g.bufs["uoff"][0]),
          flush=True)
    va, vb = prob.A.val.clone(), prob.B.val.clone()
    prob.A.val.copy_(va * 2.0)
    z.zero_()
    g._col_payload(g.Bp, g.cb)
    g._val_payload(g.Bp, g.vb)
    g.comm.all_gather_into(g.gc, g.cb)()
    g.comm.all_gather_into(g.gv, g.vb)()
    g.g1.replay()
    z.zero_()
    g.g2.replay()
    torch.cuda.synchronize()
    C1, C2 = g.result(), SG.spgemm(prob.A, prob.B)
    bad = ~torch.isclose(C1.val, C2.val, atol=1e-5, rtol=1e-5)
    print(n, "graph-2 replay with z zeroed by hand: bad", int(bad.sum()), "z", z.tolist(), flush=True)
comm.close()
