"""RowblockGraph: z after graph 1 in the normal step order (payloads, gathers, graph 1), with and without
writing z from the host first (diagnostic; graph 2 is never replayed here)."""
import os
import socket
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.parallel import comm as CM  # noqa: E402

s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
os.environ.update(SPMM_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                  LOCAL_RANK="0")
comm = CM.init(backend="nccl", device="cuda")
n, d = int(sys.argv[1]), float(sys.argv[2])
prob = MS.UniformProblem.build(n, d, comm, seed=5)
g = MS.RowblockGraph(prob.A, prob.B, comm)
z = g.bufs["z"]
print(n, "cfg", g.plan.raw.cfg, "z ptr", hex(z.data_ptr()), "uoff ptr", hex(g.bufs["uoff"].data_ptr()),
      "ws ptr", hex(g.bufs["ws"].data_ptr()), "ws bytes", g.bufs["ws"].numel(), flush=True)


def front_only(tag):
    g._col_payload(g.Bp, g.cb)
    g._val_payload(g.Bp, g.vb)
    wc = g.comm.all_gather_into(g.gc, g.cb)
    wv = g.comm.all_gather_into(g.gv, g.vb)
    wc()
    g.g1.replay()
    wv()
    torch.cuda.synchronize()
    print(n, tag, z.tolist(), flush=True)


front_only("normal order, z as left by the eager step:")
front_only("again:")
z.fill_(5)
torch.cuda.synchronize()
front_only("after z.fill_(5):")
g.g1.replay()
torch.cuda.synchronize()
print(n, "bare graph-1 replay:", z.tolist(), flush=True)
comm.close()
