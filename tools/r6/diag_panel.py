"""diagnostic: RowblockGraph through PanelComm as in test_rowblock_graph_panel_comm, with checks"""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
import spmm_amd  # noqa
from spmm_amd.models import spgemm as MS
from spmm_amd.ops import spgemm as SG, csr as CS
from spmm_amd.parallel.loopback import PanelComm
from spmm_amd.utils import gen_csr
dev = torch.device("cuda")
world = int(os.environ.get("W", "2"))
m, k, n = 4000, 20000, 300000
A = gen_csr.uniform_csr(m, k, 0.002, seed=95)
B = gen_csr.uniform_csr(k, n, 2.7e-4, seed=96)
rc = [0] + [m * (r + 1) // world for r in range(world)]
kc = [0] + [k * (r + 1) // world for r in range(world)]
if world >= 3:
    kc[2] = kc[1]
for r in range(world):
    panels = [B.row_slice(kc[q], kc[q + 1]).to(dev) for q in range(world)]
    Ap = A.row_slice(rc[r], rc[r + 1]).to(dev)
    g = MS.RowblockGraph(Ap, panels[r], PanelComm(r, world, dev, panels))
    torch.cuda.synchronize()
    print("rank", r, "after build z", g.bufs["z"].tolist(), flush=True)
    for s in (1.0, -2.0, 1.0, 0.5):
        for q in range(world):
            panels[q].val.mul_(s)
        torch.cuda.synchronize()
        g.run()
        torch.cuda.synchronize()
        z = g.bufs["z"].tolist()
        Bfull_col = torch.cat([p.col for p in panels]); Bfull_val = torch.cat([p.val for p in panels])
        ok_col = torch.equal(g.B.col, Bfull_col); ok_val = torch.equal(g.B.val, Bfull_val)
        print(f" s={s}: z={z} B.col ok {ok_col} B.val ok {ok_val} nnz={int(g.bufs['uoff'][-1])}", flush=True)
