"""diagnostic: the test's exact sequence, z snapshots around each sub-step"""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
import spmm_amd  # noqa
from spmm_amd.models import spgemm as MS
from spmm_amd.ops import spgemm as SG, csr as CS
from spmm_amd.parallel.loopback import PanelComm
from spmm_amd.utils import gen_csr
dev = torch.device("cuda")
world = 2
m, k, n = 4000, 20000, 300000
A = gen_csr.uniform_csr(m, k, 0.002, seed=95)
B = gen_csr.uniform_csr(k, n, 2.7e-4, seed=96)
rc = [0] + [m * (r + 1) // world for r in range(world)]
kc = [0] + [k * (r + 1) // world for r in range(world)]
zs = lambda g: g.bufs["z"].tolist()
for r in range(world):
    panels = [B.row_slice(kc[q], kc[q + 1]).to(dev) for q in range(world)]
    Ap = A.row_slice(rc[r], rc[r + 1]).to(dev)
    g = MS.RowblockGraph(Ap, panels[r], PanelComm(r, world, dev, panels))
    print("rank", r, "z ptr", hex(g.bufs["z"].data_ptr()), "uoff", hex(g.bufs["uoff"].data_ptr()), flush=True)
    for s in (1.0, -2.0, 3.0):
        for q in range(world):
            panels[q].val.mul_(s)
        print(f" s={s} before run z={zs(g)}", flush=True)
        g.run()
        print(f"   after run z={zs(g)}", flush=True)
        info = SG.SpgemmInfo()
        C = g.result(info)
        print(f"   result None? {C is None} z={zs(g)}", flush=True)
        ri = SG.SpgemmInfo()
        ref = SG.spgemm(A.to(dev), CS.CSR(k, n, B.rowptr.to(dev), torch.cat([p.col for p in panels]),
                                          torch.cat([p.val for p in panels])), ri).row_slice(rc[r], rc[r + 1])
        torch.cuda.synchronize()
        print(f"   after ref z={zs(g)} ref path {ri.rows_per_bin_num}", flush=True)
