import sys, time, json, os
sys.path.insert(0, "/root/repo")
import torch
import spmm_amd
from spmm_amd import _native
from spmm_amd.ops import spgemm as SG
from spmm_amd.utils.config import CONFIG
from spmm_amd.utils.gen_csr import uniform_csr
from spmm_amd.parallel.partition import row_panels
dev = torch.device("cuda"); _native.hip()
n = 1 << 20
B = uniform_csr(n, n, 1e-4, seed=2, device=dev)
for w in (2, 4):
    lo, hi = row_panels(n, w)[0]
    A = uniform_csr(n, n, 1e-4, seed=1, device=dev, rows=(lo, hi))
    for mode in ("on", "off"):
        CONFIG.spgemm_ordered = mode
        info = SG.SpgemmInfo(); C = SG.spgemm(A, B, info); del C
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(3):
            C = SG.spgemm(A, B); del C
        torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 3
        print(json.dumps(dict(world=w, ordered=mode, ms=round(dt * 1e3, 1), bins={str(k): v for k, v in info.rows_per_bin_num.items()})), flush=True)
