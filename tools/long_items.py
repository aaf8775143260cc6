"""Item-size histogram of the long-row path on R-MAT A.A^T (one GPU):
python tools/long_items.py SCALE [MAX_ROWS].  Items are (row, column chunk)
pairs; long_rank takes items of <= 1024 products, long_dense the rest."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import spmm_amd  # noqa: F401,E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

scale = int(sys.argv[1])
max_rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
dev = torch.device("cuda")
A = gen_csr.rmat_csr(scale, 16, seed=1, device=dev)
At = A.transpose()
nprod = SG.row_nprod(A, At)
cap = SG.bin_caps(1)[10]
rows = (nprod > cap).nonzero().flatten()[:max_rows].to(torch.int32)
print(f"scale {scale}: total products {int(nprod.sum()):.4g}, long rows {rows.numel()}, "
      f"products in them {int(nprod[rows.long()].sum()):.4g}", flush=True)
lgw, epw, maxch = SG._long_params()
print(f"chunk 2^{lgw}, {(At.n + (1 << lgw) - 1) >> lgw} chunks per row", flush=True)
SG.LONG_STATS = {}
out = torch.zeros(A.m, dtype=torch.int32, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
SG._long_rows(0, A, At, rows, nprod[rows.long()], torch.cuda.current_stream().cuda_stream, out_nnz=out)
torch.cuda.synchronize()
print(f"count pass {time.perf_counter() - t0:.3f} s, nnz of long rows {int(out.sum()):.4g}")
tot_i = sum(v[0] for v in SG.LONG_STATS.values())
tot_p = sum(v[1] for v in SG.LONG_STATS.values())
print("bucket(products) items %items products %products")
for k in sorted(SG.LONG_STATS):
    it, pr = SG.LONG_STATS[k]
    print(f"[{(1 << k) - 1:>8}, {(1 << (k + 1)) - 2:>8}] {it:>10} {100 * it / tot_i:6.2f} {pr:12.4g} {100 * pr / tot_p:6.2f}")
