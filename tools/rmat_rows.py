"""Long-row statistics of R-MAT A.A^T: rows by log2(products), their A entries, entries
on long B rows (>= 4 per 2^15-column chunk) and the products those carry.
usage: python tools/rmat_rows.py [scale]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import spmm_amd  # noqa: F401,E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
dev = torch.device("cuda")
A = gen_csr.rmat_csr(scale, 16, seed=1, device=dev)
At = A.transpose()
nprod = SG.row_nprod(A, At).long()
nch = (At.n + (1 << 15) - 1) >> 15
blen = (At.rowptr[1:] - At.rowptr[:-1]).long()
alen = (A.rowptr[1:] - A.rowptr[:-1]).long()
row = torch.repeat_interleave(torch.arange(A.m, device=dev), alen)
w = blen[A.col.long()]
isl = w >= 4 * nch
L = torch.zeros(A.m, dtype=torch.int64, device=dev).index_add_(0, row, isl.long())
PL = torch.zeros(A.m, dtype=torch.int64, device=dev).index_add_(0, row, torch.where(isl, w, 0))
print(f"scale {scale}: m {A.m}, nnz {A.nnz}, products {int(nprod.sum()):.4g}, long B rows {int((blen >= 4 * nch).sum())} "
      f"(>= {4 * nch} entries)")
print("log2(prod) rows  products  %prod  A-entries  long-entries  long-products  %long  mean-L")
b = torch.floor(torch.log2(nprod.double().clamp(min=1))).long()
tot = int(nprod.sum())
for k in range(int(b.max()) + 1):
    m = b == k
    r = int(m.sum())
    if not r:
        continue
    p = int(nprod[m].sum())
    print(f"{k:>3} {r:>9} {p:12.4g} {100 * p / tot:6.2f} {int(alen[m].sum()):>11} {int(L[m].sum()):>11} "
          f"{int(PL[m].sum()):12.4g} {100 * int(PL[m].sum()) / max(p, 1):6.1f} {int(L[m].sum()) / r:9.1f}")
