"""Probe the MFMA SpMM lane/layout mapping with exact integer data."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import spmm_amd  # noqa
from spmm_amd.ops import csr as CS, spmm as SM

dev = torch.device("cuda")
n, D = 64, 128
I = CS.from_dense(torch.eye(n, device=dev).to(torch.bfloat16))
for name, X in (("rowid", torch.arange(n, device=dev).view(n, 1).expand(n, D)),
                ("colid", torch.arange(D, device=dev).view(1, D).expand(n, D))):
    X = X.to(torch.bfloat16).contiguous()
    Y = SM.spmm(I, X, method="mfma")
    bad = (Y != X.float()).nonzero()
    print(name, "mismatches", bad.shape[0])
    if bad.shape[0]:
        for r in (0, 1, 2, 3, 4, 8, 16, 17, 31, 32, 63):
            print(" row", r, "got", Y[r, :20].int().tolist(), "... want", X[r, :4].float().int().tolist())
# single entry A[5][9] = 1 -> Y[5] = X[9]
A = torch.zeros(n, n, device=dev); A[5, 9] = 1
A = CS.from_dense(A.to(torch.bfloat16))
X = torch.arange(n, device=dev).view(n, 1).expand(n, D).to(torch.bfloat16).contiguous()
Y = SM.spmm(A, X, method="mfma")
print("single: nonzero rows", Y.abs().sum(1).nonzero().flatten().tolist(), "row5 vals", Y[5, :8].tolist())
nz = Y.nonzero()
print("nonzero positions sample", nz[:10].tolist(), "count", nz.shape[0])
