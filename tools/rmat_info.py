import sys, time, torch
sys.path.insert(0, '/root/repo')
import spmm_amd
from spmm_amd.ops import spgemm as SG
from spmm_amd.utils import gen_csr
scale = int(sys.argv[1])
dev = torch.device('cuda')
A = gen_csr.rmat_csr(scale, 16, seed=1, device=dev)
At = A.transpose()
nprod = SG.row_nprod(A, At)
print("rows", A.m, "nnzA", A.nnz, "total products", int(nprod.sum()), "max row", int(nprod.max()))
for t in [2048, 7680, 13824, 27648, 55296]:
    print(" rows with nprod >", t, int((nprod > t).sum()), "products in them", int(nprod[nprod > t].sum()))
info = SG.SpgemmInfo()
torch.cuda.synchronize(); t0 = time.perf_counter()
C = SG.spgemm(A, At, info)
torch.cuda.synchronize(); t1 = time.perf_counter()
print("time", t1 - t0, "nnzC", C.nnz, "bins", info.rows_per_bin_num)
rn = (C.rowptr[1:] - C.rowptr[:-1])
print("max row nnz", int(rn.max()), "rows nnz>100k", int((rn > 100000).sum()))
