import sys; sys.path.insert(0,'.')
import torch, spmm_amd
from spmm_amd.ops import spgemm as SG
from spmm_amd.utils import gen_csr
dev=torch.device('cuda')
A=gen_csr.uniform_csr(65536,65536,1e-3,seed=1,device=dev); B=gen_csr.uniform_csr(65536,65536,1e-3,seed=2,device=dev)
i=SG.SpgemmInfo(); C=SG.spgemm(A,B,i); print(sys.argv[1], i.rows_per_bin_num, C.nnz)
