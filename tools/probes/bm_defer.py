"""Deferred-unit count of the 65536^2 @ 0.1 % bitmap SpGEMM (units the fast
numeric kernel hands to the reload kernel) with the loaded library: compare
register-round variants (tools/bm_variants.py) via SPMM_HIP_LIB.
usage: python tools/probes/bm_defer.py [label]"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

dev = torch.device("cuda")
A = gen_csr.uniform_csr(65536, 65536, 1e-3, seed=1, device=dev)
B = gen_csr.uniform_csr(65536, 65536, 1e-3, seed=2, device=dev)
info = SG.SpgemmInfo()
C = SG.spgemm(A, B, info)
print(sys.argv[1] if len(sys.argv) > 1 else "lib", info.rows_per_bin_num, C.nnz)
