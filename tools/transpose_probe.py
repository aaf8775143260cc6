"""Time A^T of an R-MAT matrix on the GPU: gfx950 transpose kernels vs the
sort-based path (torch device sort of row * n + col)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.ops import csr as CS  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
dev = torch.device("cuda", 0)
A = gen_csr.rmat_csr(scale, 16, seed=1, device=dev)
print(f"R-MAT scale {scale}: nnz {A.nnz}", flush=True)


def timed(f, reps=3):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


tk, Tk = timed(lambda: CS.transpose_gpu(A))
ts, Ts = timed(lambda: CS.from_coo(A.col.long(), A.row_ids(), A.val, A.n, A.m))
same = torch.equal(Tk.rowptr, Ts.rowptr) and torch.equal(Tk.col, Ts.col) and torch.equal(Tk.val, Ts.val)
print(f"transpose kernels {tk:.1f} ms, sort path {ts:.1f} ms, identical {same}", flush=True)
