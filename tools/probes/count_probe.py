"""Count-kernel timing probe (1M config): the row-major count kernel alone,
4 timed launches, with the exact total as a check.  Compare library variants
(tools/bm_variants.py) with SPMM_HIP_LIB=<variant> python tools/probes/count_probe.py.
(A 16-bit copy of the columns was probed this way too: PERF_LOG round 3.)"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _native  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

n, d = 1 << 20, 1e-4
dev = torch.device("cuda")
A = gen_csr.uniform_csr(n, n, d, seed=1, device=dev)
B = gen_csr.uniform_csr(n, n, d, seed=2, device=dev)
lib, P = _native.hip(), _native.ptr
st = _native.stream_ptr(dev)
lgw, nwin = 17, 8
ws = torch.empty(B.m * (nwin + 1), dtype=torch.int32, device=dev)
lib.spmm_spgemm_bm_splits(P(B.rowptr), P(B.col), B.m, lgw, nwin, P(ws), st)
err = torch.zeros(2, dtype=torch.int32, device=dev)
ws8 = torch.empty(B.m * 8, dtype=torch.int32, device=dev)
lib.spmm_spgemm_bm_pack_ws8(P(ws), B.m, nwin, P(ws8), P(err), st)
src = B.col
ucnt = torch.empty(A.m * nwin, dtype=torch.int32, device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for it in range(4):
    ev[0].record()
    _native.check(lib.spmm_spgemm_bm_count_rows(0, P(A.rowptr), P(A.col), P(ws8), P(src), A.m, nwin, 4, 2, P(ucnt),
                                                P(err), B.nnz, st), "count")
    ev[1].record()
    torch.cuda.synchronize()
    print(f"count kernel {ev[0].elapsed_time(ev[1]):.2f} ms  sum={int(ucnt.long().sum())}",
          flush=True)
