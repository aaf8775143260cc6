"""SpMM kernels vs panel column reuse: a 65536^2 operand with ~65 entries per
row whose rows, in 64-row panels, draw their columns from a shared pool of
`pool` columns (reuse = 64 * 65 / pool when the pool is small), times the
MFMA panel kernel, the row kernel and the row-owning sweep (HIP events,
50 calls each after warm-up).  usage: python tools/probes/spmm_reuse.py"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.ops import csr as CS  # noqa: E402
from spmm_amd.ops import spmm as SM  # noqa: E402

dev = torch.device("cuda")
n, per_row, D = 65536, 65, 128
g = torch.Generator(device=dev).manual_seed(7)
X = (torch.rand(n, D, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
for pool in (65536, 4096, 1024, 256, 128):
    npan = n // 64
    base = torch.randint(0, n, (npan, pool), generator=g, device=dev)                  # each panel's column pool
    pick = torch.randint(0, pool, (n, per_row), generator=g, device=dev)
    cols = torch.gather(base.repeat_interleave(64, 0), 1, pick)
    rows = torch.arange(n, device=dev).repeat_interleave(per_row)
    vals = (torch.rand(n * per_row, generator=g, device=dev) * 2 - 1)
    A = CS.from_coo(rows, cols.reshape(-1), vals, n, n)   # (duplicate columns of a row merged)
    A = A.with_values(A.val.to(torch.bfloat16))
    plan = SM.plan_panels(A)
    out = {}
    for meth in ("mfma", "rowwise", "sweep"):
        if meth == "sweep" and not SM.sweep_ok(A):
            continue
        for _ in range(3):
            SM.spmm(A, X, method=meth, plan=plan)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(50):
            SM.spmm(A, X, method=meth, plan=plan)
        ev[1].record()
        torch.cuda.synchronize()
        out[meth] = round(ev[0].elapsed_time(ev[1]) / 50, 4)
    print(f"pool {pool:6d}  nnz {A.nnz}  panel reuse {plan.reuse:6.2f}  ms per call {out}", flush=True)
