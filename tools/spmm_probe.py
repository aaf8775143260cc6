"""Kernel time of Y = A . X for BASELINE config 3 (65536^2 @ 0.1 % x dense
128, bf16) with every SpMM method, from HIP events over many launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.ops import spmm as SM  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

n, d, D = 65536, 1e-3, 128
dev = torch.device("cuda", 0)
A = gen_csr.uniform_csr(n, n, d, seed=1, device=dev, dtype=torch.bfloat16)
X = (torch.rand((n, D), device=dev) * 2 - 1).to(torch.bfloat16)
plan = SM.plan_panels(A)
ref = SM.spmm(A, X, method="rowwise")
flops = 2.0 * A.nnz * D
for method in ("rowwise", "mfma"):
    f = lambda: SM.spmm(A, X, method=method, plan=plan)  # noqa: E731
    Y = f()
    err = (Y - ref).abs().max().item()
    for _ in range(5):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(f"{method:8s} {ms * 1e3:7.1f} us/launch  {flops / ms / 1e9:7.3f} TFLOP/s  max|diff| vs rowwise {err:.2e}",
          flush=True)
