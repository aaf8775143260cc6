"""torch.profiler view of one streamed R-MAT A.A^T product (which Python line
launches which device kernels).  usage: python tools/rmat_torchprof.py [scale]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.parallel import comm as PC  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
comm = PC.init()
prob = MS.RmatProblem.build(scale, 16, comm, seed=1)
B = prob.right_operand(comm)
budget = MS.stream_budget(comm.device) // int(os.environ.get("PANEL_DIV", "8"))
n = [0]


def consume(lo, hi, C):
    n[0] += C.nnz


MS.streamed_spgemm(prob.A, B, consume, budget=budget)   # warm-up (memoised B tables)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as p:
    MS.streamed_spgemm(prob.A, B, consume, budget=budget)
    torch.cuda.synchronize()
print(p.key_averages(group_by_stack_n=int(os.environ.get("STACK_N", "4"))).table(
    sort_by="self_cuda_time_total", row_limit=int(os.environ.get("ROWS", "30")), max_name_column_width=60,
    max_src_column_width=160))
