"""torch.profiler view of one bench workload step (host ops with their device
time, grouped by input shapes): finds PyTorch glue around the HIP kernels.
usage: python tools/torchprof.py [rmat SCALE | spgemm N DENSITY]"""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd.models import spgemm as MS  # noqa: E402
from spmm_amd.parallel import comm as CM  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "rmat"
comm = CM.init(backend="auto", device="auto")
if wl == "rmat":
    prob = MS.RmatProblem.build(int(sys.argv[2]) if len(sys.argv) > 2 else 22, 16, comm, seed=1)
    nnz = [0]

    def step():
        prob.step(comm, None, lambda lo, hi, C: nnz.__setitem__(0, nnz[0] + C.nnz))
else:
    n, d = int(sys.argv[2]), float(sys.argv[3])
    prob = MS.UniformProblem.build(n, d, comm, seed=1)

    def step():
        MS.rowblock_spgemm(prob.A, prob.B, comm)
step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="device_time_total", row_limit=30,
                                                          max_name_column_width=40, max_shapes_column_width=60))
