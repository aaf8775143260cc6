"""Host-side cost of the SpGEMM dispatcher's calls (per call, microseconds)."""
import time

import torch

import spmm_amd  # noqa: F401
from spmm_amd.ops import spgemm as SG
from spmm_amd.utils import gen_csr

dev = torch.device("cuda", 0)
A = gen_csr.uniform_csr(65536, 65536, 1e-3, seed=1, device=dev)
B = gen_csr.uniform_csr(65536, 65536, 1e-3, seed=2, device=dev)
for _ in range(3):
    SG.spgemm(A, B)
torch.cuda.synchronize()


def t(name, f, n=50):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    print(f"{name:28s} {(time.perf_counter() - t0) / n * 1e6:9.1f} us", flush=True)


t("mem_get_info", lambda: torch.cuda.mem_get_info(dev))
t("memory_reserved+allocated", lambda: torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev))
t("row_plan+tolist", lambda: SG.row_plan(A, B)[2].tolist())
t("zeros(131074)", lambda: torch.zeros(131074, dtype=torch.int32, device=dev))
t("cumsum(65536)", lambda: torch.cumsum(torch.ones(65536, dtype=torch.int64, device=dev), 0))
t("spgemm", lambda: SG.spgemm(A, B), n=20)

import cProfile  # noqa: E402
import pstats  # noqa: E402

pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    SG.spgemm(A, B)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
