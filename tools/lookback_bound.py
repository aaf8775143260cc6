"""Upper bound on the look-back wait of the ordered one-pass SpGEMM: the 1M
config's step with the real look-back vs with g_nowait (every unit publishes
at once; offsets are wrong, so the output is discarded — timing only)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _native  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils.gen_csr import uniform_csr  # noqa: E402

dev = torch.device("cuda", 0)
lib = _native.hip()
n = 1 << 20
A = uniform_csr(n, n, 1e-4, seed=1, device=dev)
B = uniform_csr(n, n, 1e-4, seed=2, device=dev)
for mode, flag in (("lookback", 0), ("nowait", 2), ("lookback", 0)):
    _native.check(lib.spmm_spgemm_stamps(flag, None), "stamps")
    C = SG.spgemm(A, B)
    del C
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        C = SG.spgemm(A, B)
        del C
    torch.cuda.synchronize()
    print(f"{mode:9s} {(time.perf_counter() - t) / 3 * 1e3:.1f} ms/step", flush=True)
_native.check(lib.spmm_spgemm_stamps(0, None), "stamps")
