"""SpGEMM phase diagnostics on the GPU: per-phase shader cycles per row for the
symbolic and numeric LDS kernels (diagnostic stamps in csr_spgemm.hip, taken
by thread 0 of every workgroup between the barriers that delimit a phase).
usage: python tools/spgemm_diag.py [n] [density]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _native  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
d = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
dev = torch.device("cuda")
A = gen_csr.uniform_csr(n, n, d, seed=1, device=dev)
B = gen_csr.uniform_csr(n, n, d, seed=2, device=dev)
lib = _native.hip()
buf = (C.c_ulonglong * 8)()
info = SG.SpgemmInfo()
C_ = SG.spgemm(A, B, info)  # warm
del C_
torch.cuda.synchronize()
nprod = SG.row_nprod(A, B)
row_nnz = SG.symbolic(A, B, nprod, info)
for mode in (0,):
    for phase in ("symbolic", "numeric", "onepass", "ordered"):
        lib.spmm_spgemm_stamps(1, None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if phase == "symbolic":
            SG.symbolic(A, B, nprod, info)
        elif phase == "numeric":
            Cm = SG.numeric(A, B, row_nnz, info, nprod)
            del Cm
        elif phase == "onepass":
            Cm = SG.onepass(A, B, nprod, info)
            del Cm
        else:   # ordered one-pass: units (row, column eighths) in row order, look-back offsets
            Cm = SG.onepass_ordered(A, B, nprod, info)
            del Cm
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        lib.spmm_spgemm_stamps(-1, buf)
        rows = max(buf[7], 1)
        names = ["init+staging", "inserts", "rank", "write", "count+lookback"]
        per = {names[i]: buf[i] / rows for i in range(5)}
        tot = sum(per.values())
        print(f"mode {mode} {phase}: wall {dt * 1e3:.1f} ms, rows {buf[7]}, cycles/row " +
              ", ".join(f"{k} {v:.0f} ({v / max(tot, 1) * 100:.0f}%)" for k, v in per.items()), flush=True)
lib.spmm_spgemm_stamps(0, None)
print("bins sym", info.rows_per_bin_sym, "num", info.rows_per_bin_num, "flops", info.flops, "nnz", info.nnz)
