"""Shader-clock phase stamps of the bitmap-rank SpGEMM kernels (diagnostic build
path: the stamps are off in normal runs).  usage: python tools/bm_stamps.py [n] [density] [cfg]"""
import ctypes as C
import sys
import time

sys.path.insert(0, ".")
import os  # noqa: E402

# the stamps are compiled in only in a diagnostic variant of the library
from spmm_amd import _build  # noqa: E402

_stamps_lib = os.path.join(_build.LIB_DIR, "diag", "libspmm_hip_stamps.so")
if os.environ.get("SPMM_STAMPS_PREBUILT") and os.path.exists(_stamps_lib):   # built on the CPU host beforehand
    os.environ["SPMM_HIP_LIB"] = _stamps_lib
else:
    os.environ["SPMM_HIP_LIB"] = _build.build_hip(out=_stamps_lib, extra=["-DSPMM_BM_STAMPS"])
import torch  # noqa: E402

import spmm_amd  # noqa: E402,F401
from spmm_amd import _native  # noqa: E402
from spmm_amd.ops import spgemm as SG  # noqa: E402
from spmm_amd.utils import gen_csr  # noqa: E402
from spmm_amd.utils.config import CONFIG  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
d = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
if len(sys.argv) > 3:
    CONFIG.spgemm_bitmap_cfg = int(sys.argv[3])
dev = torch.device("cuda")
A = gen_csr.uniform_csr(n, n, d, seed=1, device=dev)
B = gen_csr.uniform_csr(n, n, d, seed=2, device=dev)
lib = _native.hip()
SG.spgemm(A, B)
torch.cuda.synchronize()
t = time.perf_counter()
SG.spgemm(A, B)
torch.cuda.synchronize()
plain = time.perf_counter() - t
lib.spmm_spgemm_bm_stamps(1, None)
info = SG.SpgemmInfo()
SG.spgemm(A, B, info)
out = (C.c_ulonglong * 8)()
lib.spmm_spgemm_bm_stamps(-1, out)
lib.spmm_spgemm_bm_stamps(0, None)
st = list(out)
units = max(st[7], 1)
names = ["num staging", "num pass1", "num scan", "num pass2", "num writeout", "count stage+OR", "count pop+clear"]
if os.environ.get("SPMM_SPGEMM_BITMAP_PIPE", "1") != "0":   # pipelined kernel: [0] = the NEXT unit staged + its loads issued
    names[0] = "num stage next+ld"
if info.rows_per_bin_num.get("bitmap_fused"):
    names[5:7] = ["fused count phase", "fused look-back"]
tot = sum(st[:5])
print(f"n={n} d={d} plain step {plain * 1e3:.2f} ms  info={info.rows_per_bin_num}")
if os.environ.get("SPMM_SPGEMM_BITMAP_PIPE", "1") != "0":   # pipelined count kernel: [5] ORs (+ next scan), [6] the rest
    names[5:7] = ["count ORs", "count stage+pop"]
for i, nm in enumerate(names):
    share = f"{100 * st[i] / tot:5.1f} %" if i < 5 and tot else ""
    per = units if i < 5 else max(units // 2, 1)   # (count units: two windows)
    print(f"{nm:18s} {st[i] / per:10.0f} cycles/unit {share}")
