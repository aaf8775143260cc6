"""Build diagnostic variants of libspmm_hip.so (``-D`` flags) under _lib/diag/
for A/B runs: ``SPMM_HIP_LIB=<path> python bench.py ...``.

usage: python tools/bm_variants.py NAME=-DFLAG[,-DFLAG2] ...
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from spmm_amd import _build  # noqa: E402

for spec in sys.argv[1:]:
    name, flags = spec.split("=", 1)
    out = os.path.join(_build.LIB_DIR, "diag", f"libspmm_hip_{name}.so")
    _build.build_hip(out=out, extra=flags.split(","))
    print(out)
