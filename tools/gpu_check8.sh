#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
timeout -k 10 60 ./tools/probes/lds_bench | grep add_f32
echo "== pytest gpu spgemm" && timeout -k 10 600 python -m pytest tests/test_spgemm.py -m gpu -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== diag 1M" && timeout -k 10 400 python tools/spgemm_diag.py 1048576 0.0001 0,1 2>&1 | grep -v amdgpu.ids
echo "== diag 64k" && timeout -k 10 300 python tools/spgemm_diag.py 65536 0.001 0 2>&1 | grep -v amdgpu.ids
