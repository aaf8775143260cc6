#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
echo "== pytest gpu spgemm" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; grep -E "passed|failed|Error|error" $O/pytest_gpu.log | head -8; [ $rc -eq 0 ] || exit $rc
echo "== diag 1M" && timeout -k 10 400 python tools/spgemm_diag.py 1048576 0.0001 0 2>&1 | grep -v amdgpu.ids
echo "== diag 64k" && timeout -k 10 300 python tools/spgemm_diag.py 65536 0.001 0 2>&1 | grep -v amdgpu.ids
