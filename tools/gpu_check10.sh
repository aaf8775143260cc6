#!/bin/bash
# GPU tests + SpGEMM diagnostics + default/64k benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; grep -E "passed|failed|Error|error" $O/pytest_gpu.log | head -8; [ $rc -eq 0 ] || exit $rc
echo "== diag 1M" && timeout -k 10 300 python tools/spgemm_diag.py 1048576 0.0001 2>&1 | grep -v amdgpu.ids || exit 1
echo "== bench default" && timeout -k 10 300 python bench.py --steps 5 --warmup 2 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
echo "== bench 64k" && timeout -k 10 300 python bench.py --workload spgemm64k --steps 10 --warmup 3 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
