#!/bin/bash
# a4: concurrency test, then report-sized e2e (small, medium)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_a4_native.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_a4.log 2>&1 || { tail -30 $O/pytest_a4.log; exit 1; }
grep -E "passed|failed" $O/pytest_a4.log | tail -2
PRESETS="${PRESETS:-small medium}" bash tools/gpu_e2e.sh
