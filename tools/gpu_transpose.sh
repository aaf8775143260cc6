#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_spgemm.py -m gpu -x -v --timeout 120 --timeout-method thread -k "transpose or csr_sum or innerdim or rmat" > $O/pytest_transpose.log 2>&1 || { tail -30 $O/pytest_transpose.log; exit 1; }
grep -E "passed|failed" $O/pytest_transpose.log | tail -2
timeout -k 10 300 python -u tools/transpose_probe.py 24 > $O/transpose_probe.log 2>&1 || { tail -20 $O/transpose_probe.log; exit 1; }
cat $O/transpose_probe.log
