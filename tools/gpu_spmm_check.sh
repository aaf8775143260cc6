#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_spmm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_spmm.log 2>&1 || { tail -30 $O/pytest_spmm.log; exit 1; }
grep -E "passed|failed" $O/pytest_spmm.log | tail -1
timeout -k 10 300 python -u bench.py --workload spmm --steps 50 --warmup 5 > $O/bench_spmm.log 2>&1 || { tail -20 $O/bench_spmm.log; exit 1; }
grep metric $O/bench_spmm.log | cut -c1-260
