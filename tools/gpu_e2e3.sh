#!/bin/bash
# a4 after the arena change: gpu tests, medium with one product stream, medium default, small
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_a4_native.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_a4.log 2>&1 || { tail -30 $O/pytest_a4.log; exit 1; }
grep -E "passed|failed" $O/pytest_a4.log | tail -2
run() {  # name, extra args
  echo "== a4 e2e $1"
  timeout -k 10 600 python -u benches/bench_a4_e2e.py --device hip --json $O/a4_e2e_$1.json "${@:2}" > $O/a4_e2e_$1.log 2>&1 || { tail -20 $O/a4_e2e_$1.log; return 1; }
  grep metric $O/a4_e2e_$1.log | cut -c1-300
}
run medium_s1 --preset medium --streams 1 && run medium --preset medium && run small --preset small
