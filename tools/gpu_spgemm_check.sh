#!/bin/bash
# SpGEMM change check: GPU spgemm tests, then the CSR benches, then phase stamps for 1M
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_spgemm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_spgemm.log 2>&1 || { tail -30 $O/pytest_spgemm.log; exit 1; }
grep -E "passed|failed" $O/pytest_spgemm.log | tail -2
for wl in ${WLS:-spgemm spgemm64k rmat}; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 > $O/bench_$wl.log 2>&1 || { tail -20 $O/bench_$wl.log; exit 1; }
  grep '"metric"' $O/bench_$wl.log > $O/bench_$wl.json
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', d['value'], d['unit'], d['ms_per_step'], 'ms')"
done
[ -n "$NO_DIAG" ] || timeout -k 10 300 python tools/spgemm_diag.py 1048576 0.0001 2>&1 | grep -v amdgpu.ids | grep onepass
