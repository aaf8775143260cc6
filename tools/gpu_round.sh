#!/bin/bash
# Full GPU check: gpu tests, smoke, every bench workload (JSON lines -> gpurun_out/bench_*.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -8; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for wl in ${WLS:-spgemm spgemm64k spmm rmat chain}; do
  echo "== bench $wl"
  args="--steps ${STEPS:-5} --warmup 2"
  [ $wl = rmat ] && args="--steps 2 --warmup 1"   # scale 24: ~25 s per step on one GPU
  timeout -k 10 600 python -u bench.py --workload $wl $args > $O/bench_$wl.log 2>&1 || { tail -20 $O/bench_$wl.log; exit 1; }
  grep '"metric"' $O/bench_$wl.log > $O/bench_$wl.json; cut -c1-400 $O/bench_$wl.json
done
