#!/bin/bash
# Bitmap-rank SpGEMM: GPU tests, CSR benches, rocprofv3 kernel stats of the 1M step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest bitmap"
timeout -k 10 600 python -u -m pytest tests/test_spgemm.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "${TESTS:-bitmap or row_plan}" > $O/pytest_bm.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/pytest_bm.log | tail -20; [ $rc -eq 0 ] || { tail -40 $O/pytest_bm.log; exit $rc; }
for wl in ${WLS:-spgemm spgemm64k}; do
  echo "== bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps ${STEPS:-5} --warmup 2 > $O/bench_$wl.log 2>&1 || { tail -20 $O/bench_$wl.log; exit 1; }
  grep '"metric"' $O/bench_$wl.log | cut -c1-600
done
[ -n "$NOPROF" ] && exit 0
echo "== rocprof spgemm"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bm -o prof --output-format csv -- python3 $R/bench.py --workload spgemm --steps 3 --warmup 1 > $O/prof_bm.log 2>&1 || { tail -20 $O/prof_bm.log; exit 1; }
cd $R
f=$(find $O/prof_bm -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f $O/prof_bm.md "1M SpGEMM (bitmap) kernel stats" && head -24 $O/prof_bm.md
