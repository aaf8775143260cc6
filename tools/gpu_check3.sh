#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
for wl in spgemm64k spmm spgemm; do
  echo "== bench $wl" && timeout -k 10 400 python bench.py --workload $wl > $O/bench_$wl.log 2>&1 || { tail $O/bench_$wl.log; exit 1; }
  tail -1 $O/bench_$wl.log
done
cd /tmp && export TMPDIR=/tmp
echo "== rocprof 1M" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sp1m -o prof --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sp1m.log 2>&1 || exit 1
echo "== rocprof spmm" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_spmm -o prof --output-format csv -- python3 $R/bench.py --workload spmm --steps 3 --warmup 1 > $O/prof_spmm.log 2>&1 || exit 1
echo done
