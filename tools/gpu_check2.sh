#!/bin/bash
# SpGEMM GPU pass: tests, smoke, benches, rocprof of the 64k config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
echo "== bench 64k" && timeout -k 10 300 python bench.py --workload spgemm64k --steps 5 --warmup 2 > $O/bench_64k.log 2>&1 || { tail $O/bench_64k.log; exit 1; }
tail -1 $O/bench_64k.log
echo "== bench default" && timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { tail $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
cd /tmp && export TMPDIR=/tmp
echo "== rocprof 64k" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sp64k -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 3 --warmup 1 > $O/prof_sp64k.log 2>&1 || exit 1
echo "== rocprof 1M" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sp1m -o prof --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sp1m.log 2>&1 || exit 1
echo done
