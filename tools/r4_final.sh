#!/bin/bash
# round-4 validation: full GPU test suite, smoke, default bench (N=1), 64k bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4final; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-300
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/bench64k.json 2> $O/bench64k.err || { tail -5 $O/bench64k.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench64k.json
