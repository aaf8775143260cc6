#!/bin/bash
# round-5: full GPU suite + smoke on the current tree; 1M / 64k bench; kernel stats of the 1M step
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g07; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
echo "gpu suite: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b64.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp7 -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find /tmp/pp7 -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof.md "1M graph step" && head -20 $O/prof.md | cut -c1-150
