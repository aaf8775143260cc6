#!/bin/bash
# round-5: bitmap layout change -- bitmap GPU tests, 1M / 64k bench, 1M kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g18; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "bitmap or graph or bench_scale or dist" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp18 -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 > $O/prof1m.log 2>&1 || { tail -20 $O/prof1m.log; exit 1; }
f=$(find /tmp/pp18 -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof1m.md "1M" && grep -i "pad_pairs\|splits\|pack_ws8\|scan" $O/prof1m.md | cut -c1-140
