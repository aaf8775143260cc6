#!/bin/bash
# round-5: 1M / 64k bench + kernel stats of both graph-replayed steps (current tree)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g16; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b64.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp16a -o prof --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $O/prof1m.log 2>&1 || { tail -20 $O/prof1m.log; exit 1; }
f=$(find /tmp/pp16a -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof1m.md "1M graph step (10 steps + 2 warm-up + setup)" && sed -n 5,22p $O/prof1m.md | cut -c1-140
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp16b -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
f=$(find /tmp/pp16b -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof64.md "64k graph step (50 steps + 5 warm-up + setup)" && sed -n 5,22p $O/prof64.md | cut -c1-140
