#!/bin/bash
# round-5: count-unit width (windows per count unit 2 / 4 / 8) on the 1M step, kernel stats each
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g28; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cw in 2 4 8; do
  SPMM_SPGEMM_BITMAP_COUNT_WINDOWS=$cw timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp28_$cw -o prof --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 > $O/prof_$cw.log 2>&1 || { tail -20 $O/prof_$cw.log; exit 1; }
  f=$(find /tmp/pp28_$cw -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_$cw.md "1M count windows $cw" && echo "== $cw $(grep -o '"ms_per_step": [0-9.]*' $O/prof_$cw.log)" && grep -i "count" $O/prof_$cw.md | cut -c1-140
done
