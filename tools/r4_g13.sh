#!/bin/bash
# round-4: count units of 1 / 2 / 4 windows (padded layouts), kernel stats of the 1M step
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g13; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cw in ${CWS:-1 4}; do
  SPMM_SPGEMM_BITMAP_COUNT_WINDOWS=$cw timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc_$cw -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --graph off > $O/prof_cw$cw.log 2>&1 || { tail -20 $O/prof_cw$cw.log; exit 1; }
  f=$(find /tmp/pc_$cw -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_cw$cw.md "count windows $cw" && grep -E "count|spgemm_bm_rows<" $O/prof_cw$cw.md | cut -c1-140
  grep -o '"ms_per_step": [0-9.]*' $O/prof_cw$cw.log
done
