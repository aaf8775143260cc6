#!/bin/bash
# round-4: 65536^2 config: per-unit vs row numeric kernel (padded), graph replay; kernel stats of each
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g16; mkdir -p $O
cd $R
for mode in auto on auto on; do
  SPMM_SPGEMM_BITMAP_ROWS=$mode timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$mode.json 2> $O/b64_$mode.err || { tail -5 $O/b64_$mode.err; exit 1; }
  echo "64k rows=$mode $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$mode.json)"
done
cd /tmp && export TMPDIR=/tmp
for mode in auto on; do
  SPMM_SPGEMM_BITMAP_ROWS=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p64_$mode -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 20 --warmup 3 --graph off > $O/prof_$mode.log 2>&1 || { tail -20 $O/prof_$mode.log; exit 1; }
  f=$(find /tmp/p64_$mode -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof64_$mode.md "64k rows=$mode" && sed -n 5,16p $O/prof64_$mode.md | cut -c1-150
done
