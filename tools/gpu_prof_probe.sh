#!/bin/bash
# rocprofv3 kernel stats of the R-MAT per-rank probe (rank 0 of $WORLD, scale $SCALE)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_probe -o prof --output-format csv -- python3 $R/tools/rmat_rank_probe.py --scale ${SCALE:-24} --world ${WORLD:-8} --ranks 0 --steps 1 > $O/prof_probe.log 2>&1 || { tail -20 $O/prof_probe.log; exit 1; }
cd $R
grep '"rank"' $O/prof_probe.log
f=$(find $O/prof_probe -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f $O/prof_probe.md "R-MAT scale-${SCALE:-24} rank 0 of ${WORLD:-8} kernel stats" && head -24 $O/prof_probe.md
rm -rf $O/prof_probe
