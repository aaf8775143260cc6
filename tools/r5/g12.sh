#!/bin/bash
# round-5: R-MAT 24 direct long-row products with the compare-swap LDS adds (two modes), kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g12; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mode in d1024 d0; do
  if [ $mode = d0 ]; then export SPMM_LONG_DIRECT_MIN=0; fi
  SPMM_SPGEMM_LONG_DIRECT=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pp12$mode -o prof --output-format csv -- python3 $R/tools/r5/rmat_steps.py 24 2 > $O/prof_$mode.log 2>&1 || { tail -20 $O/prof_$mode.log; exit 1; }
  grep "^step" $O/prof_$mode.log
  f=$(find /tmp/pp12$mode -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_$mode.md "R-MAT 24 direct $mode, two steps" && sed -n 5,14p $O/prof_$mode.md | cut -c1-130
done
