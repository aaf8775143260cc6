#!/bin/bash
# R-MAT 24, one streamed step (overlapped panels, side-stream accumulation at 75 %): kernel stats + concurrency
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g56; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d /tmp/prm -o prof --output-format csv -- python3 $R/tools/rmat_steps.py 24 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep "^step" $O/trace.log
f=$(find /tmp/prm -name "*kernel_trace.csv" | head -1)
python3 $R/tools/overlap.py $f long_place long_dense long_rank long_route spgemm_esc compact > $O/rmat_overlap.txt
cp $(find /tmp/prm -name "*kernel_stats.csv" | head -1) $O/rmat_kernel_stats.csv
cat $O/rmat_overlap.txt
