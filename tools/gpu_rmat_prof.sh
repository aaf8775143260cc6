#!/bin/bash
# R-MAT A.A^T kernel stats of K streamed steps with no setup product (tools/rmat_steps.py):
#   SCALE=24 STEPS=2 bash tools/gpu_rmat_prof.sh   ->  gpurun_out/rmat_prof/prof.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rmat_prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/pprm -o prof --output-format csv -- python3 $R/tools/rmat_steps.py ${SCALE:-24} ${STEPS:-2} > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep "^step" $O/prof.log
f=$(find /tmp/pprm -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv
python3 $R/tools/prof_summary.py $f $O/prof.md "R-MAT ${SCALE:-24}, ${STEPS:-2} streamed steps" && head -20 $O/prof.md | cut -c1-170
