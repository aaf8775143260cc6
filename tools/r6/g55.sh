#!/bin/bash
# R-MAT: long-row scratch budget per batch (more, smaller batches = finer dense / routing overlap)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g55; mkdir -p $O
cd $R
for gb in ${GBS:-4 8 2 4}; do
  SPMM_GLOBAL_WS_GB=$gb timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_$gb.json 2> $O/rm_$gb.err || { tail -20 $O/rm_$gb.err; exit 1; }
  echo "rmat ws $gb GB $(grep -o '"ms_per_step": [0-9.]*' $O/rm_$gb.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_$gb.json) $(grep -o '"sum_val": [-0-9.e]*' $O/rm_$gb.json)"
done
