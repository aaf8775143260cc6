#!/bin/bash
# R-MAT: long_dense / long_rank persistent grids at a share of the resident capacity (beside the routing)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g51; mkdir -p $O
cd $R
for pct in ${PCTS:-50 100 75}; do
  SPMM_LONG_GRID_PCT=$pct timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_$pct.json 2> $O/rm_$pct.err || { tail -20 $O/rm_$pct.err; exit 1; }
  echo "rmat grid $pct % $(grep -o '"ms_per_step": [0-9.]*' $O/rm_$pct.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_$pct.json) $(grep -o '"sum_val": [-0-9.e]*' $O/rm_$pct.json)"
done
