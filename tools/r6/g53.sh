#!/bin/bash
# R-MAT: long_rank's grid share apart from long_dense's (75 %)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g53; mkdir -p $O
cd $R
for rp in 50 100 34 75; do
  SPMM_LONG_RANK_PCT=$rp timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_$rp.json 2> $O/rm_$rp.err || { tail -20 $O/rm_$rp.err; exit 1; }
  echo "rmat rank $rp % $(grep -o '"ms_per_step": [0-9.]*' $O/rm_$rp.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_$rp.json) $(grep -o '"sum_val": [-0-9.e]*' $O/rm_$rp.json)"
done
