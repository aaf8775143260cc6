#!/bin/bash
# R-MAT overlap: side stream at normal vs high priority
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g45; mkdir -p $O
cd $R
for pr in 0 -1; do
  SPMM_SIDE_PRIO=$pr timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_p$pr.json 2> $O/rm_p$pr.err || { tail -20 $O/rm_p$pr.err; exit 1; }
  echo "rmat prio $pr $(grep -o '"ms_per_step": [0-9.]*' $O/rm_p$pr.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_p$pr.json)"
done
