#!/bin/bash
# R-MAT with long-row accumulation on the side stream: side stream at normal vs high priority
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g49; mkdir -p $O
cd $R
for pr in 0 -1 0; do
  SIDE_PRIO=$pr timeout -k 10 400 python -u tools/r6/rmat_side_prio.py --workload rmat --steps 2 --warmup 1 > $O/rm_p$pr.json 2> $O/rm_p$pr.err || { tail -20 $O/rm_p$pr.err; exit 1; }
  echo "rmat prio $pr $(grep -o '"ms_per_step": [0-9.]*' $O/rm_p$pr.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_p$pr.json)"
done
