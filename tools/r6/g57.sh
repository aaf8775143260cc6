#!/bin/bash
# R-MAT with the overlap: direct hub-row products (long_dense reads the long B rows, no scratch) on / off
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g57; mkdir -p $O
cd $R
for d in 1 0; do
  SPMM_SPGEMM_LONG_DIRECT=$d timeout -k 10 500 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_d$d.json 2> $O/rm_d$d.err || { tail -20 $O/rm_d$d.err; exit 1; }
  echo "rmat direct $d $(grep -o '"ms_per_step": [0-9.]*' $O/rm_d$d.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_d$d.json) $(grep -o '"sum_val": [-0-9.e]*' $O/rm_d$d.json)"
done
