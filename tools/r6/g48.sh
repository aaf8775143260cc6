#!/bin/bash
# R-MAT streamed panel size: share of free memory a panel may take
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g48; mkdir -p $O
cd $R
for fr in ${FRACS:-0.55 0.4 0.7}; do
  SPMM_STREAM_MEM_FRACTION=$fr timeout -k 10 400 python -u tools/r6/rmat_memstats.py --workload rmat --steps 2 --warmup 1 > $O/rm_f$fr.json 2> $O/rm_f$fr.err || { tail -20 $O/rm_f$fr.err; exit 1; }
  echo "rmat frac $fr $(grep -o '"ms_per_step": [0-9.]*' $O/rm_f$fr.json) $(grep -o '"panels": [0-9]*' $O/rm_f$fr.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_f$fr.json)"
  grep memstats $O/rm_f$fr.err
done
