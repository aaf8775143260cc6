#!/bin/bash
# round-4: R-MAT scale 24 -- long-row scratch budget per batch (SPMM_GLOBAL_WS_GB) and 2^14-column chunks
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g19; mkdir -p $O
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
cd $R
for cfg in "8 main" "32 main" "64 main" "32 lw14"; do
  set -- $cfg
  if [ $2 = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$2.so; fi
  SPMM_HIP_LIB=$lib SPMM_GLOBAL_WS_GB=$1 timeout -k 10 400 python -u bench.py --workload rmat --steps 1 --warmup 0 > $O/rmat_$1_$2.json 2> $O/rmat_$1_$2.err || { tail -5 $O/rmat_$1_$2.err; exit 1; }
  echo "ws=$1 lib=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/rmat_$1_$2.json) $(grep -o '"nnz_C": [0-9]*' $O/rmat_$1_$2.json)"
done
