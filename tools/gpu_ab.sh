#!/bin/bash
# A/B of diagnostic library variants on the 1M SpGEMM bench: VARIANTS="base rr16 ..."
# (base = the real library; others lib/diag/libspmm_hip_<name>.so), one bench per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in ${VARIANTS:-base}; do
  lib=""
  [ "$v" = base ] || lib=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag/libspmm_hip_$v.so
  for wl in ${WLS:-spgemm}; do
    SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --steps ${STEPS:-5} --warmup 2 > $O/ab_${v}_$wl.log 2>&1 || { tail -20 $O/ab_${v}_$wl.log; exit 1; }
    echo "$v $wl $(grep -o '"ms_per_step": [0-9.]*' $O/ab_${v}_$wl.log) $(grep -o '"value": [0-9.]*' $O/ab_${v}_$wl.log)"
  done
done
