#!/bin/bash
# round-5: long_rank capacity (register rounds 8 / 16 / 24), same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g31; mkdir -p $O
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
cd $R
for v in base lr8 lr24; do
  L=""; [ $v != base ] && L=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$L timeout -k 10 200 python -u tools/r5/rmat_steps.py 24 2 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^step' $O/$v.log | tr '\n' ' ')"
done
