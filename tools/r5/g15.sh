#!/bin/bash
# round-5: R-MAT 24 route variants (entries per routing workgroup, windows per step): step times
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g15; mkdir -p $O
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
cd $R
for v in epw16 epw32 ppu8; do
  echo "== $v"
  SPMM_HIP_LIB=$D/libspmm_hip_$v.so timeout -k 10 200 python -u tools/r5/rmat_steps.py 24 2 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep "^step" $O/$v.log
done
