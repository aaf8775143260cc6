#!/bin/bash
# round-4: vectorised long_place ($V): long-row GPU tests, R-MAT step vs main
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
V=${V:-lp4}
O=$R/gpurun_out/r4g30; mkdir -p $O
cd $R
SPMM_HIP_LIB=$L/diag/libspmm_hip_$V.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "long or rmat or stream or hub" -m gpu > $O/pytest_$V.log 2>&1 || { tail -30 $O/pytest_$V.log; exit 1; }
echo "$V $(tail -1 $O/pytest_$V.log)"
for v in main $V; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$v.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --workload rmat --steps 1 --warmup 0 > $O/rmat_$v.json 2> $O/rmat_$v.err || { tail -5 $O/rmat_$v.err; exit 1; }
  echo "$v rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rmat_$v.json) $(grep -o '"nnz_C": [0-9]*' $O/rmat_$v.json) $(grep -o '"sum_val": [0-9.e+-]*' $O/rmat_$v.json)"
done
