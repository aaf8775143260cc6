#!/bin/bash
# round-4: a count/numeric variant: bitmap GPU tests, kernel stats, bench vs main (interleaved)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
V=${V:-cw}
O=$R/gpurun_out/r4g15; mkdir -p $O
cd $R
SPMM_HIP_LIB=$L/diag/libspmm_hip_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "bitmap or bench_scale or graph" -m gpu > $O/pytest_$V.log 2>&1 || { tail -30 $O/pytest_$V.log; exit 1; }
tail -1 $O/pytest_$V.log
VARS=$V bash tools/r4_g9.sh | grep -E "count|spgemm_bm_rows<" | cut -c1-150
VARS="$V ${EXTRA:-}" bash tools/r4_g14.sh
