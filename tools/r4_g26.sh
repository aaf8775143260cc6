#!/bin/bash
# round-4: fixed-count load variants ($VARS) -- tests of the last, kernel stats, 1M bench interleaved with main
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
O=$R/gpurun_out/r4g26; mkdir -p $O
cd $R
for v in ${VARS:-ul ul2}; do
  SPMM_HIP_LIB=$L/diag/libspmm_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_spgemm.py -k "bitmap or bench_scale" -m gpu > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
VARS="${VARS:-ul ul2}" bash tools/r4_g9.sh | grep -E "count|spgemm_bm_rows<" | cut -c1-150
VARS="${VARS:-ul ul2}" bash tools/r4_g14.sh
