#!/bin/bash
# round-4: wide loads + wide stores: all bitmap GPU tests, kernel stats, 1M and 64k benches vs main
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
O=$R/gpurun_out/r4g28; mkdir -p $O
cd $R
for v in ${VARS:-all3}; do
  SPMM_HIP_LIB=$L/diag/libspmm_hip_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_spgemm.py tests/test_a4_native.py -k "bitmap or bench_scale or graph or mtx" -m gpu > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
VARS="${VARS:-all3}" bash tools/r4_g9.sh | grep -E "count|spgemm_bm_rows<" | cut -c1-150
for v in main ${VARS:-all3} main ${VARS:-all3}; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$v.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m_$v.json 2> $O/b1m_$v.err || { tail -5 $O/b1m_$v.err; exit 1; }
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -5 $O/b64_$v.err; exit 1; }
  echo "$v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$v.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
