#!/bin/bash
# round-4: variant $V on both bitmap configs: tests, 1M + 64k benches interleaved with main
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
V=${V:-wo4}
O=$R/gpurun_out/r4g23; mkdir -p $O
cd $R
SPMM_HIP_LIB=$L/diag/libspmm_hip_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "bitmap or bench_scale or graph" -m gpu > $O/pytest_$V.log 2>&1 || { tail -30 $O/pytest_$V.log; exit 1; }
tail -1 $O/pytest_$V.log
for v in main $V main $V; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$v.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m_$v.json 2> $O/b1m_$v.err || { tail -5 $O/b1m_$v.err; exit 1; }
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -5 $O/b64_$v.err; exit 1; }
  echo "$v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$v.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
