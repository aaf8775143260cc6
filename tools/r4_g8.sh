#!/bin/bash
# round-4: count-kernel variants: correctness on the bitmap tests, 1M kernel stats (eager, so every kernel is traced)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
R=$PWD
O=gpurun_out/r4g8; mkdir -p $O
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
VARS=${VARS:-chalf}
for v in $VARS; do
  SPMM_HIP_LIB=$L/diag/libspmm_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_spgemm.py -k "bitmap or bench_scale or graph" -m gpu > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
cd /tmp && export TMPDIR=/tmp
for v in main $VARS; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$v.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/prof_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph off > $R/$O/prof_bench_$v.json 2> $R/$O/prof_bench_$v.err || exit 1
  python3 $R/tools/prof_top.py /tmp/prof_$v/run_results.db $v 6 | tee $R/$O/top_$v.txt
  SPMM_HIP_LIB=$lib timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/bench_$v.json 2> $R/$O/bench_$v.err || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $R/$O/bench_$v.json)"
done
