#!/bin/bash
# round-4: numeric-kernel tuning variants on the 1M bench (graph replay), main library interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g14; mkdir -p $O
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
cd $R
for v in main ${VARS:-sg4 r9 r11} main; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$v.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.json)"
done
