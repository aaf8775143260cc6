#!/bin/bash
# round-4: per-kernel stats of the 1M step for the main library and diagnostic variants ($VARS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g9; mkdir -p $O
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
cd /tmp && export TMPDIR=/tmp
for v in main ${VARS:-chalf}; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$v.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_$v -o prof --output-format csv -- python3 $R/bench.py --workload ${WL:-spgemm} --steps 3 --warmup 1 --graph off > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  f=$(find /tmp/p_$v -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_$v.md "$v kernel stats" && sed -n 5,14p $O/prof_$v.md
done
