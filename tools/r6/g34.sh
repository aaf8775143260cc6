#!/bin/bash
# 65536^2 lane-group A/B (numeric 32-pair chunks, count 16- / 64-column chunks) and kernel stats of the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g34; mkdir -p $O
cd $R
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
for v in base lgn24 lgc24 lgc96 base lgc24 lgc96; do
  lib=""; [ "$v" = base ] || lib=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -20 $O/b64_$v.err; exit 1; }
  echo "64k $v $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json) $(grep -o '"bitmap_deferred": [0-9]*' $O/b64_$v.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppvb -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
cp $(find /tmp/ppvb -name "*kernel_stats.csv" | head -1) $O/spgemm64k_kernel_stats.csv
head -5 $O/spgemm64k_kernel_stats.csv | cut -c1-150
