#!/bin/bash
# A/B of one environment knob on a bench workload:
#   VAR=SPMM_SPGEMM_BITMAP_ROWS VALUES="auto on auto on" BENCH_ARGS="--workload spgemm64k" bash tools/gpu_env_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
i=0
for val in ${VALUES}; do
  i=$((i + 1))
  env $VAR=$val timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > $O/ab_$i.log 2>&1 || { tail -20 $O/ab_$i.log; exit 1; }
  echo "$VAR=$val $(grep -o '"ms_per_step": [0-9.]*' $O/ab_$i.log) $(grep -o '"value": [0-9.]*' $O/ab_$i.log)"
done
