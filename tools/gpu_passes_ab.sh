#!/bin/bash
# window-major passes of the bitmap row kernels: tests with passes on, then 1M / 64k benches per setting
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
SPMM_BM_NUM_PASS_WINDOWS=1 SPMM_BM_COUNT_PASS_WINDOWS=2 timeout -k 10 400 python -u -m pytest tests/test_spgemm.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bitmap or bench_scale" > $O/pytest_passes.log 2>&1; rc=$?
tail -2 $O/pytest_passes.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-"0 0" "1 2" "0 0" "1 2" "2 2" "1 4"}; do
  set -- $cfg
  for wl in ${WLS:-spgemm}; do
    SPMM_BM_NUM_PASS_WINDOWS=$1 SPMM_BM_COUNT_PASS_WINDOWS=$2 timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 > $O/passes_$1_$2_$wl.log 2>&1 || { tail -20 $O/passes_$1_$2_$wl.log; exit 1; }
    echo "num=$1 count=$2 $wl $(grep -o '"ms_per_step": [0-9.]*' $O/passes_$1_$2_$wl.log)"
  done
done
