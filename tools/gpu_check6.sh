#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -8 $O/pytest_gpu.log
echo "== diag 64k" && timeout -k 10 300 python tools/spgemm_diag.py 65536 0.001 2>&1 | grep -v amdgpu.ids
echo "== diag 1M" && timeout -k 10 300 python tools/spgemm_diag.py 2>&1 | grep -v amdgpu.ids
for wl in spgemm64k spgemm spmm; do
  echo "== bench $wl" && timeout -k 10 400 python bench.py --workload $wl > $O/bench_$wl.log 2>&1 || { tail $O/bench_$wl.log; exit 1; }
  tail -1 $O/bench_$wl.log
done
echo done
