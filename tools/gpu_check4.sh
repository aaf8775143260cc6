#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== spmm layout probe" && timeout -k 10 300 python tools/debug_spmm_layout.py > $O/spmm_probe.log 2>&1; cat $O/spmm_probe.log | grep -v amdgpu.ids
for wl in spgemm64k spgemm; do
  echo "== bench $wl" && timeout -k 10 400 python bench.py --workload $wl > $O/bench_$wl.log 2>&1 || { tail $O/bench_$wl.log; exit 1; }
  tail -1 $O/bench_$wl.log
done
cd /tmp && export TMPDIR=/tmp
echo "== rocprof 1M" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sp1m -o prof --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sp1m.log 2>&1 || exit 1
echo done
