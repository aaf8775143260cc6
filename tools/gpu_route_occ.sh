#!/bin/bash
# R-MAT 24 long-row scatter occupancy sweep: dynamic LDS pads limit route<true>
# workgroups per CU (PADS, bytes); kernel stats per pad under gpurun_out/route_occ/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/route_occ
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pad in ${PADS:-0 49152 114688}; do
  echo "== pad $pad"
  SPMM_LONG_ROUTE_LDS_PAD=$pad timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/ro_$pad -o prof --output-format csv -- python3 $R/bench.py --workload rmat --steps 1 --warmup 0 > $O/pad_$pad.log 2>&1 || { tail -20 $O/pad_$pad.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/pad_$pad.log
  f=$(find /tmp/ro_$pad -name "*kernel_stats.csv" | head -1)
  (cd $R && python tools/prof_summary.py $f $O/pad_$pad.md "route pad $pad" > /dev/null && grep -E "long_route|long_dense" $O/pad_$pad.md | cut -c1-90)
done
