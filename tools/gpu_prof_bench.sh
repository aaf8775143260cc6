#!/bin/bash
# rocprofv3 kernel stats of bench.py (default workload unless $WL set); PDIR = trace
# directory (default gpurun_out/prof_$WL; put long runs' traces in /tmp, gpurun_out is capped)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
WL=${WL:-spgemm}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${PDIR:=$O/prof_$WL} -o prof --output-format csv -- python3 $R/bench.py --workload $WL --steps ${STEPS:-3} --warmup ${WARMUP:-1} ${BENCH_ARGS} > $O/prof_$WL.log 2>&1 || { tail -20 $O/prof_$WL.log; exit 1; }
cd $R
grep metric $O/prof_$WL.log | cut -c1-220
f=$(find $PDIR -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f $O/prof_$WL.md "$WL kernel stats" && head -20 $O/prof_$WL.md
