#!/bin/bash
# round-4 final: PMC (SQ, LDS, fetch, write) and kernel stats of the 1M step's bitmap kernels (16-byte gathers)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g32; mkdir -p $O
cd $R
PASSES="pmcA pmcB pmcC pmcD" FILTER=spgemm_bm KREGEX=spgemm_bm BENCH_ARGS="--graph off" PMC_DIR=/tmp/pmc1m bash tools/gpu_pmc.sh > $O/pmc_1m.txt 2>&1 || { tail -20 $O/pmc_1m.txt; exit 1; }
grep -c "" $O/pmc_1m.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p1m -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --graph off > $O/prof1m.log 2>&1 || { tail -20 $O/prof1m.log; exit 1; }
f=$(find /tmp/p1m -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof1m.md "1M kernel stats (16-byte gathers, eager, 3 steps + warm-up + setup)" && sed -n 5,16p $O/prof1m.md | cut -c1-150
