#!/bin/bash
# round-4: PMC of the 65536^2 step's bitmap kernels (per-unit numeric with 16-byte gathers, row count)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g33; mkdir -p $O
cd $R
WL=spgemm64k PASSES="pmcA pmcB pmcC pmcD" FILTER=spgemm_bm KREGEX=spgemm_bm BENCH_ARGS="--graph off" PMC_DIR=/tmp/pmc64 bash tools/gpu_pmc.sh > $O/pmc_64k.txt 2>&1 || { tail -20 $O/pmc_64k.txt; exit 1; }
cat $O/pmc_64k.txt
