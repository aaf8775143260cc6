#!/bin/bash
# round-4: PMC of the 1M step's bitmap kernels (bytes through the fabric, VALU/LDS activity)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g24; mkdir -p $O
cd $R
PASSES="pmcA pmcC pmcD" FILTER=spgemm_bm KREGEX=spgemm_bm BENCH_ARGS="--graph off" PMC_DIR=/tmp/pmc1m bash tools/gpu_pmc.sh > $O/pmc_1m.txt 2>&1 || { tail -20 $O/pmc_1m.txt; exit 1; }
cat $O/pmc_1m.txt | head -80
