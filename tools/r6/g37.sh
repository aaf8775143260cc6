#!/bin/bash
# PMC of the 65536^2 row kernels (numeric pipe + flat count): one bench step per pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g37; mkdir -p $O
cd $R
WL=spgemm64k FILTER=spgemm_bm_rows KREGEX="spgemm_bm_rows" PASSES="pmcA pmcB pmcC pmcD" PMC_DIR=$O/pmc \
  bash tools/gpu_pmc.sh > $O/pmc.txt 2>&1 || { tail -30 $O/pmc.txt; exit 1; }
grep -v "^==" $O/pmc.txt | head -60
