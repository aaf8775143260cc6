#!/bin/bash
# Two PMC passes over the SpGEMM 1M diagnostics (counters only, no tracing domains)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "== pass 1" && timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmcA -o pmc --output-format csv -- python3 $R/tools/spgemm_diag.py 1048576 0.0001 > $O/pmcA.log 2>&1 || { tail -20 $O/pmcA.log; exit 1; }
echo "== pass 2" && timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $O/pmcB -o pmc --output-format csv -- python3 $R/tools/spgemm_diag.py 1048576 0.0001 > $O/pmcB.log 2>&1 || { tail -20 $O/pmcB.log; exit 1; }
cd $R
for p in pmcA pmcB; do f=$(find $O/$p -name "*counter_collection.csv" | head -1); python tools/pmc_summary.py $f spgemm_lds; done
