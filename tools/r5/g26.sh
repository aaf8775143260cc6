#!/bin/bash
# round-5: PMC of the product-parallel route + dense kernels, one R-MAT 24 step (two counter passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g26; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "long_(route_pp|dense)" --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d /tmp/pm26a -o pmc --output-format csv -- python3 $R/tools/r5/rmat_steps.py 24 1 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
f=$(find /tmp/pm26a -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_summary.py $f long_ --md $O/pmc_a.md > $O/pmc_a.txt && cat $O/pmc_a.txt | head -80
timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex "long_(route_pp|dense)" --pmc FETCH_SIZE TCC_HIT_sum SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -d /tmp/pm26b -o pmc --output-format csv -- python3 $R/tools/r5/rmat_steps.py 24 1 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
f=$(find /tmp/pm26b -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_summary.py $f long_ --md $O/pmc_b.md > $O/pmc_b.txt && cat $O/pmc_b.txt | head -80
