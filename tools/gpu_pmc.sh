#!/bin/bash
# PMC passes over one bench step (counters only, kernel-trace; no tracing domains), summarised per
# kernel.  WL = bench workload (default spgemm), FILTER = kernel-name filter (default spgemm_),
# PASSES = subset of pmcA..pmcE (E: MFMA), KREGEX = kernels to collect, BENCH_ARGS, PMC_DIR
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
pass() {  # name, counters...
  echo "== $1"
  timeout -k 10 300 rocprofv3 --kernel-trace ${KREGEX:+--kernel-include-regex "$KREGEX"} --pmc "${@:2}" -d ${PMC_DIR:-$O}/$1 -o pmc --output-format csv -- python3 $R/bench.py --workload ${WL:-spgemm} --steps 1 --warmup 0 ${BENCH_ARGS} > $O/$1.log 2>&1 || { tail -20 $O/$1.log; return 1; }
}
PASSES=${PASSES:-pmcA pmcB pmcC pmcD}
declare -A CTR=(
  [pmcA]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
  [pmcB]="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
  [pmcC]="SQ_WAVES FETCH_SIZE TCC_HIT_sum"
  [pmcD]="SQ_WAVES WRITE_SIZE TCC_MISS_sum SQ_INSTS_VMEM_WR"
  [pmcE]="SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE")
for p in $PASSES; do pass $p ${CTR[$p]} || exit 1; done
cd $R
for p in $PASSES; do
  f=$(find ${PMC_DIR:-$O}/$p -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $f ${FILTER:-spgemm_} > $O/$p.txt && cat $O/$p.txt
done
