#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
echo "== pmc 1M" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d $O/pmc_1m -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $O/pmc_1m.log 2>&1 || { tail -20 $O/pmc_1m.log; exit 1; }
echo done
