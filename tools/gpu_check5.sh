#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== tr16 probe" && timeout -k 10 60 ./tools/probes/tr16_probe > $O/tr16_probe.log 2>&1; head -70 $O/tr16_probe.log | tail -66 | head -20
echo "== diag 64k" && timeout -k 10 300 python tools/spgemm_diag.py 65536 0.001 2>&1 | grep -v amdgpu.ids
echo "== diag 1M" && timeout -k 10 300 python tools/spgemm_diag.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
echo "== pmc" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $O/pmc_64k -o pmc --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 1 --warmup 0 > $O/pmc_64k.log 2>&1 || { tail -20 $O/pmc_64k.log; exit 1; }
echo done
