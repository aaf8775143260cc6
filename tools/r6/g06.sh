#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g07; mkdir -p $O
cd $R
SPMM_LINK_PRIO=-1 timeout -k 10 120 python -u tools/r6/diag_panel2.py > $O/prio_hi.log 2>&1; echo "rc $?"


grep -v amdgpu.ids $O/prio_hi.log
