#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g04; mkdir -p $O
cd $R
SPMM_LINK_PRIO=-1 timeout -k 10 120 python -u tools/r6/diag_panel.py > $O/prio_hi.log 2>&1 || { tail -30 $O/prio_hi.log; exit 1; }
SPMM_LINK_PRIO=0 timeout -k 10 120 python -u tools/r6/diag_panel.py > $O/prio_0.log 2>&1 || { tail -30 $O/prio_0.log; exit 1; }
cat $O/prio_hi.log $O/prio_0.log
