#!/bin/bash
# SpGEMM 1M diag under several sliced-table load factors
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for L in ${LOADS:-0.35 0.5 0.6}; do
  echo "== load $L"
  SPMM_SPGEMM_LOAD_SLICED=$L timeout -k 10 300 python tools/spgemm_diag.py 1048576 0.0001 2>&1 | grep -v amdgpu.ids || exit 1
done
