#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
echo "== diag 1M" && timeout -k 10 400 python tools/spgemm_diag.py 1048576 0.0001 0,1,2 2>&1 | grep -v amdgpu.ids
echo "== diag 64k" && timeout -k 10 300 python tools/spgemm_diag.py 65536 0.001 0,1,2 2>&1 | grep -v amdgpu.ids
