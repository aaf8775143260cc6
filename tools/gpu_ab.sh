#!/bin/bash
# A/B: SpGEMM 1M diag + bench under two env settings ($AB_VAR = values in $AB_VALUES)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 300 python -m pytest tests/test_spgemm.py -m gpu -x -q 2>&1 | tail -2 || exit 1
for v in $AB_VALUES; do
  echo "== $AB_VAR=$v"
  env $AB_VAR=$v timeout -k 10 300 python tools/spgemm_diag.py 1048576 0.0001 2>&1 | grep -v amdgpu.ids | grep -v symbolic || exit 1
  env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 || exit 1
done
