#!/bin/bash
# tests changed in the docs pass: SpMM (row-group kernel on one-sided / unsorted rows), bitmap row-kernel selectors
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g21; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spmm.py tests/test_spgemm.py -k "spmm or row_kernels" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
