#!/bin/bash
# R-MAT streamed panels handed over before their last copies finish (overlap): tests, bench + allocator counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g41; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "overlap or pipelined or long_rows or streamed or rmat" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
timeout -k 10 400 python -u tools/r6/rmat_memstats.py --workload rmat --steps 2 --warmup 1 > $O/rmat.json 2> $O/rmat.err || { tail -20 $O/rmat.err; exit 1; }
echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rmat.json) $(grep -o '"nnz_C": [0-9]*' $O/rmat.json) $(grep -o '"sum_col": [0-9]*' $O/rmat.json)"
grep memstats $O/rmat.err
