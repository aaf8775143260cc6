#!/bin/bash
# long-row grids at 75 % beside the routing: long-row / streamed / native-engine tests, R-MAT x2
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g52; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_a4_native.py -k "side_stream or overlap or pipelined or long_rows or streamed or rmat or onepass or a4" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_$i.json 2> $O/rm_$i.err || { tail -20 $O/rm_$i.err; exit 1; }
  echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rm_$i.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_$i.json) $(grep -o '"sum_col": [0-9]*' $O/rm_$i.json) $(grep -o '"sum_val": [-0-9.e]*' $O/rm_$i.json)"
done
