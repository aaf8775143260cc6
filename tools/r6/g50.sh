#!/bin/bash
# LDS / ESC bins on the side stream beside the hub rows' routing: tests, R-MAT (side on / off), trace overlap
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g50; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "side_stream or overlap or pipelined or long_rows or streamed or rmat or onepass or vs_dense" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
for sd in 1 0 1; do
  SPMM_SPGEMM_LONG_SIDE=$sd timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_s$sd.json 2> $O/rm_s$sd.err || { tail -20 $O/rm_s$sd.err; exit 1; }
  echo "rmat side $sd $(grep -o '"ms_per_step": [0-9.]*' $O/rm_s$sd.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_s$sd.json) $(grep -o '"sum_col": [0-9]*' $O/rm_s$sd.json) $(grep -o '"sum_val": [-0-9.e]*' $O/rm_s$sd.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace -d /tmp/prm -o prof --output-format csv -- python3 $R/tools/rmat_steps.py 24 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
f=$(find /tmp/prm -name "*kernel_trace.csv" | head -1)
python3 $R/tools/overlap.py $f long_place long_dense long_rank long_route spgemm_esc compact > $O/rmat_overlap.txt
cat $O/rmat_overlap.txt
