#!/bin/bash
# R-MAT overlap with a high-priority side stream: tests, bench + allocator counters, kernel trace windows
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g42; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "overlap or pipelined or long_rows or streamed or rmat" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
timeout -k 10 400 python -u tools/r6/rmat_memstats.py --workload rmat --steps 2 --warmup 1 > $O/rmat.json 2> $O/rmat.err || { tail -20 $O/rmat.err; exit 1; }
echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rmat.json) $(grep -o '"nnz_C": [0-9]*' $O/rmat.json) $(grep -o '"sum_col": [0-9]*' $O/rmat.json)"
grep memstats $O/rmat.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace -d /tmp/prm -o prof --output-format csv -- python3 $R/tools/rmat_steps.py 24 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep "^step" $O/trace.log
f=$(find /tmp/prm -name "*kernel_trace.csv" | head -1)
python3 $R/tools/r6/timeline_window.py $f long_place 300 40 40 > $O/win_place300.txt
python3 $R/tools/overlap.py $f long_place long_dense long_rank long_route spgemm_esc compact > $O/rmat_overlap.txt
cat $O/rmat_overlap.txt; awk '{print $3}' $O/win_place300.txt | sort | uniq -c
