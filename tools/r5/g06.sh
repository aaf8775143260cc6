#!/bin/bash
# round-5: window-major unit order experiment (per-unit numeric kernel, 1M): does one window's B slice stay in the MALL?
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g06; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "bitmap_matches_binned or bench_scale" -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "tests (pipe+scan): $(tail -1 $O/pytest.log)"
SPMM_SPGEMM_BITMAP_WMAJOR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "bitmap_matches_binned or bench_scale" -m gpu > $O/pytest_wm.log 2>&1 || { tail -30 $O/pytest_wm.log; exit 1; }
echo "tests (wmajor): $(tail -1 $O/pytest_wm.log)"
for e in "SPMM_SPGEMM_BITMAP_WMAJOR=0" "SPMM_SPGEMM_BITMAP_WMAJOR=1" "SPMM_SPGEMM_BITMAP_WMAJOR=2"; do
  env $e timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --graph off > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "1M [$e] $(grep -o '"ms_per_step": [0-9.]*' $O/b.json)"
done
cd /tmp && export TMPDIR=/tmp
for x in 2 1; do
  SPMM_SPGEMM_BITMAP_WMAJOR=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pw$x -o prof --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --graph off > $O/prof$x.log 2>&1 || { tail -20 $O/prof$x.log; exit 1; }
  f=$(find /tmp/pw$x -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof$x.md "wmajor=$x" && grep -E "spgemm_bm" $O/prof$x.md | cut -c1-150
done
