#!/bin/bash
# round-5: pipelined numeric + count row kernels (row inputs in the peeled last unit) -- bitmap GPU tests, then 1M / 64k bench A/B (pipe vs flat), kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g04; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "bitmap or bench_scale or graph or count or mtx" -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
for x in 1 0 1 0; do
  SPMM_SPGEMM_BITMAP_PIPE=$x timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m_$x.json 2> $O/b1m_$x.err || { tail -20 $O/b1m_$x.err; exit 1; }
  SPMM_SPGEMM_BITMAP_PIPE=$x timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$x.json 2> $O/b64_$x.err || { tail -20 $O/b64_$x.err; exit 1; }
  echo "pipe=$x 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$x.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$x.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --graph off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find /tmp/pp -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof.md "1M pipe" && grep -E "spgemm_bm" $O/prof.md | cut -c1-160
grep -E "spgemm_bm" $O/prof.md | cut -c1-160 > /dev/null; SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_stamps.py > $O/stamps.log 2>&1 && tail -8 $O/stamps.log
