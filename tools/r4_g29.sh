#!/bin/bash
# round-4: per-unit numeric on padded pairs (16-byte loads): bitmap + mtx GPU tests, 64k / 1M benches, 64k kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g29; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py tests/test_a4_native.py -k "bitmap or bench_scale or graph or mtx or deterministic" -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$i.json 2> $O/b64_$i.err || { tail -5 $O/b64_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m_$i.json 2> $O/b1m_$i.err || { tail -5 $O/b1m_$i.err; exit 1; }
  echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$i.json) 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$i.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p64w -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 20 --warmup 3 --graph off > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
f=$(find /tmp/p64w -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof64.md "64k kernel stats (wide per-unit numeric)" && sed -n 5,14p $O/prof64.md | cut -c1-150
