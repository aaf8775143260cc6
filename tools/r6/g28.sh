#!/bin/bash
# cfg 1 on the pipelined row kernel by default: SpGEMM GPU tests, 64k / 1M benches, 64k kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g28; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_dist_device.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$i.json 2> $O/b64_$i.err || { tail -20 $O/b64_$i.err; exit 1; }
  echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$i.json)"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppvb -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
cp $(find /tmp/ppvb -name "*kernel_stats.csv" | head -1) $O/spgemm64k_kernel_stats.csv
head -4 $O/spgemm64k_kernel_stats.csv | cut -c1-160
