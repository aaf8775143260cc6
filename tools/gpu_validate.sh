#!/bin/bash
# validation run: full GPU suite + smoke, 1M / 64k benches, kernel stats of both graph steps (full CSVs),
# rank emulation N = 1 / 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/validate; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
echo "gpu suite: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b64.json)"
: > $O/rank_emulate.jsonl
for w in 1 8; do
  timeout -k 10 300 python -u tools/rank_emulate.py --world $w --rank 0 >> $O/rank_emulate.jsonl 2> $O/rank_emulate.err || { tail -20 $O/rank_emulate.err; exit 1; }
done
cat $O/rank_emulate.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppva -o prof --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof1m.log 2>&1 || { tail -20 $O/prof1m.log; exit 1; }
cp $(find /tmp/ppva -name "*kernel_stats.csv" | head -1) $O/spgemm1m_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppvb -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
cp $(find /tmp/ppvb -name "*kernel_stats.csv" | head -1) $O/spgemm64k_kernel_stats.csv
echo profiles done
