#!/bin/bash
# round 6: row tickets in the pipelined bitmap kernels -- correctness (bitmap / bench-scale / graph tests),
# benches, per-WG timeline, rank-0-of-8 emulation, kernel stats of the 1M step
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g03; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_dist_device.py -k "bitmap or bench_scale or panel_comm or rccl_one_rank or graph" > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 8 > $O/wg8.json 2> $O/wg8.err || { tail -20 $O/wg8.err; exit 1; }
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 1 > $O/wg1.json 2> $O/wg1.err || { tail -20 $O/wg1.err; exit 1; }
cat $O/wg8.json $O/wg1.json
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp03 -o prof --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $O/prof1m.log 2>&1 || { tail -20 $O/prof1m.log; exit 1; }
cp $(find /tmp/pp03 -name "*kernel_stats.csv" | head -1) $O/spgemm1m_kernel_stats.csv
echo profiled
