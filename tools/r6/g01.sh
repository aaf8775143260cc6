#!/bin/bash
# round 6, first GPU call: new tests (count descriptor batches, lazy rerun, RowblockGraph at W=1 RCCL and
# W=2/7/8 loopback), the 1M / 64k benches, rank-0-of-8 step emulation with the gather, per-WG numeric timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g01; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "descriptor_batches or truncated_window or rccl_one_rank or count_units or bitmap_matches_binned" \
  > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py -k "rowblock_graph or bench_problem" > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
echo "tests b: $(tail -1 $O/pytest_b.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,150,300,600 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 8 > $O/wg8.json 2> $O/wg8.err || { tail -20 $O/wg8.err; exit 1; }
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 1 > $O/wg1.json 2> $O/wg1.err || { tail -20 $O/wg1.err; exit 1; }
cat $O/wg8.json $O/wg1.json
