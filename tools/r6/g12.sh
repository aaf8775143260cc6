#!/bin/bash
# packed column payloads + faster unpack + async long-row placement: tests (packing, RCCL one-rank
# graph, long rows / R-MAT), 1M bench, emulated rank 0 of 8 at 0 / 300 GB/s, R-MAT 24 x2;
# LAST the multi-graph tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g12; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py tests/test_spgemm.py -k "packed or rccl_one_rank or long or rmat or device_branches" > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm$i.json 2> $O/rm$i.err || { tail -20 $O/rm$i.err; exit 1; }
  echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rm$i.json) $(grep -o '"nnz_C": [0-9]*' $O/rm$i.json) $(grep -o '"c_checksum": {[^}]*}' $O/rm$i.json)"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py -k "panel_comm or rowblock_graph" > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
echo "tests b: $(tail -1 $O/pytest_b.log)"
