#!/bin/bash
# front reset as a kernel: the row-block graph test (cfg 1 / cfg 0 with row tickets), the replay diagnostic,
# SpGEMM + device-collective GPU tests, 64k / 1M benches, rank 0 of 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g33; mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/r6/diag_rows_graph4.py 65536 1e-3 > $O/diag4.log 2>&1 || { tail -20 $O/diag4.log; exit 1; }
grep "^[0-9]" $O/diag4.log
timeout -k 10 120 python -u tools/r6/diag_rows_graph.py > $O/diag.log 2>&1 || { grep -v "^frame" $O/diag.log | tail -20; exit 1; }
grep "s=" $O/diag.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_dist_device.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$i.json 2> $O/b64_$i.err || { tail -20 $O/b64_$i.err; exit 1; }
  echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$i.json)"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
