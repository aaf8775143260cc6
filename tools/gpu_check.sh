#!/bin/bash
# GPU check: distributed-device tests (loopback ranks on one GPU), the
# full GPU suite, smoke, the headline bench at 1 rank and at 2 gloo ranks on the
# one card (self-launched by bench.py --gpus 2).  STEPS selects what runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3}
mkdir -p $O
cd $R
for st in ${STEPS:-dist gpu smoke bench bench2}; do
  case $st in
    dist)
      echo "== pytest dist-device"
      timeout -k 10 600 python -u -m pytest tests/test_dist_device.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 1; }
      grep -E "passed|failed" $O/pytest_dist.log | tail -2 ;;
    gpu)
      echo "== pytest gpu (all)"
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYARGS} > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
      grep -E "passed|failed" $O/pytest_gpu.log | tail -2 ;;
    det)
      echo "== pytest deterministic"
      timeout -k 10 600 python -u -m pytest tests/test_spgemm.py -m gpu -k deterministic -x -v --timeout 300 --timeout-method thread > $O/pytest_det.log 2>&1 || { grep -E "FAILED|Error|assert|passed|failed" $O/pytest_det.log | tail -20; exit 1; }
      grep -E "passed|failed" $O/pytest_det.log | tail -2 ;;
    benchdet)
      echo "== bench 1 rank, deterministic"
      SPMM_SPGEMM_DETERMINISTIC=1 timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench1_det.log 2>&1 || { tail -20 $O/bench1_det.log; exit 1; }
      grep '"metric"' $O/bench1_det.log > $O/bench1_det.json; cut -c1-300 $O/bench1_det.json ;;
    spmm)
      echo "== pytest spmm"
      timeout -k 10 600 python -u -m pytest tests/test_spmm.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_spmm.log 2>&1 || { grep -E "FAILED|Error|assert|passed|failed" $O/pytest_spmm.log | tail -20; exit 1; }
      grep -E "passed|failed" $O/pytest_spmm.log | tail -2
      for db in 0 1 0 1; do
        SPMM_SPMM_MFMA_DB=$db timeout -k 10 300 python -u bench.py --workload spmm --steps 20 --warmup 5 > $O/bench_spmm_db$db.log 2>&1 || { tail -20 $O/bench_spmm_db$db.log; exit 1; }
        echo "db=$db $(grep -o '"ms_per_step": [0-9.]*' $O/bench_spmm_db$db.log) $(grep -o '"value": [0-9.]*' $O/bench_spmm_db$db.log) $(grep -o '"spmm_method": "[a-z]*"' $O/bench_spmm_db$db.log) $(grep -o '"inspector_ms": [0-9.]*' $O/bench_spmm_db$db.log) $(grep -o '"inspector_first_ms": [0-9.]*' $O/bench_spmm_db$db.log)"
      done
      for meth in rowwise; do
        SPMM_MFMA_MIN_REUSE=100 timeout -k 10 300 python -u bench.py --workload spmm --steps 20 --warmup 5 > $O/bench_spmm_row.log 2>&1 || { tail -20 $O/bench_spmm_row.log; exit 1; }
        echo "rowwise $(grep -o '"ms_per_step": [0-9.]*' $O/bench_spmm_row.log) $(grep -o '"spmm_method": "[a-z]*"' $O/bench_spmm_row.log)"
      done ;;
    rows64k)
      for v in auto on auto on; do
        SPMM_SPGEMM_BITMAP_ROWS=$v timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 20 --warmup 3 > $O/bench64k_rows_$v.log 2>&1 || { tail -20 $O/bench64k_rows_$v.log; exit 1; }
        echo "rows=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench64k_rows_$v.log)"
      done ;;
    long)
      echo "== pytest long rows / rmat"
      timeout -k 10 900 python -u -m pytest tests/test_spgemm.py -m gpu -x -v --timeout 300 --timeout-method thread -k "long or rmat or streamed or onepass or column_sliced" > $O/pytest_long.log 2>&1 || { grep -E "FAILED|Error|assert|passed|failed" $O/pytest_long.log | tail -20; exit 1; }
      grep -E "passed|failed" $O/pytest_long.log | tail -2 ;;
    smoke)
      echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      echo "== bench 1 rank"
      timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench1.log 2>&1 || { tail -20 $O/bench1.log; exit 1; }
      grep '"metric"' $O/bench1.log > $O/bench1.json; cut -c1-300 $O/bench1.json ;;
    bench2)
      echo "== bench 2 gloo ranks, self-launched"
      timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 ${BENCH_ARGS} > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
      grep '"metric"' $O/bench2.log > $O/bench2.json; cut -c1-300 $O/bench2.json ;;
    wl)
      for wl in ${WLS:-spgemm64k spmm rmat chain}; do
        echo "== bench $wl"
        args="--steps 5 --warmup 2"
        [ $wl = rmat ] && args="--steps 2 --warmup 1"
        timeout -k 10 600 python -u bench.py --workload $wl $args > $O/bench_$wl.log 2>&1 || { tail -20 $O/bench_$wl.log; exit 1; }
        grep '"metric"' $O/bench_$wl.log > $O/bench_$wl.json; cut -c1-300 $O/bench_$wl.json
      done ;;
  esac
done
