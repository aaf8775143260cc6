cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spgemm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_spgemm.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_spgemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload rmat --steps 2 --warmup 1 > gpurun_out/bench_rmat.log 2>&1 || { tail -20 gpurun_out/bench_rmat.log; exit 1; }
grep metric gpurun_out/bench_rmat.log | cut -c1-330
