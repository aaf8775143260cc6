#!/bin/bash
# row-group MFMA SpMM (tests + config-3 bench per method), R-MAT with placement beside the next
# batch's accumulation (x2), long-row tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g13; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spmm.py > $O/pytest_spmm.log 2>&1 || { tail -40 $O/pytest_spmm.log; exit 1; }
echo "spmm tests: $(tail -1 $O/pytest_spmm.log)"
for meth in mfma sweep panel mfma sweep; do
  timeout -k 10 200 python -u bench.py --workload spmm --spmm-method $meth --steps 50 --warmup 10 > $O/spmm_$meth.json 2> $O/spmm_$meth.err || { tail -20 $O/spmm_$meth.err; exit 1; }
  echo "spmm $meth $(grep -o '"ms_per_step": [0-9.]*' $O/spmm_$meth.json)"
done
timeout -k 10 200 python -u bench.py --workload spmm --steps 50 --warmup 10 > $O/spmm_auto.json 2> $O/spmm_auto.err || { tail -20 $O/spmm_auto.err; exit 1; }
echo "spmm auto $(grep -o '"ms_per_step": [0-9.]*' $O/spmm_auto.json) $(grep -o '"autotune_ms": {[^}]*}' $O/spmm_auto.json)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "long or rmat" > $O/pytest_long.log 2>&1 || { tail -40 $O/pytest_long.log; exit 1; }
echo "long tests: $(tail -1 $O/pytest_long.log)"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm$i.json 2> $O/rm$i.err || { tail -20 $O/rm$i.err; exit 1; }
  echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rm$i.json) $(grep -o '"nnz_C": [0-9]*' $O/rm$i.json) $(grep -o '"c_checksum": {[^}]*}' $O/rm$i.json)"
done
