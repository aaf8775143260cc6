#!/bin/bash
# row-group MFMA SpMM with slice-major staging: tests, bench (mfma vs sweep), PMC of the new kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g20; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spmm.py > $O/pytest_spmm.log 2>&1 || { tail -40 $O/pytest_spmm.log; exit 1; }
echo "spmm tests: $(tail -1 $O/pytest_spmm.log)"
for meth in mfma sweep mfma sweep; do
  timeout -k 10 200 python -u bench.py --workload spmm --spmm-method $meth --steps 50 --warmup 10 > $O/spmm_$meth.json 2> $O/spmm_$meth.err || { tail -20 $O/spmm_$meth.err; exit 1; }
  echo "spmm $meth $(grep -o '"ms_per_step": [0-9.]*' $O/spmm_$meth.json)"
done
WL=spmm BENCH_ARGS="--spmm-method mfma" FILTER=spmm_ KREGEX="spmm_rows_mfma" PASSES="pmcA pmcC" \
  PMC_DIR=$O/pmc_mfma bash tools/gpu_pmc.sh > $O/pmc_mfma.txt 2>&1 || { tail -30 $O/pmc_mfma.txt; exit 1; }
grep -v "^==" $O/pmc_mfma.txt | head -30
