#!/bin/bash
# flat row count kernel restored for one-unit rows, count tickets removed: GPU suites, headline, 64k,
# emulated rank 0 of 8; PMC of the SpMM kernels (row-group MFMA vs sweep); multi-graph tests last
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g17; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_spmm.py > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
for meth in mfma sweep; do
  WL=spmm BENCH_ARGS="--spmm-method $meth" FILTER=spmm_ KREGEX="spmm_(rows_mfma|sweep)" PASSES="pmcA pmcB pmcC pmcE" \
    PMC_DIR=$O/pmc_$meth bash tools/gpu_pmc.sh > $O/pmc_$meth.txt 2>&1 || { tail -30 $O/pmc_$meth.txt; exit 1; }
done
tail -40 $O/pmc_mfma.txt; tail -40 $O/pmc_sweep.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
echo "tests b: $(tail -1 $O/pytest_b.log)"
