#!/bin/bash
# round-5: 64-byte segment padding (pairs and/or count columns) vs 128-byte: tests, bench A/B, FETCH_SIZE
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
O=$R/gpurun_out/r5g08; mkdir -p $O
cd $R
SPMM_HIP_LIB=$L/diag/libspmm_hip_pad64.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py -k "bitmap or bench_scale or graph" -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "pad64 tests: $(tail -1 $O/pytest.log)"
for x in main pad64 padn64 padc64 main pad64; do
  if [ $x = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$x.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b_$x.json 2> $O/b_$x.err || { tail -5 $O/b_$x.err; exit 1; }
  echo "$x 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b_$x.json)"
done
cd /tmp && export TMPDIR=/tmp
for x in main pad64; do
  if [ $x = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$x.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk_$x -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $O/prof_$x.log 2>&1 || { tail -20 $O/prof_$x.log; exit 1; }
  f=$(find /tmp/pk_$x -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_$x.md "$x" && grep -E "spgemm_bm_rows|pad_pairs" $O/prof_$x.md | cut -c1-130
  SPMM_HIP_LIB=$lib timeout -k 60 120 rocprofv3 --kernel-trace --kernel-include-regex spgemm_bm_rows --pmc SQ_WAVES FETCH_SIZE -d /tmp/pf_$x -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --graph off > $O/pmc_$x.log 2>&1 || { tail -20 $O/pmc_$x.log; exit 1; }
  f=$(find /tmp/pf_$x -name "*counter_collection.csv" | head -1)
  python3 $R/tools/pmc_summary.py $f spgemm_bm_rows > $O/pmc_$x.txt && cat $O/pmc_$x.txt
done
