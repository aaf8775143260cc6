#!/bin/bash
# round-4: bm_pad_pairs with lane-shuffle window bounds (VARS=pshfl) vs main: tests incl. loopback dist, kernel stats, benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
O=$R/gpurun_out/r4g37; mkdir -p $O
cd $R
v=${VARS:-pshfl}
SPMM_HIP_LIB=$L/diag/libspmm_hip_$v.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py tests/test_a4_native.py tests/test_dist_device.py -k "bitmap or bench_scale or graph or mtx or loopback" -m gpu > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
echo "$v $(tail -1 $O/pytest_$v.log)"
cd /tmp && export TMPDIR=/tmp
for x in main $v; do
  if [ $x = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$x.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp_$x -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --graph off > $O/prof_$x.log 2>&1 || { tail -20 $O/prof_$x.log; exit 1; }
  f=$(find /tmp/pp_$x -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_$x.md "$x" && grep -E "pad_pairs|spgemm_bm_rows" $O/prof_$x.md | cut -c1-140
done
cd $R
for x in main $v main $v; do
  if [ $x = main ]; then lib=$L/libspmm_hip.so; else lib=$L/diag/libspmm_hip_$x.so; fi
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m_$x.json 2> $O/b1m_$x.err || { tail -5 $O/b1m_$x.err; exit 1; }
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$x.json 2> $O/b64_$x.err || { tail -5 $O/b64_$x.err; exit 1; }
  echo "$x 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$x.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$x.json)"
done
