#!/bin/bash
# round-4: 65536^2 on the row-major numeric kernel (cfg 1 rows at 12 / 14 register rounds) vs the per-unit default
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
O=$R/gpurun_out/r4g31; mkdir -p $O
cd $R
for v in r14; do
  SPMM_SPGEMM_BITMAP_ROWS=on SPMM_HIP_LIB=$L/diag/libspmm_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_spgemm.py -k "bitmap and not det" -m gpu > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for v in main r14 r12 main r14 r12; do
  if [ $v = main ]; then lib=$L/libspmm_hip.so; rows=auto; else lib=$L/diag/libspmm_hip_$v.so; rows=on; fi
  SPMM_SPGEMM_BITMAP_ROWS=$rows SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -5 $O/b64_$v.err; exit 1; }
  echo "$v 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
cd /tmp && export TMPDIR=/tmp
SPMM_SPGEMM_BITMAP_ROWS=on SPMM_HIP_LIB=$L/diag/libspmm_hip_r14.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p64r -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 20 --warmup 3 --graph off > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
f=$(find /tmp/p64r -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof64.md "64k kernel stats (row kernel r14)" && sed -n 5,14p $O/prof64.md | cut -c1-150
