#!/bin/bash
# 65536^2 row kernel at 512 threads (8 / 10 rounds, 4 waves per SIMD) vs 256 threads (14 rounds, 3 per SIMD)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g35; mkdir -p $O
cd $R
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
SPMM_HIP_LIB=$D/libspmm_hip_n512r8.so timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "bitmap or bench_scale or rowblock" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests (n512r8): $(tail -1 $O/pytest.log)"
for v in base n512r8 n512r10 base n512r8 n512r10; do
  lib=""; [ "$v" = base ] || lib=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -20 $O/b64_$v.err; exit 1; }
  echo "64k $v $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json) $(grep -o '"bitmap_deferred": [0-9]*' $O/b64_$v.json)"
done
