#!/bin/bash
# 65536^2 on the pipelined row numeric kernel (cfg 1 at 12 / 14 register rounds, 3 waves per SIMD)
# vs the per-unit kernel: bitmap tests on the variant, 64k A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g27; mkdir -p $O
cd $R
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
SPMM_HIP_LIB=$D/libspmm_hip_rp14w3.so SPMM_SPGEMM_BITMAP_ROWS=on timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "bitmap or bench_scale" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
for v in base rp14w3 rp12w3 base rp14w3; do
  lib=""; rows=""; [ "$v" = base ] || { lib=$D/libspmm_hip_$v.so; rows=on; }
  SPMM_SPGEMM_BITMAP_ROWS=$rows SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -20 $O/b64_$v.err; exit 1; }
  echo "64k $v $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
