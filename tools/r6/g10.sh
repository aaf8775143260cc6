#!/bin/bash
# per-unit tickets removed: the RCCL one-rank graph test first, 1M A/B (numeric tickets vs
# numeric + count tickets), 64k, R-MAT scale 24 A/B (long_dense item tickets vs static);
# LAST the multi-graph tests (graphs kept alive)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g10; mkdir -p $O
cd $R
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "rccl_one_rank or graph_replay or bitmap_matches" > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
for v in base tk3 base tk3; do
  lib=""; [ "$v" = base ] || lib=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  echo "$v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/ab_$v.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/ab_$v.json)"
done
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
for v in base lt0 base lt0; do
  lib=""; [ "$v" = base ] || lib=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_$v.json 2> $O/rm_$v.err || { tail -20 $O/rm_$v.err; exit 1; }
  echo "$v rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rm_$v.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_$v.json) $(grep -o '"checksum[a-z_]*": [-0-9.e]*' $O/rm_$v.json)"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py -k "panel_comm or rowblock_graph" > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
echo "tests b: $(tail -1 $O/pytest_b.log)"
