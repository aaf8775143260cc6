#!/bin/bash
# round-5: row-kernel register rounds (10 / 12 / 14) -- 1M step, 64k step with the row kernels forced on
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g22; mkdir -p $O
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
cd $R
for v in base rr12 rr14; do
  L=""; [ $v != base ] && L=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m_$v.json 2> $O/b1m_$v.err || { tail -20 $O/b1m_$v.err; exit 1; }
  SPMM_HIP_LIB=$L SPMM_SPGEMM_BITMAP_ROWS=on timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64r_$v.json 2> $O/b64r_$v.err || { tail -20 $O/b64r_$v.err; exit 1; }
  echo "$v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$v.json) 64k-rows $(grep -o '"ms_per_step": [0-9.]*' $O/b64r_$v.json) $(grep -o '"bitmap_deferred": [0-9]*' $O/b64r_$v.json)"
done
