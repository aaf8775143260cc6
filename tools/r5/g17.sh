#!/bin/bash
# round-5: A/B on one box -- 1M / 64k step with the compare-swap LDS adds vs plain ds_add_f32 in the bitmap kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g17; mkdir -p $O
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
cd $R
for rep in 1 2; do
for v in cas nat; do
  L=""; [ $v = nat ] && L=$D/libspmm_hip_faddnat.so
  SPMM_HIP_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m_$v.json 2> $O/b1m_$v.err || { tail -20 $O/b1m_$v.err; exit 1; }
  SPMM_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -20 $O/b64_$v.err; exit 1; }
  echo "$rep $v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m_$v.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
done
: > $O/rank_emulate.jsonl
for w in 1 8; do
  timeout -k 10 300 python -u tools/rank_emulate.py --world $w --rank 0 >> $O/rank_emulate.jsonl 2> $O/rank_emulate.err || { tail -20 $O/rank_emulate.err; exit 1; }
done
cat $O/rank_emulate.jsonl
