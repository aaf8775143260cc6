#!/bin/bash
# round-4: count-kernel time decomposition (diagnostic builds with wrong counts: the bench step is
# expected to fail its count check; only the kernel times are read)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g12; mkdir -p $O
L=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-dnold dnoor}; do
  SPMM_HIP_LIB=$L/diag/libspmm_hip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_$v -o prof --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --graph off > $O/prof_$v.log 2>&1
  rc=$?
  [ $rc -ge 124 ] && { echo "$v rc=$rc"; exit 1; }
  f=$(find /tmp/p_$v -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && python3 $R/tools/prof_summary.py $f $O/prof_$v.md "$v kernel stats" && grep -E "count|spgemm_bm_rows<" $O/prof_$v.md | cut -c1-140
done
echo ok
