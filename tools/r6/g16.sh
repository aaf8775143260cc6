#!/bin/bash
# 64k on the pipelined count kernel (static vs ticket rows), bitmap tests at 65536; then the traces of g15
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g16; mkdir -p $O
cd $R
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "bitmap_matches or graph_replay or bench_scale_sampled or deterministic" > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
for v in base tk3 base tk3; do
  lib=""; [ "$v" = base ] || lib=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -20 $O/b64_$v.err; exit 1; }
  echo "64k $v $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
bash $R/tools/r6/g15.sh
