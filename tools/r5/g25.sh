#!/bin/bash
# round-5: long_dense fresh-slot skip A/B (same box) + R-MAT 24 bench in driver form
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g25; mkdir -p $O
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "long or rmat" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in fresh nofresh; do
  L=""; [ $v = nofresh ] && L=$D/libspmm_hip_nofresh.so
  SPMM_HIP_LIB=$L timeout -k 10 200 python -u tools/r5/rmat_steps.py 24 2 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^step' $O/$v.log | tr '\n' ' ')"
done
timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 0 > $O/brmat.json 2> $O/brmat.err || { tail -20 $O/brmat.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/brmat.json')); print('rmat', d['ms_per_step'], d['nnz_C'], d['c_checksum'], d['value'])"
