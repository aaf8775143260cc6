#!/bin/bash
# round-4: chain tile kernel (mul_lo cross terms) + counter-order tree: GPU chain tests, a4 medium timing, traces
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/r4g7; mkdir -p $O
W=/tmp/a4ab; mkdir -p $W
A4=$PWD/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/bin/a4
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bsr_chain.py tests/test_a4_native.py tests/test_dist_chain.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'benches'); sys.path.insert(0,'.')
from bench_a4_e2e import generate; print(generate('$W/in','medium',7))" > $O/gen.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 $A4 $W/in --quiet --out $W/matrix --metrics-json $O/m_$i.json --device hip > $O/a4_$i.log 2>&1 || exit 1
  echo "$i $(cat $O/a4_$i.log) $(grep -o '"kernel_s": [0-9.e-]*' $O/m_$i.json) $(grep -o '"wall_s": [0-9.e-]*' $O/m_$i.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace -d $GRAFT_REPO_ROOT/$O/trace -o run -- $A4 $W/in --quiet --out $W/matrix --device hip > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
echo rc=$?
