#!/bin/bash
# round-4: A/B of the chain tile kernel's MAC (speculative 3x mad / speculative mul_lo cross terms / exact only)
# on the native a4 medium preset, plus a kernel-stats profile and one PMC pass of the default build.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/r4g6; mkdir -p $O
W=/tmp/a4ab; mkdir -p $W
L=sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib
A4=sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/bin/a4
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'benches'); sys.path.insert(0,'.')
from bench_a4_e2e import generate; print(generate('$W/in','medium',7))" > $O/gen.log 2>&1 || exit 1
rc=0
for v in main spec0 xmul main spec0 xmul; do
  d=$W/lib_$v; mkdir -p $d
  if [ $v = main ]; then ln -sf $PWD/$L/libspmm_hip.so $d/libspmm_hip.so; else ln -sf $PWD/$L/diag/libspmm_hip_$v.so $d/libspmm_hip.so; fi
  ln -sf $PWD/$L/libspmm_host.so $d/libspmm_host.so
  LD_LIBRARY_PATH=$d:$LD_LIBRARY_PATH timeout -k 10 120 $A4 $W/in --quiet --out $W/matrix --metrics-json $O/m_$v.json --device hip > $O/a4_$v.log 2>&1 || { rc=$?; break; }
  echo "$v $(grep -o '"kernel_s": [0-9.e-]*' $O/m_$v.json)" | tee -a $O/ab.txt
done
[ $rc = 0 ] || { echo rc=$rc; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- $GRAFT_REPO_ROOT/$A4 $W/in --quiet --out $W/matrix --device hip > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex bsr_u64 -d $GRAFT_REPO_ROOT/$O/pmc -o run -- $GRAFT_REPO_ROOT/$A4 $W/in --quiet --out $W/matrix --device hip > $GRAFT_REPO_ROOT/$O/pmc.log 2>&1
echo rc=$?
