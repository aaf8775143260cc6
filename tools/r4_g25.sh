#!/bin/bash
# round-4: where the native a4's host gaps go -- HIP API trace of a medium chain (no counters)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g25; mkdir -p $O
W=/tmp/a4m; mkdir -p $W
A4=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/bin/a4
cd $R
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'benches'); sys.path.insert(0,'.')
from bench_a4_e2e import generate; print(generate('$W/in','${PRESET:-medium}',7))" > $O/gen.log 2>&1 || { tail -5 $O/gen.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace -d /tmp/pa -o prof --output-format csv -- $A4 $W/in --quiet --out $W/matrix --device hip > $O/a4.log 2>&1 || { tail -5 $O/a4.log; exit 1; }
cat $O/a4.log
f=$(find /tmp/pa -name "*hip_api_trace.csv" | head -1)
python3 $R/tools/api_top.py $f 15 | tee $O/api_top.txt
k=$(find /tmp/pa -name "*kernel_trace.csv" | head -1)
python3 $R/tools/busy_union.py $k | tee -a $O/api_top.txt
