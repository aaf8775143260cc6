#!/bin/bash
# round-4: chain Large preset: kernel-phase busy time of the tile kernel (kernel trace of the native a4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g18; mkdir -p $O
W=/tmp/a4l; mkdir -p $W
A4=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/bin/a4
cd $R
timeout -k 10 600 python -u -c "
import sys; sys.path.insert(0,'benches'); sys.path.insert(0,'.')
from bench_a4_e2e import generate; print(generate('$W/in','large',7))" > $O/gen.log 2>&1 || { tail -5 $O/gen.log; exit 1; }
tail -1 $O/gen.log
timeout -k 10 300 $A4 $W/in --quiet --out $W/matrix --metrics-json $O/m_large.json --device hip > $O/a4_large.log 2>&1 || exit 1
cat $O/a4_large.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pl -o prof --output-format csv -- $A4 $W/in --quiet --out $W/matrix --device hip > $O/prof_large.log 2>&1 || { tail -5 $O/prof_large.log; exit 1; }
f=$(find /tmp/pl -name "*kernel_trace.csv" | head -1)
python3 $R/tools/busy_union.py $f numeric_lds | tee $O/busy_large.txt
python3 $R/tools/busy_union.py $f | tee -a $O/busy_large.txt
