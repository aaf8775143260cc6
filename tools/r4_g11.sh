#!/bin/bash
# round-4: SpMM config 3 on each executor (+ MFMA PMC), chain kernel PMC of the default build, R-MAT step
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g11; mkdir -p $O
cd $R
for mth in mfma sweep rowwise auto; do
  timeout -k 10 300 python -u bench.py --workload spmm --spmm-method $mth --steps 20 --warmup 5 > $O/spmm_$mth.json 2> $O/spmm_$mth.err || { tail -5 $O/spmm_$mth.err; exit 1; }
  echo "spmm $mth $(grep -o '"ms_per_step": [0-9.]*' $O/spmm_$mth.json) $(grep -o '"spmm_kernel": "[a-z_]*"' $O/spmm_$mth.json)"
done
WL=spmm BENCH_ARGS="--spmm-method mfma" FILTER=spmm PASSES=pmcE PMC_DIR=/tmp/pmc_spmm bash tools/gpu_pmc.sh > $O/pmc_spmm_mfma.txt 2>&1 || { tail -20 $O/pmc_spmm_mfma.txt; exit 1; }
WL=spmm BENCH_ARGS="--spmm-method sweep" FILTER=spmm PASSES=pmcE PMC_DIR=/tmp/pmc_spmm2 bash tools/gpu_pmc.sh > $O/pmc_spmm_sweep.txt 2>&1 || { tail -20 $O/pmc_spmm_sweep.txt; exit 1; }
W=/tmp/a4c; mkdir -p $W
A4=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/bin/a4
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0,'benches'); sys.path.insert(0,'.')
from bench_a4_e2e import generate; print(generate('$W/in','medium',7))" > $O/gen.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex bsr_u64 -d /tmp/pmc_chain -o run --output-format csv -- $A4 $W/in --quiet --out $W/matrix --device hip > $O/pmc_chain.log 2>&1 || { tail -5 $O/pmc_chain.log; exit 1; }
f=$(find /tmp/pmc_chain -name "*counter_collection.csv" | head -1); cp $f $O/chain_counters.csv
cd $R
timeout -k 10 600 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rmat.json 2> $O/rmat.err || { tail -5 $O/rmat.err; exit 1; }
echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rmat.json)"
