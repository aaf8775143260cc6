#!/bin/bash
# round-5: buffer range-check probe; phase stamps of the pipelined vs flat numeric row kernel; PMC A/B of the 1M kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g03; mkdir -p $O
cd $R
timeout -k 5 60 ./tools/probes/buffer_oob > $O/buffer_oob.txt 2>&1 || { tail -5 $O/buffer_oob.txt; exit 1; }
tail -1 $O/buffer_oob.txt
for x in 1 0; do
  SPMM_SPGEMM_BITMAP_PIPE=$x SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_stamps.py > $O/stamps_$x.log 2>&1 || { tail -20 $O/stamps_$x.log; exit 1; }
  echo "== pipe=$x"; tail -8 $O/stamps_$x.log
done
for x in 1 0; do
  SPMM_SPGEMM_BITMAP_PIPE=$x PASSES="pmcA pmcB" PMC_DIR=/tmp/pmc_$x KREGEX=spgemm_bm_rows FILTER=spgemm_bm_rows timeout -k 10 600 bash tools/gpu_pmc.sh > $O/pmc_$x.log 2>&1 || { tail -30 $O/pmc_$x.log; exit 1; }
  cp $R/gpurun_out/pmcA.txt $O/pmcA_$x.txt; cp $R/gpurun_out/pmcB.txt $O/pmcB_$x.txt
  echo "== pmc pipe=$x"; cat $O/pmcA_$x.txt $O/pmcB_$x.txt | grep -v "^$"
done
