#!/bin/bash
# round-5: stamps of both pipelined kernels; PMC (A, B, C) of the 1M bitmap kernels; 64k bench check
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g05; mkdir -p $O
cd $R
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_stamps.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
tail -8 $O/stamps.log
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
PASSES="pmcA pmcB pmcC pmcD" PMC_DIR=/tmp/pmc5 KREGEX=spgemm_bm_rows FILTER=spgemm_bm_rows timeout -k 10 600 bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -30 $O/pmc.log; exit 1; }
for x in A B C D; do cp $R/gpurun_out/pmc$x.txt $O/; done
cat $O/pmcA.txt $O/pmcB.txt $O/pmcC.txt $O/pmcD.txt | grep -v "^$"
for e in "SPMM_SPGEMM_BITMAP_ROWS=on" "SPMM_SPGEMM_BITMAP_ROWS=on SPMM_SPGEMM_BITMAP_PIPE=0"; do
  env $e timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64r.json 2> $O/b64r.err || { tail -20 $O/b64r.err; exit 1; }
  echo "64k [$e] $(grep -o '"ms_per_step": [0-9.]*' $O/b64r.json) deferred $(grep -o '"bitmap_deferred": [0-9]*' $O/b64r.json)"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json)"
