#!/bin/bash
# round-5 baseline: 1M + 64k bench, phase stamps of the 1M bitmap kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g01; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_stamps.py > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
tail -9 $O/stamps.log
