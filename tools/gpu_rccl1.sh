#!/bin/bash
# RCCL code paths at world size 1 (SPMM_FORCE_DIST=1): bench workloads through the distributed branches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for wl in spgemm64k spmm chain; do
  SPMM_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29477 bench.py --gpus 1 --workload $wl --steps 3 --warmup 1 > $O/bench_rccl1_$wl.log 2>&1 || { tail -30 $O/bench_rccl1_$wl.log; exit 1; }
  grep metric $O/bench_rccl1_$wl.log | cut -c1-220
done
SPMM_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29478 bench.py --gpus 1 --steps 3 --warmup 1 > $O/bench_rccl1_spgemm.log 2>&1 || { tail -30 $O/bench_rccl1_spgemm.log; exit 1; }
grep metric $O/bench_rccl1_spgemm.log | cut -c1-220
