#!/bin/bash
# Multi-rank rehearsal of bench.py on one GPU (gloo transport, same code path as RCCL apart from the wire)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for n in ${NRANKS:-2 4}; do
  echo "== $n ranks"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2941$n \
    bench.py --gpus $n --steps 2 --warmup 1 --backend gloo ${ARGS} > $O/bench_gloo$n.log 2>&1 || { tail -30 $O/bench_gloo$n.log; exit 1; }
  grep metric $O/bench_gloo$n.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench_spgemm.log 2>&1 || { tail -20 $O/bench_spgemm.log; exit 1; }
grep metric $O/bench_spgemm.log | cut -c1-200
