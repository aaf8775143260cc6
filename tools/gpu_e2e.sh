#!/bin/bash
# a4 end-to-end on report-sized inputs (Table 1) + a 2-rank bench.py rehearsal over gloo on one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
df -h /tmp | tail -1
for p in ${PRESETS:-small medium}; do
  echo "== a4 e2e $p"
  timeout -k 10 600 python -u benches/bench_a4_e2e.py --preset $p --device hip --json $O/a4_e2e_$p.json > $O/a4_e2e_$p.log 2>&1 || { tail -20 $O/a4_e2e_$p.log; exit 1; }
  cut -c1-600 $O/a4_e2e_$p.log | grep metric
done
[ -n "$NO_REHEARSAL" ] && exit 0
echo "== bench rehearsal: 2 ranks, gloo, one GPU"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29411 \
  bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --matrix-n 262144 > $O/bench_gloo2.log 2>&1 || { tail -30 $O/bench_gloo2.log; exit 1; }
grep metric $O/bench_gloo2.log | cut -c1-400
