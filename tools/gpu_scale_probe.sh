#!/bin/bash
# Strong-scaling probe on one GPU: per-rank local cost at N = 1, 2, 4, 8 (rank 0 and last rank),
# a 2-rank gloo rehearsal of bench.py, and the a4 medium e2e (writer check)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
: > $O/rank_emulate.jsonl
for w in 1 2 4 8; do
  timeout -k 10 300 python -u tools/rank_emulate.py --world $w --rank 0 >> $O/rank_emulate.jsonl 2> $O/rank_emulate.err || { tail -20 $O/rank_emulate.err; exit 1; }
done
timeout -k 10 300 python -u tools/rank_emulate.py --world 8 --rank 7 >> $O/rank_emulate.jsonl 2>> $O/rank_emulate.err || { tail -20 $O/rank_emulate.err; exit 1; }
cat $O/rank_emulate.jsonl
echo "== bench rehearsal: 2 ranks, gloo, one GPU"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29411 \
  bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo > $O/bench_gloo2.log 2>&1 || { tail -30 $O/bench_gloo2.log; exit 1; }
grep metric $O/bench_gloo2.log | cut -c1-300
echo "== a4 e2e medium"
timeout -k 10 600 python -u benches/bench_a4_e2e.py --device hip --preset medium --json $O/a4_e2e_medium.json > $O/a4_e2e_medium.log 2>&1 || { tail -20 $O/a4_e2e_medium.log; exit 1; }
python -c "import json; d=json.load(open('$O/a4_e2e_medium.json')); p=d['phases']; print(d['value'], 's reduce', p['t_reduce_s'], 'write', p['t_write_s'])"
