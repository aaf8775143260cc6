#!/bin/bash
# round-4: per-rank cost of the 1M row-block step at N = 1/2/4/8 on the current kernels (eager and graph-replayed local product)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g34; mkdir -p $O
cd $R
: > $O/rank_emulate_1m.jsonl
for w in 1 2 4 8; do
  timeout -k 10 240 python -u tools/rank_emulate.py --world $w --steps 5 >> $O/rank_emulate_1m.jsonl 2> $O/err_$w.log || { tail -5 $O/err_$w.log; exit 1; }
  timeout -k 10 240 python -u tools/rank_emulate.py --world $w --steps 5 --graph >> $O/rank_emulate_1m.jsonl 2> $O/errg_$w.log || { tail -5 $O/errg_$w.log; exit 1; }
done
SPMM_SPGEMM_BITMAP_LAZY=1 timeout -k 10 240 python -u tools/rank_emulate.py --world 8 --steps 5 > $O/lazy8.jsonl 2> $O/errl.log || { tail -5 $O/errl.log; exit 1; }
cat $O/rank_emulate_1m.jsonl $O/lazy8.jsonl | cut -c1-220
