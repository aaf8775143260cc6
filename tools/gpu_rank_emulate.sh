#!/bin/bash
# per-rank local cost of the 1M row-block step at N = 1, 2, 4, 8 (rank 0) on one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
: > $O/rank_emulate.jsonl
for w in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 300 python -u tools/rank_emulate.py --world $w --rank 0 >> $O/rank_emulate.jsonl 2> $O/rank_emulate.err || { tail -20 $O/rank_emulate.err; exit 1; }
done
cat $O/rank_emulate.jsonl
