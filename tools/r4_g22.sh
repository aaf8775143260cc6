#!/bin/bash
# round-4: multi-rank rehearsal on one GPU (gloo ranks sharing the card): per-rank fields, 120 s collective timeout
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g22; mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --workload spmm --gpus 4 --backend gloo --steps 5 --warmup 2 > $O/spmm_4gloo.json 2> $O/spmm_4gloo.err || { tail -20 $O/spmm_4gloo.err; exit 1; }
cut -c1-400 $O/spmm_4gloo.json
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > $O/spgemm_2gloo.json 2> $O/spgemm_2gloo.err || { tail -20 $O/spgemm_2gloo.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/spgemm_2gloo.json').readline())
print({k: d[k] for k in ('value','ms_per_step','n_gpus','torch_dist_world','rank_step_ms','per_rank')})"
