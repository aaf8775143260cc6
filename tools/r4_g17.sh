#!/bin/bash
# round-4: chain Large preset (native a4 end to end, kernel phase) and the R-MAT step's kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g17; mkdir -p $O
cd $R
timeout -k 10 900 python -u bench.py --workload chain --chain-preset large --steps 1 --warmup 0 > $O/chain_large.json 2> $O/chain_large.err || { tail -5 $O/chain_large.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/chain_large.json').readline()); m=d['a4_phases']
print('chain large', d['ms_per_step'], 'ms/step; a4', d['a4_time_taken_s'], 's; kernel_s', m['phases']['kernel_s'], 'int_ops', m['int_ops'], '->', round(m['int_ops']/m['phases']['kernel_s']/1e12,2), 'TOP/s (sum of per-product stream time)')"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prm -o prof --output-format csv -- python3 $R/bench.py --workload rmat --steps 1 --warmup 0 > $O/prof_rmat.log 2>&1 || { tail -20 $O/prof_rmat.log; exit 1; }
f=$(find /tmp/prm -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/rmat_kernel_stats.md "R-MAT 24 (1 step, no warm-up)" && sed -n 5,30p $O/rmat_kernel_stats.md | cut -c1-160
grep -o '"ms_per_step": [0-9.]*' $O/prof_rmat.log
