#!/bin/bash
# round-4: why the eager world-4 rank product is 2x its graph replay (per-step times, path, kernel stats)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r4g35; mkdir -p $O
cd $R
timeout -k 10 240 python -u tools/rank_emulate.py --world 4 --steps 6 --per-step > $O/w4.jsonl 2> $O/w4.err || { tail -5 $O/w4.err; exit 1; }
grep -v amdgpu.ids $O/w4.err | cut -c1-400; cat $O/w4.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pw4 -o prof --output-format csv -- python3 $R/tools/rank_emulate.py --world 4 --steps 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find /tmp/pw4 -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py $f $O/prof_w4.md "world-4 rank 0 eager kernel stats" && sed -n 5,22p $O/prof_w4.md | cut -c1-170
