#!/bin/bash
# round-5: R-MAT scale-24 step timing + kernel stats of two steps (no setup checksum)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g11; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "long or rmat or bitmap" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pp11 -o prof --output-format csv -- python3 $R/tools/r5/rmat_steps.py 24 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cat $O/prof.log | tail -4
f=$(find /tmp/pp11 -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv
python3 $R/tools/prof_summary.py $f $O/prof.md "R-MAT 24, two streamed steps" && head -40 $O/prof.md | cut -c1-170
