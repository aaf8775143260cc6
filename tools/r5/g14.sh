#!/bin/bash
# round-5: R-MAT 24 route variants (per-phase launches vs one launch), kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g14; mkdir -p $O
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "long or rmat" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
for pp in 1 2; do
  SPMM_LONG_ROUTE_PP=$pp timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pp14_$pp -o prof --output-format csv -- python3 $R/tools/r5/rmat_steps.py 24 2 > $O/prof_$pp.log 2>&1 || { tail -20 $O/prof_$pp.log; exit 1; }
  grep "^step" $O/prof_$pp.log
  f=$(find /tmp/pp14_$pp -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py $f $O/prof_$pp.md "R-MAT 24 route pp=$pp, two steps" && sed -n 5,13p $O/prof_$pp.md | cut -c1-120
done
