#!/bin/bash
# First GPU pass: GPU tests, smoke, chain bench, rocprof kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== pytest gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
echo "== chain bench" && timeout -k 10 300 python benches/bench_chain.py --preset medium --steps 3 > $O/chain_medium.log 2>&1 || exit $?
cat $O/chain_medium.log
cd /tmp && export TMPDIR=/tmp
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_chain -o prof --output-format csv -- python3 $R/benches/bench_chain.py --preset small --steps 2 > $O/prof_chain.log 2>&1 || exit $?
find $O/prof_chain -name "*stats*" | head
