#!/bin/bash
# round-5: shared native bitmap planner -- full GPU suite, 1M / 64k bench, native mtx chain vs Python
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g20; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
echo "gpu suite: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
timeout -k 10 600 python -u tools/a4_chain_bench.py --dir /tmp/a4c > $O/chain.json 2> $O/chain.err || { tail -20 $O/chain.err; exit 1; }
cat $O/chain.json
