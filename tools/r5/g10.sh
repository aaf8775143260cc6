#!/bin/bash
# round-5: LDS float adds as read + compare-swap -- GPU suite, R-MAT 24 bench (nnz + checksum), 1M / 64k bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g10; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
echo "gpu suite: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u bench.py --workload rmat --steps 2 --warmup 0 > $O/brmat.json 2> $O/brmat.err || { tail -20 $O/brmat.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/brmat.json')); print('rmat', d['ms_per_step'], d['nnz_C'], d['c_checksum'])"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json) eager $(grep -o '"eager_ms_per_step": [0-9.]*' $O/b64.json)"
