#!/bin/bash
# round-5: R-MAT 24 bench (driver form: nnz_C + checksum of the setup product, 2 timed steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g24; mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 0 > $O/brmat.json 2> $O/brmat.err || { tail -20 $O/brmat.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/brmat.json')); print('rmat', d['ms_per_step'], d['nnz_C'], d['c_checksum'], d['value'])"
