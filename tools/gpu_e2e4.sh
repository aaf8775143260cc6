#!/bin/bash
# a4 e2e on report Table 1 sizes (small, medium, large)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_a4_native.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_a4.log 2>&1 || { tail -30 $O/pytest_a4.log; exit 1; }
grep -E "passed|failed" $O/pytest_a4.log | tail -2
run() {  # name, extra args
  echo "== a4 e2e $1"
  timeout -k 10 ${TMO:-600} python -u benches/bench_a4_e2e.py --device hip --json $O/a4_e2e_$1.json "${@:2}" > $O/a4_e2e_$1.log 2>&1 || { tail -20 $O/a4_e2e_$1.log; return 1; }
  python -c "import json; d=json.load(open('$O/a4_e2e_$1.json')); p=d['phases']; print(d['value'], 's  in', d['input_bytes']>>20, 'MiB  out', d['output_bytes']>>20, 'MiB  reduce', p['t_reduce_s'], 'write', p['t_write_s'], 'GOPs', p['reduce_gops'])"
}
run small --preset small && run medium --preset medium && TMO=900 run large --preset large
