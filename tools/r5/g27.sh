#!/bin/bash
# round-5: native engine device binning -- a4 / prim / spgemm GPU tests, chain bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5g27; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "a4 or prim or sort_rows" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u tools/a4_chain_bench.py --dir /tmp/a4c > $O/chain.json 2> $O/chain.err || { tail -20 $O/chain.err; exit 1; }
cat $O/chain.json
