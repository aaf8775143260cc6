#!/bin/bash
# round-4: padded layouts + graph: GPU tests of the bitmap path, 1M / 64k benches (graph on/off), chain bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/r4g5; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_spgemm.py tests/test_a4_native.py -k "bitmap or bench_scale or graph or mtx" -m gpu > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench1m.json 2> $O/bench1m.err &&
SPMM_SPGEMM_BITMAP_PAD=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --graph off > $O/bench1m_nopad.json 2> $O/bench1m_nopad.err &&
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 20 --warmup 3 > $O/bench64k.json 2> $O/bench64k.err &&
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 20 --warmup 3 --graph off > $O/bench64k_eager.json 2> $O/bench64k_eager.err &&
timeout -k 10 300 python -u bench.py --workload chain --steps 3 --warmup 1 > $O/chain.json 2> $O/chain.err
rc=$?
tail -3 $O/pytest.log
for f in $O/*.json; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f)"; done
echo rc=$rc
