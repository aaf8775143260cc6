#!/bin/bash
# round-4 validation: gather calibration, GPU tests of the pruned bitmap path,
# the speculative chain kernel and the SpMM sweep gate; 1M + chain benches
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/r4g4; mkdir -p $O
timeout -k 10 120 ./tools/probes/seg_gather > $O/seg0.csv &&
SEG_ALIGN=1 timeout -k 10 120 ./tools/probes/seg_gather > $O/seg1.csv &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_bsr_chain.py tests/test_spmm.py tests/test_spgemm.py -k "bitmap or bsr or chain or spmm or sweep or bench_scale" -m gpu > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench1m.json 2> $O/bench1m.err &&
timeout -k 10 300 python -u bench.py --workload chain --steps 3 --warmup 1 > $O/chain.json 2> $O/chain.err
rc=$?
tail -3 $O/pytest.log
echo rc=$rc
