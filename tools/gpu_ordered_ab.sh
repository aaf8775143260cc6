#!/bin/bash
# A/B of the ordered one-pass ESC unit size (SPMM_SPGEMM_ORDERED_PCAP 7680 vs 3840) on the
# SpGEMM benches, plus the new SpGEMM GPU tests and the inner-dimension decomposition.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_spgemm.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_spgemm_gpu.log 2>&1 || { tail -30 $O/pytest_spgemm_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_spgemm_gpu.log | tail -2
for pc in ${PCAPS:-7680 3840}; do
  for wl in spgemm spgemm64k; do
    SPMM_SPGEMM_ORDERED_PCAP=$pc timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 > $O/ab_${wl}_$pc.log 2>&1 || { tail -20 $O/ab_${wl}_$pc.log; exit 1; }
    echo "pcap=$pc $wl $(grep '"metric"' $O/ab_${wl}_$pc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 python -u bench.py --workload spgemm --decomp inner --steps 3 --warmup 1 > $O/bench_spgemm_inner.log 2>&1 || { tail -20 $O/bench_spgemm_inner.log; exit 1; }
grep '"metric"' $O/bench_spgemm_inner.log | cut -c1-250
