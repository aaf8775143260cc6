#!/bin/bash
# after removing the unpipelined row kernels: the GPU suites of spgemm / spmm / dist_device (multi-graph
# tests last), headline + 64k benches, SpMM row-group MFMA A/B (3 vs 2 chunks in flight), rank-0-of-8
# emulation (copy and link-only models)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g14; mkdir -p $O
cd $R
D=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_spmm.py > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json)"
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
for v in base rm2 base rm2; do
  lib=""; [ "$v" = base ] || lib=$D/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --workload spmm --spmm-method mfma --steps 50 --warmup 10 > $O/spmm_$v.json 2> $O/spmm_$v.err || { tail -20 $O/spmm_$v.err; exit 1; }
  echo "spmm mfma $v $(grep -o '"ms_per_step": [0-9.]*' $O/spmm_$v.json)"
done
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
echo "tests b: $(tail -1 $O/pytest_b.log)"
