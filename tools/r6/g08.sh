#!/bin/bash
# ticket protocol v2: the scenario that faulted, tests, ticket A/B on 1M, per-WG timelines, N=8 emulation
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g08; mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/r6/diag_panel2.py > $O/diag.log 2>&1 || { tail -30 $O/diag.log; exit 1; }
grep -c "result None? False" $O/diag.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py tests/test_dist_device.py -k "bitmap or bench_scale or panel_comm or rccl_one_rank or graph" > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
for v in base tk0 tk1 tk2 base; do
  lib=""; [ "$v" = base ] || lib=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  echo "$v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/ab_$v.json)"
done
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
echo "64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json)"
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 8 > $O/wg8.json 2> $O/wg8.err || { tail -20 $O/wg8.err; exit 1; }
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 1 > $O/wg1.json 2> $O/wg1.err || { tail -20 $O/wg1.err; exit 1; }
cat $O/wg8.json $O/wg1.json
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
