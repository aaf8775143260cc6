#!/bin/bash
# ticket protocol v2 validation: bitmap tests (live tickets: 20000-row and 1M sampled-row products),
# ticket A/B on 1M, per-WG timelines, N=8 emulation; LAST the multi-graph tests (graphs kept alive)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g09; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spgemm.py -k "bitmap or bench_scale or graph_replay" > $O/pytest_a.log 2>&1 || { tail -40 $O/pytest_a.log; exit 1; }
echo "tests a: $(tail -1 $O/pytest_a.log)"
for v in base tk0 tk1 base; do
  lib=""; [ "$v" = base ] || lib=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -20 $O/ab_$v.err; exit 1; }
  echo "$v 1M $(grep -o '"ms_per_step": [0-9.]*' $O/ab_$v.json) $(grep -o '"eager_ms_per_step": [0-9.]*' $O/ab_$v.json)"
done
for v in base tk3 base tk3; do
  lib=""; [ "$v" = base ] || lib=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag/libspmm_hip_$v.so
  SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64_$v.json 2> $O/b64_$v.err || { tail -20 $O/b64_$v.err; exit 1; }
  echo "$v 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64_$v.json)"
done
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 1 --n 65536 --density 1e-3 > $O/wg64k.json 2> $O/wg64k.err || { tail -20 $O/wg64k.err; exit 1; }
cat $O/wg64k.json
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 8 > $O/wg8.json 2> $O/wg8.err || { tail -20 $O/wg8.err; exit 1; }
SPMM_STAMPS_PREBUILT=1 timeout -k 10 300 python -u tools/bm_wg_times.py --world 1 > $O/wg1.json 2> $O/wg1.err || { tail -20 $O/wg1.err; exit 1; }
cat $O/wg8.json $O/wg1.json
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --no-local --gather-gbps 300 --link-priority -1 > $O/emu8_hi.json 2> $O/emu8_hi.err || { tail -20 $O/emu8_hi.err; exit 1; }
cat $O/emu8.json $O/emu8_hi.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_dist_device.py tests/test_spgemm.py -k "panel_comm or rowblock_graph or rccl_one_rank" > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
echo "tests b: $(tail -1 $O/pytest_b.log)"
