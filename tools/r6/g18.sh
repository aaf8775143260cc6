#!/bin/bash
# HW queues: with GPU_MAX_HW_QUEUES=4 HIP maps streams round-robin onto 4 queues and a side stream can
# share the compute stream's queue (no concurrency).  R-MAT and the emulated rank step at 4 vs 8 queues.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g18; mkdir -p $O
cd $R
for q in 8 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rm_q$q.json 2> $O/rm_q$q.err || { tail -20 $O/rm_q$q.err; exit 1; }
  echo "q$q rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rm_q$q.json) $(grep -o '"nnz_C": [0-9]*' $O/rm_q$q.json)"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --no-local --gather-gbps 0,300 > $O/emu_q$q.json 2> $O/emu_q$q.err || { tail -20 $O/emu_q$q.err; exit 1; }
  echo "q$q $(cat $O/emu_q$q.json)"
done
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_spmm.py > $O/pytest_spmm.log 2>&1 || { tail -40 $O/pytest_spmm.log; exit 1; }
echo "spmm tests: $(tail -1 $O/pytest_spmm.log)"
for meth in mfma sweep mfma; do
  timeout -k 10 200 python -u bench.py --workload spmm --spmm-method $meth --steps 50 --warmup 10 > $O/spmm_$meth.json 2> $O/spmm_$meth.err || { tail -20 $O/spmm_$meth.err; exit 1; }
  echo "spmm $meth $(grep -o '"ms_per_step": [0-9.]*' $O/spmm_$meth.json)"
done
