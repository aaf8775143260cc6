#!/bin/bash
# round-6 validation in the driver's order: full GPU suite, smoke, benches (1M, 64k, SpMM auto, R-MAT),
# rank 0 of 8 emulation, kernel stats of the 1M and 64k graph steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${OUT:-r6g19}; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
echo "gpu suite: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
echo "default $(grep -o '"ms_per_step": [0-9.]*' $O/bench_default.json)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b1m.json 2> $O/b1m.err || { tail -20 $O/b1m.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload spmm --steps 50 --warmup 10 > $O/spmm.json 2> $O/spmm.err || { tail -20 $O/spmm.err; exit 1; }
echo "1M $(grep -o '"ms_per_step": [0-9.]*' $O/b1m.json) 64k $(grep -o '"ms_per_step": [0-9.]*' $O/b64.json) spmm $(grep -o '"ms_per_step": [0-9.]*' $O/spmm.json)"
timeout -k 10 400 python -u tools/rank_emulate.py --world 8 --rank 0 --graph --gather-gbps 0,300 > $O/emu8.json 2> $O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
cat $O/emu8.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppva -o prof --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof1m.log 2>&1 || { tail -20 $O/prof1m.log; exit 1; }
cp $(find /tmp/ppva -name "*kernel_stats.csv" | head -1) $O/spgemm1m_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ppvb -o prof --output-format csv -- python3 $R/bench.py --workload spgemm64k --steps 50 --warmup 5 > $O/prof64.log 2>&1 || { tail -20 $O/prof64.log; exit 1; }
cp $(find /tmp/ppvb -name "*kernel_stats.csv" | head -1) $O/spgemm64k_kernel_stats.csv
cd $R
timeout -k 10 400 python -u bench.py --workload rmat --steps 2 --warmup 1 > $O/rmat.json 2> $O/rmat.err || { tail -20 $O/rmat.err; exit 1; }
echo "rmat $(grep -o '"ms_per_step": [0-9.]*' $O/rmat.json) $(grep -o '"nnz_C": [0-9]*' $O/rmat.json)"
