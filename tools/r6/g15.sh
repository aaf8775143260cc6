#!/bin/bash
# kernel traces: R-MAT 24 one streamed step (does long_place now overlap the accumulation?), and the
# emulated rank 0 of 8 step, link-only model at 300 GB/s (what the step adds to the local product)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g15; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d /tmp/prm -o prof --output-format csv -- python3 $R/tools/rmat_steps.py 24 1 > $O/rmat.log 2>&1 || { tail -20 $O/rmat.log; exit 1; }
grep "^step" $O/rmat.log
f=$(find /tmp/prm -name "*kernel_trace.csv" | head -1)
python3 $R/tools/overlap.py $f long_place long_dense long_rank long_route spgemm_esc compact > $O/rmat_overlap.txt; cat $O/rmat_overlap.txt
f=$(find /tmp/prm -name "*kernel_stats.csv" | head -1); cp $f $O/rmat_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pe8 -o prof --output-format csv -- python3 $R/tools/rank_emulate.py --world 8 --rank 0 --no-local --gather-gbps 300 --steps 3 > $O/emu.log 2>&1 || { tail -20 $O/emu.log; exit 1; }
f=$(find /tmp/pe8 -name "*kernel_trace.csv" | head -1); cp $f $O/emu_trace.csv
python3 $R/tools/overlap.py $f unpack pad_pairs rows_count rows_pipe splits pack_bits spin > $O/emu_overlap.txt; cat $O/emu_overlap.txt
