#!/bin/bash
# R-MAT 24, one streamed step under a kernel trace: what long_place runs beside (queues, streams)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6g40; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace -d /tmp/prm -o prof --output-format csv -- python3 $R/tools/rmat_steps.py 24 1 > $O/rmat.log 2>&1 || { tail -20 $O/rmat.log; exit 1; }
grep "^step" $O/rmat.log
f=$(find /tmp/prm -name "*kernel_trace.csv" | head -1)
head -1 $f > $O/trace_header.txt
python3 $R/tools/r6/timeline_window.py $f long_place 300 40 40 > $O/win_place300.txt
python3 $R/tools/r6/timeline_window.py $f spgemm_compact 60 40 40 > $O/win_compact60.txt
python3 $R/tools/overlap.py $f long_place long_dense long_rank long_route spgemm_esc compact > $O/rmat_overlap.txt
cat $O/trace_header.txt; cat $O/rmat_overlap.txt; wc -l $O/win_place300.txt $O/win_compact60.txt
