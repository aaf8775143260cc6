#!/bin/bash
# Memory counters of the bitmap kernels, one pass per numeric-kernel variant (SPMM_SPGEMM_BITMAP_ROWS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-pipe nopipe off}; do
  for ctr in "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    tag=bmpmc_${v}_$(echo $ctr | cut -c1-5)
    echo "== $tag"
    SPMM_SPGEMM_BITMAP_ROWS=$v timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/$tag -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  done
done
cd $R
for d in $O/bmpmc_*; do
  [ -d $d ] || continue
  f=$(find $d -name "*counter_collection.csv" | head -1)
  echo "### $(basename $d)"; python tools/pmc_summary.py $f spgemm_bm | grep -v "^$"
done
