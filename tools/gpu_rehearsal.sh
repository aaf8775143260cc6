#!/bin/bash
# Multi-rank rehearsal of every bench.py workload on ONE GPU: N gloo ranks share the card
# (same code path as RCCL apart from the wire).  For each workload the 1-rank and N-rank runs
# must report the same whole-job work (flops_per_step, nnz_C / nnz_A when present).
#   NRANKS="1 8" WORKLOADS="spgemm spgemm64k spmm rmat chain" bash tools/gpu_rehearsal.sh
# R-MAT runs at --scale 20 here (eight ranks sharing one card would each size their streamed
# panels from the same free memory) and spgemm at n = 2^18 (gloo stages every collective
# through host memory).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
port=29410
for wl in ${WORKLOADS:-spgemm spgemm64k spmm rmat chain}; do
  extra=""
  [ "$wl" = rmat ] && extra="--scale ${RMAT_SCALE:-20}"
  [ "$wl" = spgemm ] && extra="--matrix-n ${SPGEMM_N:-262144}"   # gloo moves B through the host: keep it small
  [ "$wl" = chain ] && extra="--chain-preset small"                 # (one chain; its split over N ranks shares the card)
  for n in ${NRANKS:-1 8}; do
    port=$((port + 1))
    log=$O/rehearsal_${wl}_$n.log
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n --workload $wl --steps 2 --warmup 1 --backend gloo $extra ${ARGS} \
      > $log 2>&1 || { echo "FAILED $wl n=$n"; tail -30 $log; exit 1; }
  done
done
python - "$O" ${WORKLOADS:-spgemm spgemm64k spmm rmat chain} <<'PY'
import json, os, sys
O, wls = sys.argv[1], sys.argv[2:]
ns = os.environ.get("NRANKS", "1 8").split()
bad = 0
print("| workload | ranks | ms/step | value | flops/step | nnz_C | parallelism |")
print("|---|---:|---:|---:|---:|---:|---|")
for wl in wls:
    recs = {}
    for n in ns:
        with open(os.path.join(O, f"rehearsal_{wl}_{n}.log")) as f:
            recs[n] = json.loads([l for l in f if l.startswith("{")][-1])
    for n, r in recs.items():
        print(f"| {wl} | {n} | {r['ms_per_step']} | {r['value']} {r['unit'].split()[0]} | {r.get('flops_per_step')} | "
              f"{r.get('nnz_C', '')} | {r['config'].get('parallelism')} |")
    if True:   # every workload, the chain too (a4 sums the ranks' tile pairs)
        ref = recs[ns[0]]
        for n, r in recs.items():
            for k in ("flops_per_step", "nnz_C", "nnz_A"):
                if k in ref and int(float(ref[k])) != int(float(r[k])):
                    print(f"MISMATCH {wl} n={n} {k}: {r[k]} vs {ref[k]}")
                    bad += 1
sys.exit(1 if bad else 0)
PY
