#!/bin/bash
# Kernel experiments: A/B of library variants (VARIANTS, WLS), the
# shader-clock phase stamps of the bitmap kernels, and PMC passes (PASSES) of the 1M step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
cd $R
if [ -n "${VARIANTS}" ]; then
  echo "== A/B ${VARIANTS}"
  for v in ${VARIANTS}; do
    lib=""
    [ "$v" = base ] || lib=$R/sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd/lib/diag/libspmm_hip_$v.so
    for wl in ${WLS:-spgemm}; do
      SPMM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --steps ${NSTEPS:-5} --warmup 2 > $O/ab_${v}_$wl.log 2>&1 || { tail -20 $O/ab_${v}_$wl.log; exit 1; }
      echo "$v $wl $(grep -o '"ms_per_step": [0-9.]*' $O/ab_${v}_$wl.log) $(grep -o '"value": [0-9.]*' $O/ab_${v}_$wl.log)"
    done
  done
fi
if [ -n "${ENVS}" ]; then
  # ENVS="base;VAR=1;VAR=2,OTHER=3": one bench run per ';'-separated environment set
  echo "== env A/B"
  IFS=';' read -ra SETS <<< "${ENVS}"
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    envs=""
    [ "$set" = base ] || envs=$(echo "$set" | tr ',' ' ')
    for wl in ${WLS:-spgemm}; do
      env $envs timeout -k 10 300 python -u bench.py --workload $wl --steps ${NSTEPS:-5} --warmup 2 > $O/env_${i}_$wl.log 2>&1 || { tail -20 $O/env_${i}_$wl.log; exit 1; }
      echo "[$set] $wl $(grep -o '"ms_per_step": [0-9.]*' $O/env_${i}_$wl.log) $(grep -o '"value": [0-9.]*' $O/env_${i}_$wl.log)"
    done
  done
fi
if [ -n "${STAMPS}" ]; then
  echo "== stamps ${STAMPS}"
  timeout -k 10 300 python -u tools/bm_stamps.py ${STAMPS} > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
  cat $O/stamps.log | tail -9
fi
if [ -n "${PASSES}" ]; then
  PMC_DIR=/tmp/pmc_r3 KREGEX=${KREGEX:-spgemm_bm} bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -30 $O/pmc.log; exit 1; }
  cp $R/gpurun_out/pmc*.txt $O/ 2>/dev/null
  tail -40 $O/pmc.log
fi
