export SPMM_STAMPS_PREBUILT=1
timeout -k 10 200 python tools/bm_stamps.py 1048576 1e-4 3 > gpurun_out/st3.log 2>&1
timeout -k 10 200 python tools/bm_stamps.py 1048576 1e-4 0 > gpurun_out/st0.log 2>&1
WL=spgemm STEPS=3 bash tools/gpu_prof_bench.sh > /dev/null 2>&1; cp gpurun_out/prof_spgemm.md gpurun_out/prof3.md
SPMM_SPGEMM_BITMAP_CFG=0 WL=spgemm STEPS=3 bash tools/gpu_prof_bench.sh >/dev/null 2>&1; cp gpurun_out/prof_spgemm.md gpurun_out/prof0.md; rm -rf gpurun_out/prof_spgemm
