#!/bin/bash
# Diagnostics A/B of the fp16 pair core stream (core_kernel_hpm): the product library against FDR_HPM_PROBE builds
# (1: no theta loads, 2: no HBM stream).  Build them first (container):
#   make -C dfd-starter_amd/csrc variant VSRC=fdr_impala_h VFLAGS=-DFDR_HPM_PROBE=1 VOUT=../fdr/libfdr_hpm1.so  (and =2)
# Usage (GPU box): bash tools/ab_hpm_probe.sh -> gpurun_out/abh_<lib>.log
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in libfdr libfdr_hpm1 libfdr_hpm2; do
    log=gpurun_out/abh_${lib}_${rep}.log
    FDR_LIB=$PWD/dfd-starter_amd/fdr/$lib.so timeout -k 10 300 python bench.py --config impala_fp16 --steps 2 --warmup 1 \
      --episode-len 100 --no-cpu-baseline --no-novelty > $log 2>&1 || { echo "$lib FAIL"; tail -5 $log; exit 3; }
    tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('$lib rep $rep step %.1f ms conv %.4f ms core %.4f replay %.1f' % (l['ms_per_step'], r['conv_launch_ms'], r['core_kernel']['launch_ms'], r['entropy_replay_ms']))"
  done
done
