#!/bin/bash
# Same-box A/B of two builds of libfdr (FDR_LIB) on one bench config, alternating.  Usage (GPU box):
#   LIBS="libfdr_old libfdr" REPS=2 CONFIG=impala_fp16 T=100 bash tools/ab_lib.sh
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-libfdr_old libfdr}; do
    log=gpurun_out/abl_${lib}_${rep}.log
    FDR_LIB=$PWD/dfd-starter_amd/fdr/$lib.so timeout -k 10 300 python bench.py --config ${CONFIG:-impala_fp16} --steps 2 \
      --warmup 1 --episode-len ${T:-100} --no-cpu-baseline ${EXTRA:-} > $log 2>&1 || { echo "$lib FAIL"; tail -5 $log; exit 3; }
    tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('$lib rep $rep step %.1f ms conv %.4f ms core %.4f replay %.2f ms rollout %.2f ms' % (l['ms_per_step'], r['conv_launch_ms'], r['core_kernel']['launch_ms'], r['entropy_replay_ms'], r['rollout_ms']))"
  done
done
