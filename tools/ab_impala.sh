#!/bin/bash
# A/B of Impala builds (GPU box): bench.py --config <c> at a short episode, per-phase times.
# Usage: RUNS="libfdr libfdr_v1 ..." CONFIGS="impala impala_fp16" bash tools/ab_impala.sh
set -u
mkdir -p gpurun_out
for lib in ${RUNS:-libfdr}; do
  for c in ${CONFIGS:-impala impala_fp16}; do
    log=gpurun_out/abi_${lib}_${c}.log
    FDR_LIB=$PWD/dfd-starter_amd/fdr/$lib.so timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 \
      --episode-len ${T:-100} --no-cpu-baseline > $log 2>&1 || { echo "$lib $c FAIL"; tail -5 $log; exit 3; }
    tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('$lib $c step %.1f ms conv %.3f core %.3f replay %.1f' % (l['ms_per_step'], r['conv_launch_ms'], r['core_kernel']['launch_ms'], r['entropy_replay_ms']))"
  done
done
