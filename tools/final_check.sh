#!/bin/bash
# End-of-round GPU session: parity + smoke + default bench (tools/gpu_check.sh), then one bench line per
# BASELINE config that fits one GPU.  Stops at the first fault / timeout.
set -u
bash tools/gpu_check.sh "$@" || exit $?
for c in cartpole impala impala_fp16; do
  extra=""
  [ "$c" = cartpole ] || extra="--steps 2 --warmup 1"
  timeout -k 10 600 python bench.py --config $c $extra --no-cpu-baseline > gpurun_out/final_bench_$c.log 2>&1 \
    || { echo "bench $c rc=$?"; tail -5 gpurun_out/final_bench_$c.log; exit 3; }
  echo "== bench $c"; tail -1 gpurun_out/final_bench_$c.log | cut -c1-200
done
