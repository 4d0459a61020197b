#!/bin/bash
# Same-box A/B of an environment switch through bench.py, alternating values.
#   VAR=FDR_PREFETCH_WAIT VALUES="always default" CONFIGS="halfcheetah cartpole" REPS=3 bash tools/ab_env.sh
# ("default" leaves the variable unset)
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for c in ${CONFIGS:-halfcheetah}; do
    for v in ${VALUES:-default}; do
      log=gpurun_out/abe_${c}_${v}_${rep}.log
      if [ "$v" = default ]; then unset "$VAR"; else export "$VAR=$v"; fi
      timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-variant ${BENCH_ARGS:-} > $log 2>&1 \
        || { echo "$c $v FAIL"; tail -5 $log; exit 3; }
      unset "$VAR"
      tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('%-12s %-8s rep $rep value %.4g ms/step %.4f rollout_ms %s' % ('$c', '$v', l['value'], l['ms_per_step'], r.get('rollout_ms')))"
    done
  done
done
