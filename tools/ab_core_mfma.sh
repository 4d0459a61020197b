#!/bin/bash
# Same-box A/B of the fp16 pair core forms (fdr_ctx_set_core_mfma / FDR_CORE_MFMA: 1 one pair per workgroup,
# 2 two pairs): config 5 (CONFIG overrides) at a short episode, alternating.  Usage: MODES="1 2" REPS=3 T=100 bash tools/ab_core_mfma.sh
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for m in ${MODES:-1 2}; do
    log=gpurun_out/abm_${m}_${rep}.log
    FDR_CORE_MFMA=$m timeout -k 10 300 python bench.py --config ${CONFIG:-impala_fp16} --steps 2 --warmup 1 \
      --episode-len ${T:-100} --no-cpu-baseline > $log 2>&1 || { echo "mode $m FAIL"; tail -5 $log; exit 3; }
    tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('core_mfma $m rep $rep step %.1f ms conv %.4f ms core %.4f replay %.1f' % (l['ms_per_step'], r['conv_launch_ms'], r['core_kernel']['launch_ms'], r['entropy_replay_ms']))"
  done
done
