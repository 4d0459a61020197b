#!/bin/bash
# Same-box A/B of one environment switch on config 5 (tools/ab_env_impala.sh <tag> <VAR=value> [episode_len]):
# alternates the default run and the run with the variable set, twice -> gpurun_out/<tag>_{new,prev}<i>.log.
set -u
TAG=$1; SW=$2; T=${3:-300}
mkdir -p gpurun_out
for i in 1 2; do
  for v in new prev; do
    log=gpurun_out/${TAG}_${v}$i.log
    if [ $v = prev ]; then export "$SW"; else unset "${SW%%=*}"; fi
    timeout -k 10 300 python -u bench.py --config impala_fp16 --steps 3 --warmup 1 --no-cpu-baseline \
      --episode-len $T > $log 2>&1 || { echo "$v FAIL"; tail -5 $log; exit 3; }
    tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('$v $i step %.2f ms conv %.4f core %.4f replay %.2f' % (l['ms_per_step'], r['conv_launch_ms'], r['core_kernel']['launch_ms'], r['entropy_replay_ms']))"
  done
done
