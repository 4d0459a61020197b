#!/bin/bash
# Same-box A/B of the in-tree libfdr.so against another build (FDR_LIB) on the MLP configs, alternating:
#   bash tools/ab_lib_mlp.sh <tag> <other lib> [configs...]   -> gpurun_out/<tag>_<config>_{new,prev}<i>.log
set -u
TAG=$1; OTHER=$2; shift 2
CONFIGS=${*:-halfcheetah cartpole}
mkdir -p gpurun_out
for cfg in $CONFIGS; do
  for i in 1 2; do
    for v in new prev; do
      log=gpurun_out/${TAG}_${cfg}_${v}$i.log
      if [ $v = prev ]; then export FDR_LIB=$OTHER; else unset FDR_LIB; fi
      timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-variant > $log 2>&1 \
        || { echo "$cfg $v FAIL"; tail -5 $log; exit 3; }
      tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('$cfg $v $i FD step %.4f ms rollout %.4f ms frac %.4f' % (l['ms_per_step'], r['rollout_ms'], r['frac']))"
    done
  done
done
unset FDR_LIB
