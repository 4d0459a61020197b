#!/bin/bash
# r07h: conv_kernel_h2<512> without spills (stage-2 entry fragments streamed too) -- tests, phases, A/B vs <256>.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_impala.py -k "h2" \
  > gpurun_out/r07h_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r07h_tests.log; exit 3; }
tail -1 gpurun_out/r07h_tests.log
FDR_CONV_H2=2 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_impala.py \
  tests/test_gpu_impala_novelty.py -k "fp16 or strateg or forward" > gpurun_out/r07h_tests2.log 2>&1 \
  || { echo "tests2 rc=$?"; tail -30 gpurun_out/r07h_tests2.log; exit 3; }
tail -1 gpurun_out/r07h_tests2.log
for m in 1 2; do
  timeout -k 10 120 python -u tools/impala_phases_h2.py --mode $m > gpurun_out/r07h_phases_m$m.txt 2>&1 || { echo "phases rc=$?"; exit 3; }
  tail -1 gpurun_out/r07h_phases_m$m.txt
done
for round in 1 2; do
  for m in 1 2; do
    log=gpurun_out/r07h_bench_m$m.log
    FDR_CONV_H2=$m timeout -k 10 300 python bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 60 \
      --no-cpu-baseline > $log 2>&1 || { echo "bench m$m FAIL"; tail -5 $log; exit 3; }
    tail -1 $log | python -c "import json,sys; l=json.loads(sys.stdin.read()); r=l['roofline']; print('mode $m step %.1f ms conv %.4f core %.3f' % (l['ms_per_step'], r['conv_launch_ms'], r['core_kernel']['launch_ms']))"
  done
done
