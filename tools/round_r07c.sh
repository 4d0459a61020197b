#!/bin/bash
# r07c: conv_kernel_h2 (frame bands spread + exact /255, fma_mix epilogues) -- bit-identity + fp16 parity, phases, A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
FDR_CONV_H2=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_impala.py \
  tests/test_gpu_impala_novelty.py -k "h2 or fp16 or strateg or forward" > gpurun_out/r07c_tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/r07c_tests.log; exit 3; }
tail -2 gpurun_out/r07c_tests.log
timeout -k 10 120 python -u tools/impala_phases_h2.py > gpurun_out/r07c_phases_h2.txt 2>&1 || { echo "phases rc=$?"; exit 3; }
tail -1 gpurun_out/r07c_phases_h2.txt
for h2 in 0 1; do
  FDR_CONV_H2=$h2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r07c_prof_h$h2 -o run -- \
    python3 bench.py --config impala_fp16 --episode-len 100 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r07c_prof_h$h2.log 2>&1 || { echo "prof rc=$?"; exit 3; }
  grep -E "conv_kernel" gpurun_out/r07c_prof_h$h2/run_kernel_stats.csv | cut -c1-200
done
