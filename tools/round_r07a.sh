#!/bin/bash
# r07a: conv_kernel_h2 parity + A/B against conv_kernel_h; SrcC probe.  Each GPU step under its own limit.
set -e
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/srcc_probe > gpurun_out/r07a_srcc.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_impala.py \
  -k "h2 or fp16" > gpurun_out/r07a_tests_h.log 2>&1
FDR_CONV_H2=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_impala.py tests/test_gpu_impala_novelty.py -k "fp16 or h2 or strateg or forward" \
  > gpurun_out/r07a_tests_h2.log 2>&1
for h2 in 0 1; do
  FDR_CONV_H2=$h2 timeout -k 10 300 python -u bench.py --config impala_fp16 --episode-len 100 --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r07a_bench_h$h2.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for h2 in 0 1; do
  FDR_CONV_H2=$h2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r07a_prof_h$h2 -o run -- \
    python3 bench.py --config impala_fp16 --episode-len 100 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r07a_prof_h$h2.log 2>&1
done
