#!/bin/bash
# r08j: conv_kernel_h2<512> register pressure (wave index in an SGPR, weight-block remainder as one dword per thread):
# spills 52 -> 32 B/lane; parity + A/B against the previous build (libfdr_prev).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_impala.py tests/test_gpu_impala_novelty.py \
  > gpurun_out/r08j_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r08j_tests.log; exit 3; }
tail -1 gpurun_out/r08j_tests.log
RUNS="libfdr_prev libfdr libfdr_prev libfdr libfdr_prev libfdr" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
echo r08j done
