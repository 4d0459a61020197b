#!/bin/bash
# r08d: LDS conflict fixes (exchange-slot layout, rotated frame stores): parity of the default build, A/B, LDS PMC.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_impala.py tests/test_gpu_impala_novelty.py \
  > gpurun_out/r08d_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r08d_tests.log; exit 3; }
tail -1 gpurun_out/r08d_tests.log
RUNS="libfdr_base libfdr_exonly libfdr_new libfdr_base libfdr_new libfdr_exonly" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
LDS="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $LDS --kernel-trace --output-format csv -d gpurun_out/r08d_pmc_lds -o run -- \
  python3 bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-cpu-baseline --no-novelty > gpurun_out/r08d_pmc_lds.log 2>&1 \
  || { echo "pmc failed"; tail -5 gpurun_out/r08d_pmc_lds.log; exit 3; }
echo r08d done
