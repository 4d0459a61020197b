#!/bin/bash
# r07m: stage-3 residual convs split over (pixel tile, channel tile) per wave -- bit identity, A/B vs FDR_H2_SPLIT=0, PMC.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_impala.py -k "h2" \
  > gpurun_out/r07m_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r07m_tests.log; exit 3; }
tail -1 gpurun_out/r07m_tests.log
RUNS="libfdr libfdr_old libfdr libfdr_old" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
MFMA="SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $MFMA --kernel-trace --output-format csv -d gpurun_out/r07m_pmc_1 -o run -- \
  python3 bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-cpu-baseline > gpurun_out/r07m_pmc_1.log 2>&1 \
  || { echo "pmc failed"; tail -5 gpurun_out/r07m_pmc_1.log; exit 3; }
echo r07m done
