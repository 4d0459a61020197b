#!/bin/bash
# r08b: fp16 conv A/B -- one workgroup per CU (LDS padded) and a staggered second workgroup vs the default build;
# LDS / VALU PMC pass of conv_kernel_h2<512>.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS="libfdr_base libfdr_one libfdr_stag libfdr_base libfdr_stag" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
LDS="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $LDS --kernel-trace --output-format csv -d gpurun_out/r08b_pmc_lds -o run -- \
  python3 bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-cpu-baseline --no-novelty > gpurun_out/r08b_pmc_lds.log 2>&1 \
  || { echo "pmc failed"; tail -5 gpurun_out/r08b_pmc_lds.log; exit 3; }
echo r08b done
