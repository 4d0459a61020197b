#!/bin/bash
# r08a (round 3, re-entry): full parity suite + smoke + default bench, every config's bench line,
# config-5 / config-3 rocprof kernel trace + MFMA PMC of the current build.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/mfma_rate_probe > gpurun_out/r08a_mfma_rate.txt 2>&1 || exit 3
bash tools/gpu_check.sh || exit $?
bash tools/bench_round.sh r08a || exit $?
MFMA_PMC="SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  bash tools/profile.sh r08a_impala_fp16 --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-novelty || exit $?
timeout -k 10 120 python tools/impala_phases_h2.py --mode 2 > gpurun_out/r08a_phases.txt 2>&1 || exit 3
FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr_fine.so timeout -k 10 120 python tools/impala_phases_h2.py --mode 2 > gpurun_out/r08a_phases_fine.txt 2>&1 || exit 3
echo r08a done
