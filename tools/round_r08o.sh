#!/bin/bash
# r08o: the round's final build -- full GPU suite + smoke + default bench, every config's bench line, config-5 rocprof
# (kernel trace + FETCH / WRITE / SQ / MFMA PMC) and phase clocks.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit $?
bash tools/bench_round.sh r08o || exit $?
MFMA_PMC="SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  bash tools/profile.sh r08o_impala_fp16 --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-novelty || exit $?
timeout -k 10 120 python tools/impala_phases_h2.py --mode 2 > gpurun_out/r08o_phases.txt 2>&1 || exit 3
echo r08o done
