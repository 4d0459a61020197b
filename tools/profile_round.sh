#!/bin/bash
# All rocprofv3 passes of one round (GPU box): config 3 (headline), config 2, configs 4/5 (short episodes).
# Usage: bash tools/profile_round.sh <tag>     -> gpurun_out/prof_<tag>_<config>/...
set -u
TAG=${1:-r05}
export TMPDIR=/tmp
run_cfg() {  # run_cfg <config> <extra bench args...>
  local cfg=$1; shift
  bash tools/profile.sh "${TAG}_${cfg}" --config "$cfg" "$@" || exit $?
}
# issue/wait breakdown of the MLP rollout kernels (DESIGN.md 3.0 ceiling table)
ISSUE_PMC="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
EXTRA_PMC="$ISSUE_PMC" run_cfg halfcheetah --no-variant
EXTRA_PMC="$ISSUE_PMC" run_cfg cartpole
MFMA_PMC="SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  run_cfg impala --steps 2 --warmup 1 --episode-len 40
MFMA_PMC="SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
  run_cfg impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-novelty
echo profile_round done
