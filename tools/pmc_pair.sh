#!/bin/bash
# PMC passes over the pair rollout kernel (one counter group per pass), GPU box.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_pair
export FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr.so
i=0
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES}"
for g in "${GROUPS_[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $g --kernel-trace --output-format csv -d gpurun_out/pmc_pair/p$i -o run -- \
    python3 tools/rollout_phases.py --iters 4 ${PHASE_ARGS:-} > gpurun_out/pmc_pair/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_pair/p$i.log; exit 3; }
  echo "pass $i ok"
  i=$((i + 1))
done
