#!/bin/bash
# r07l: PMC of the fp16 conv with h3 entries (issue / MFMA / LDS; HBM traffic) on a short config-5 run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ISSUE="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
MFMA="SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for ctrs in "$ISSUE" "$MFMA" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/r07l_pmc_$i -o run -- \
    python3 bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-cpu-baseline > gpurun_out/r07l_pmc_$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 gpurun_out/r07l_pmc_$i.log; exit 3; }
  i=$((i + 1))
done
echo r07l done
