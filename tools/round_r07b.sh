#!/bin/bash
# r07b: conv_kernel_h2 phase clocks + issue / MFMA PMC of both fp16 conv kernels (short config-5 runs).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/impala_phases_h2.py > gpurun_out/r07b_phases_h2.txt 2>&1 || { echo "phases h2 rc=$?"; tail -5 gpurun_out/r07b_phases_h2.txt; exit 3; }
timeout -k 10 120 python -u tools/impala_phases.py --fp16 > gpurun_out/r07b_phases_h.txt 2>&1 || { echo "phases h rc=$?"; exit 3; }
ISSUE="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
MFMA="SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for h2 in 0 1; do
  i=0
  for ctrs in "$ISSUE" "$MFMA"; do
    FDR_CONV_H2=$h2 timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/r07b_pmc_h${h2}_$i -o run -- \
      python3 bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 40 --no-cpu-baseline > gpurun_out/r07b_pmc_h${h2}_$i.log 2>&1 \
      || { echo "pmc h2=$h2 pass $i failed"; tail -5 gpurun_out/r07b_pmc_h${h2}_$i.log; exit 3; }
    i=$((i + 1))
  done
done
echo r07b done
