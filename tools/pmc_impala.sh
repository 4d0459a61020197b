#!/bin/bash
# MFMA utilisation of the Impala conv stack (f32 and fp16 modes): one PMC pass per config, short episodes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_impala
mkdir -p $OUT
CTRS=${CTRS:-SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE}
for c in ${CONFIGS:-impala impala_fp16}; do
  timeout -s KILL 150 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/$c -o run -- \
    python3 bench.py --config $c --steps 2 --warmup 1 --episode-len 40 --no-cpu-baseline > $OUT/$c.log 2>&1 \
    || { echo "$c failed"; tail -5 $OUT/$c.log; exit 3; }
  echo "$c ok"
done
