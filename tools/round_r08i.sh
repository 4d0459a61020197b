#!/bin/bash
# r08i: instruction-fetch counters of conv_kernel_h2<512> (is the 45 KB straight-line kernel I-cache bound?)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r08i_avail.txt 2>&1 || true
grep -iE "icache|ifetch|SQ_WAIT_INST|INST_LEVEL" gpurun_out/r08i_avail.txt | head -40
B="python3 bench.py --config impala_fp16 --steps 2 --warmup 1 --episode-len 20 --no-cpu-baseline --no-novelty"
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/r08i_pmc_a -o run -- $B > gpurun_out/r08i_pmc_a.log 2>&1 || { echo "pass a failed"; tail -3 gpurun_out/r08i_pmc_a.log; exit 3; }
echo pass a ok
if grep -q "SQC_ICACHE_MISSES" gpurun_out/r08i_avail.txt; then
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/r08i_pmc_b -o run -- $B > gpurun_out/r08i_pmc_b.log 2>&1 || { echo "pass b failed"; tail -3 gpurun_out/r08i_pmc_b.log; exit 3; }
  echo pass b ok
fi
echo r08i done
