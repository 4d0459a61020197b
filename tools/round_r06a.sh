#!/bin/bash
# r06a GPU session: bench lines (configs 3, 2, 1) then the config-3 rocprofv3 passes (trace, FETCH, WRITE, SQ, issue).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r06a_bench_halfcheetah.log 2>&1 || { echo "bench halfcheetah rc=$?"; tail -5 gpurun_out/r06a_bench_halfcheetah.log; exit 3; }
tail -1 gpurun_out/r06a_bench_halfcheetah.log | cut -c1-400
timeout -k 10 300 python bench.py --config cartpole > gpurun_out/r06a_bench_cartpole.log 2>&1 || { echo "bench cartpole rc=$?"; exit 3; }
timeout -k 10 300 python bench.py --config trap --steps 20 > gpurun_out/r06a_bench_trap.log 2>&1 || { echo "bench trap rc=$?"; tail -5 gpurun_out/r06a_bench_trap.log; exit 3; }
tail -1 gpurun_out/r06a_bench_trap.log | cut -c1-300
ISSUE_PMC="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
EXTRA_PMC="$ISSUE_PMC" bash tools/profile.sh r06a_halfcheetah --config halfcheetah --no-variant || exit $?
echo r06a done
