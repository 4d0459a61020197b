#!/bin/bash
# r07i: baseline of the current build on a fresh box -- full GPU suite + smoke, config 3 and 5 bench lines,
# config-5 kernel trace (conv_kernel_h2<512> default).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress|GPU core dump'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rf \
  > gpurun_out/r07i_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r07i_pytest.log; exit 3; }
tail -2 gpurun_out/r07i_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r07i_smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -10 gpurun_out/r07i_smoke.log; exit 3; }
tail -1 gpurun_out/r07i_smoke.log
timeout -k 10 120 python -u tools/impala_phases_h2.py --mode 2 > gpurun_out/r07i_phases_m2.txt 2>&1 || { echo "phases rc=$?"; exit 3; }
cat gpurun_out/r07i_phases_m2.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r07i_bench_halfcheetah.log 2>&1 || { echo "bench3 rc=$?"; tail -5 gpurun_out/r07i_bench_halfcheetah.log; exit 3; }
tail -1 gpurun_out/r07i_bench_halfcheetah.log | cut -c1-600
timeout -k 10 400 python -u bench.py --config impala_fp16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r07i_bench_impala_fp16.log 2>&1 \
  || { echo "bench5 rc=$?"; tail -5 gpurun_out/r07i_bench_impala_fp16.log; exit 3; }
tail -1 gpurun_out/r07i_bench_impala_fp16.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r07i_prof_fp16 -o run -- \
  python3 bench.py --config impala_fp16 --episode-len 100 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r07i_prof_fp16.log 2>&1 || { echo "prof rc=$?"; exit 3; }
head -12 gpurun_out/r07i_prof_fp16/run_kernel_stats.csv | cut -c1-200
if grep -qE "$FAULT" gpurun_out/*.log; then echo FAULT; fi
echo r07i done
