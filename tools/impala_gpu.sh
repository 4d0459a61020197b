# Impala path on the GPU box: parity tests, short bench, rocprof kernel stats, phase clocks.
set -u
mkdir -p gpurun_out
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress'
timeout -k 10 400 python -m pytest tests/test_gpu_impala.py -q -x -rf > gpurun_out/impala_t.log 2>&1; rc=$?
tail -5 gpurun_out/impala_t.log
grep -qE "$FAULT" gpurun_out/impala_t.log && exit 3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config impala --steps 2 --warmup 1 --episode-len ${T:-20} --no-cpu-baseline > gpurun_out/impala_bench.log 2>&1 || { tail -20 gpurun_out/impala_bench.log; exit 4; }
tail -1 gpurun_out/impala_bench.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_imp -o run -- python3 bench.py --config impala --steps 1 --warmup 1 --episode-len 10 --no-cpu-baseline > gpurun_out/impala_prof.log 2>&1 || { tail -20 gpurun_out/impala_prof.log; exit 5; }
find gpurun_out/prof_imp -name "*kernel_stats.csv" | head -3
timeout -k 10 120 python tools/impala_phases.py > gpurun_out/phases.log 2>&1; head -1 gpurun_out/phases.log
