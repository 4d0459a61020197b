set -u
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_impala.py -q -x -rf > gpurun_out/impala_t2.log 2>&1; rc=$?
tail -15 gpurun_out/impala_t2.log
grep -qE "HSA_STATUS_ERROR|Memory access fault" gpurun_out/impala_t2.log && exit 3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config impala --steps 2 --warmup 1 --episode-len 20 --no-cpu-baseline > gpurun_out/impala_bench.log 2>&1 || { tail -20 gpurun_out/impala_bench.log; exit 4; }
tail -2 gpurun_out/impala_bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_imp -o run -- python bench.py --config impala --steps 1 --warmup 1 --episode-len 10 --no-cpu-baseline > gpurun_out/impala_prof.log 2>&1 || { tail -20 gpurun_out/impala_prof.log; exit 5; }
find gpurun_out/prof_imp -name "*stats*" | head
