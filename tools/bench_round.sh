#!/bin/bash
# The round's bench lines (GPU box): every BASELINE config that fits one GPU, CPU baseline included.
# Usage: bash tools/bench_round.sh <tag>  -> gpurun_out/bench_<tag>_<config>.log (last line = the JSON line)
set -u
TAG=${1:-r05}
mkdir -p gpurun_out
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress'
b() {  # b <config> <timeout> <args...>
  local cfg=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py --config "$cfg" "$@" > "gpurun_out/bench_${TAG}_${cfg}.log" 2>&1
  local rc=$?
  echo "== $cfg rc=$rc"; tail -1 "gpurun_out/bench_${TAG}_${cfg}.log" | cut -c1-400
  if grep -qE "$FAULT" "gpurun_out/bench_${TAG}_${cfg}.log"; then echo "GPU FAULT"; exit 3; fi
  [ "$rc" -eq 0 ] || exit "$rc"
}
b halfcheetah 300 ${BENCH_ARGS:-}
b cartpole 300
b impala 400 --steps 5 --warmup 1
b impala_fp16 300 --steps 5 --warmup 1
