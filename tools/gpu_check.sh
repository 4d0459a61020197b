#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first fault / abort / timeout.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_check.sh [bench args...]
set -u
mkdir -p gpurun_out
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress|GPU core dump'
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -25 "gpurun_out/$name.log"
  if grep -qE "$FAULT" "gpurun_out/$name.log"; then echo "GPU FAULT in $name -- stopping"; exit 3; fi
  [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || exit "$rc"   # 1 = test failures, not a fault
}
# (N-rank == 1-rank: tests/test_gpu_dist_equivalence.py drives tools/dist_check.py inside the suite)
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py "$@"
