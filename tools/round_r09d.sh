#!/bin/bash
# r09d: Impala pair rollouts as two lane ranges on two HIP streams -- bitwise tests, then same-box A/B of
# configs 5 and 4 with FDR_IMPALA_STREAMS=1 (one sequence) / 2 (default), alternating.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/dfd-starter_amd:$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_impala.py \
  -k "side_streams or full_size_rollout_properties" > gpurun_out/r09d_pytest.log 2>&1 || { tail -30 gpurun_out/r09d_pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r09d_pytest.log | tail -10
ab() {  # ab <config> <runs>
  for i in $(seq 1 $2); do
    for s in 1 2; do
      FDR_IMPALA_STREAMS=$s timeout -k 10 300 python -u bench.py --config $1 --steps 5 --warmup 1 --no-cpu-baseline \
        > gpurun_out/r09d_${1}_${s}_$i.log 2>&1 || exit 1
      python3 - gpurun_out/r09d_${1}_${s}_$i.log $1 $s <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("%s streams=%s: %.1f ms per FD step, value %.4g" % (sys.argv[2], sys.argv[3], d["ms_per_step"], d["value"]))
PY
    done
  done
}
ab impala_fp16 3
ab impala 2
echo r09d done
