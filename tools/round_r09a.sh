#!/bin/bash
# r09a: rollout_pair_kernel launched in rounds (lane_base) -- new multi-round test, then a same-box A/B of the
# 4096-pair variant (8192 lanes) with FDR_PAIR_ROUNDS=0 (one launch) / 1 (rounds), alternating.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/dfd-starter_amd:$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_kernels.py \
  -k "multi_round or full_size_properties or pair_and_single" > gpurun_out/r09a_pytest.log 2>&1 || { tail -30 gpurun_out/r09a_pytest.log; exit 1; }
tail -3 gpurun_out/r09a_pytest.log
for i in 1 2 3; do
  for r in 0 1; do
    FDR_PAIR_ROUNDS=$r timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/r09a_ab_${r}_$i.log 2>&1 || exit 1
    python3 - gpurun_out/r09a_ab_${r}_$i.log $r <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
v = d["variants"]["4096_pairs"]
print("rounds=%s base %.4f ms (rollout %.4f)  variant %.4f ms rollout %.4f frac %.4f" % (
    sys.argv[2], d["ms_per_step"], d["roofline"]["rollout_ms"], v["ms_per_step"], v["rollout_ms"], v["roofline_frac"]))
PY
  done
done
echo r09a done
