#!/bin/bash
# r09e: rollout_pair_kernel with 4-wave workgroups (2 per CU; libfdr_pw4.so, -DFDR_PAIR_WAVES=4) vs the default
# 2-wave workgroups (4 per CU): parity subset on the variant, then alternating same-box bench runs (config 3).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/dfd-starter_amd:$PWD
FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr_pw4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_kernels.py -k "multi_round or full_size_properties or pair_and_single" > gpurun_out/r09e_pytest.log 2>&1 || { tail -30 gpurun_out/r09e_pytest.log; exit 1; }
tail -1 gpurun_out/r09e_pytest.log
for i in 1 2 3; do
  for v in default pw4; do
    if [ $v = pw4 ]; then export FDR_LIB=$PWD/dfd-starter_amd/fdr/libfdr_pw4.so; else unset FDR_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/r09e_${v}_$i.log 2>&1 || exit 1
    python3 - gpurun_out/r09e_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
v = d["variants"]["4096_pairs"]
print("%-7s base %.4f ms (rollout %.4f, frac %.4f)  variant rollout %.4f" % (
    sys.argv[2], d["ms_per_step"], d["roofline"]["rollout_ms"], d["roofline"]["frac"], v["rollout_ms"]))
PY
  done
done
echo r09e done
