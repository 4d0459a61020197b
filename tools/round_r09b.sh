#!/bin/bash
# r09b: final build after the round-split pair launches -- full GPU suite + smoke, every config's bench line,
# config-3 rocprof (kernel trace incl. the 8192-lane variant's two launches + FETCH / WRITE / SQ PMC).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit $?
bash tools/bench_round.sh r09b || exit $?
bash tools/profile.sh r09b_halfcheetah --config halfcheetah || exit $?
echo r09b done
