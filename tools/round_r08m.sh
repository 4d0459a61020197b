#!/bin/bash
# r08m: fdr_impala_h.hip built with other AMDGPU machine-scheduler settings (conv_kernel_h2<512> spills: default 32 B/lane,
# -amdgpu-use-amdgpu-trackers 0, max-ilp 20, both 0): A/B, config 5 at T = 60; fdr_rollout.hip with max-ilp on config 3.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS="libfdr libfdr_trk libfdr_ilp libfdr_trkilp libfdr libfdr_trk libfdr_ilp libfdr_trkilp" CONFIGS="impala_fp16" T=60 bash tools/ab_impala.sh || exit 3
timeout -k 10 600 bash tools/ab_pair.sh 3 halfcheetah libfdr libfdr_roilp || exit 3
echo r08m done
