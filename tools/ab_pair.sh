#!/bin/bash
# Alternating A/B of rollout builds on the GPU box (tools/ab_pair.py per build and round).
#   bash tools/ab_pair.sh <rounds> <config> libfdr libfdr_v1 ...      -> gpurun_out/ab_pair_<config>.txt
set -u
mkdir -p gpurun_out
rounds=$1; cfg=$2; shift 2
out=gpurun_out/ab_pair_${cfg}.txt
: > "$out"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    timeout -k 10 150 python tools/ab_pair.py --lib dfd-starter_amd/fdr/$v.so --config "$cfg" >> "$out" 2>&1 \
      || { echo "$v FAILED rc=$?" >> "$out"; tail -5 "$out"; exit 3; }
    tail -1 "$out"
  done
done
