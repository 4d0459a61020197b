#!/bin/bash
# rocprofv3 runs for the bench workload (GPU box).  Kernel trace + stats, then separate PMC passes.
# Usage: bash tools/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress'
run() {  # run <name> <rocprof args...> -- handled by caller
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if grep -qE "$FAULT" "$OUT/$name.log"; then echo "GPU FAULT -- stopping"; exit 3; fi
  [ "$rc" -eq 0 ] || exit "$rc"
}
BENCH="bench.py --steps 20 --warmup 3 --no-cpu-baseline $*"
[ -n "${SKIP_BASE:-}" ] || run trace --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH
[ -n "${SKIP_BASE:-}" ] || run pmc_fetch --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH
[ -n "${SKIP_BASE:-}" ] || run pmc_write --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 $BENCH
[ -n "${SKIP_BASE:-}" ] || run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $BENCH
if [ -n "${MFMA_PMC:-}" ]; then
  run pmc_mfma --pmc $MFMA_PMC --kernel-trace --output-format csv -d "$OUT/pmc_mfma" -o run -- python3 $BENCH
fi
# EXTRA_PMC="C1 C2;C3 C4": one more pass per ';'-separated counter group
if [ -n "${EXTRA_PMC:-}" ]; then
  i=0
  IFS=';' read -ra GROUPS_ <<< "$EXTRA_PMC"
  for g in "${GROUPS_[@]}"; do
    run pmc_extra$i --pmc $g --kernel-trace --output-format csv -d "$OUT/pmc_extra$i" -o run -- python3 $BENCH
    i=$((i + 1))
  done
fi
ls -R "$OUT" > "$OUT/ls.txt"
