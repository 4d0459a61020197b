set -u
mkdir -p gpurun_out
for impl in pair single; do for L in 1024 2048 4096; do
  FDR_ROLLOUT=$impl timeout -k 10 120 python tools/rollout_phases.py --lanes $L --iters 8 > gpurun_out/ph_${impl}_$L.log 2>&1 || exit 3
  echo "== $impl $L"; cat gpurun_out/ph_${impl}_$L.log | grep -v amdgpu.ids
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/parity.log
