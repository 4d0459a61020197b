#!/bin/bash
# Focused GPU session: the given pytest node ids / files, then optional bench args.  Stops at a fault.
set -u
mkdir -p gpurun_out
FAULT='HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorIllegalAddress|GPU core dump'
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_new.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_new.log
if grep -qE "$FAULT" gpurun_out/pytest_new.log; then echo "GPU FAULT"; exit 3; fi
exit $rc
