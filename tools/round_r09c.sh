#!/bin/bash
# r09c: two-stream feasibility probe for config 5 (lane halves on two HIP streams vs one sequence)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/impala_two_stream.py --T 100 --reps 3 > gpurun_out/r09c_two_stream.log 2>&1 || { cat gpurun_out/r09c_two_stream.log | tail -20; exit 1; }
timeout -k 10 240 python -u tools/impala_two_stream.py --T 100 --reps 2 --splits 4 >> gpurun_out/r09c_two_stream.log 2>&1 || { tail -20 gpurun_out/r09c_two_stream.log; exit 1; }
cat gpurun_out/r09c_two_stream.log
