#!/bin/bash
# Round 3: the driver's bench command, its rocprofv3 kernel trace and HBM counter passes
# (config 5 primary; config 3 alone for its own counter record).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_v19.log 2>&1 || exit $?
PROF_OUT=gpurun_out/prof5 bash scripts/profile.sh > gpurun_out/r03_prof5.log 2>&1 || exit $?
