#!/bin/bash
# Round 3 final state: the whole -m gpu suite, then rocprofv3 kernel trace + HBM counters of the
# driver's bench command (scripts/profile.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu_final2.txt 2>&1 || exit $?
PROF_OUT=gpurun_out/prof_final2 PROF_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/profile.sh > gpurun_out/r03_prof_final2.log 2>&1
