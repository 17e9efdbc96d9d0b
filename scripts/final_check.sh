#!/bin/bash
# The whole -m gpu suite, then rocprofv3 kernel trace + HBM counters of the driver's bench
# command (scripts/profile.sh) into gpurun_out/prof_$1.
set -o pipefail
T=${1:-final}
R=${ROUND:-r04}
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_pytest_gpu_$T.txt 2>&1 || exit $?
PROF_OUT=gpurun_out/prof_$T PROF_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/profile.sh > gpurun_out/${R}_prof_$T.log 2>&1
