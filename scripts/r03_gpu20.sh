#!/bin/bash
# Round 3: the driver's bench command on the final defaults (two stages from 4096 rows).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_v20.log 2>&1
