#!/bin/bash
# Round 3: the bench line with two-stage batches (default command).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/r03_bench_v11.log 2>&1
