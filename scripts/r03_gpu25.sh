#!/bin/bash
# Round 3: fp64 matrix / vector rate ceilings (f64_rate_probe).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/f64_rate_probe > gpurun_out/r03_f64_rate_probe.txt 2>&1
