#!/bin/bash
# Round 3: 64-slot sweep layouts with the pivot rows in LDS (msweep64_probe V7/V8).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/msweep64_probe > gpurun_out/r03_msweep64_probe_v7.txt 2>&1
