#!/bin/bash
# Round 3: the 64-slot sweep on the vector units with DPP-broadcast factors (vsweep_probe).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/vsweep_probe > gpurun_out/r03_vsweep_probe.txt 2>&1
