#!/bin/bash
# Round 3, first GPU probe: the reference's -t sweep (36 instances, TIMER CSVs), the MX250's
# failing instance (n=1024, m=8192, seed 110592).
set -o pipefail
mkdir -p gpurun_out/r03_cli_t
export SIMPLEX_DATA_DIR=$PWD/gpurun_out/r03_cli_t
timeout -k 10 300 ./simplexoncuda_amd/simplex_cli -t > gpurun_out/r03_cli_t.log 2>&1 && \
timeout -k 10 120 python3 -u -c '
import sys, time; sys.path.insert(0, ".")
import torch; torch.cuda.set_device(0)
import simplexoncuda_amd as sx
for seed in (110592, 110593):
    p = sx.generateRandomProblem(1024, 8192, seed, 1, 100)
    t0 = time.time(); r = sx.twoPhaseMethodEx(p); dt = time.time() - t0
    print("n=1024 m=8192 seed", seed, "status", r.status_name, "pivots", r.pivots, "objective", repr(r.optimal_value), "s", round(dt, 3), flush=True)
' > gpurun_out/r03_seed110592.log 2>&1
