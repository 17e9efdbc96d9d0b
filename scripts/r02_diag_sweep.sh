#!/bin/bash
# Why did the driver's `bench.py --steps 20 --warmup 5` sweep run at 1498 us (vs 868 us)?
# 1) the driver's own command under rocprofv3 kernel trace; 2) 2000 pivots with 20-pivot
# batches vs 32-pivot batches (HIP events per sweep).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/diag
mkdir -p $OUT
Q="--no-cpu-baseline --secondary= --no-full-solve"
echo "== driver cmd under rocprofv3 ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt20 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 $Q > $OUT/kt20.log 2>&1 || exit 1
tail -1 $OUT/kt20.log
for b in 20 32; do
  echo "== batch $b ($(date +%T))"
  timeout -k 10 300 python3 bench.py --steps 640 --warmup 64 --batch $b $Q > $OUT/batch$b.log 2>&1 || exit 1
  tail -1 $OUT/batch$b.log
done
