#!/bin/bash
# Deactivation cadence: bench lines (window, config 3, whole solves) with SIMPLEX_DEACTIVATE=4 / 8 / 16 / 32.
# (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
for v in 4 8 16 32 8 4; do
  export SIMPLEX_DEACTIVATE=$v; step bench_$v 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  python3 - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fs = {x["instance"]: (round(x["seconds"], 3), [round(v) for v in x["pivots_per_s"]], (x.get("parity") or {}).get("match")) for x in d["full_solve"]}
print("every", sys.argv[2], "c5", round(d["value"]), "frac", round(d["roofline"]["frac"], 3), "c3", round(d["secondary"]["value"]), "parity", d["parity"]["match"], fs)
PY
done
