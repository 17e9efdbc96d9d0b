#!/bin/bash
# Basic-slack deactivation, final form: the whole GPU suite, a kernel trace of the bench (k_deact_*
# durations), then same-box bench lines with SIMPLEX_DEACTIVATE=8 / 0 alternating.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
export TMPDIR=/tmp
step suite 1000 python -u -m pytest tests -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu || exit $?
tail -1 $O/suite.log
step kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
for v in 8 0 8 0; do
  export SIMPLEX_DEACTIVATE=$v; step bench_$v 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  python3 - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fs = {x["instance"]: (round(x["seconds"], 3), x["pivots"], [round(v) for v in x["pivots_per_s"]], (x.get("parity") or {}).get("match")) for x in d["full_solve"]}
print("deact", sys.argv[2], "c5", round(d["value"]), "frac", round(d["roofline"]["frac"], 3), "c3", round(d["secondary"]["value"]), "parity", d["parity"]["match"], fs)
PY
done
