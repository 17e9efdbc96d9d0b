#!/bin/bash
# Basic-slack deactivation, part 2: the rest of the GPU suite, then same-box bench lines with it on
# and off (SIMPLEX_DEACTIVATE), window + whole solves.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
step suite2 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_published.py tests/test_gpu_tabular.py tests/test_gpu_deactivate.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu || exit $?
tail -1 $O/suite2.log
for v in 1 0 1 0; do
  export SIMPLEX_DEACTIVATE=$v; step bench_$v 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  python3 - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fs = {x["instance"]: (round(x["seconds"], 3), x["pivots"], [round(v) for v in x["pivots_per_s"]], (x.get("parity") or {}).get("match")) for x in d["full_solve"]}
print("deact", sys.argv[2], "c5", round(d["value"]), "frac", round(d["roofline"]["frac"], 3), "c3", round(d["secondary"]["value"]), "parity", d["parity"]["match"], fs)
PY
done
