#!/bin/bash
# Basic-slack deactivation every few sweeps: its tests, the compaction / two-phase / long-pin tests,
# then same-box bench lines with SIMPLEX_DEACTIVATE=8 and 0 alternating.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
step deact 400 python -u -m pytest tests/test_gpu_deactivate.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu || exit $?
tail -1 $O/deact.log
step subset 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_published.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "compaction or two_phase or region or long_pins or whole_solve or published or config2 or session or pivots" || exit $?
tail -1 $O/subset.log
for v in 8 0 8 0; do
  export SIMPLEX_DEACTIVATE=$v; step bench_$v 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  python3 - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fs = {x["instance"]: (round(x["seconds"], 3), x["pivots"], [round(v) for v in x["pivots_per_s"]], (x.get("parity") or {}).get("match")) for x in d["full_solve"]}
print("deact", sys.argv[2], "c5", round(d["value"]), "frac", round(d["roofline"]["frac"], 3), "c3", round(d["secondary"]["value"]), "parity", d["parity"]["match"], fs)
PY
done
