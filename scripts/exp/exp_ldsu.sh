#!/bin/bash
# The two-stage sweep with U in LDS (SIMPLEX_SWEEP_LDSU=1, k_msweep_lu) vs the register form: parity
# subset with it on, then bench lines alternating.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
export SIMPLEX_SWEEP_LDSU=1
step parity 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_deactivate.py -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -m gpu -k "sweep or batch or leaves or fused or compaction or two_phase or long_pins or deactivated" || exit $?
tail -1 $O/parity.log
for v in 1 0 1 0; do
  export SIMPLEX_SWEEP_LDSU=$v; step bench_$v 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --full-solves=config4 || exit $?
  python3 - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fs = {x["instance"]: (round(x["seconds"], 3), (x.get("parity") or {}).get("match")) for x in d["full_solve"]}
print("ldsu", sys.argv[2], "c5", round(d["value"]), "us/piv", round(d["ms_per_pivot"] * 1000, 2), "sweep_us", round(d["roofline"]["avg_launch_us"], 1), "frac", round(d["roofline"]["frac"], 3), "c3", round(d["secondary"]["value"]), "parity", d["parity"]["match"], fs)
PY
done
