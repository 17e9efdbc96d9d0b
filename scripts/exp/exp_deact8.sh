#!/bin/bash
# Deactivation with failed columns remembered: its tests, the long-pin / whole-solve subset, a kernel
# trace of the bench and two bench lines.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
export TMPDIR=/tmp
step deact 400 python -u -m pytest tests/test_gpu_deactivate.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu || exit $?
tail -1 $O/deact.log
step subset 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "compaction or two_phase or long_pins or whole_solve or config2" || exit $?
tail -1 $O/subset.log
step kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
for v in 1 2; do
  step bench_$v 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  python3 - $O/bench_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
fs = {x["instance"]: (round(x["seconds"], 3), [round(v) for v in x["pivots_per_s"]], (x.get("parity") or {}).get("match")) for x in d["full_solve"]}
print("bench c5", round(d["value"]), "frac", round(d["roofline"]["frac"], 3), "c3", round(d["secondary"]["value"]), "parity", d["parity"]["match"], fs)
PY
done
