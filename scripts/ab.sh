#!/bin/bash
# Same-box A/B of engine variants on the driver's bench command (config 5 + config 3 + the
# synthetic update bench).  VARIANTS: space-separated list of NAME=ENV[,ENV...] ("base=" for the
# defaults); REPS rounds, the variants interleaved in each.  Every bench run under its own time
# limit; a failure ends the script.  Summary: gpurun_out/$TAG/summary.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-ab}
O=gpurun_out/$TAG
mkdir -p $O
REPS=${REPS:-3}
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --full-solves=}
for rep in $(seq 1 $REPS); do
  for v in ${VARIANTS:-base=}; do
    name=${v%%=*}; envs=${v#*=}
    echo "== $name rep $rep ($(date +%T))"
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python -u bench.py $BENCH_ARGS > "$O/${name}_$rep.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "== $name rc=$rc"; tail -20 "$O/${name}_$rep.log"; exit $rc; fi
  done
done
python3 - "$O" <<'PY' | tee "$O/summary.txt"
import glob, json, os, sys
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_*.log"))):
    name = os.path.basename(f).rsplit("_", 1)[0]
    line = [l for l in open(f) if l.startswith("{")]
    if not line:
        continue
    d = json.loads(line[-1])
    pr = d["config"]["per_rank"][0]
    s = d.get("secondary") or {}
    ub = d.get("update_bench") or {}
    v64 = (ub.get("variants") or [None, None])[1] or {}
    rows.setdefault(name, []).append((d["value"], pr["sweep_us_per_pivot"], pr["chain_us_per_pivot"],
                                     d["roofline"]["frac"], d["roofline"]["avg_launch_us"], s.get("value", 0),
                                     (s.get("roofline") or {}).get("frac", 0), ub.get("frac", 0),
                                     v64.get("frac", 0), (ub.get("out_of_cache") or {}).get("frac", 0)))
print("variant        c5 piv/s  sweep  chain  frac  sweep_us | c3 piv/s  frac | ub32  ub64  ub32big")
for name, rs in rows.items():
    for r in rs:
        print(f"{name:12s} {r[0]:9.0f} {r[1]:6.2f} {r[2]:6.2f} {r[3]:.3f} {r[4]:8.1f} | {r[5]:8.0f} {r[6]:.3f} | {r[7]:.3f} {r[8]:.3f} {r[9]:.3f}")
    med = [sorted(x)[len(x) // 2] for x in zip(*rs)]
    print(f"{name + ' med':12s} {med[0]:9.0f} {med[1]:6.2f} {med[2]:6.2f} {med[3]:.3f} {med[4]:8.1f} | {med[5]:8.0f} {med[6]:.3f} | {med[7]:.3f} {med[8]:.3f} {med[9]:.3f}")
PY
