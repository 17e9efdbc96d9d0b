"""Harvest the reference's published pivot counts into tests/golden/published_pivots.json.

Run in the build container only (reads /root/reference, which the GPU box does not have).
Source: data/measures/<gpu>/benchmark_<n>_<m>.txt -- one CSV row per timed operation
(chrono.cu:35-50).  Each `solve` row is one call of solve() (solver.cu:78-126); the rows
column is 1+n+2m in phase 1 and 1+n+m in phase 2 (tabular.cu:30, twoPhaseMethod.cu:288).
Pivots per phase = solve rows - 1 (the last call only detects termination), except when
the phase ended UNBOUNDED, which the file cannot distinguish (never happens in this set).
Seeds follow main.cu:63 (n*100+m, +1 for n=1024/m=8192), values in [+1,+100] (main.cu:64).
"""
import csv
import glob
import json
import os
import sys

REF = "/root/reference/data/measures"
OUT = os.path.join(os.path.dirname(__file__), "..", "published_pivots.json")


def parse(path, n, m):
    p1 = p2 = 0
    ops = set()
    with open(path) as f:
        rd = csv.reader(f)
        next(rd)
        for row in rd:
            rows, _cols, op = int(row[0]), int(row[1]), row[2]
            ops.add(op)
            if op == "solve":
                if rows == 1 + n + 2 * m:
                    p1 += 1
                elif rows == 1 + n + m:
                    p2 += 1
    ended_p1_infeasible = "checkDegeneracy" not in ops
    return {
        "p1_pivots": p1 - 1,
        "p2_pivots": (p2 - 1) if p2 else None,
        "status": "infeasible" if ended_p1_infeasible else ("optimal" if p2 else "degenerate"),
    }


def main():
    out = []
    for gpu in ("rtx2070super", "mx250_2"):
        for path in sorted(glob.glob(os.path.join(REF, gpu, "benchmark_*_*.txt"))):
            n, m = map(int, os.path.basename(path)[len("benchmark_"):-4].split("_"))
            seed = n * 100 + m + (1 if (n == 1024 and m == 8192) else 0)
            rec = {"gpu": gpu, "n": n, "m": m, "seed": seed, "lo": 1, "hi": 100}
            rec.update(parse(path, n, m))
            out.append(rec)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(out)} records to {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
