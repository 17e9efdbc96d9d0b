"""Harvest the reference's per-phase pivot-loop times into tests/golden/published_timings.json.

Run in the build container only (reads /root/reference).  Source: data/measures/<gpu>/
benchmark_<n>_<m>.txt (chrono.cu:35-50: one `solve` row per iteration of the pivot loop, in
microseconds; rows column 1+n+2m in phase 1, 1+n+m in phase 2).  Per phase: the sum of the
`solve` rows (the pivot loop's wall time) and the number of rows.  tools/compare_t_sweep.py sets
the MI355X -t sweep (simplex_cli -t, same CSV format) beside it.
"""
import csv
import glob
import json
import os
import sys

REF = "/root/reference/data/measures"
OUT = os.path.join(os.path.dirname(__file__), "..", "published_timings.json")


def parse(path, n, m):
    sums = {1: 0.0, 2: 0.0}
    rows_ = {1: 0, 2: 0}
    with open(path) as f:
        rd = csv.reader(f)
        next(rd)
        for row in rd:
            rows, op, us = int(row[0]), row[2], float(row[3])
            if op != "solve":
                continue
            ph = 1 if rows == 1 + n + 2 * m else 2 if rows == 1 + n + m else 0
            if ph:
                sums[ph] += us
                rows_[ph] += 1
    return {"p1_solve_us": sums[1], "p1_solve_rows": rows_[1], "p2_solve_us": sums[2], "p2_solve_rows": rows_[2]}


def main():
    out = []
    for gpu in ("rtx2070super", "mx250_2"):
        for path in sorted(glob.glob(os.path.join(REF, gpu, "benchmark_*_*.txt"))):
            n, m = map(int, os.path.basename(path)[len("benchmark_"):-4].split("_"))
            rec = {"gpu": gpu, "n": n, "m": m}
            rec.update(parse(path, n, m))
            out.append(rec)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(out)} records to {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
