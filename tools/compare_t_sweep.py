"""The reference's -t benchmark (main.cu:50-77) on MI355X beside its published runs (diagnostic).

Reads the TIMER CSVs that `simplex_cli -t` wrote (benchmark_<n>_<m>.txt, chrono.cu:35-50 format:
one `solve` row per pivot-loop iteration) and tests/golden/published_{pivots,timings}.json
(harvested from data/measures/rtx2070super), and prints a markdown table: per instance the
pivot counts (must equal the published ones), the phase-1 pivot rate on both GPUs and the ratio.
usage: python tools/compare_t_sweep.py <dir of benchmark_*.txt> [> table.md]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def phase_rows(path, n, m):
    out = {1: [], 2: []}
    with open(path) as f:
        rd = csv.reader(f)
        next(rd)
        for row in rd:
            rows, op, us = int(row[0]), row[2], float(row[3])
            if op == "solve":
                ph = 1 if rows == 1 + n + 2 * m else 2 if rows == 1 + n + m else 0
                if ph:
                    out[ph].append(us)
    return out


def main():
    d = sys.argv[1]
    with open(os.path.join(GOLDEN, "published_pivots.json")) as f:
        piv = {(r["n"], r["m"]): r for r in json.load(f) if r["gpu"] == "rtx2070super"}
    with open(os.path.join(GOLDEN, "published_timings.json")) as f:
        tim = {(r["n"], r["m"]): r for r in json.load(f) if r["gpu"] == "rtx2070super"}
    print("| n | m | P1 / P2 pivots (MI355X) | published (RTX 2070S) | equal | MI355X P1 pivots/s | "
          "RTX 2070S P1 pivots/s | ratio |")
    print("|---|---|---|---|---|---|---|---|")
    allsame, tot = True, 0
    for path in sorted(glob.glob(os.path.join(d, "benchmark_*_*.txt")),
                       key=lambda p: tuple(int(x) for x in os.path.basename(p)[10:-4].split("_"))):
        n, m = map(int, os.path.basename(path)[len("benchmark_"):-4].split("_"))
        ph = phase_rows(path, n, m)
        p1, p2 = len(ph[1]) - 1, (len(ph[2]) - 1) if ph[2] else None
        ref = piv[(n, m)]
        same = (p1, p2) == (ref["p1_pivots"], ref["p2_pivots"])
        allsame &= same
        tot += 1
        ours = p1 / (sum(ph[1]) * 1e-6)
        t = tim[(n, m)]
        theirs = ref["p1_pivots"] / (t["p1_solve_us"] * 1e-6)
        print(f"| {n} | {m} | {p1} / {p2} | {ref['p1_pivots']} / {ref['p2_pivots']} | {'yes' if same else 'NO'} | "
              f"{ours:,.0f} | {theirs:,.1f} | {ours / theirs:,.0f}x |")
    print(f"\n{tot} instances; pivot counts equal to the published ones on all: {allsame}")


if __name__ == "__main__":
    main()
