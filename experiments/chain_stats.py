"""Per-pivot kernel breakdown from a rocprofv3 kernel trace of bench.py: duration of each
pivot-path kernel (mean / median / p10 / p90, microseconds), the gaps between consecutive
ones, and the device time per pivot.

usage: python scripts/chain_stats.py <run_kernel_trace.csv> [pivots]   (pivots: the count the
trace covers, for the per-pivot figure when whole batches run in one launch)"""
import collections
import csv
import sys

import numpy as np

KINDS = [("k_ratio_select", "ratio"), ("k_select_row", "select_row"), ("k_select_gathered", "select_gathered"),
         ("k_pivot_row", "pivot_row"), ("k_sweep", "sweep"), ("k_batch", "batch")]


def kind(name):
    for key, short in KINDS:
        if key in name:
            return short
    return None


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    seq = [r for r in rows if kind(r["Kernel_Name"])]
    dur, gap = collections.defaultdict(list), collections.defaultdict(list)
    for i, r in enumerate(seq):
        dur[kind(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        if i:
            gap[kind(seq[i - 1]["Kernel_Name"]) + ">" + kind(r["Kernel_Name"])].append(
                int(r["Start_Timestamp"]) - int(seq[i - 1]["End_Timestamp"]))
    for k, v in dur.items():
        v = np.array(v) / 1e3
        print(f"{k:16s} n={len(v):6d} mean {v.mean():8.2f} med {np.median(v):8.2f} p10 {np.percentile(v, 10):8.2f} "
              f"p90 {np.percentile(v, 90):8.2f} us")
    for k, v in gap.items():
        v = np.array(v) / 1e3
        print(f"gap {k:24s} n={len(v):6d} mean {v.mean():6.2f} us")
    npiv = int(sys.argv[2]) if len(sys.argv) > 2 else len(dur.get("pivot_row", dur.get("batch", [1])))
    tot = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
    print(f"device time {tot:.1f} us over {npiv} pivots: {tot / max(npiv, 1):.2f} us per pivot")


if __name__ == "__main__":
    main()
