"""Summarise a scripts/profile.sh run into profiles/<tag>_*.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc_update.json    per-launch HBM bytes of the update kernel:
      traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes -- gfx950 FETCH_SIZE counts half
      the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact
      for 16-B-per-lane streaming stores.
usage: python scripts/analyze_profile.py <prof_dir> <tag> [kernel_substring] [publish_as.json]
"""
import collections
import csv
import json
import os
import shutil
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    sub = sys.argv[3] if len(sys.argv) > 3 else "k_sweep"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(prof, "kt", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    stats = {}
    with open(os.path.join(prof, "kt", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            # the instantiation of the kernel with the most launches
            if sub in r["Name"] and int(r["Calls"]) > stats.get("calls", 0):
                stats = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                         "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    fetch = per_kernel(os.path.join(prof, "FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(prof, "WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {"kernel_trace": stats}
    for k in fetch:
        if k == stats.get("name") and k in write:
            fs = sum(fetch[k]) / len(fetch[k])
            ws = sum(write[k]) / len(write[k])
            res.update({"pmc_kernel": k, "launches": len(fetch[k]), "FETCH_SIZE_KB_avg": fs, "WRITE_SIZE_KB_avg": ws,
                        "hbm_bytes_per_launch": (2 * fs + ws) * 1024.0,
                        "correction": "traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)"})
    res["tag"] = tag
    with open(os.path.join(out, f"{tag}_pmc_update.json"), "w") as f:
        json.dump(res, f, indent=1)
    if len(sys.argv) > 4:  # also publish as the file bench.py reads for roofline.traffic
        with open(os.path.join(out, sys.argv[4]), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
