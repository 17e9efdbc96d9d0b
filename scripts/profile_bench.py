"""Summarise a scripts/profile.sh run of the driver's bench command into profiles/.

The bench runs its primary workload first: `warmup` + `steps` steps, one sweep (k_msweep or
k_sweep) each, so the first warmup+steps k_sweep dispatches of the trace are the primary workload's
and the last `steps` of those are its timed sweeps -- the ones the bench line's roofline
averages with HIP events.  Outputs:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the command
  profiles/<tag>_sweep.json         the timed sweeps' durations (trace) and HBM bytes (PMC):
      traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch -- gfx950 FETCH_SIZE
      counts half the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM); WRITE_SIZE
      is exact for 16-B-per-lane streaming stores
  profiles/pmc_sweep_<config>.json  (with --publish) the record bench.py reads for roofline.traffic
usage: python scripts/profile_bench.py <prof_dir> <tag> <warmup> <steps> "<command>" [--publish config5]
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sweep_rows(path, counter=None):
    """sweep dispatches (k_msweep / k_sweep) in dispatch order: (dispatch id, name, value) -- value = duration
    in ns (trace) or the counter's value (PMC)."""
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "k_sweep" not in r["Kernel_Name"] and "k_msweep" not in r["Kernel_Name"]:
                continue
            if counter is None:
                v = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            elif r.get("Counter_Name") == counter:
                v = float(r["Counter_Value"])
            else:
                continue
            out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], v))
    out.sort()
    return out


def find(prof, sub, name):
    for dp, _, files in os.walk(os.path.join(prof, sub)):
        if name in files:
            return os.path.join(dp, name)
    return None


def main():
    prof, tag, warmup, steps, command = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    publish = sys.argv[sys.argv.index("--publish") + 1] if "--publish" in sys.argv else None
    out = os.path.join(ROOT, "profiles")
    shutil.copy(find(prof, "kt", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    trace = sweep_rows(find(prof, "kt", "run_kernel_trace.csv"))
    timed = trace[warmup:warmup + steps]
    res = {"tag": tag, "command": command, "kernel": timed[0][1] if timed else None,
           "timed_launches": len(timed),
           "avg_ns": sum(v for _, _, v in timed) / max(len(timed), 1),
           "min_ns": min((v for _, _, v in timed), default=None),
           "max_ns": max((v for _, _, v in timed), default=None),
           "selection": f"sweep dispatches {warmup}..{warmup + steps - 1} in dispatch order: the primary "
                        "workload's timed sweeps"}
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = find(prof, c, "run_counter_collection.csv")
        if p:
            rows = sweep_rows(p, c)[warmup:warmup + steps]
            if rows:
                pmc[c] = sum(v for _, _, v in rows) / len(rows)
    if len(pmc) == 2:
        res.update({"FETCH_SIZE_KB_avg": pmc["FETCH_SIZE"], "WRITE_SIZE_KB_avg": pmc["WRITE_SIZE"],
                    "hbm_bytes_per_launch": (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0,
                    "correction": "traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)"})
    with open(os.path.join(out, f"{tag}_sweep.json"), "w") as f:
        json.dump(res, f, indent=1)
    if publish:
        with open(os.path.join(out, f"pmc_sweep_{publish}.json"), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
