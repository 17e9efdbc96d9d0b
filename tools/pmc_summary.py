"""Per-dispatch summaries of rocprofv3 --pmc counter CSVs (diagnostic; the profiles/r04_* records).

  python tools/pmc_summary.py sq  <run_counter_collection.csv> [kernel-substring]
      effective clock (GRBM_GUI_ACTIVE / 8 / duration, MI355X_MICROARCH.md "DVFS give-back"),
      f64 MFMA count (SQ_INSTS_VALU_MFMA_MOPS_F64 / 4: 512-flop units, 2048 flops per
      v_mfma_f64_16x16x4f64), matrix-pipe busy fraction (SQ_VALU_MFMA_BUSY_CYCLES per SIMD over the
      dispatch's cycles), and the wave-state split (SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY /
      SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES)
  python tools/pmc_summary.py tcp <csv> [kernel-substring]      UTCL1 (L1 TLB) hits / misses
  python tools/pmc_summary.py hbm <FETCH csv> <WRITE csv> <algorithmic bytes> [kernel-substring]
      HBM bytes per dispatch, (2 FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 correction)
"""
import collections
import csv
import re
import sys

SIMDS = 1024  # 256 CUs x 4


def dispatches(path, filt):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if filt not in r["Kernel_Name"]:
            continue
        k = r["Dispatch_Id"]
        e = d.setdefault(k, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                             "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(d.values())


def kname(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if xs else float("nan")


def main():
    mode = sys.argv[1]
    if mode == "sq":
        ds = dispatches(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
        by = collections.defaultdict(list)
        for v in ds:
            by[kname(v["name"])].append(v)
        for name, vs in by.items():
            rows = []
            for v in vs:
                cyc = v["GRBM_GUI_ACTIVE"] / 8
                mf = v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) / 4
                rows.append({
                    "dur_us": v["dur"] * 1e6, "clock_GHz": cyc / v["dur"] / 1e9, "mfma_f64": mf,
                    "tflops": mf * 2048 / v["dur"] / 1e12,
                    "mfma_busy_frac": v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / SIMDS / cyc,
                    "active": v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"],
                    "wait_any": v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"],
                    "wait_inst": v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"]})
            keys = rows[0].keys()
            print(f"{name}: {len(rows)} dispatches, medians: " +
                  ", ".join(f"{k} {med([r[k] for r in rows]):.4g}" for k in keys))
    elif mode == "tcp":
        ds = dispatches(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
        by = collections.defaultdict(list)
        for v in ds:
            by[kname(v["name"])].append(v)
        for name, vs in by.items():
            print(f"{name}: {len(vs)} dispatches, medians: " + ", ".join(
                f"{k} {med([v[k] for v in vs]):.4g}" for k in vs[0] if k.startswith("TCP_")))
    elif mode == "hbm":
        filt = sys.argv[5] if len(sys.argv) > 5 else "msweep"
        f = [v["FETCH_SIZE"] for v in dispatches(sys.argv[2], filt)]
        w = [v["WRITE_SIZE"] for v in dispatches(sys.argv[3], filt)]
        alg = float(sys.argv[4])
        hbm = (2 * med(f) + med(w)) * 1024
        print(f"{filt}: {len(f)} / {len(w)} dispatches; HBM bytes per dispatch (2*FETCH+WRITE)*1024 = {hbm / 1e6:.1f} MB "
              f"(read {2 * med(f) * 1024 / 1e6:.1f}, write {med(w) * 1024 / 1e6:.1f}); algorithmic {alg / 1e6:.1f} MB; "
              f"ratio {hbm / alg:.3f}")


if __name__ == "__main__":
    main()
