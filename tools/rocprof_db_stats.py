#!/usr/bin/env python3
"""Kernel statistics CSV from a rocprofv3 --kernel-trace database (run_results.db):
per kernel name the calls, total / average / min / max / std-dev duration (ns), the share of
all kernel time and the launch resources (LDS, VGPR, AGPR, SGPR, scratch), as the
profiles/r05/rocprof_*_kernel_stats.csv files hold.
  python3 tools/rocprof_db_stats.py gpurun_out/TAG/NN_prof/run_results.db OUT.csv"""
import csv
import sqlite3
import statistics
import sys


def main(db_path, out_path):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, duration, lds_size, vgpr_count, accum_vgpr_count, sgpr_count, scratch_size "
                      "from kernels").fetchall()
    by = {}
    for name, dur, lds, vgpr, agpr, sgpr, scr in rows:
        e = by.setdefault(name, {"d": [], "res": (lds, vgpr, agpr, sgpr, scr)})
        e["d"].append(dur)
    total = sum(sum(e["d"]) for e in by.values()) or 1
    out = []
    for name, e in by.items():
        d = e["d"]
        out.append([name, len(d), sum(d), round(sum(d) / len(d), 3), round(100.0 * sum(d) / total, 2), min(d), max(d),
                    round(statistics.pstdev(d), 3), *e["res"]])
    out.sort(key=lambda r: -r[2])
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev",
                    "LdsBytes", "Vgpr", "Agpr", "Sgpr", "ScratchBytes"])
        w.writerows(out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
