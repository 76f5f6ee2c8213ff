"""Per-kernel summary (rocprofv3 --stats layout) from a rocprofv3 output: a rocpd SQLite
database (`*_results.db`, the default format) or a `*_kernel_trace.csv`.

    python tools/prof_summary.py gpurun_out/prof_r01/run_results.db > profiles/r01_kernel_stats.csv
"""
from __future__ import annotations

import csv
import sqlite3
import sys
from collections import defaultdict


def rows_from_db(path: str):
    con = sqlite3.connect(path)
    for name, dur in con.execute("select name, duration from kernels"):
        yield name, int(dur)


def rows_from_csv(path: str):
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main(path: str) -> None:
    src = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    agg = defaultdict(list)
    for name, dur in src:
        agg[name].append(dur)
    total = sum(sum(v) for v in agg.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        w.writerow([name, len(v), s, round(s / len(v), 3), round(100.0 * s / total, 2), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
