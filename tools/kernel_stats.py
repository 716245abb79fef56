#!/usr/bin/env python3
"""rocprofv3 --kernel-trace output (rocpd database run_results.db, or a
kernel_trace.csv) -> the per-kernel summary rocprofv3 --stats prints
(Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).

usage: tools/kernel_stats.py TRACE(.db|.csv) OUT.csv
"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict


def durations(path):
    d = defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for s, e, name in c.execute("select start, end, name from kernels"):
            d[name].append(e - s)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                d[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return d


def main():
    d = durations(sys.argv[1])
    total = sum(sum(v) for v in d.values())
    rows = []
    for name, v in d.items():
        avg = sum(v) / len(v)
        sd = math.sqrt(sum((x - avg) ** 2 for x in v) / len(v))
        rows.append((name, len(v), sum(v), avg, 100.0 * sum(v) / total, min(v), max(v), sd))
    rows.sort(key=lambda r: -r[2])
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 1), round(r[4], 2), r[5], r[6], round(r[7], 1)])
    for r in rows[:12]:
        print(f"{r[1]:6d} {r[3] / 1000:10.1f} us  {r[4]:5.1f}%  {r[0][:90]}")


if __name__ == "__main__":
    main()
