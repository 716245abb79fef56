#!/usr/bin/env python3
"""Development-only: print the kernel timeline of the last search steps from a
rocprofv3 --kernel-trace database (gpurun_out/<dir>/run_results.db)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select start, end, name from kernels order by start").fetchall()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 26
last = rows[-n:]
t0, prev = last[0][0], None
for s, e, name in last:
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{(s - t0) / 1000:9.1f} gap {gap:6.1f} dur {(e - s) / 1000:7.1f}  {name[:70]}")
    prev = e
