#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, with the
pool_refine launches split by their order in a step (tau mode first, then the
final mode).  usage: tools/trace_kernels.py run_kernel_trace.csv [last_n_steps [skip_last]]
(skip_last: steps at the end to leave out, e.g. bench.py's time_kernels leg)"""
import csv
import statistics
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
d = defaultdict(list)
seq = []
for r in rows:
    n = r["Kernel_Name"]
    if "lhip" not in n:
        continue
    short = n.split("(")[0].replace("void ", "").replace("lhip::", "")
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    seq.append((short, dur, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
# steps start at ivf_prep (IVF configs) or else query_absmax (int8 path) / prep_queries
if any(s[0].startswith("ivf_prep_kernel") for s in seq):
    starts = [i for i, s in enumerate(seq) if s[0].startswith("ivf_prep_kernel")]
elif any(s[0].startswith("query_absmax") for s in seq):
    starts = [i for i, s in enumerate(seq) if s[0].startswith("query_absmax") or s[0].startswith("prep_queries_kernel")]
else:  # (a few queries per call: the int8 prep is one fused launch)
    starts = [i for i, s in enumerate(seq) if s[0].startswith("prep_queries")]
steps = [seq[a:b] for a, b in zip(starts, starts[1:] + [len(seq)])]
steps = steps[:len(steps) - skip][-last:]
for st in steps:
    npr = 0
    for (n, dur, _, _) in st:
        if n.startswith("pool_refine"):
            n = n + (" [tau]" if npr == 0 else " [final]")
            npr += 1
        d[n].append(dur)
span = [(st[-1][3] - st[0][2]) / 1000.0 for st in steps]
gaps = [(b[0][2] - a[-1][3]) / 1000.0 for a, b in zip(steps, steps[1:])]
for n, v in d.items():
    print(f"{n:55s} n={len(v):3d} avg={statistics.mean(v):8.1f} med={statistics.median(v):8.1f} min={min(v):7.1f} max={max(v):7.1f}")
print(f"step GPU span (first kernel start -> last kernel end): med {statistics.median(span):.1f} us")
if gaps:
    print(f"gap between steps (last kernel end -> next first kernel start): med {statistics.median(gaps):.1f} us")
