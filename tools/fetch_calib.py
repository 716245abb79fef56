#!/usr/bin/env python3
"""FETCH_SIZE calibration from tools/_fetch_probe under rocprofv3 --pmc
FETCH_SIZE: per probe kernel, bytes read / (FETCH_SIZE KiB x 1024) = the
factor that turns that access pattern's FETCH_SIZE into bytes.
usage: tools/fetch_calib.py PMC_DIR PROBE_STDOUT OUT.json"""
import csv
import json
import os
import re
import sys

d, log, out = sys.argv[1:4]
nbytes = {}
for ln in open(log):
    m = re.match(r"(k\w+) bytes (\d+)", ln.strip())
    if m:
        nbytes[m.group(1)] = int(m.group(2))
vals = {}
for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    if r["Counter_Name"] != "FETCH_SIZE":
        continue
    n = r["Kernel_Name"]
    key = "k16" if "k16" in n else ("k12c" if ("k12<0>" in n or "k12ILi0E" in n) else
                                     "k12" if ("k12<2>" in n or "k12ILi2E" in n) else None)
    if key:
        vals.setdefault(key, []).append(float(r["Counter_Value"]))
res = {}
for k, v in vals.items():
    fk = sum(v) / len(v)
    res[k] = {"launches": len(v), "fetch_size_kib": fk, "bytes": nbytes[k],
              "factor_bytes_per_fetch_byte": nbytes[k] / (fk * 1024.0)}
res["note"] = ("k16: 16 B/lane global_load_dwordx4 (the guide's calibrated pattern, factor ~2); k12: the "
               "pq_fast_scan_bank_kernel<3> row stream (96-B rows, 8 lanes x buffer_load_dwordx3, nt); k12c: same, "
               "default cache policy; 1 GiB per launch")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
