#!/usr/bin/env python3
"""DuckDB's one-query-per-call path timed from C++ (no Python in the loop):
tests/cpp/abi_caller.cpp (the reference's RustFFI + LanceIndex::Search
restated over the C-ABI, torch-free, /opt/rocm's HIP runtime) loads the C2
table (--n rows x --d, seeded N(0,1) float32) through Append, then times
`--reps` passes of one Search per query over --nq queries after `--settle`
untimed calls.  Prints one JSON line (per-call mean / median microseconds).
Development / measurement tool; needs a GPU."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--d", type=int, default=768)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--settle", type=int, default=2000)
ap.add_argument("--reps", type=int, default=4)
a = ap.parse_args()

lib = os.path.join(ROOT, "duckdb-lancedb_amd", "lib")
tmp = tempfile.mkdtemp(prefix="lhip_pc_")
exe = os.path.join(tmp, "abi_caller")
subprocess.run(["g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "abi_caller.cpp"), "-o", exe,
                f"-L{lib}", "-llancedb_hip", f"-Wl,-rpath,{lib}"], check=True, timeout=180)
rng = np.random.default_rng(1234)
rows = os.path.join(tmp, "rows.f32")
with open(rows, "wb") as f:
    for lo in range(0, a.n, 1 << 17):
        rng.standard_normal((min(a.n, lo + (1 << 17)) - lo, a.d), dtype=np.float32).tofile(f)
qf = os.path.join(tmp, "q.f32")
rng.standard_normal((a.nq, a.d), dtype=np.float32).tofile(qf)
script = os.path.join(tmp, "script.txt")
with open(script, "w") as f:
    f.write(f"bulk {a.d} l2 {rows} {a.n} 65536\n")
    f.write(f"time_percall {qf} {a.nq} {a.k} {a.settle} {a.reps}\n")
t0 = time.perf_counter()
r = subprocess.run([exe, "gpu", script], capture_output=True, text=True, timeout=900)
os.remove(rows)
out = r.stdout.split("\n")
line = [l for l in out if l.startswith("time_percall")]
if r.returncode != 0 or not line or any(l.startswith("error") for l in out):
    print(r.stdout + r.stderr, file=sys.stderr)
    sys.exit(1)
_, calls, secs, mean_us, med_us, got = line[0].split()
print(json.dumps({"metric": "per-call latency, lance_search()'s one Search per query from C++ (torch-free)",
                  "n": a.n, "dim": a.d, "k": a.k, "calls": int(calls), "settle_calls": a.settle,
                  "us_per_call": float(mean_us), "median_us": float(med_us),
                  "queries_per_s": round(int(calls) / float(secs), 1), "results": int(got),
                  "path": "abi_caller MiniIndex::Search -> RustFFI::Search -> lance_detached_search (host buffers)",
                  "wall_s": round(time.perf_counter() - t0, 1)}))
