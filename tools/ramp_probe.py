#!/usr/bin/env python3
"""Per-step time of bench.py's pipelined device-API step from a cold start
(development tool): builds the C2 store (or --n rows), then, twice with an idle
second between, runs --steps steps recording each step's wall time.  Shows how
many steps the GPU needs before the step time settles (clock / power state
ramp).  Output: one JSON line per run with the per-step ms and summaries."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--steps", type=int, default=400)
a = ap.parse_args()
lh = bench._load_lib()
L = lh.lib()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
e = bench.err_buf()
D, B, K = 768, 256, 10
h = L.lance_create_detached(b"", D, b"l2", b"ramp", e, 2048)
lh.LanceHipSetOption(h, "reserve_rows", str(a.n))
for lo in range(0, a.n, 1 << 18):
    hi = min(a.n, lo + (1 << 18))
    X = bench.gen_rows(lo, hi, D, dev)
    torch.cuda.synchronize()
    L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, D, e, 2048)
    del X
lh.LanceHipSetOption(h, "prepare", "1")
g = torch.Generator(device=dev)
g.manual_seed(5678)
Q = torch.randn((B, D), generator=g, device=dev, dtype=torch.float32)
from lance_hip.sharded import AsyncPipeline  # noqa: E402

pipe = AsyncPipeline(L, h, D)
for run in range(2):
    torch.cuda.synchronize()
    time.sleep(1.0)  # idle: the clocks drop
    ts = []
    t_prev = time.perf_counter()
    for i in range(a.steps):
        pipe.step(Q, K)
        t = time.perf_counter()
        ts.append(1000 * (t - t_prev))
        t_prev = t
    pipe.drain()
    ts = np.array(ts)
    blocks = [round(float(np.median(ts[i:i + 20])), 4) for i in range(0, a.steps, 20)]
    print(json.dumps({"run": run, "n": a.n, "median_ms_per_20_steps": blocks,
                      "first_20_mean_ms": round(float(ts[:20].mean()), 4),
                      "last_100_mean_ms": round(float(ts[-100:].mean()), 4)}), flush=True)
