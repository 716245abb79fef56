#!/usr/bin/env python3
"""Interleaved A/B of handle options on ONE flat store (development tool).

Builds bench.py's synthetic store once (default: the north_star shape, 10M x
768 f32, B = 256, k = 10), then for each repetition and each option setting:
sets the options, runs warmup + timed pipelined steps (bench.py's device API)
and reads the append scan's in-library HIP-event time.  Results are exact for
every setting these options accept; the first setting's ids are compared with
every other's.

usage: tools/ab_opts.py [--n N] [--steps K] [--reps R] "s8_couple=0" "s8_couple=8" ...
(a setting may hold several options separated by commas)
"""
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
ap.add_argument("settings", nargs="+")
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--dim", type=int, default=768)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--settle-steps", type=int, default=300, help="untimed steps first (the GPU clock ramp)")
a = ap.parse_args()

lh = bench._load_lib()
L = lh.lib()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
e = bench.err_buf()
h = L.lance_create_detached(b"", a.dim, b"l2", b"ab", e, 2048)
lh.LanceHipSetOption(h, "reserve_rows", str(a.n))
for lo in range(0, a.n, 1 << 18):
    hi = min(a.n, lo + (1 << 18))
    X = bench.gen_rows(lo, hi, a.dim, dev)
    torch.cuda.synchronize()
    if L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, a.dim, e, 2048) < 0:
        raise RuntimeError(e.value.decode())
    del X
lh.LanceHipSetOption(h, "prepare", "1")
g = torch.Generator(device=dev)
g.manual_seed(5678)
Q = torch.randn((a.batch, a.dim), generator=g, device=dev, dtype=torch.float32)
from lance_hip.sharded import AsyncPipeline  # noqa: E402

ref_ids = None
_p = AsyncPipeline(L, h, a.dim)
for _ in range(a.settle_steps):
    _p.step(Q, a.k)
_p.drain()
del _p
for rep in range(a.reps):
    for s in a.settings:
        for kv in s.split(","):
            k, _, v = kv.partition("=")
            lh.LanceHipSetOption(h, k, v)
        pipe = AsyncPipeline(L, h, a.dim)
        for _ in range(a.warmup):
            pipe.step(Q, a.k)
        pipe.drain()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for _ in range(a.steps):
            r = pipe.step(Q, a.k)
            out = r if r is not None else out
        r = pipe.drain()
        out = r if r is not None else out
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ids = out[0].cpu().numpy().copy()
        lh.LanceHipSetOption(h, "time_kernels", "1")
        for _ in range(5):
            pipe.step(Q, a.k)
        pipe.drain()
        kt = lh.LanceHipKernelTimes(h)
        lh.LanceHipSetOption(h, "time_kernels", "0")
        st = lh.LanceHipLastSearchStats(h)
        if ref_ids is None:
            ref_ids = ids
        line = {"setting": s, "rep": rep, "qps": round(a.batch * a.steps / dt, 1),
                "ms_per_step": round(1000 * dt / a.steps, 4), "append_ms": round(kt["scan_ms_total"] / max(1, kt["scan_launches"]), 4),
                "ids_equal_first": bool((ids == ref_ids).all()), "fallbacks": st.get("fallback_queries")}
        print(json.dumps(line), flush=True)
