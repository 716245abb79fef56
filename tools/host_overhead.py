#!/usr/bin/env python3
"""Development-only: per-call host costs on the search path (GPU box)."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "duckdb-lancedb_amd"))
import lance_hip  # noqa: E402

L = lance_hip.lib()
dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
torch.cuda.synchronize()


def bench(name, f, n=2000):
    for _ in range(50):
        f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    print(f"{name:40s} {(time.perf_counter() - t0) / n * 1e6:8.2f} us")


bench("torch current_stream().synchronize()", lambda: torch.cuda.current_stream().synchronize())
bench("ctypes lance_hip_version()", lambda: L.lance_hip_version())
bench("ctypes lance_hip_device_count()", lambda: L.lance_hip_device_count())
x = torch.empty(10, device=dev)
bench("torch.empty x3", lambda: (torch.empty((256, 10), dtype=torch.int64, device=dev),
                                  torch.empty((256, 10), device=dev), torch.empty((256,), dtype=torch.int32, device=dev)))
bench("ctypes.create_string_buffer(2048)", lambda: ctypes.create_string_buffer(2048))
# a tiny index: one full search call (GPU work small)
e = ctypes.create_string_buffer(2048)
h = L.lance_create_detached(b"", 64, b"l2", b"t", e, 2048)
X = torch.randn(100_000, 64, device=dev)
torch.cuda.synchronize()
assert L.lance_hip_add_batch_device(h, X.data_ptr(), 100_000, 64, e, 2048) >= 0, e.value
from lance_hip.sharded import hip_device_search  # noqa: E402

s = hip_device_search(L, h, 64)
Q = torch.randn(256, 64, device=dev)
bench("search 100k x 64, 256 q (sampled path)", lambda: s(Q, 10, reuse_outputs=True), n=300)
