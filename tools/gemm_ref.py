#!/usr/bin/env python3
"""Development-only: time the library (hipBLASLt via torch.matmul) GEMM of the
scan's shape, rows[N][D] bf16 x queries[D][B] bf16 -> [N][B] bf16, as a
reference for the MFMA throughput a tuned GEMM reaches on this shape."""
import sys

import torch

N, D, B = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (1_000_000, 768, 256)))
X = torch.randn(N, D, device="cuda", dtype=torch.bfloat16)
Q = torch.randn(D, B, device="cuda", dtype=torch.bfloat16)
Y = torch.empty(N, B, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    torch.matmul(X, Q, out=Y)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
it = 20
e0.record()
for _ in range(it):
    torch.matmul(X, Q, out=Y)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / it
fl = 2.0 * N * D * B
print(f"N={N} D={D} B={B}: {ms:.4f} ms  {fl / ms / 1e9:.1f} TFLOP/s  "
      f"X stream {N * D * 2 / ms / 1e6:.1f} GB/s  + Y write {N * B * 2 / ms / 1e6:.1f} GB/s")
