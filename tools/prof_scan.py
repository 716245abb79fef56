#!/usr/bin/env python3
"""Development-only: per-phase cycle breakdown of the scan kernel.

Run with a LHIP_PROF=1 build (tools/ablate.sh PROF):
    LANCE_HIP_LIB=abl/lib_PROF.so python tools/prof_scan.py [--n N --dim D --batch B]
Prints, per scan mode (0 dense sample pass, 1 append pass), the average per
wave and per stage / per tile of the s_memtime cycles spent in the DMA wait,
the barrier, the fragment reads + MFMA issue and the epilogue.
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "duckdb-lancedb_amd"))

import lance_hip  # noqa: E402
from bench import gen_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--scan-copy", choices=["on", "off"], default="on")
    ap.add_argument("--scan-i8", choices=["on", "off"], default="on")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = lance_hip.lib()
    if not hasattr(L, "lhip_prof_read"):
        raise SystemExit("not a LHIP_PROF build")
    L.lhip_prof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    e = ctypes.create_string_buffer(2048)
    h = L.lance_create_detached(b"", a.dim, b"l2", b"prof", e, 2048)
    lance_hip.LanceHipSetOption(h, "reserve_rows", str(a.n))
    lance_hip.LanceHipSetOption(h, "scan_copy", a.scan_copy)
    lance_hip.LanceHipSetOption(h, "scan_i8", a.scan_i8)
    for lo in range(0, a.n, 1 << 18):
        hi = min(a.n, lo + (1 << 18))
        X = gen_rows(lo, hi, a.dim, dev)
        torch.cuda.synchronize()
        if L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, a.dim, e, 2048) < 0:
            raise RuntimeError(e.value.decode())
        del X
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    Q = torch.randn((a.batch, a.dim), generator=g, device=dev, dtype=torch.float32)
    from lance_hip.sharded import hip_device_search

    search = hip_device_search(L, h, a.dim)
    search(Q, a.k)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 24)()
    L.lhip_prof_read(buf, 1)
    for _ in range(a.iters):
        search(Q, a.k)
    torch.cuda.synchronize()
    L.lhip_prof_read(buf, 1)
    for mode in (0, 1):
        v = [buf[mode * 8 + i] for i in range(8)]
        waves, stages, tiles = v[4], v[5], v[6]
        if waves == 0:
            continue
        print(f"mode {mode}: waves {waves // a.iters}/launch, stages/wave {stages / waves:.1f}, "
              f"tiles/wave {tiles / waves:.2f}")
        print(f"  survivors {buf[16 + mode * 2] / a.iters:.0f}/launch ({buf[16 + mode * 2] / max(tiles, 1):.1f} per wave-tile), "
              f"list overflow {buf[17 + mode * 2] / a.iters:.0f}/launch; survivor write path "
              f"{buf[20 + mode * 2] / max(waves, 1):.0f} cyc/wave over {buf[21 + mode * 2] / max(waves, 1):.1f} entries")
        tot = sum(v[:4])
        for name, x in zip(("wait", "barrier", "mfma", "epilogue"), v[:4]):
            print(f"  {name:9s} {x / waves:12.0f} cyc/wave  {100.0 * x / tot:5.1f}%  "
                  f"{x / max(stages, 1):8.0f} cyc/stage  {x / max(tiles, 1):9.0f} cyc/tile")
    lance_hip.LanceFreeDetached(h)


if __name__ == "__main__":
    main()
