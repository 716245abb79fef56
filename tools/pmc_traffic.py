#!/usr/bin/env python3
"""Turns rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (run separately, as
/opt/skills/guides/MI355X_MICROARCH.md 'HBM' prescribes) into the per-launch HBM
traffic of the scan kernel, for bench.py's roofline.traffic.

gfx950 correction (same guide): FETCH_SIZE reports exactly half the bytes of a
wide coalesced streaming read (16 B/lane, global_load and *_lds alike) -> x2;
WRITE_SIZE is exact for 16 B/lane stores (other widths uncalibrated).  Both
counters are in KiB.

usage: tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json --n N --dim D --batch B
"""
import argparse
import csv
import json
import os


def per_launch(path, counter, kernel_sub):
    vals = []
    with open(os.path.join(path, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and kernel_sub in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--dim", type=int, required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--elem-bytes", type=int, default=4, help="bytes per element the scan streams")
    ap.add_argument("--kernel", default="scan_kernel<0, 1>")
    ap.add_argument("--bench-kernel", default=None, help="bench.py's roofline.kernel name the passes belong to")
    ap.add_argument("--fetch-factor", type=float, default=2.0,
                    help="bytes per FETCH_SIZE byte of this kernel's access pattern (2.0: 16-B/lane streams, "
                         "MI355X_MICROARCH.md 'HBM'; the PQ scan's 12-B/lane row stream: profiles/r06b_fetch_calib.json)")
    a = ap.parse_args()
    fk, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    wk, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel)
    read_b = a.fetch_factor * fk * 1024.0
    write_b = wk * 1024.0
    out = {"kernel": a.kernel, "n": a.n, "dim": a.dim, "batch": a.batch, "scan_elem_bytes": a.elem_bytes, "launches": [nf, nw],
           "fetch_size_kib_per_launch": fk, "write_size_kib_per_launch": wk,
           "hbm_read_bytes_corrected": read_b, "hbm_write_bytes": write_b,
           "traffic_bytes_per_launch": read_b + write_b,
           "correction": f"FETCH_SIZE x{a.fetch_factor:g} (gfx950 wide-read undercount, calibrated for this access pattern), "
                         "WRITE_SIZE as is; KiB -> bytes"}
    if a.bench_kernel:
        out["bench_kernel"] = a.bench_kernel
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
