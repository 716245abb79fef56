#!/usr/bin/env python3
"""Copies a closing run's evidence from gpurun_out/ into profiles/ (tracked):
the bench JSON lines, rocprofv3 kernel stats, the scan kernel's PMC traffic
(tools/pmc_traffic.py: FETCH_SIZE x2 per MI355X_MICROARCH.md 'HBM') and a
summary of its SQ / TCC / LDS counters with the derived rates.

usage: tools/collect_round.py TAG OUT_PREFIX   (e.g. r03f r03)
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def last_json(path):
    line = None
    with open(path) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = ln
    return json.loads(line) if line else None


def counters(d, kernel_sub):
    """per-launch averages of every counter in a rocprofv3 --pmc directory"""
    acc, disp = defaultdict(float), set()
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kernel_sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    return {k: v / n for k, v in acc.items()}, len(disp)


def main():
    tag, out = sys.argv[1], sys.argv[2]
    os.makedirs(P, exist_ok=True)
    for log in sorted(glob.glob(os.path.join(G, f"{tag}_bench_*.log")) + glob.glob(os.path.join(G, f"{tag}_rank_*.log"))):
        j = last_json(log)
        if j:
            name = os.path.basename(log)[len(tag) + 1:-4]
            with open(os.path.join(P, f"{out}_{name}.json"), "w") as f:
                json.dump(j, f, indent=1)
    for d in sorted(glob.glob(os.path.join(G, f"{tag}_prof_*"))):
        if os.path.isdir(d) and os.path.exists(os.path.join(d, "run_kernel_stats.csv")):
            shutil.copy(os.path.join(d, "run_kernel_stats.csv"),
                        os.path.join(P, f"{out}_{os.path.basename(d)[len(tag) + 6:]}_kernel_stats.csv"))
    shapes = {"c2": (1_000_000, 768, 256), "nstar": (10_000_000, 768, 256)}
    for cfg, (n, dim, batch) in shapes.items():
        fd, wd = os.path.join(G, f"{tag}_pmc_{cfg}_fetch"), os.path.join(G, f"{tag}_pmc_{cfg}_write")
        if os.path.isdir(fd) and os.path.isdir(wd):
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), fd, wd,
                            os.path.join(P, f"{out}_{cfg}_scan_traffic.json"), "--n", str(n), "--dim", str(dim),
                            "--batch", str(batch), "--elem-bytes", "1", "--kernel", "scan8_kernel",
                            "--bench-kernel", "scan8_kernel<L2,append,i8>"], check=True)
        summ = {"kernel": "scan8_kernel", "config": cfg}
        for grp in ("tcc", "sq", "lds"):
            d = os.path.join(G, f"{tag}_pmc_{cfg}_{grp}")
            if os.path.isdir(d):
                c, nd = counters(d, "scan8_kernel")
                summ[grp] = {"dispatches": nd, **{k: round(v, 1) for k, v in c.items()}}
        if "tcc" in summ:
            t = summ["tcc"]
            summ["l2_hit_rate"] = round(t["TCC_HIT_sum"] / max(t["TCC_HIT_sum"] + t["TCC_MISS_sum"], 1), 4)
        if "sq" in summ:
            s = summ["sq"]
            # GRBM_GUI_ACTIVE sums the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES sums the 1024 SIMDs
            gui = s["GRBM_GUI_ACTIVE"] / 8.0
            summ["mfma_busy_frac"] = round(s["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / gui, 4)
            wc = s["SQ_WAVE_CYCLES"]
            summ["wave_cycle_split"] = {"issue_stall": round(s["SQ_WAIT_INST_ANY"] / wc, 3),
                                        "waitcnt_parked": round(s["SQ_WAIT_ANY"] / wc, 3),
                                        "active": round(s["SQ_ACTIVE_INST_ANY"] / wc, 3)}
        if "lds" in summ:
            l = summ["lds"]
            summ["lds_conflict_cycles_per_inst"] = round(l["SQ_LDS_BANK_CONFLICT"] / max(l["SQ_INSTS_LDS"], 1), 4)
        if len(summ) > 2:
            with open(os.path.join(P, f"{out}_{cfg}_scan_pmc.json"), "w") as f:
                json.dump(summ, f, indent=1)
    print("\n".join(sorted(os.path.basename(x) for x in glob.glob(os.path.join(P, f"{out}_*")))))


if __name__ == "__main__":
    main()
