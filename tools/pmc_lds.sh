#!/bin/bash
# Development-only (GPU box): SQ LDS counters of the append scan for base vs NOLISTWRITE
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base NOLISTWRITE; do
	L=abl/lib_$v.so; [ "$v" = base ] && L=duckdb-lancedb_amd/lib/liblancedb_hip.so
	for c in "SQ_INSTS_LDS SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_SALU SQ_INSTS_VALU"; do
		LANCE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --pmc $c -d gpurun_out/pmc_$v -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-recall > /dev/null 2>&1 || exit 1
		python3 - "$v" "$c" <<'PY'
import csv, glob, sys
v, cs = sys.argv[1], sys.argv[2].split()
f = sorted(glob.glob(f"gpurun_out/pmc_{v}/**/*counter_collection.csv", recursive=True))[-1]
acc = {}
for r in csv.DictReader(open(f)):
    if "scan_kernel<0, 1, true>" in r["Kernel_Name"] and r["Counter_Name"] in cs:
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(v, {k: f"{sum(x)/len(x):.4g}" for k, x in acc.items()})
PY
		rm -rf gpurun_out/pmc_$v
	done
done
